/* pbrt-v2 lights/diffuse.h -> the boundary stub (see ../pbrt_stub.h) */
#pragma once
#include "../pbrt_stub.h"
