/* pbrt-v2 shapes/trianglemesh.h -> the boundary stub (see ../pbrt_stub.h) */
#pragma once
#include "../pbrt_stub.h"
