/* pbrt-v2 core/pbrt.h -> the boundary stub (see ../pbrt_stub.h) */
#pragma once
#include "../pbrt_stub.h"
