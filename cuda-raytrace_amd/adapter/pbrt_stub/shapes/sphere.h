/* pbrt-v2 shapes/sphere.h -> the boundary stub (see ../pbrt_stub.h) */
#pragma once
#include "../pbrt_stub.h"
