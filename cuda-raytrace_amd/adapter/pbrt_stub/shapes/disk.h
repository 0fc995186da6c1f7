/* pbrt-v2 shapes/disk.h -> the boundary stub (see ../pbrt_stub.h) */
#pragma once
#include "../pbrt_stub.h"
