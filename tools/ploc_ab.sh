#!/bin/bash
# C3 trace on the host PLOC tree (radius sweep) vs the SAH tree.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
BENCH_ARGS="--config c3 --no-census" bash tools/gpu_quick.sh ploc "" "PM_X=1" "PM_BVH_BUILD=ploc-host PM_PLOC_RADIUS=1" "PM_BVH_BUILD=ploc-host PM_PLOC_RADIUS=2" "PM_BVH_BUILD=ploc-host PM_PLOC_RADIUS=3" "PM_BVH_BUILD=ploc-host PM_PLOC_RADIUS=4" "PM_X=2"
