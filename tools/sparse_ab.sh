#!/bin/bash
# k_gather_tile's sparse pass (PM_TILE_SPARSE): parity tests, then C3 / C5 / C2 bench A/B.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
BENCH_ARGS="--config c3 --no-census" bash tools/gpu_quick.sh sp3 "kernels_agree or c3_full or c5_prog or record_order or adaptive_grid or c2_full or c4_share" "PM_TILE_SPARSE=0" "PM_TILE_SPARSE=1" "PM_TILE_SPARSE=0" "PM_TILE_SPARSE=1" || exit $?
BENCH_ARGS="--config c5 --no-census" bash tools/gpu_quick.sh sp5 "" "PM_TILE_SPARSE=0" "PM_TILE_SPARSE=1" "PM_TILE_SPARSE=0" "PM_TILE_SPARSE=1" || exit $?
BENCH_ARGS="--config c2 --no-census" bash tools/gpu_quick.sh sp2 "" "PM_TILE_SPARSE=0" "PM_TILE_SPARSE=1" "PM_TILE_SPARSE=0" "PM_TILE_SPARSE=1"
