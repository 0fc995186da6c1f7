#!/bin/bash
# C5 gather knobs (union cap, grid quantile), C2 under the same union cap, and
# the C4 all-gather per-rank cost.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
V=cuda-raytrace_amd/lib/variants
BENCH_ARGS="--config c5 --no-census" bash tools/gpu_quick.sh c5ab "" "PM_X=1" "PM_GRID_QUANTILE=0.9" "PMHIP_LIB=$V/libpmhip_umax512.so" "PMHIP_LIB=$V/libpmhip_umax512.so PM_GRID_QUANTILE=0.9" "PM_X=2" "PM_GRID_QUANTILE=0.9 PM_X=2" || exit $?
BENCH_ARGS="--config c2 --no-census" bash tools/gpu_quick.sh c2ab "" "PM_X=1" "PMHIP_LIB=$V/libpmhip_umax512.so" "PM_X=2" || exit $?
timeout -k 10 300 python tools/c4_allgather_cost.py 8 > gpurun_out/c5ab/c4_allgather.json 2> gpurun_out/c5ab/c4_allgather.err; echo "[c4 allgather] rc=$?"; cat gpurun_out/c5ab/c4_allgather.json; tail -5 gpurun_out/c5ab/c4_allgather.err
