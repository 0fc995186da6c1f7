#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_quick.sh ab3 "adaptive_grid or record_order or write_modes or c5_progressive or kernels_agree" "PM_GRID_QUANTILE=0.99" "PM_GRID_QUANTILE=0" "PM_TRACE_HOLD=0" || exit $?
BENCH_ARGS="--config c5" bash tools/gpu_quick.sh ab3c5 "" "PM_GRID_QUANTILE=0" "PM_GRID_QUANTILE=0.99" "PM_GRID_QUANTILE=0.9"
