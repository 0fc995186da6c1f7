#!/bin/bash
# Round-3 A/B session: GPU suite, held trace deposits (PM_TRACE_HOLD) on C2,
# adaptive grid radius (PM_GRID_QUANTILE) on C5, trace write traffic.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_quick.sh ab "${AB_TESTS:-not test_c2_full_knn}" "PM_TRACE_HOLD=1" "PM_TRACE_HOLD=0" "PM_TRACE_HOLD=1" "PM_TRACE_HOLD=0" || exit $?
BENCH_ARGS="--config c5" bash tools/gpu_quick.sh abc5 "" "PM_GRID_QUANTILE=0" "PM_GRID_QUANTILE=0.99" "PM_GRID_QUANTILE=0.95" "PM_GRID_QUANTILE=1" || exit $?
bash tools/pmc_write_ab.sh abw c2 "PM_TRACE_HOLD=1" "PM_TRACE_HOLD=0"
