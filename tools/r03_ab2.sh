#!/bin/bash
# C2 per-step overhead hunt (adaptive-grid histogram / record order) and the
# C3 record-order A/B; record-order GPU tests first.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_quick.sh ab2 "record_order or kernels_agree or write_modes" "PM_GRID_QUANTILE=0 PM_REC_ORDER=0" "PM_GRID_QUANTILE=0.99 PM_REC_ORDER=0" "PM_GRID_QUANTILE=0 PM_REC_ORDER=-1" "PM_TRACE_HOLD=0" || exit $?
BENCH_ARGS="--config c3" bash tools/gpu_quick.sh ab2c3 "" "PM_REC_ORDER=0" "PM_REC_ORDER=1"
