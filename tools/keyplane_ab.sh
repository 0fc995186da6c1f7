#!/bin/bash
# Plane-major fused bucket keys / ranks (PM_KEY_PLANES): parity, bench A/B at C2 and C3, trace WRITE_SIZE.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
BENCH_ARGS="--config c2 --no-census" bash tools/gpu_quick.sh kp2 "write_modes or c2_full or c3_full or kernels_agree or c4_share or c5_prog or dist or group or adaptive" "PM_KEY_PLANES=0" "PM_KEY_PLANES=1" "PM_KEY_PLANES=0" "PM_KEY_PLANES=1" || exit $?
BENCH_ARGS="--config c3 --no-census" bash tools/gpu_quick.sh kp3 "" "PM_KEY_PLANES=0" "PM_KEY_PLANES=1" || exit $?
bash tools/pmc_write_ab.sh kpw c2 "PM_KEY_PLANES=0" "PM_KEY_PLANES=1" || exit $?
bash tools/pmc_write_ab.sh kpw3 c3 "PM_KEY_PLANES=0" "PM_KEY_PLANES=1"
