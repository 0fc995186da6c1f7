#!/bin/bash
# Pooled trace with a capped LDS stack (PM_POOL_STACK, deeper entries spilled to global) and forced occupancy variants.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
V=$R/cuda-raytrace_amd/lib/variants
mkdir -p gpurun_out/stk
PM_POOL_STACK=12 timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_bvh_gpu.py -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -k "c3_full or soup or renders_as" > gpurun_out/stk/pytest.log 2>&1
rc=$?; echo "[pytest spill 12] rc=$rc"; tail -3 gpurun_out/stk/pytest.log; [ $rc -ne 0 ] && exit $rc
PMHIP_LIB=$V/libpmhip_eu5.so PM_POOL_STACK=12 timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -k "c3_full" > gpurun_out/stk/pytest2.log 2>&1
rc=$?; echo "[pytest eu5 spill 12] rc=$rc"; tail -3 gpurun_out/stk/pytest2.log; [ $rc -ne 0 ] && exit $rc
BENCH_ARGS="--config c3 --no-census" bash tools/gpu_quick.sh stk "" "PM_X=1" "PM_POOL_STACK=31" "PMHIP_LIB=$V/libpmhip_eu5.so PM_POOL_STACK=31" "PMHIP_LIB=$V/libpmhip_eu5.so PM_POOL_STACK=24" "PMHIP_LIB=$V/libpmhip_eu6.so PM_POOL_STACK=26" "PMHIP_LIB=$V/libpmhip_eu6.so PM_POOL_STACK=20" "PM_X=2"
