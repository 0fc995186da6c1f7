#!/bin/bash
# Pooled trace with dynamic chunks from a global counter (PM_POOL_CHUNK) vs static pools: parity, C3 A/B.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out/chunk
PM_POOL_CHUNK=64 timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_bvh_gpu.py -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -k "c3_full or soup or renders_as or write_modes" > gpurun_out/chunk/pytest.log 2>&1
rc=$?; echo "[pytest chunk 64] rc=$rc"; tail -3 gpurun_out/chunk/pytest.log; [ $rc -ne 0 ] && exit $rc
BENCH_ARGS="--config c3 --no-census" bash tools/gpu_quick.sh chunk "" "PM_X=1" "PM_POOL_CHUNK=64" "PM_POOL_CHUNK=128" "PM_POOL_CHUNK=32" "PM_X=2" "PM_POOL_CHUNK=64 PM_POOL_WAVES=10240"
