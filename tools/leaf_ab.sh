#!/bin/bash
# Pooled trace leaf batching (PM_POOL_LEAF_MIN): C3 parity with it on, then C3 bench A/B.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out/leaf
PM_POOL_LEAF_MIN=32 timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_bvh_gpu.py -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -k "c3_full or soup or renders_as" > gpurun_out/leaf/pytest.log 2>&1
rc=$?; echo "[pytest] rc=$rc"; tail -3 gpurun_out/leaf/pytest.log; [ $rc -ne 0 ] && exit $rc
BENCH_ARGS="--config c3 --no-census" bash tools/gpu_quick.sh leaf "" "PM_POOL_LEAF_MIN=0" "PM_POOL_LEAF_MIN=16" "PM_POOL_LEAF_MIN=32" "PM_POOL_LEAF_MIN=48" "PM_POOL_LEAF_MIN=0" "PM_POOL_LEAF_MIN=24"
