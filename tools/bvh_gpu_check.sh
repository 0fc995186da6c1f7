#!/bin/bash
# Device BVH build: its GPU tests, the C3 oracle parity on it, then C3 bench
# lines (setup_s, trace) for the device build (default) and the host SAH build.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/bvhgpu
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_bvh_gpu.py tests/test_gpu_configs.py -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -k "bvh_gpu or c3_full" > $O/pytest.log 2>&1
rc=$?; echo "[pytest] rc=$rc"; tail -12 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
BENCH_ARGS="--config c3 --no-census" PM_COMMIT_TIMES=1 bash tools/gpu_quick.sh bvhgpu "" "PM_X=1" "PM_BVH_BUILD=host" "PM_X=2"
rc=$?; grep -h "pm_commit" $O/bench*.err; for f in $O/bench*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f', d['setup_s'], d['stages_ms'])"; done; exit $rc
