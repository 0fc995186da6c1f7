#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out/grp
timeout -k 10 600 python -u -m pytest tests/test_group_gpu.py tests/test_dist_gpu.py tests/test_pbrt_boundary.py -v -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/grp/pytest.log 2>&1
rc=$?; tail -25 gpurun_out/grp/pytest.log
[ $rc -gt 1 ] && exit $rc
bash tools/nodelet_ab.sh
