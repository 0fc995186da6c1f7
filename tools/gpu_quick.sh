#!/bin/bash
# Short GPU iteration: selected GPU tests, then bench lines under given env
# settings. Stops at the first crash / timeout (never retries a GPU step).
# usage: tools/gpu_quick.sh TAG "pytest -k expr" "ENV=.. ENV2=.." ["ENV=.." ...]
set -u
TAG=$1; K=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread -k "$K" > "$O/pytest.log" 2>&1
  rc=$?; echo "[pytest] rc=$rc" | tee -a "$O/steps.log"; tail -3 "$O/pytest.log"
  [ $rc -ne 0 ] && exit $rc
fi
i=0
for envs in "$@"; do
  i=$((i+1))
  env $envs timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > "$O/bench$i.json" 2> "$O/bench$i.err"
  rc=$?; echo "[bench$i $envs] rc=$rc" | tee -a "$O/steps.log"
  [ $rc -ne 0 ] && exit $rc
  python3 -c "import json;d=json.load(open('$O/bench$i.json'));print('$envs', d['value'], d['ms_per_step'], d['stages_ms'], d['roofline']['avg_launch_ms'] if d.get('roofline') else None)"
done
exit 0
