#!/bin/bash
# Wavefront trace (PM_TRACE_WAVEFRONT) parity tests, then the C3 A/B against
# the pooled megakernel: bench lines per setting (stage-timed trace).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; O=gpurun_out/wf; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread \
    -k "${WF_TESTS:-wavefront or write_modes}" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
i=0
for envs in "PM_TRACE_WAVEFRONT=0" ${WF_ARMS:-"PM_TRACE_WAVEFRONT=1" "PM_TRACE_WAVEFRONT=1 PM_WF_SORT=0" "PM_TRACE_WAVEFRONT=1 PM_WF_BITS=3" "PM_TRACE_WAVEFRONT=1 PM_WF_BITS=5"} "PM_TRACE_WAVEFRONT=0"; do
  i=$((i+1))
  env $envs timeout -k 10 300 python bench.py --config ${WF_CFG:-c3} --steps 5 --warmup 1 --no-cpu-baseline --no-census > $O/b$i.json 2> $O/b$i.err
  rc=$?; [ $rc -ne 0 ] && { echo "[$envs] rc=$rc"; tail -5 $O/b$i.err; exit $rc; }
  python3 -c "import json;d=json.loads(open('$O/b$i.json').read().strip().splitlines()[-1]);print('$envs', d['value'], d['stages_ms'])"
done
