#!/bin/bash
# C3 trace-stage sweep of the pooled kernel's knobs (one bench per setting).
# usage: tools/trace_pool_sweep.sh "ENV=.. ENV=.." ...
for envs in "$@"; do
  env $envs timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --no-census --steps 5 --warmup 1 \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$envs', d['value'], d['stages_ms']['trace'])" || exit $?
done
