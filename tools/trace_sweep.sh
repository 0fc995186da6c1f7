#!/bin/bash
# trace pool / refill sweep on C2 (bench stages_ms.trace)
mkdir -p gpurun_out/sw
for cfg in "64 32" "128 16" "128 32" "96 16" "128 8" "256 16" "192 24"; do
  set -- $cfg
  PM_TRACE_WAVE_PATHS=$1 PM_TRACE_REFILL_MIN=$2 timeout -k 10 120 python bench.py --no-cpu-baseline --no-census --steps 20 --warmup 3 > gpurun_out/sw/b_$1_$2.json 2>/dev/null || exit $?
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/sw/b_$1_$2.json').read().strip().splitlines()[-1]); print('$1 $2', d['value'], d['stages_ms'])"
done
