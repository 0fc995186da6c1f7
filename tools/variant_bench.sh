#!/bin/bash
# C2 bench of experiment builds (make -C cuda-raytrace_amd variant NAME=x VFLAGS=...):
#   tools/variant_bench.sh default x y ...   -> gpurun_out/var/<name>.json + one summary line each
mkdir -p gpurun_out/var
for v in "$@"; do
  if [ "$v" = default ]; then L=cuda-raytrace_amd/lib/libpmhip.so; else L=cuda-raytrace_amd/lib/variants/libpmhip_$v.so; fi
  PMHIP_LIB=$L timeout -k 10 120 python bench.py --no-cpu-baseline --no-census --steps 20 --warmup 3 \
      > gpurun_out/var/$v.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.loads(open('gpurun_out/var/$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['stages_ms'])"
done
