#!/bin/bash
# bench one config across experiment builds (lib/variants/libpmhip_<name>.so, "default" = lib/libpmhip.so)
# usage: tools/variant_bench_cfg.sh CONFIG name...   (BENCH_ARGS: extra bench.py arguments)
CFG=$1; shift
mkdir -p gpurun_out/var
for v in "$@"; do
  if [ "$v" = default ]; then L=cuda-raytrace_amd/lib/libpmhip.so; else L=cuda-raytrace_amd/lib/variants/libpmhip_$v.so; fi
  PMHIP_LIB=$L timeout -k 10 300 python bench.py --config $CFG --no-cpu-baseline --no-census --steps 5 --warmup 1 ${BENCH_ARGS:-} \
      > gpurun_out/var/$v.$CFG.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.loads(open('gpurun_out/var/$v.$CFG.json').read().strip().splitlines()[-1]); print('$v $CFG', d['value'], d['stages_ms'])"
done
