for v in default gm4 gm24; do
  if [ $v = default ]; then L=cuda-raytrace_amd/lib/libpmhip.so; else L=cuda-raytrace_amd/lib/variants/libpmhip_$v.so; fi
  for c in c3 c2; do
    PMHIP_LIB=$L timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-census --steps 10 --warmup 2 > gpurun_out/var/$v$c.json 2>/dev/null || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/var/$v$c.json').read().strip().splitlines()[-1]); print('$v $c', d['value'], d['stages_ms'])"
  done
done
PM_GATHER_KERNEL=lane timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --no-census --steps 10 --warmup 2 | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('lane c3', d['value'], d['stages_ms'])"
