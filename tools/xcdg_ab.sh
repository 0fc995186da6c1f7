#!/bin/bash
# XCD-grouped tile mapping A/B (lib/variants/libpmhip_xg1 = off, xg8; default = 4): C2 / C3 / C5
# bench lines and the C2 gather's FETCH_SIZE per arm
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; O=$R/gpurun_out/xg; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread -k "kernels_agree or c2_full" > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/variant_bench.sh default ${XG_ARMS:-xg1 xg8} default ${XG_ARMS:-xg1 xg8} || exit $?
for c in c3 c5; do bash tools/variant_bench_cfg.sh $c default ${XG_CMP:-xg1} default ${XG_CMP:-xg1} || exit $?; done
for v in default ${XG_PMC:-xg1}; do
  if [ $v = default ]; then L=$R/cuda-raytrace_amd/lib/libpmhip.so; else L=$R/cuda-raytrace_amd/lib/variants/libpmhip_$v.so; fi
  (cd /tmp && PMHIP_LIB=$L timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/f_$v -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-census > $O/f_$v.log 2>&1) || exit $?
  python3 -c "
import csv,glob
v=[float(r['Counter_Value']) for f in glob.glob('$O/f_$v/**/*counter_collection.csv', recursive=True) for r in csv.DictReader(open(f)) if 'k_gather_tile' in r['Kernel_Name'] and r['Counter_Name']=='FETCH_SIZE']
print('$v gather FETCH_SIZE x2 MB per launch', round(2*sum(v)/len(v)*1024/1e6,1), len(v))"
done
