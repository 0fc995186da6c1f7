#!/bin/bash
# HBM bytes of the wavefront trace bounces at C3, sorted vs queue order
# (separate FETCH_SIZE / WRITE_SIZE passes, tools/pmc_traffic.py)
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/wfpmc; mkdir -p $O; export TMPDIR=/tmp
for arm in sort nosort off; do
  case $arm in sort) E="PM_TRACE_WAVEFRONT=1";; nosort) E="PM_TRACE_WAVEFRONT=1 PM_WF_SORT=0";; off) E="PM_TRACE_WAVEFRONT=0";; esac
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && export $E && timeout -k 10 300 rocprofv3 --pmc $c -d $O/${arm}_$c -o run --output-format csv -- python3 $R/bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-census > $O/${arm}_$c.log 2>&1) || exit $?
  done
  python3 $R/tools/pmc_traffic.py $O/${arm}_FETCH_SIZE $O/${arm}_WRITE_SIZE $O/traffic_$arm.json c3 > /dev/null || exit $?
done
