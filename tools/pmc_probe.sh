#!/bin/bash
# Counter passes over a short bench run, one rocprofv3 --pmc invocation per
# pass (each pass its own process; no trace domains combined with --pmc).
# usage: tools/pmc_probe.sh OUTDIR "C1 C2" "C3" ... [-- extra bench args]
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/$1; shift
mkdir -p "$O"
passes=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do passes+=("$1"); shift; done
[ "${1:-}" = "--" ] && shift
export TMPDIR=/tmp
cd /tmp
i=0
for p in "${passes[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $p -d "$O/p$i" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-census "$@" > "$O/p$i.log" 2>&1
  rc=$?
  echo "pass $i ($p) rc=$rc" | tee -a "$O/steps.log"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
