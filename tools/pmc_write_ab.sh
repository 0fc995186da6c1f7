#!/bin/bash
# WRITE_SIZE per kernel launch under env settings (one rocprofv3 --pmc pass
# each, bench.py --steps 5): A/B of write traffic (e.g. PM_TRACE_HOLD=0/1).
# usage: tools/pmc_write_ab.sh TAG CONFIG "ENV=.." ["ENV=.." ...]
set -u
TAG=$1; CFG=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
i=0
for envs in "$@"; do
  i=$((i+1))
  cd /tmp
  env $envs timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$O/w$i" -o run --output-format csv -- python3 "$R/bench.py" --config "$CFG" --steps 5 --warmup 1 --no-cpu-baseline --no-census > "$O/w$i.log" 2>&1
  rc=$?; echo "[pmc_write $i $envs] rc=$rc" | tee -a "$O/steps.log"
  [ $rc -ne 0 ] && exit $rc
  cd "$R"
  python3 - "$O/w$i" "$envs" <<'PY'
import csv, glob, os, sys
from collections import defaultdict
v = defaultdict(list)
for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        if row.get("Counter_Name") == "WRITE_SIZE":
            v[row["Kernel_Name"].split("(")[0]].append(float(row["Counter_Value"]))
for k, xs in sorted(v.items()):
    print(sys.argv[2], k[:60], "launches", len(xs), "MB/launch %.2f" % (sum(xs) / len(xs) * 1024 / 1e6))
PY
done
