# Same-box A/B of a run-time switch on one bench config, alternated REPS times,
# plus one WRITE_SIZE PMC pass per arm (the switch's effect on HBM writes).
# usage: bash tools/env_ab.sh TAG CONFIG REPS VAR "VAL_A VAL_B" [extra bench args]
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/env_$1; mkdir -p $O; cd $R
CFG=$2; REPS=$3; VAR=$4; VALS=$5; shift 5
export TMPDIR=/tmp
for i in $(seq 1 $REPS); do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 300 python bench.py --config $CFG --steps 20 --warmup 3 --no-cpu-baseline --no-census "$@" \
      > $O/${v}_$i.json 2> $O/${v}_$i.err || exit $?
  done
done
for v in $VALS; do
  env $VAR=$v timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_w_$v -o run --output-format csv -- python3 $R/bench.py \
    --config $CFG --steps 5 --warmup 1 --no-cpu-baseline --no-census "$@" > $O/pmc_w_$v.log 2>&1 || exit $?
done
python3 - $O "$VALS" <<'PY' > $O/summary.txt
import csv, glob, json, os, sys
from collections import defaultdict
o = sys.argv[1]
for f in sorted(glob.glob(os.path.join(o, "*.json"))):
    d = json.load(open(f)); print(os.path.basename(f), d["value"], d["ms_per_step"], d["stages_ms"])
for v in sys.argv[2].split():
    w = defaultdict(list)
    for f in glob.glob(os.path.join(o, "pmc_w_" + v, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") == "WRITE_SIZE":
                w[row["Kernel_Name"].split("(")[0]].append(float(row["Counter_Value"]))
    for k, x in sorted(w.items()):
        if len(x) >= 5:
            print(f"WRITE_SIZE {v} {k}: {sum(x) / len(x) * 1024 / 1e6:.1f} MB per launch ({len(x)} launches)")
PY
cat $O/summary.txt
