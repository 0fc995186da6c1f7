# Same-box A/B of the cost-sorted tile list (PM_TILE_SORT=1, default) against
# record order (PM_TILE_SORT=0) on a bench config, alternated REPS times.
# usage: bash tools/sort_ab.sh TAG CONFIG REPS [extra bench args]
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/sort_$1; mkdir -p $O; cd $R
CFG=$2; REPS=$3; shift 3
for i in $(seq 1 $REPS); do
  for v in 1 0; do
    PM_TILE_SORT=$v timeout -k 10 300 python bench.py --config $CFG --steps 20 --warmup 3 --no-cpu-baseline --no-census "$@" \
      > $O/sort${v}_$i.json 2> $O/sort${v}_$i.err || exit $?
  done
done
python3 - $O <<'PY' > $O/summary.txt
import glob, json, os, sys
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.json"))):
    d = json.load(open(f)); print(os.path.basename(f), d["value"], d["ms_per_step"], d["stages_ms"], d["roofline"]["avg_launch_ms"])
PY
cat $O/summary.txt
