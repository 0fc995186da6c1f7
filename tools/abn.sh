# Same-box A/B/n of variant libraries on one bench config, alternated REPS times.
# usage: bash tools/abn.sh TAG CONFIG REPS "VARIANTS" [extra bench args]
#   VARIANTS: space-separated names; "base" is the default library, any other
#   name X runs with PMHIP_LIB=cuda-raytrace_amd/lib/variants/libpmhip_X.so
# writes gpurun_out/abn_TAG/<name>_<i>.json and summary.txt (value, ms/step, stage ms)
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/abn_$1; mkdir -p $O; cd $R
CFG=$2; REPS=$3; VS=$4; shift 4
for i in $(seq 1 $REPS); do
  for v in $VS; do
    L=""; [ $v != base ] && L="PMHIP_LIB=$R/cuda-raytrace_amd/lib/variants/libpmhip_$v.so"
    env $L timeout -k 10 300 python bench.py --config $CFG --steps 20 --warmup 3 --no-cpu-baseline --no-census "$@" \
      > $O/${v}_$i.json 2> $O/${v}_$i.err || exit $?
  done
done
python - $O <<'PY' > $O/summary.txt
import glob, json, os, sys
o = sys.argv[1]
for f in sorted(glob.glob(os.path.join(o, "*.json"))):
    d = json.load(open(f))
    print(os.path.basename(f), d["value"], d["ms_per_step"], d["stages_ms"])
PY
cat $O/summary.txt
