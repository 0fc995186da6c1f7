# Same-box comparison of library variants on one bench config, alternated REPS times.
# usage: bash tools/abn_libs.sh TAG CONFIG REPS "name1 name2 ..."   (name "base" = the default library)
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/abn_$1; mkdir -p $O; cd $R
CFG=$2; REPS=$3; NAMES=$4
for i in $(seq 1 $REPS); do
  for v in $NAMES; do
    if [ $v = base ]; then E=""; else E="PMHIP_LIB=cuda-raytrace_amd/lib/variants/libpmhip_$v.so"; fi
    env $E timeout -k 10 300 python bench.py --config $CFG --steps 20 --warmup 3 --no-cpu-baseline --no-census \
      > $O/${v}_$i.json 2> $O/${v}_$i.err || exit $?
  done
done
python3 - $O <<'PY' > $O/summary.txt
import glob, json, os, sys
o = sys.argv[1]
for f in sorted(glob.glob(os.path.join(o, "*.json"))):
    d = json.load(open(f))
    print(os.path.basename(f), d["value"], d["ms_per_step"], d["stages_ms"])
PY
cat $O/summary.txt
