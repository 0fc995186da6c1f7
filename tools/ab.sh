# Same-box A/B of two environments on one bench config, alternated REPS times
# (box-to-box spread is +-2-4 %, so A/Bs are only compared within one call).
# usage: bash tools/ab.sh TAG CONFIG REPS "ENV_A" "ENV_B" [extra bench args]
#   e.g. bash tools/ab.sh box c2 3 "PM_TILE_BOX=1" "PM_TILE_BOX=0"
#        bash tools/ab.sh coop c3 2 "" "PMHIP_LIB=cuda-raytrace_amd/lib/variants/libpmhip_nocoop.so"
# writes gpurun_out/ab_TAG/{a,b}_<i>.json and summary.txt (value, ms/step, stage ms)
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/ab_$1; mkdir -p $O; cd $R
CFG=$2; REPS=$3; EA=$4; EB=$5; shift 5
for i in $(seq 1 $REPS); do
  for v in a b; do
    if [ $v = a ]; then E=$EA; else E=$EB; fi
    env $E timeout -k 10 300 python bench.py --config $CFG --steps 20 --warmup 3 --no-cpu-baseline --no-census "$@" \
      > $O/${v}_$i.json 2> $O/${v}_$i.err || exit $?
  done
done
python - $O <<'EOF' > $O/summary.txt
import glob, json, os, sys
o = sys.argv[1]
for f in sorted(glob.glob(os.path.join(o, "*.json"))):
    d = json.load(open(f))
    print(os.path.basename(f), d["value"], d["ms_per_step"], d["stages_ms"])
EOF
cat $O/summary.txt
