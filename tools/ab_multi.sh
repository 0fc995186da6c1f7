# Same-box A/B/n of (variant library, environment) pairs on one bench config,
# alternated REPS times (box-to-box spread is +-2-4 %: compare within a call).
# usage: bash tools/ab_multi.sh TAG CONFIG REPS SPEC [SPEC...] [-- bench args]
#   SPEC = label[:lib][:ENV=v,ENV=v]   lib "-" or empty = the default library,
#          else cuda-raytrace_amd/lib/variants/libpmhip_<lib>.so
#   e.g. bash tools/ab_multi.sh pf c2 3 base:r05base new new_nopf::PM_TILE_PF=0
# writes gpurun_out/abm_TAG/<label>_<i>.json and summary.txt (value, ms/step,
# event-timed gather launch, stage ms)
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/abm_$1; mkdir -p $O; cd $R
CFG=$2; REPS=$3; shift 3
SPECS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do SPECS+=("$1"); shift; done
[ $# -gt 0 ] && shift
for i in $(seq 1 $REPS); do
  for s in "${SPECS[@]}"; do
    IFS=: read -r label lib envs <<< "$s"
    E=()
    [ -n "$lib" ] && [ "$lib" != "-" ] && E+=("PMHIP_LIB=$R/cuda-raytrace_amd/lib/variants/libpmhip_$lib.so")
    [ -n "${envs:-}" ] && IFS=, read -r -a EV <<< "$envs" && E+=("${EV[@]}")
    env "${E[@]}" timeout -k 10 300 python bench.py --config $CFG --steps 20 --warmup 3 --no-cpu-baseline --no-census "$@" \
      > $O/${label}_$i.json 2> $O/${label}_$i.err || exit $?
  done
done
python - $O <<'PY' > $O/summary.txt
import glob, json, os, sys
o = sys.argv[1]
for f in sorted(glob.glob(os.path.join(o, "*.json"))):
    d = json.load(open(f))
    print(os.path.basename(f), d["value"], d["ms_per_step"], "gather_launch", d["roofline"]["avg_launch_ms"], d["stages_ms"])
PY
cat $O/summary.txt
