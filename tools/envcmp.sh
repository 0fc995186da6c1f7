# same-box bench of one config under several environment settings, each run twice:
#   CFG=c3 QTAG=x tools/envcmp.sh "A=1" "B=2 C=3" ...
set -u
O=gpurun_out/${QTAG:-envcmp}; mkdir -p $O
b() { n=$1; shift; env $@ timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-census --config ${CFG:-c3} > $O/$n.json 2> $O/$n.err || exit $?; python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n', '$*', d['value'], d['ms_per_step'], d['stages_ms'])" | tee -a $O/summary.txt; }
for r in 1 2; do i=0; for e in "$@"; do i=$((i+1)); b s${i}_$r $e; done; done
