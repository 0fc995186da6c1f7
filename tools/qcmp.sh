# same-box A/B on C3 under two environment settings: tools/qcmp.sh "ENV_A=.." "ENV_B=.."
set -u
O=gpurun_out/${QTAG:-q3}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread -k "soup or figure or killeroo or c3_full or scene_parity or photon_trace or eye" > $O/pytest.log 2>&1 || exit $?
b() { n=$1; shift; env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-census $BA > $O/$n.json 2> $O/$n.err || exit $?; python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n', d['value'], d['ms_per_step'], d['stages_ms'])" | tee -a $O/summary.txt; }
BA="--config c3"; b A1 $1; b B1 $2; b A2 $1; b B2 $2
