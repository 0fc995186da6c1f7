# same-box A/B of trace builds on C3 (default library vs lib/variants/libpmhip_$1.so)
set -u
O=gpurun_out/q2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread -k "soup or figure or killeroo or c3_full or scene_parity or photon_trace" > $O/pytest.log 2>&1 || exit $?
b() { n=$1; shift; env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-census $BA > $O/$n.json 2> $O/$n.err || exit $?; python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n', d['value'], d['ms_per_step'], d['stages_ms'])" | tee -a $O/summary.txt; }
V=cuda-raytrace_amd/lib/variants/libpmhip_$1.so
BA="--config c3"; b c3_def X=1; b c3_$1 PMHIP_LIB=$V; b c3_def2 X=1; b c3_${1}2 PMHIP_LIB=$V
