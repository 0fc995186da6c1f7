# One bench line per config at the committed sources (the lines' roofline
# traffic comes from the committed PMC profiles of the same source hash).
# usage: bash tools/bench_all.sh TAG
set -u
T=${1:-bench_all}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$T; mkdir -p "$O"; cd "$R"
for c in c2 c1 c3 c4 c5; do
  timeout -k 10 600 python bench.py --config $c --steps 20 --warmup 3 > "$O/bench_$c.json" 2> "$O/bench_$c.err" || exit $?
done
timeout -k 10 600 python bench.py --config c2 --estimator knn --steps 20 --warmup 3 > "$O/bench_c2_knn.json" 2> "$O/bench_c2_knn.err" || exit $?
echo done
