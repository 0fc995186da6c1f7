set -u
O=gpurun_out/r05a; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -k "allgather_map or from_bands or adaptive" > $O/new.log 2>&1; echo "new rc=$?" >> $O/steps.log
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread --durations=15 > $O/pytest.log 2>&1 || { echo "suite rc=$?" >> $O/steps.log; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c2.json 2> $O/c2.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --estimator knn > $O/knn.json 2> $O/knn.err || exit 1
bash tools/abn.sh tile c2 3 "base noloop w4 w4nopf"
