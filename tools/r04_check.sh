# full GPU suite + C2 / C3 / C5 / C2-kNN bench lines at the current sources
# and the C3 / C5 lines of the no-cooperative-scan variant (lib/variants, if built)
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r04_check}; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" | tee -a $O/steps.log
case $rc in 0|1) ;; *) exit $rc ;; esac   # a crash or time limit: nothing more on the GPU
for c in c2 c3 c5; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || exit $?
done
V=$R/cuda-raytrace_amd/lib/variants/libpmhip_nocoop.so
if [ -f $V ]; then
  for c in c3 c5; do
    PMHIP_LIB=$V timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_${c}_nocoop.json 2> $O/bench_${c}_nocoop.err || exit $?
  done
fi
timeout -k 10 300 python bench.py --estimator knn --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_c2_knn.json 2> $O/bench_c2_knn.err
