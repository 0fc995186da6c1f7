# round 4: kNN histogram A/B + bench N=1 / N=2 rehearsal (weak + strong) on one GPU
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r04_s1; mkdir -p $O; cd $R
L=$R/cuda-raytrace_amd/lib/variants
BENCH_ARGS="--estimator knn" bash tools/gpu_quick.sh r04_s1 "knn_kernels_agree or c2_full_knn" \
  "PMHIP_LIB=$L/libpmhip_pk6.so" "PMHIP_LIB=$L/libpmhip_u4.so" "PMHIP_LIB=$L/libpmhip_u5.so" "PMHIP_LIB=$L/libpmhip_pk6.so" "PMHIP_LIB=$L/libpmhip_u5.so" || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/c2.json 2> $O/c2.err || exit $?
for ex in reduce allgather; do
  PM_BENCH_ONE_DEVICE=1 PM_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 4 --warmup 1 --exchange $ex --config c4 \
    --total-paths 1048576 --no-census > $O/n2_strong_$ex.json 2> $O/n2_strong_$ex.err || exit $?
done
timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --config c4 --total-paths 1048576 > $O/n1_strong.json 2> $O/n1_strong.err
