# bench.py's N > 1 paths rehearsed on a one-GPU box: two ranks on device 0
# over gloo (PM_BENCH_ONE_DEVICE=1 PM_BENCH_BACKEND=gloo; the exchange moves
# through the host, so its times are not measurements), both exchanges, in
# strong scaling (C4 scene, --total-paths); then the N = 1 strong line.
# usage: bash tools/multi_rank_rehearsal.sh [TAG]
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-rehearsal}; mkdir -p $O; cd $R
for ex in reduce allgather; do
  PM_BENCH_ONE_DEVICE=1 PM_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 4 --warmup 1 --exchange $ex --config c4 \
    --total-paths 1048576 > $O/n2_strong_$ex.out 2> $O/n2_strong_$ex.err || exit $?
  # gloo prints its connection notice on stdout: keep the bench's JSON line
  python3 -c "import sys; print([l for l in open(sys.argv[1]) if l.startswith('{')][-1], end='')" \
    $O/n2_strong_$ex.out > $O/n2_strong_$ex.json || exit $?
done
timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --config c4 --total-paths 1048576 > $O/n1_strong.json 2> $O/n1_strong.err
