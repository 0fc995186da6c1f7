# Round-end measurement of every config at the committed sources: GPU suite,
# smoke, C2 (+ SQ counters) and C2-kNN sessions, then C1, C4, C5, C3.
set -u
PM_TESTS=1 bash tools/gpu_session.sh r02 c2 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02/smoke.log 2>&1 || exit $?
PM_NAME=c2_knn bash tools/gpu_session.sh r02 c2 --estimator knn || exit $?
for c in c1 c4 c5 c3; do PM_SQ=0 bash tools/gpu_session.sh r02 $c || exit $?; done
