# Round-end measurement of every config at the committed sources, in two
# gpurun calls: A = GPU suite, C2 (+ SQ counters), smoke, C2-kNN;
# B = C1, C4, C5, C3 (bench + kernel stats + FETCH/WRITE passes each).
set -u
T=${PM_ROUND:-r03}
case "${1:-A}" in
A)
  PM_TESTS=1 bash tools/gpu_session.sh $T c2 || exit $?
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || exit $?
  PM_SQ=0 PM_NAME=c2_knn bash tools/gpu_session.sh $T c2 --estimator knn || exit $?
  ;;
B)
  for c in c1 c4 c5 c3; do PM_SQ=0 bash tools/gpu_session.sh $T $c || exit $?; done
  ;;
esac
