#!/bin/bash
# GPU suite + smoke at the current sources, then the tile-gather block-size A/B
# (lib/variants/libpmhip_tb64 / _tb128 vs the default 256-thread blocks) at C2, C3, C5.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; O=gpurun_out/tb; mkdir -p $O
if [ "${PM_TESTS:-1}" = 1 ]; then
  timeout -k 10 500 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
fi
bash tools/variant_bench.sh default ${TB_VARIANTS:-tb64 tb128} default ${TB_VARIANTS:-tb64} || exit $?
for c in c3 c5; do bash tools/variant_bench_cfg.sh $c default ${TB_VARIANTS:-tb64} default || exit $?; done
