#!/bin/bash
# k_gather_tile event counts (PM_TILE_STATS variant) at C2 and C3.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
for c in c2 c3; do
  echo "== $c"
  PMHIP_LIB=$R/cuda-raytrace_amd/lib/variants/libpmhip_tstats.so timeout -k 10 300 python tools/tile_stats.py $c || exit $?
done
