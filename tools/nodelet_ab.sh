#!/bin/bash
# C3 trace: LDS nodelets (top BVH4 levels in LDS, breadth-first node order)
# A/B against the depth-first tree without nodelets; soup parity tests first.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
PM_NODELETS=85 bash tools/gpu_quick.sh nl "soup or figure or c3_full or write_modes" || exit $?
BENCH_ARGS="--config c3 --no-census" bash tools/gpu_quick.sh nlc3 "" "PM_NODELETS=0" "PM_BVH4_BFS=1" "PM_NODELETS=21" "PM_NODELETS=85" "PM_NODELETS=341" "PM_NODELETS=0"
