#!/bin/bash
# Pooled trace: shade threshold (PM_POOL_SHADE_MIN) and steps per decision (PM_POOL_STEPS) variants at C3.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
V=cuda-raytrace_amd/lib/variants
BENCH_ARGS="--config c3 --no-census" bash tools/gpu_quick.sh pool "" "PM_X=1" "PMHIP_LIB=$V/libpmhip_sm8.so" "PMHIP_LIB=$V/libpmhip_sm24.so" "PMHIP_LIB=$V/libpmhip_sm32.so" "PMHIP_LIB=$V/libpmhip_st1.so" "PMHIP_LIB=$V/libpmhip_st2.so" "PMHIP_LIB=$V/libpmhip_st8.so" "PM_X=2"
