#!/bin/bash
# Tile gather test-loop unroll (PM_TEST_UNROLL 1/2/4/8: 4 = 110 VGPRs, 4 waves/SIMD; others 95-96 VGPRs, 5 waves).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
V=cuda-raytrace_amd/lib/variants
BENCH_ARGS="--config c2 --no-census" bash tools/gpu_quick.sh un2 "" "PM_X=1" "PMHIP_LIB=$V/libpmhip_u2.so" "PMHIP_LIB=$V/libpmhip_u8.so" "PMHIP_LIB=$V/libpmhip_u1.so" "PM_X=2" "PMHIP_LIB=$V/libpmhip_u2.so" "PMHIP_LIB=$V/libpmhip_u8.so" || exit $?
BENCH_ARGS="--config c3 --no-census" bash tools/gpu_quick.sh un3 "" "PM_X=1" "PMHIP_LIB=$V/libpmhip_u2.so" "PMHIP_LIB=$V/libpmhip_u8.so" || exit $?
BENCH_ARGS="--config c5 --no-census" bash tools/gpu_quick.sh un5 "" "PM_X=1" "PMHIP_LIB=$V/libpmhip_u2.so" "PMHIP_LIB=$V/libpmhip_u8.so"
