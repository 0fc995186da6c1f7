#!/bin/bash
# Tile gather: paired LDS positions + sign-bit masks (default; pw5 variant: 5 waves/SIMD forced) vs SoA variant.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
V=cuda-raytrace_amd/lib/variants
BENCH_ARGS="--config c2 --no-census" bash tools/gpu_quick.sh pr2 "kernels_agree or nan_photons or c2_full or c3_full or c5_prog or adaptive" "PMHIP_LIB=$V/libpmhip_soa.so" "PM_X=1" "PMHIP_LIB=$V/libpmhip_pw5.so" "PMHIP_LIB=$V/libpmhip_soa.so" "PM_X=1" "PMHIP_LIB=$V/libpmhip_pw5.so" || exit $?
BENCH_ARGS="--config c5 --no-census" bash tools/gpu_quick.sh pr5 "" "PMHIP_LIB=$V/libpmhip_soa.so" "PM_X=1" "PMHIP_LIB=$V/libpmhip_pw5.so" || exit $?
BENCH_ARGS="--config c3 --no-census" bash tools/gpu_quick.sh pr3 "" "PMHIP_LIB=$V/libpmhip_soa.so" "PM_X=1" "PMHIP_LIB=$V/libpmhip_pw5.so"
