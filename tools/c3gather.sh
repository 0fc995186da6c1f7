# C3 gather: tile-kernel event counts and same-box group-parameter variants
set -u
O=gpurun_out/c3g; mkdir -p $O
PMHIP_LIB=cuda-raytrace_amd/lib/variants/libpmhip_tstats.so timeout -k 10 300 python tools/tile_stats.py c3 > $O/tstats_c3.txt 2>&1 || exit $?
V=cuda-raytrace_amd/lib/variants
CFG=c3 QTAG=c3g bash tools/envcmp.sh X=1 PMHIP_LIB=$V/libpmhip_g12.so PMHIP_LIB=$V/libpmhip_r2.so PMHIP_LIB=$V/libpmhip_r1.so || exit $?
