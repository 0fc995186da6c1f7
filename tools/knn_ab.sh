set -u
L=$PWD/cuda-raytrace_amd/lib/variants
BENCH_ARGS="--estimator knn" bash tools/gpu_quick.sh r04_knn5 "knn" "PM_KNN_SS=1" "PMHIP_LIB=$L/libpmhip_w6.so" "PMHIP_LIB=$L/libpmhip_w7.so" "PM_KNN_SS=1" || exit $?
PMHIP_LIB=$L/libpmhip_tstats.so timeout -k 10 200 python tools/tile_stats.py knn > gpurun_out/r04_knn5/stats.txt 2>&1 || exit $?
PMHIP_LIB=$L/libpmhip_gprof.so timeout -k 10 200 python tools/gather_profile.py knn > gpurun_out/r04_knn5/prof.txt 2>&1
