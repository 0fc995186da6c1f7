# Gather diagnostics at C2 / C3 / C5 from the variant builds (if built):
# phase clocks (libpmhip_gprof.so, tools/gather_profile.py) and event counts
# (libpmhip_tstats.so, tools/tile_stats.py), into gpurun_out/TAG/.
#   make -C cuda-raytrace_amd variant NAME=gprof VFLAGS=-DPM_GATHER_PROFILE
#   make -C cuda-raytrace_amd variant NAME=tstats VFLAGS=-DPM_TILE_STATS
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-gather_diag}; mkdir -p $O; cd $R
V=$R/cuda-raytrace_amd/lib/variants
for c in c2 c3 c5; do
  PMHIP_LIB=$V/libpmhip_gprof.so timeout -k 10 300 python tools/gather_profile.py $c >> $O/gather_phases.txt 2>> $O/diag.err || exit $?
  PMHIP_LIB=$V/libpmhip_tstats.so timeout -k 10 300 python tools/tile_stats.py $c > $O/tile_stats_$c.txt 2>> $O/diag.err || exit $?
done
cat $O/gather_phases.txt
