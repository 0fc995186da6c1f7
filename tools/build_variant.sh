# Builds cuda-raytrace_amd/lib/variants/libpmhip_NAME.so from the current
# sources with extra compile flags (A/B runs: tools/ab_multi.sh NAME specs).
# usage: bash tools/build_variant.sh NAME "-DPM_X=1 -DPM_Y=2"
set -eu
NAME=$1; DEFS=${2:-}
R=$(cd "$(dirname "$0")/.." && pwd)
P=$R/cuda-raytrace_amd
B=$P/build/v_$NAME
mkdir -p "$B" "$P/lib/variants"
HIPCC=/opt/rocm/bin/hipcc
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-function -Wno-unused-result -I$R/include"
PIDS=""
for f in pm_trace pm_bucket pm_gather pm_bvh_gpu; do
  X=""; [ $f = pm_trace ] && X="-fno-slp-vectorize"
  $HIPCC $F $X $DEFS -c "$P/csrc/$f.hip" -o "$B/$f.o" & PIDS="$PIDS $!"
done
$HIPCC $F $DEFS -x hip -c "$P/csrc/pm_api.cpp" -o "$B/pm_api.o" & PIDS="$PIDS $!"
$HIPCC -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -I$R/include $DEFS -c "$P/csrc/pm_build.cpp" -o "$B/pm_build.o" & PIDS="$PIDS $!"
for p in $PIDS; do wait $p; done
$HIPCC -shared --offload-arch=gfx950 -fPIC -o "$P/lib/variants/libpmhip_$NAME.so" \
  "$B"/pm_trace.o "$B"/pm_bucket.o "$B"/pm_gather.o "$B"/pm_bvh_gpu.o "$B"/pm_api.o "$B"/pm_build.o \
  -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "built $P/lib/variants/libpmhip_$NAME.so"
