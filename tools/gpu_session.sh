#!/bin/bash
# One GPU measurement session for one config: bench, rocprofv3 kernel trace +
# stats of the same bench command, two separate PMC passes (FETCH_SIZE,
# WRITE_SIZE -> per-launch HBM bytes) and SQ/TA counter passes. Stops at the
# first step that crashes / times out (never retries a GPU step).
# usage: tools/gpu_session.sh TAG CONFIG [extra bench args...]
#   PM_TESTS=1  also run the GPU test suite first
#   PM_NAME=x   file-name suffix instead of CONFIG (runs with extra args, e.g. c2_knn)
set -u
TAG=${1:-r02}; CFG=${2:-c2}; shift 2 || true
N=${PM_NAME:-$CFG}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
ok() {  # tolerate ordinary failures (exit 1/2: test failures), stop on crashes/timeouts
  local rc=$1 name=$2
  echo "[$name] exit=$rc" | tee -a "$O/steps.log"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ] && [ "$rc" -ne 2 ]; then echo "stopping after $name" | tee -a "$O/steps.log"; exit "$rc"; fi
}
cd "$R"
if [ "${PM_TESTS:-0}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1; ok $? pytest
fi
B="--config $CFG $*"
timeout -k 10 900 python bench.py --steps 20 --warmup 3 $B > "$O/bench_$N.json" 2> "$O/bench_$N.err"; ok $? bench
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/prof_$N" -o run --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline $B > "$O/prof_$N.log" 2>&1; ok $? rocprof_stats
find "$O/prof_$N" -name '*kernel_stats.csv' -exec cp {} "$O/kernel_stats_$N.csv" \;
[ "${PM_QUICK:-0}" = "1" ] && { echo done | tee -a "$O/steps.log"; exit 0; }
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_fetch_$N" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-census $B > "$O/pmc_fetch_$N.log" 2>&1; ok $? pmc_fetch
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d "$O/pmc_write_$N" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-census $B > "$O/pmc_write_$N.log" 2>&1; ok $? pmc_write
cd "$R"
python3 tools/pmc_traffic.py "$O/pmc_fetch_$N" "$O/pmc_write_$N" "$O/pmc_traffic_$N.json" "$CFG" > /dev/null 2>&1; ok $? pmc_summary
if [ "${PM_SQ:-1}" = "1" ]; then
  P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
  P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
  P3="TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum"
  bash tools/pmc_probe.sh "gpurun_out/$TAG/sq_$N" "$P1" "$P2" "$P3" -- $B; ok $? pmc_sq
  python3 tools/pmc_table.py "gpurun_out/$TAG/sq_$N" > "$O/counters_$N.txt"; ok $? pmc_table
fi
echo done | tee -a "$O/steps.log"
