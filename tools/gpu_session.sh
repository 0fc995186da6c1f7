#!/bin/bash
# One GPU session: parity tests, bench, rocprofv3 kernel trace + stats, and
# two separate PMC passes (FETCH_SIZE, WRITE_SIZE). Stops at the first step
# that ends in a crash / fault / timeout (never retries a GPU step).
# usage: tools/gpu_session.sh TAG [extra bench args...]
set -u
TAG=${1:-r01}; shift || true
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
timeout -k 10 900 python -m pytest tests -q -m gpu -p no:cacheprovider > "$O/pytest_gpu.log" 2>&1; ok $? pytest
timeout -k 10 600 python bench.py --steps 20 --warmup 3 "$@" > "$O/bench.json" 2> "$O/bench.err"; ok $? bench
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline "$@" > "$O/prof.log" 2>&1; ok $? rocprof_stats
if [ "${PM_QUICK:-0}" = "1" ]; then
  find "$O/prof" -name '*kernel_stats.csv' -exec cp {} "$O/kernel_stats.csv" \;
  echo done | tee -a "$O/steps.log"; exit 0
fi
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_fetch" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-census "$@" > "$O/pmc_fetch.log" 2>&1; ok $? pmc_fetch
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d "$O/pmc_write" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-census "$@" > "$O/pmc_write.log" 2>&1; ok $? pmc_write
cd "$R"
python3 tools/pmc_traffic.py "$O/pmc_fetch" "$O/pmc_write" "$O/pmc_traffic.json" > /dev/null 2>&1; ok $? pmc_summary
find "$O/prof" -name '*kernel_stats.csv' -exec cp {} "$O/kernel_stats.csv" \;

# optional: SQ counters of every kernel (issue/wait anatomy), its own pass
if [ "${PM_SQ:-0}" = "1" ]; then
  cd /tmp
  timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_ANY -d "$O/pmc_sq" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-census "$@" > "$O/pmc_sq.log" 2>&1; ok $? pmc_sq
  cd "$R"
fi
echo done | tee -a "$O/steps.log"
