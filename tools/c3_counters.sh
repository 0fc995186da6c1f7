#!/bin/bash
# SQ / TA / TCP / TCC counter passes of the C3 bench (trace kernel study).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
P3="TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum"
bash tools/pmc_probe.sh gpurun_out/c3sq "$P1" "$P2" "$P3" -- --config c3 || exit $?
python3 tools/pmc_table.py gpurun_out/c3sq > gpurun_out/c3sq/counters_c3.txt
grep -A20 "k_trace_pool" gpurun_out/c3sq/counters_c3.txt
