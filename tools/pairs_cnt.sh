#!/bin/bash
# LDS / VALU counters of the C2 tile gather: paired layout (default) vs SoA variant.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
bash tools/pmc_probe.sh gpurun_out/prc/pairs "$P1" "$P2" -- --config c2 || exit $?
PMHIP_LIB=$R/cuda-raytrace_amd/lib/variants/libpmhip_soa.so bash tools/pmc_probe.sh gpurun_out/prc/soa "$P1" "$P2" -- --config c2 || exit $?
for v in pairs soa; do python3 tools/pmc_table.py gpurun_out/prc/$v > gpurun_out/prc/$v.txt; echo "== $v"; grep -A16 "k_gather_tile" gpurun_out/prc/$v.txt; done
