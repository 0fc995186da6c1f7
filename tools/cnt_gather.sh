set -e
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
P3="TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum"
for k in ${KERNELS:-tile lane}; do
  PM_GATHER_KERNEL=$k bash tools/pmc_probe.sh gpurun_out/${TAG:-r02e}/$k "$P1" "$P2" "$P3"
  python3 tools/pmc_table.py gpurun_out/${TAG:-r02e}/$k k_gather > gpurun_out/${TAG:-r02e}/$k.txt
done
