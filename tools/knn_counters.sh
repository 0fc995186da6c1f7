set -u
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
PM_KNN_SS=1 bash tools/pmc_probe.sh gpurun_out/r04_cnt/ss "$P1" "$P2" -- --estimator knn || exit $?
python3 tools/pmc_table.py gpurun_out/r04_cnt/ss > gpurun_out/r04_cnt/ss.txt
PM_KNN_SS=0 bash tools/pmc_probe.sh gpurun_out/r04_cnt/old "$P1" "$P2" -- --estimator knn || exit $?
python3 tools/pmc_table.py gpurun_out/r04_cnt/old > gpurun_out/r04_cnt/old.txt
