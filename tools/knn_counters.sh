# Issue / wait / scalar-cache counters of the kNN gather (k_gather_knn_ss) at C2
# kNN, one rocprofv3 --pmc pass each (tools/pmc_probe.sh), table into
# gpurun_out/knn_cnt/table.txt
set -u
R=$GRAFT_REPO_ROOT; O=gpurun_out/knn_cnt
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM GRBM_GUI_ACTIVE"
P3="SQ_INST_LEVEL_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LEVEL_WAVES SQ_BUSY_CU_CYCLES SQ_INST_CYCLES_SALU SQ_IFETCH"
P4="SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_MISSES_DUPLICATE SQC_DCACHE_BUSY_CYCLES"
P5="SQC_TC_STALL SQC_TC_DATA_READ_REQ SQC_DCACHE_REQ"
bash $R/tools/pmc_probe.sh $O "$P1" "$P2" "$P3" "$P4" "$P5" -- --estimator knn || exit $?
python3 $R/tools/pmc_table.py $R/$O knn_ss knn_tile knn_pack > $R/$O/table.txt
cat $R/$O/table.txt
