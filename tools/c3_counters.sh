# SQ / TA / TCC counters of the C3 bench (the pooled trace dominates), one
# rocprofv3 --pmc pass each (tools/pmc_probe.sh), table into gpurun_out/c3_cnt/table.txt
set -u
R=$GRAFT_REPO_ROOT; O=gpurun_out/c3_cnt
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
P3="TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum"
P4="TCP_TCC_READ_REQ_sum"
bash $R/tools/pmc_probe.sh $O "$P1" "$P2" "$P3" "$P4" -- --config c3 || exit $?
python3 $R/tools/pmc_table.py $R/$O > $R/$O/table.txt
