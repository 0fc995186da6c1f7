# Scalar-cache counters of the kNN gather (one rocprofv3 --pmc pass each, killed at 120 s)
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r04_sqc; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
i=0
for p in "SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_MISSES_DUPLICATE SQC_DCACHE_BUSY_CYCLES" \
         "SQC_TC_STALL SQC_TC_DATA_READ_REQ SQC_DCACHE_REQ" \
         "SQ_INST_LEVEL_SMEM SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $p -d $O/p$i -o run --output-format csv -- python3 $R/bench.py --estimator knn --steps 5 --warmup 1 --no-cpu-baseline --no-census > $O/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc" | tee -a $O/steps.log; [ $rc -ne 0 ] && exit $rc
done
cd $R && python3 tools/pmc_table.py $O > $O/table.txt
