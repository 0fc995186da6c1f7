# rocprofv3's counter list on the box (names for the PMC passes)
set -u
mkdir -p gpurun_out/r04_list
cd /tmp && timeout -k 10 120 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/r04_list/counters.txt 2>&1
