#!/bin/bash
# kernel-time stats over bench steps + PMC passes (MFMA busy, HBM fetch / write bytes)
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --steps 10 --warmup 3"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/fstats -o r18 -- $B > $R/gpurun_out/fstats.log 2>&1
B="python3 $R/bench.py --steps 2 --warmup 1"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d $R/gpurun_out/fpmc1 -o p -- $B > $R/gpurun_out/fpmc1.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/fpmc3 -o p -- $B > $R/gpurun_out/fpmc3.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/fpmc4 -o p -- $B > $R/gpurun_out/fpmc4.log 2>&1
cd $R
python3 tools/prof_summary.py $(find gpurun_out/fstats -name "*kernel_stats.csv" | head -1) 15 45 > gpurun_out/final_kernel_summary.txt
python3 tools/pmc_summary.py $(find gpurun_out/fpmc1 gpurun_out/fpmc3 gpurun_out/fpmc4 -name "*counter_collection.csv") > gpurun_out/final_pmc_summary.txt
find gpurun_out/fstats gpurun_out/fpmc1 gpurun_out/fpmc3 gpurun_out/fpmc4 -name "*.csv" -size +2M -delete
head -5 gpurun_out/final_kernel_summary.txt
