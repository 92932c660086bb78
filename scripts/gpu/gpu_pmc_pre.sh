#!/bin/bash
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace --output-format csv -d $R/gpurun_out/ppmc -o p -- python3 $R/tools/bench_pre.py 512 3 > $R/gpurun_out/ppmc.log 2>&1 || exit 1
cd $R && python3 tools/pmc_summary.py gpurun_out/ppmc/p_counter_collection.csv | grep -A3 preprocess
