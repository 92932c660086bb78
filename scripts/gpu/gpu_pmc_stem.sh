#!/bin/bash
mkdir -p gpurun_out
timeout -k 5 100 python tools/bench_stem_wgrad.py 512 10 2>&1 | grep -v amdgpu || exit 1
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d $R/gpurun_out/spmc1 -o p -- python3 $R/tools/bench_stem_wgrad.py 512 2 > $R/gpurun_out/spmc1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA TA_BUSY_avr TCC_HIT_sum --kernel-trace --output-format csv -d $R/gpurun_out/spmc2 -o p -- python3 $R/tools/bench_stem_wgrad.py 512 2 > $R/gpurun_out/spmc2.log 2>&1 || exit 1
cd $R && python3 tools/pmc_summary.py gpurun_out/spmc1/p_counter_collection.csv gpurun_out/spmc2/p_counter_collection.csv | grep -A4 "stem_wgrad\|wgrad_dma_inc"
