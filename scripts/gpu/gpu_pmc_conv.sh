#!/bin/bash
# PMC passes over selected conv shapes: scripts/gpu/gpu_pmc_conv.sh BATCH SHAPES TAG
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
P="python3 $R/tools/pmc_conv.py $1 $2"
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d $R/gpurun_out/cpmc1_$3 -o p -- $P > $R/gpurun_out/cpmc1_$3.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA TA_BUSY_avr TCC_HIT_sum --kernel-trace --output-format csv -d $R/gpurun_out/cpmc2_$3 -o p -- $P > $R/gpurun_out/cpmc2_$3.log 2>&1 &&
cd $R && python3 tools/pmc_summary.py gpurun_out/cpmc1_$3/p_counter_collection.csv gpurun_out/cpmc2_$3/p_counter_collection.csv > gpurun_out/cpmc_$3.txt && cat gpurun_out/cpmc_$3.txt
