set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d $R/gpurun_out/pmc1 -o p -- python3 $R/tools/pmc_conv.py > $R/gpurun_out/pmc1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA TA_BUSY_avr TCC_HIT_sum --kernel-trace --output-format csv -d $R/gpurun_out/pmc2 -o p -- python3 $R/tools/pmc_conv.py > $R/gpurun_out/pmc2.log 2>&1 || echo "pmc2 failed rc=$?"
ls -R $R/gpurun_out/pmc1 | head
