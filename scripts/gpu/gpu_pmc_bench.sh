set -e
# PMC passes over two bench.py steps (every kernel of the training step gets counters)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
B="python3 $R/bench.py --steps 2 --warmup 1"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d $R/gpurun_out/bpmc1 -o p -- $B > $R/gpurun_out/bpmc1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA TA_BUSY_avr TCC_HIT_sum --kernel-trace --output-format csv -d $R/gpurun_out/bpmc2 -o p -- $B > $R/gpurun_out/bpmc2.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/bpmc3 -o p -- $B > $R/gpurun_out/bpmc3.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/bpmc4 -o p -- $B > $R/gpurun_out/bpmc4.log 2>&1
