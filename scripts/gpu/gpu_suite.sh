#!/bin/bash
# full GPU suite + smoke + bench + one-step kernel sequence
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { echo "gpu tests rc=$?"; tail -30 gpurun_out/t_all.log; exit 1; }
tail -1 gpurun_out/t_all.log
timeout -k 10 120 python __graft_entry__.py smoke 2>&1 | tail -1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 || exit 1
scripts/gpu/gpu_seq2.sh ${1:-new}
