#!/bin/bash
# halo kernel tests + bench + one-step kernel sequence
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "halo" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_halo.log 2>&1 || { echo "halo tests rc=$?"; tail -30 gpurun_out/t_halo.log; exit 1; }
tail -1 gpurun_out/t_halo.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 || exit 1
scripts/gpu/gpu_seq2.sh ${1:-new}
