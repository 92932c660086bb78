#!/bin/bash
# halo conv kernel timing with and without the in-loop next-item DMAs (MPA_HALO_DBG=1 skips
# them: the result is wrong, the time shows what waiting for the DMAs costs)
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
export MPA_BENCH_ENGINES=1h MPA_SWEEP_SHAPES=l1.3x3,l2.3x3,l3.3x3,l4.3x3
timeout -k 10 200 python -u tools/bench_kernels.py ${1:-512} 20 > gpurun_out/halo_dbg0.txt 2>&1 || exit 1
MPA_HALO_DBG=1 timeout -k 10 200 python -u tools/bench_kernels.py ${1:-512} 20 > gpurun_out/halo_dbg1.txt 2>&1 || exit 1
paste gpurun_out/halo_dbg0.txt gpurun_out/halo_dbg1.txt
MPA_HALO_DBG=2 timeout -k 10 200 python -u tools/bench_kernels.py ${1:-512} 20 > gpurun_out/halo_dbg2.txt 2>&1 || exit 1
grep 3x3 gpurun_out/halo_dbg2.txt
