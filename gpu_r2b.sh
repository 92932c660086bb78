#!/bin/bash
# halo kernel DMA-cost diagnostic: per-layer times with and without the in-loop DMAs
mkdir -p gpurun_out
MPA_BENCH_ENGINES=1h timeout -k 10 300 python tools/bench_kernels.py 512 10 > gpurun_out/halo_dbg0.log 2>&1 || exit 1
MPA_HALO_DBG=1 MPA_BENCH_ENGINES=1h timeout -k 10 300 python tools/bench_kernels.py 512 10 > gpurun_out/halo_dbg1.log 2>&1 || exit 1
cat gpurun_out/halo_dbg0.log gpurun_out/halo_dbg1.log | grep -v amdgpu.ids
