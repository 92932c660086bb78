#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_head.py 512 20 > gpurun_out/head.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/head.log | head -6
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || exit 1
tail -1 gpurun_out/bench.log
bash gpu_pmc_bench.sh || exit 1
python3 tools/pmc_summary.py gpurun_out/bpmc1/p_counter_collection.csv gpurun_out/bpmc2/p_counter_collection.csv gpurun_out/bpmc3/p_counter_collection.csv > gpurun_out/bpmc_summary.txt
rm -f gpurun_out/bpmc*/p_kernel_trace.csv
