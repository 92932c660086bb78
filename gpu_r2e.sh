#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "stem" > gpurun_out/t_e.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/t_e.log; exit 1; }
tail -2 gpurun_out/t_e.log
timeout -k 10 300 ./gpu_ab.sh - MPA_STEM_DIRECT=0 || exit 1
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/seq -o r18 -- python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/seq.log 2>&1 || { echo seq failed; exit 1; }
cd $R
f=$(find gpurun_out/seq -name "*kernel_trace.csv" | head -1)
python3 tools/prof_sequence.py $f 1 > gpurun_out/seq_step.txt
s=$(find gpurun_out/seq -name "*kernel_stats.csv" | head -1)
python3 tools/prof_summary.py $s 5 40 > gpurun_out/seq_summary.txt 2>&1 || true
rm -f $f
tail -1 gpurun_out/seq_step.txt
