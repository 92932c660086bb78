#!/bin/bash
# round-2 GPU session: stem wgrad plan test, bench, one-step kernel sequence
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "stem" > gpurun_out/stemtest.log 2>&1 || { echo "stemtest rc=$?"; tail -30 gpurun_out/stemtest.log; exit 1; }
tail -3 gpurun_out/stemtest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { echo bench failed; exit 1; }
tail -1 gpurun_out/bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/seq -o r18 -- python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/seq.log 2>&1 || { echo seq failed; exit 1; }
cd $R
f=$(find gpurun_out/seq -name "*kernel_trace.csv" | head -1)
python3 tools/prof_sequence.py $f 1 > gpurun_out/seq_step.txt
rm -f $f
tail -2 gpurun_out/seq_step.txt
