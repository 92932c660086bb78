#!/bin/bash
# end-of-round ResNet-18 b1024 kernel stats (rocprofv3 --kernel-trace --stats) and one-step sequence
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O; R=$(pwd)
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/fprof -o r18 -- python3 $R/bench.py --steps 5 --warmup 2 --small-batch 0 > $R/$O/fprof.log 2>&1 || exit 1
cd $R
f=$(find $O/fprof -name "*kernel_trace.csv" | head -1)
python3 tools/prof_sequence.py $f 1 > $O/final_seq.txt && tail -1 $O/final_seq.txt
python3 tools/step_breakdown.py $f 1 30 > $O/final_breakdown.txt && head -20 $O/final_breakdown.txt
rm -f $f
