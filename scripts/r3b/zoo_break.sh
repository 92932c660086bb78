#!/bin/bash
# DenseNet-121 / Inception-v3 step breakdowns (kernel trace of bench.py)
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O; R=$(pwd)
for m in "densenet 224 256" "inception 299 256"; do
  set -- $m
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/zb_$1 -o run -- python3 $R/bench.py --model $1 --image-size $2 --batch $3 --steps 4 --warmup 2 --small-batch 0 > $R/$O/zb_$1.json 2> $R/$O/zb_$1.err || exit 1
  cd $R
  f=$(find $O/zb_$1 -name "*kernel_trace.csv" | head -1)
  python3 tools/step_breakdown.py $f 1 40 > $O/zb_$1.txt && head -50 $O/zb_$1.txt
  rm -f $f
done
