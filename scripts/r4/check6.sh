#!/bin/bash
# round 4 call 6: per-kernel step breakdowns of the zoo models (VGG-16, DenseNet-121, Inception-v3)
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
cd /tmp
for m in "vgg16 224" "densenet 224" "inception 299"; do
  set -- $m
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/c6_$1 -o k -- python3 $R/bench.py --model $1 --image-size $2 --batch 256 --steps 3 --warmup 2 --small-batch 0 > $O/c6_$1.log 2>&1 || { echo "$1 failed"; tail -5 $O/c6_$1.log; exit 1; }
done
cd $R
for m in vgg16 densenet inception; do
  f=$(find $O/c6_$m -name "*kernel_trace.csv" | head -1)
  python3 tools/step_breakdown.py $f 1 40 > $O/c6_${m}_break.txt
  head -16 $O/c6_${m}_break.txt
  find $O/c6_$m -name "*.csv" -size +1M -delete
done
