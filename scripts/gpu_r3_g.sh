#!/bin/bash
# round-3: DenseNet / Inception kernel traces of the current tree at batch 256 + step breakdown
export TMPDIR=/tmp
O=gpurun_out
for m in "densenet 224" "inception 299"; do
  set -- $m
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof3_$1 -o run -- python bench.py --model $1 --image-size $2 --batch 256 --steps 4 --warmup 2 --small-batch 0 > $O/b3_$1.json 2> $O/b3_$1.err || exit $?
  cat $O/b3_$1.json
  python tools/step_breakdown.py $O/prof3_$1/run_kernel_trace.csv 1 20 > $O/breakdown_$1.txt && cat $O/breakdown_$1.txt
done
