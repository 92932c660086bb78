#!/bin/bash
# round-3: ResNet-34 / VGG-16 (BASELINE configs) kernel traces + step breakdowns
export TMPDIR=/tmp
O=gpurun_out
for m in "resnet34 224 512" "vgg16 224 256"; do
  set -- $m
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof3_$1 -o run -- python bench.py --model $1 --image-size $2 --batch $3 --steps 4 --warmup 2 --small-batch 0 > $O/b3_$1.json 2> $O/b3_$1.err || exit $?
  cat $O/b3_$1.json
  python tools/step_breakdown.py $O/prof3_$1/run_kernel_trace.csv 1 20 > $O/breakdown_$1.txt && cat $O/breakdown_$1.txt
done
