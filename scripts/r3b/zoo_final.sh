#!/bin/bash
# end-of-round model zoo throughput (eager, Adam, bf16, 64,500 classes, synthetic data)
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
for m in "resnet18 224 1024" "resnet34 224 512" "vgg16 224 256" "inception 299 256" "densenet 224 256" "alexnet 224 512" "squeezenet 224 512" "vgg 224 256"; do
  set -- $m
  timeout -k 10 300 python bench.py --model $1 --image-size $2 --batch $3 --steps 10 --warmup 3 --small-batch 0 > $O/zf_$1.json 2> $O/zf_$1.err || { echo "$1 failed"; tail -3 $O/zf_$1.err; exit 1; }
  python -c "import json;d=json.load(open('$O/zf_$1.json'));print('%-11s %3d px batch %4d  %9.1f img/s  %7.2f ms/step' % ('$1', $2, $3, d['value'], d['ms_per_step']))"
done
