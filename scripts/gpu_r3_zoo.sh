#!/bin/bash
# round-3 model zoo on one MI355X: eager and HIP-graph replayed
export TMPDIR=/tmp
O=gpurun_out
for m in "resnet34 224 512" "vgg16 224 256" "inception 299 256" "densenet 224 256" "alexnet 224 512" "squeezenet 224 512" "vgg 224 256"; do
  set -- $m
  for g in off on; do
    timeout -k 10 240 python bench.py --model $1 --image-size $2 --batch $3 --steps 10 --warmup 3 --small-batch 0 --graph $g > $O/zoo_$1_$g.json 2>$O/zoo_$1_$g.err || { echo "$1 $g failed"; tail -3 $O/zoo_$1_$g.err; continue; }
    python -c "import json; r=json.load(open('$O/zoo_$1_$g.json')); print('%-11s %4s px batch %4s graph %-3s %9.1f img/s %8.2f ms/step' % ('$1', '$2', '$3', '$g', r['value'], r['ms_per_step']))"
  done
done
