#!/bin/bash
# round 4 call 22: stem weight gradient on the side stream vs the compute stream (ResNet-18 / DenseNet)
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
b() { local name=$1; shift; timeout -k 10 300 env "$@" > $O/c22_$name.json 2> $O/c22_$name.err || { echo "bench $name failed"; tail -4 $O/c22_$name.err; exit 1; }; python -c "import json; d=json.load(open('$O/c22_$name.json')); print('$name', d['value'], d['ms_per_step'])"; }
b r18 python bench.py --steps 20 --warmup 5 --small-batch 0
b r18_main MPA_STEM_WGRAD_STREAM=0 python bench.py --steps 20 --warmup 5 --small-batch 0
b r18b python bench.py --steps 20 --warmup 5 --small-batch 0
b r18_mainb MPA_STEM_WGRAD_STREAM=0 python bench.py --steps 20 --warmup 5 --small-batch 0
b r18c python bench.py --steps 20 --warmup 5 --small-batch 0
b r18_mainc MPA_STEM_WGRAD_STREAM=0 python bench.py --steps 20 --warmup 5 --small-batch 0
b dense python bench.py --model densenet --batch 256 --steps 10 --warmup 3 --small-batch 0
b dense_main MPA_STEM_WGRAD_STREAM=0 python bench.py --model densenet --batch 256 --steps 10 --warmup 3 --small-batch 0
