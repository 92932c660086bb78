#!/bin/bash
# round 4 call 18: side-stream priority A/B
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
b() { local name=$1; shift; timeout -k 10 300 env "$@" > $O/c18_$name.json 2> $O/c18_$name.err || { echo "bench $name failed"; tail -4 $O/c18_$name.err; exit 1; }; python -c "import json; d=json.load(open('$O/c18_$name.json')); print('$name', d['value'], d['ms_per_step'])"; }
b r18 python bench.py --steps 20 --warmup 5 --small-batch 0
b r18_hi MPA_WGRAD_PRIO=-1 python bench.py --steps 20 --warmup 5 --small-batch 0
b r18b python bench.py --steps 20 --warmup 5 --small-batch 0
b r18_hib MPA_WGRAD_PRIO=-1 python bench.py --steps 20 --warmup 5 --small-batch 0
b inc python bench.py --model inception --image-size 299 --batch 256 --steps 10 --warmup 3 --small-batch 0
b inc_hi MPA_WGRAD_PRIO=-1 python bench.py --model inception --image-size 299 --batch 256 --steps 10 --warmup 3 --small-batch 0
b dense python bench.py --model densenet --batch 256 --steps 10 --warmup 3 --small-batch 0
b dense_hi MPA_WGRAD_PRIO=-1 python bench.py --model densenet --batch 256 --steps 10 --warmup 3 --small-batch 0
b vgg16 python bench.py --model vgg16 --batch 256 --steps 10 --warmup 3 --small-batch 0
b vgg16_hi MPA_WGRAD_PRIO=-1 python bench.py --model vgg16 --batch 256 --steps 10 --warmup 3 --small-batch 0
