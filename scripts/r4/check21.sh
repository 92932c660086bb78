#!/bin/bash
# round 4 call 21: Linear weight gradients on the side stream (A/B), bitwise side-stream tests
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
T="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $T tests/test_determinism_gpu.py tests/test_models_gpu.py > $O/c21_t1.log 2>&1
rc=$?; tail -3 $O/c21_t1.log; [ $rc -eq 0 ] || grep -E "^E |FAILED|Error" $O/c21_t1.log | head -30; [ $rc -le 1 ] || exit $rc
b() { local name=$1; shift; timeout -k 10 300 env "$@" > $O/c21_$name.json 2> $O/c21_$name.err || { echo "bench $name failed"; tail -4 $O/c21_$name.err; exit 1; }; python -c "import json; d=json.load(open('$O/c21_$name.json')); print('$name', d['value'], d['ms_per_step'])"; }
b vgg16 python bench.py --model vgg16 --batch 256 --steps 10 --warmup 3 --small-batch 0
b vgg16_off MPA_FC_WGRAD_STREAM=0 python bench.py --model vgg16 --batch 256 --steps 10 --warmup 3 --small-batch 0
b alex python bench.py --model alexnet --batch 512 --steps 10 --warmup 3 --small-batch 0
b alex_off MPA_FC_WGRAD_STREAM=0 python bench.py --model alexnet --batch 512 --steps 10 --warmup 3 --small-batch 0
b r18 python bench.py --steps 20 --warmup 5 --small-batch 0
b r18_off MPA_FC_WGRAD_STREAM=0 python bench.py --steps 20 --warmup 5 --small-batch 0
b r18b python bench.py --steps 20 --warmup 5 --small-batch 0
b r18_offb MPA_FC_WGRAD_STREAM=0 python bench.py --steps 20 --warmup 5 --small-batch 0
b inc python bench.py --model inception --image-size 299 --batch 256 --steps 10 --warmup 3 --small-batch 0
b inc_off MPA_FC_WGRAD_STREAM=0 python bench.py --model inception --image-size 299 --batch 256 --steps 10 --warmup 3 --small-batch 0
