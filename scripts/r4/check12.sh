#!/bin/bash
# round 4 call 12: side-stream weight gradients on DenseNet / Inception (bitwise + A/B)
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
T="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_determinism_gpu.py -k "side_stream" > $O/c12_t1.log 2>&1
rc=$?; tail -2 $O/c12_t1.log; [ $rc -eq 0 ] || grep -E "^E |FAILED|Error" $O/c12_t1.log | head -20; [ $rc -le 1 ] || exit $rc
b() { local name=$1; shift; timeout -k 10 300 env "$@" > $O/c12_$name.json 2> $O/c12_$name.err || { echo "bench $name failed"; tail -4 $O/c12_$name.err; exit 1; }; python -c "import json; d=json.load(open('$O/c12_$name.json')); print('$name', d['value'], d['ms_per_step'])"; }
b dense python bench.py --model densenet --batch 256 --steps 10 --warmup 3 --small-batch 0
b dense_nowgs MPA_WGRAD_STREAM=0 python bench.py --model densenet --batch 256 --steps 10 --warmup 3 --small-batch 0
b inc python bench.py --model inception --image-size 299 --batch 256 --steps 10 --warmup 3 --small-batch 0
b inc_nowgs MPA_WGRAD_STREAM=0 python bench.py --model inception --image-size 299 --batch 256 --steps 10 --warmup 3 --small-batch 0
b r34 python bench.py --model resnet34 --batch 512 --steps 10 --warmup 3 --small-batch 0
b vgg11bn python bench.py --model vgg --batch 256 --steps 10 --warmup 3 --small-batch 0
b alexnet python bench.py --model alexnet --batch 256 --steps 10 --warmup 3 --small-batch 0
b squeeze python bench.py --model squeezenet --batch 256 --steps 10 --warmup 3 --small-batch 0
timeout -k 10 120 python tools/adam_probe.py > $O/c12_adam.txt 2>&1 || { tail -5 $O/c12_adam.txt; exit 1; }
cat $O/c12_adam.txt
