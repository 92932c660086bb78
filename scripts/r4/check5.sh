#!/bin/bash
# round 4 call 5: strip-tiled halo kernel (wide images; layer1 3-stage) tests + A/B
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
T="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_kernels_gpu.py -k "strip or halo" > $O/c5_t1.log 2>&1
rc=$?; tail -2 $O/c5_t1.log; [ $rc -eq 0 ] || grep -E "^E |FAILED|Error" $O/c5_t1.log | head -20; [ $rc -le 1 ] || exit $rc
[ $rc -eq 0 ] || exit 1
b() { local name=$1; shift; timeout -k 10 300 env "$@" > $O/c5_$name.json 2> $O/c5_$name.err || { echo "bench $name failed"; tail -4 $O/c5_$name.err; exit 1; }; python -c "import json; d=json.load(open('$O/c5_$name.json')); print('$name', d['value'], d['ms_per_step'])"; }
b head python bench.py --steps 20 --warmup 5 --small-batch 0
b strip2 MPA_HALO_STRIP=2 python bench.py --steps 20 --warmup 5 --small-batch 0
b vgg16 python bench.py --model vgg16 --batch 256 --steps 10 --warmup 3 --small-batch 0
b vgg16_nostrip MPA_HALO_STRIP=0 python bench.py --model vgg16 --batch 256 --steps 10 --warmup 3 --small-batch 0
b inc python bench.py --model inception --image-size 299 --batch 256 --steps 10 --warmup 3 --small-batch 0
b inc_nostrip MPA_HALO_STRIP=0 python bench.py --model inception --image-size 299 --batch 256 --steps 10 --warmup 3 --small-batch 0
b head2 python bench.py --steps 20 --warmup 5 --small-batch 0
b strip2b MPA_HALO_STRIP=2 python bench.py --steps 20 --warmup 5 --small-batch 0
