#!/bin/bash
# round 4: the whole GPU test suite + smoke + default bench + A/B of this round's options
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/full_tests.log 2>&1
rc=$?; tail -3 $O/full_tests.log; [ $rc -eq 0 ] || grep -E "^E |FAILED|Error" $O/full_tests.log | head -30; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/full_smoke.log 2>&1; tail -2 $O/full_smoke.log
b() { local name=$1; shift; timeout -k 10 300 env "$@" > $O/f_$name.json 2> $O/f_$name.err || { echo "bench $name failed"; tail -4 $O/f_$name.err; exit 1; }; python -c "import json; d=json.load(open('$O/f_$name.json')); print('$name', d['value'], d['ms_per_step'])"; }
b default python bench.py
b wgs MPA_WGRAD_STREAM=1 python bench.py --steps 20 --warmup 5 --small-batch 0
b nores MPA_RES_MASK=0 python bench.py --steps 20 --warmup 5 --small-batch 0
b head python bench.py --steps 20 --warmup 5 --small-batch 0
b wgs2 MPA_WGRAD_STREAM=1 python bench.py --steps 20 --warmup 5 --small-batch 0
b inc python bench.py --model inception --image-size 299 --batch 256 --steps 10 --warmup 3 --small-batch 0
b inc_nokpad MPA_KPAD=0 python bench.py --model inception --image-size 299 --batch 256 --steps 10 --warmup 3 --small-batch 0
b inc_nostrip MPA_HALO_STRIP=0 python bench.py --model inception --image-size 299 --batch 256 --steps 10 --warmup 3 --small-batch 0
b vgg16 python bench.py --model vgg16 --batch 256 --steps 10 --warmup 3 --small-batch 0
b vgg16_wgs MPA_WGRAD_STREAM=1 python bench.py --model vgg16 --batch 256 --steps 10 --warmup 3 --small-batch 0
b dense python bench.py --model densenet --batch 256 --steps 10 --warmup 3 --small-batch 0
