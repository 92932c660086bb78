#!/bin/bash
# round 4 call 14: Inception side-branch streams (bitwise tests, A/B)
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
T="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $T tests/test_determinism_gpu.py tests/test_grouped_gpu.py tests/test_models_gpu.py -k "inception or branch or side_stream or replay" > $O/c14_t1.log 2>&1
rc=$?; tail -3 $O/c14_t1.log; [ $rc -eq 0 ] || grep -E "^E |FAILED|Error" $O/c14_t1.log | head -30; [ $rc -le 1 ] || exit $rc
b() { local name=$1; shift; timeout -k 10 300 env "$@" > $O/c14_$name.json 2> $O/c14_$name.err || { echo "bench $name failed"; tail -4 $O/c14_$name.err; exit 1; }; python -c "import json; d=json.load(open('$O/c14_$name.json')); print('$name', d['value'], d['ms_per_step'])"; }
b inc python bench.py --model inception --image-size 299 --batch 256 --steps 10 --warmup 3 --small-batch 0
b inc_nobr MPA_BRANCH_STREAM=0 python bench.py --model inception --image-size 299 --batch 256 --steps 10 --warmup 3 --small-batch 0
b inc2 python bench.py --model inception --image-size 299 --batch 256 --steps 10 --warmup 3 --small-batch 0
b inc_nobr2 MPA_BRANCH_STREAM=0 python bench.py --model inception --image-size 299 --batch 256 --steps 10 --warmup 3 --small-batch 0
