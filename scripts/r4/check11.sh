#!/bin/bash
# round 4 call 11: masked residual applied at the epilogue (no spills) - test + A/B
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
T="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_kernels_gpu.py -k "masked_residual or halo or strip" tests/test_models_gpu.py > $O/c11_t1.log 2>&1
rc=$?; tail -2 $O/c11_t1.log; [ $rc -eq 0 ] || grep -E "^E |FAILED|Error" $O/c11_t1.log | head -20; [ $rc -le 1 ] || exit $rc
b() { local name=$1; shift; timeout -k 10 300 env "$@" > $O/c11_$name.json 2> $O/c11_$name.err || { echo "bench $name failed"; tail -4 $O/c11_$name.err; exit 1; }; python -c "import json; d=json.load(open('$O/c11_$name.json')); print('$name', d['value'], d['ms_per_step'])"; }
b res python bench.py --steps 20 --warmup 5 --small-batch 0
b nores MPA_RES_MASK=0 python bench.py --steps 20 --warmup 5 --small-batch 0
b res2 python bench.py --steps 20 --warmup 5 --small-batch 0
b nores2 MPA_RES_MASK=0 python bench.py --steps 20 --warmup 5 --small-batch 0
b nowgs MPA_WGRAD_STREAM=0 python bench.py --steps 20 --warmup 5 --small-batch 0
