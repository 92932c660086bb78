#!/bin/bash
# round 4 call 20: side-stream weight gradients under DP (2 gloo ranks on the GPU), bench decisions at N=2
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
T="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $T tests/test_multirank_gpu.py tests/test_determinism_gpu.py > $O/c20_t1.log 2>&1
rc=$?; tail -3 $O/c20_t1.log; [ $rc -eq 0 ] || grep -E "^E |FAILED|Error" $O/c20_t1.log | head -30; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --small-batch 0 > $O/c20_r18.json 2> $O/c20_r18.err || { tail -5 $O/c20_r18.err; exit 1; }
python -c "import json; d=json.load(open('$O/c20_r18.json')); print('r18', d['value'], d['ms_per_step'])"
