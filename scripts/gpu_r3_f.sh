#!/bin/bash
# round-3: full GPU test suite, zoo throughput (inception / densenet), knob A/B on ResNet-18
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/t6.log 2>&1
rc=$?; tail -5 $O/t6.log; [ $rc -ne 0 ] && exit $rc
for m in "inception 299 256" "densenet 224 256"; do
  set -- $m
  timeout -k 10 200 python bench.py --model $1 --image-size $2 --batch $3 --steps 10 --warmup 3 --small-batch 0 > $O/z_$1.json 2>$O/z_$1.err || exit $?
  python -c "import json; r=json.load(open('$O/z_$1.json')); print('$1', r['value'], r['ms_per_step'])"
done
bash scripts/gpu_r3_e.sh
