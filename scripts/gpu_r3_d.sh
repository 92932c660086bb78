#!/bin/bash
# round-3: unit parity (tests + table), DenseNet / Inception kernel profiles at batch 256
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_layer_parity_gpu.py -q --timeout 300 --timeout-method thread > $O/t5.log 2>&1
tail -5 $O/t5.log
timeout -k 10 300 python -u tools/unit_parity.py > $O/unit_parity.txt 2>&1 || exit $?
grep "==" $O/unit_parity.txt
for m in "densenet 224" "inception 299"; do
  set -- $m
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$1 -o run -- python bench.py --model $1 --image-size $2 --batch 256 --steps 5 --warmup 3 --small-batch 0 > $O/b_$1.json 2> $O/b_$1.err || exit $?
  cat $O/b_$1.json
done
