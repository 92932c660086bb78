#!/bin/bash
# 256x256 rows tile in the autotuner: A/B on ResNet-18 (headline) and the zoo
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "autotune or linear or splitk" > $O/t_256.log 2>&1
rc=$?; tail -1 $O/t_256.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" $O/t_256.log | head -20; exit $rc; }
for t in 1 0 1 0; do
  MPA_TUNE_256=$t timeout -k 10 300 python bench.py --small-batch 0 > $O/b256_$t.json 2> $O/b256_$t.err || { tail -5 $O/b256_$t.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b256_$t.json'));print('resnet18 tune256=$t', d['value'], d['ms_per_step'])"
done
for m in "inception 299 256" "resnet34 224 512"; do
  set -- $m
  for t in 1 0; do
    MPA_TUNE_256=$t timeout -k 10 300 python bench.py --model $1 --image-size $2 --batch $3 --steps 10 --warmup 3 --small-batch 0 > $O/bz_$1_$t.json 2> $O/bz_$1_$t.err || { tail -5 $O/bz_$1_$t.err; exit 1; }
    python -c "import json;d=json.load(open('$O/bz_$1_$t.json'));print('$1 tune256=$t', d['value'], d['ms_per_step'])"
  done
done
