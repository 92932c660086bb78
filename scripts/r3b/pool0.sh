#!/bin/bash
# valid (pad 0) 3x3/s2 fused stem pool fast paths: tests + Inception bench
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 200 --timeout-method thread -k "maxpool or inception" > $O/t_pool0.log 2>&1
rc=$?; tail -1 $O/t_pool0.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" $O/t_pool0.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --model inception --image-size 299 --batch 256 --steps 10 --warmup 3 --small-batch 0 > $O/bz_inception.json 2> $O/bz_inception.err || { tail -5 $O/bz_inception.err; exit 1; }
python -c "import json;d=json.load(open('$O/bz_inception.json'));print('inception', d['value'], d['ms_per_step'])"
