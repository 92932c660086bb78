#!/bin/bash
# DenseNet transitions with BN + ReLU inside the pool pass: tests + A/B
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_grouped_gpu.py tests/test_models_gpu.py tests/test_parallel_gpu.py -x -q --timeout 200 --timeout-method thread -k "dense or avgpool or bn_relu" > $O/t_tpool.log 2>&1
rc=$?; tail -1 $O/t_tpool.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" $O/t_tpool.log | head -20; exit $rc; }
for d in 1 0 1 0; do
  MPA_DENSE_FUSE_POOL=$d timeout -k 10 300 python bench.py --model densenet --batch 256 --steps 10 --warmup 3 --small-batch 0 > $O/b_tp$d.json 2> $O/b_tp$d.err || { tail -5 $O/b_tp$d.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b_tp$d.json'));print('fuse_pool $d', d['value'], d['ms_per_step'], d['config']['mean_loss'])"
done
