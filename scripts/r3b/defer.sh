#!/bin/bash
# deferred DenseNet norm1 backward: kernel tests, DenseNet GPU block / model tests, bench
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_grouped_gpu.py tests/test_models_gpu.py -x -q --timeout 200 --timeout-method thread -k "dense or splitk" > $O/t_defer.log 2>&1
rc=$?; tail -3 $O/t_defer.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" $O/t_defer.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --model densenet --batch 256 --steps 10 --warmup 3 --small-batch 0 > $O/b_dn2.json 2> $O/b_dn2.err || { tail -5 $O/b_dn2.err; exit 1; }
cat $O/b_dn2.json
MPA_DENSE_DEFER=0 timeout -k 10 300 python bench.py --model densenet --batch 256 --steps 10 --warmup 3 --small-batch 0 > $O/b_dn0.json 2> $O/b_dn0.err || { tail -5 $O/b_dn0.err; exit 1; }
cat $O/b_dn0.json
