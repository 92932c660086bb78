#!/bin/bash
# DenseNet transitions with BN + ReLU inside the pool pass: tests + A/B
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_grouped_gpu.py tests/test_models_gpu.py tests/test_parallel_gpu.py -x -q --timeout 200 --timeout-method thread -k "dense or avgpool or bn_relu" > $O/t_tpool.log 2>&1
rc=$?; tail -1 $O/t_tpool.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" $O/t_tpool.log | head -20; exit $rc; }
for d in 1 1; do
  timeout -k 10 300 python bench.py --model densenet --batch 256 --steps 10 --warmup 3 --small-batch 0 > $O/b_tp$d.json 2> $O/b_tp$d.err || { tail -5 $O/b_tp$d.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b_tp$d.json'));print('defer_step_unroll2', d['value'], d['ms_per_step'], d['config']['mean_loss'])"
done
R=$(pwd); cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/dstep -o run -- python3 $R/bench.py --model densenet --batch 256 --steps 3 --warmup 2 --small-batch 0 > $R/$O/dstep.log 2>&1 || exit 1
cd $R; grep -h "bn_defer_step\|dense_gacc" $O/dstep/run_kernel_stats.csv | cut -c1-160
