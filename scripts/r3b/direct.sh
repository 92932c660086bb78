#!/bin/bash
# DenseNet in-place feature writes / slice handover: tests + A/B
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_grouped_gpu.py tests/test_models_gpu.py tests/test_parallel_gpu.py -x -q --timeout 200 --timeout-method thread -k "dense or splitk or halo_fwd or conv_fwd" > $O/t_direct.log 2>&1
rc=$?; tail -1 $O/t_direct.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" $O/t_direct.log | head -20; exit $rc; }
for d in 1; do
timeout -k 10 300 python bench.py --model densenet --batch 256 --steps 10 --warmup 3 --small-batch 0 > $O/b_dd$d.json 2> $O/b_dd$d.err || { tail -5 $O/b_dd$d.err; exit 1; }
python -c "import json;d=json.load(open('$O/b_dd$d.json'));print('pool_first $d', d['value'], d['ms_per_step'])"
done
