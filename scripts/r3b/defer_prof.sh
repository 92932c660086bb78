#!/bin/bash
# deferred DenseNet norm1 backward: A/B bench + kernel trace breakdown
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O; R=$(pwd)
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "dense or bnred or halo_fwd or splitk" > $O/t_defer.log 2>&1
rc=$?; tail -1 $O/t_defer.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" $O/t_defer.log | head -20; exit $rc; }
for d in 1 0; do
MPA_DENSE_DEFER=$d timeout -k 10 300 python bench.py --model densenet --batch 256 --steps 10 --warmup 3 --small-batch 0 > $O/b_dn$d.json 2> $O/b_dn$d.err || { tail -5 $O/b_dn$d.err; exit 1; }
python -c "import json;d=json.load(open('$O/b_dn$d.json'));print('defer $d', d['value'], d['ms_per_step'])"
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/zb_dd -o run -- python3 $R/bench.py --model densenet --batch 256 --steps 4 --warmup 2 --small-batch 0 > $R/$O/zb_dd.json 2> $R/$O/zb_dd.err || exit 1
cd $R
f=$(find $O/zb_dd -name "*kernel_trace.csv" | head -1)
python3 tools/step_breakdown.py $f 1 25 > $O/zb_dd.txt && head -40 $O/zb_dd.txt
rm -f $f
