#!/bin/bash
# round 4 call 10: parity/side-stream test fixes; masked-residual A/B with kernel traces
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=gpurun_out
T="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_layer_parity_gpu.py tests/test_determinism_gpu.py -k "parity or side_stream" > $O/c10_t1.log 2>&1
rc=$?; tail -2 $O/c10_t1.log; [ $rc -eq 0 ] || grep -E "^E |FAILED|Error" $O/c10_t1.log | head -20; [ $rc -le 1 ] || exit $rc
b() { local name=$1; shift; timeout -k 10 300 env "$@" > $O/c10_$name.json 2> $O/c10_$name.err || { echo "bench $name failed"; tail -4 $O/c10_$name.err; exit 1; }; python -c "import json; d=json.load(open('$O/c10_$name.json')); print('$name', d['value'], d['ms_per_step'])"; }
b res python bench.py --steps 20 --warmup 5 --small-batch 0
b nores MPA_RES_MASK=0 python bench.py --steps 20 --warmup 5 --small-batch 0
b res2 python bench.py --steps 20 --warmup 5 --small-batch 0
b nores2 MPA_RES_MASK=0 python bench.py --steps 20 --warmup 5 --small-batch 0
cd /tmp
for v in 1 0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/c10_r$v -o k -- python3 $R/bench.py --steps 3 --warmup 2 --small-batch 0 --res-mask $v > $R/$O/c10_r$v.log 2>&1 || { echo "trace $v failed"; tail -3 $R/$O/c10_r$v.log; exit 1; }
done
cd $R
for v in 1 0; do
  f=$(find $O/c10_r$v -name "*kernel_trace.csv" | head -1)
  python3 tools/step_breakdown.py $f 1 45 > $O/c10_r${v}_break.txt
  python3 tools/prof_sequence.py $f 1 > $O/c10_r${v}_seq.txt
  head -12 $O/c10_r${v}_break.txt
  find $O/c10_r$v -name "*.csv" -size +1M -delete
done
