#!/bin/bash
# round 4 call 13: zoo step breakdowns with side-stream weight gradients; Adam kernel isolation probe
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
PYTHONPATH=$R timeout -k 10 120 python tools/adam_probe.py > $O/c13_adam.txt 2>&1 || { tail -5 $O/c13_adam.txt; exit 1; }
cat $O/c13_adam.txt
cd /tmp
for m in "densenet 224" "inception 299"; do
  set -- $m
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/c13_$1 -o k -- python3 $R/bench.py --model $1 --image-size $2 --batch 256 --steps 3 --warmup 2 --small-batch 0 > $O/c13_$1.log 2>&1 || { echo "$1 failed"; tail -5 $O/c13_$1.log; exit 1; }
done
cd $R
for m in densenet inception; do
  f=$(find $O/c13_$m -name "*kernel_trace.csv" | head -1)
  python3 tools/step_breakdown.py $f 1 40 > $O/c13_${m}_break.txt
  head -16 $O/c13_${m}_break.txt
  python3 tools/prof_sequence.py $f 1 > $O/c13_${m}_seq.txt 2>&1 || true
  find $O/c13_$m -name "*.csv" -size +1M -delete
done
b() { local name=$1; shift; timeout -k 10 300 env "$@" > $O/c13_$name.json 2> $O/c13_$name.err || { echo "bench $name failed"; tail -4 $O/c13_$name.err; exit 1; }; python -c "import json; d=json.load(open('$O/c13_$name.json')); print('$name', d['value'], d['ms_per_step'])"; }
b inc_eh MPA_EARLY_HEAD_OPT=1 python bench.py --model inception --image-size 299 --batch 256 --steps 10 --warmup 3 --small-batch 0
b inc python bench.py --model inception --image-size 299 --batch 256 --steps 10 --warmup 3 --small-batch 0
b dense_eh MPA_EARLY_HEAD_OPT=1 python bench.py --model densenet --batch 256 --steps 10 --warmup 3 --small-batch 0
b dense python bench.py --model densenet --batch 256 --steps 10 --warmup 3 --small-batch 0
b r18_eh MPA_EARLY_HEAD_OPT=1 python bench.py --steps 20 --warmup 5 --small-batch 0
b r18 python bench.py --steps 20 --warmup 5
