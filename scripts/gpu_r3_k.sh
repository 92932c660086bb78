#!/bin/bash
# round-3: step-GC A/B (DenseNet), headline bench, batch-128 ResNet-18 kernel trace
export TMPDIR=/tmp
O=gpurun_out
b() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 240 python bench.py --steps 10 --warmup 3 --small-batch 0 ${ARGS} > $O/ab_$n.json 2> $O/ab_$n.err || { echo "$n failed"; tail -3 $O/ab_$n.err; return 1; }
  python -c "import json; r=json.load(open('$O/ab_$n.json')); print('%-28s %9.1f img/s %8.2f ms/step' % ('$n', r['value'], r['ms_per_step']))"
}
ARGS="--model densenet --image-size 224 --batch 256"
b dn_gcoff MPA_X=1 && b dn_gcon MPA_STEP_GC=1 && b dn_gcoff2 MPA_X=1 || exit 1
ARGS="--model inception --image-size 299 --batch 256"
b inc MPA_X=1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/b_head.json 2> $O/b_head.err || exit 1
cat $O/b_head.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_b128 -o run -- python bench.py --batch 128 --steps 10 --warmup 5 --small-batch 0 > $O/b128p.json 2> $O/b128p.err || exit 1
python tools/step_breakdown.py $O/prof_b128/run_kernel_trace.csv 1 25 > $O/breakdown_b128.txt && cat $O/breakdown_b128.txt
