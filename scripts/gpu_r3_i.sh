#!/bin/bash
# round-3 A/B on one box: DenseNet block buffer vs plain autograd, eager vs graph; Inception
# pool branch commuted vs pool-first
export TMPDIR=/tmp
O=gpurun_out
b() {  # name, env..., -- bench args
  local n=$1; shift
  env "$@" timeout -k 10 240 python bench.py --steps 10 --warmup 3 --small-batch 0 ${ARGS} > $O/ab_$n.json 2> $O/ab_$n.err || { echo "$n failed"; tail -3 $O/ab_$n.err; return 1; }
  python -c "import json; r=json.load(open('$O/ab_$n.json')); print('%-28s %9.1f img/s %8.2f ms/step' % ('$n', r['value'], r['ms_per_step']))"
}
ARGS="--model densenet --image-size 224 --batch 256"
b dn_fused MPA_X=1 && b dn_plain MPA_DENSE_BLOCK_GRAD=0 && ARGS="$ARGS --graph on" b dn_fused_graph MPA_X=1 || exit 1
ARGS="--model inception --image-size 299 --batch 256"
b inc_commuted MPA_X=1 && b inc_poolfirst MPA_POOL_FIRST=1 && ARGS="$ARGS --graph on" b inc_graph MPA_X=1
