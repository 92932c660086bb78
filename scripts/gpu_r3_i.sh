#!/bin/bash
# round-3: structural-fusion tests, then A/B on one box: DenseNet block buffer vs plain
# autograd, eager vs graph; Inception grouped heads / commuted pool branch vs the old forms
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_grouped_gpu.py tests/test_kernels_gpu.py -k "grouped or feature_buffer or channel_prefix or channel_window" -x -q --timeout 250 --timeout-method thread > $O/t9.log 2>&1
rc=$?; tail -3 $O/t9.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/t9.log | head -20; exit $rc; }
b() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 240 python bench.py --steps 10 --warmup 3 --small-batch 0 ${ARGS} > $O/ab_$n.json 2> $O/ab_$n.err || { echo "$n failed"; tail -3 $O/ab_$n.err; return 1; }
  python -c "import json; r=json.load(open('$O/ab_$n.json')); print('%-28s %9.1f img/s %8.2f ms/step' % ('$n', r['value'], r['ms_per_step']))"
}
ARGS="--model inception --image-size 299 --batch 256"
b inc_new MPA_X=1 && b inc_nomerge MPA_MERGE_1X1=0 && b inc_old MPA_MERGE_1X1=0 MPA_POOL_FIRST=1 || exit 1
ARGS="$ARGS --graph on" b inc_new_graph MPA_X=1
ARGS="--model densenet --image-size 224 --batch 256"
b dn_fused MPA_X=1 && b dn_plain MPA_DENSE_BLOCK_GRAD=0 || exit 1
b dn_fused_g16 MPA_DENSE_GRAD_BF16=1 && ARGS="$ARGS --graph on" b dn_fused_graph MPA_X=1
exit 0
