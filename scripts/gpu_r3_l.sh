#!/bin/bash
# round-3: early classifier update - determinism tests, then same-box A/B
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_determinism_gpu.py tests/test_multirank_gpu.py tests/test_models_gpu.py -x -q --timeout 300 --timeout-method thread > $O/t11.log 2>&1
rc=$?; tail -3 $O/t11.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" $O/t11.log | head -20; exit $rc; }
b() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 240 python bench.py --steps 20 --warmup 5 --small-batch 0 ${ARGS} > $O/ab_$n.json 2> $O/ab_$n.err || { echo "$n failed"; tail -3 $O/ab_$n.err; return 1; }
  python -c "import json; r=json.load(open('$O/ab_$n.json')); print('%-28s %9.1f img/s %8.3f ms/step' % ('$n', r['value'], r['ms_per_step']))"
}
ARGS="" b r18_early MPA_X=1 && ARGS="" b r18_late MPA_EARLY_HEAD_OPT=0 || exit 1
ARGS="--batch 128" b r18b128_early MPA_X=1 && ARGS="--batch 128" b r18b128_late MPA_EARLY_HEAD_OPT=0 || exit 1
ARGS="--model inception --image-size 299 --batch 256" b inc_early MPA_X=1 && ARGS="--model inception --image-size 299 --batch 256" b inc_late MPA_EARLY_HEAD_OPT=0 || exit 1
ARGS="--model densenet --image-size 224 --batch 256" b dn_early MPA_X=1 && ARGS="--model densenet --image-size 224 --batch 256" b dn_late MPA_EARLY_HEAD_OPT=0
ARGS="" b r18_early2 MPA_X=1 && ARGS="" b r18_late2 MPA_EARLY_HEAD_OPT=0
