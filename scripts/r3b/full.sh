#!/bin/bash
# full validation: every GPU test, smoke, headline bench, DenseNet / Inception bench
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tfull.log 2>&1
rc=$?; tail -3 $O/tfull.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" $O/tfull.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/b_final.json 2> $O/b_final.err || { tail -5 $O/b_final.err; exit 1; }
cat $O/b_final.json
for m in "densenet 224 256" "inception 299 256"; do
  set -- $m
  timeout -k 10 300 python bench.py --model $1 --image-size $2 --batch $3 --steps 10 --warmup 3 --small-batch 0 > $O/bz_$1.json 2> $O/bz_$1.err || { tail -5 $O/bz_$1.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bz_$1.json'));print('$1', d['value'], d['ms_per_step'])"
done
