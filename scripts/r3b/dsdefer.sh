#!/bin/bash
# deferred downsample BN: every GPU test, then a same-box A/B of the headline
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/t_dsd.log 2>&1
rc=$?; tail -1 $O/t_dsd.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" $O/t_dsd.log | head -20; exit $rc; }
for d in 1 0 1 0; do
  MPA_DS_DEFER=$d timeout -k 10 300 python bench.py --small-batch 0 > $O/b_dsd$d.json 2> $O/b_dsd$d.err || { tail -5 $O/b_dsd$d.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b_dsd$d.json'));print('ds_defer $d', d['value'], d['ms_per_step'], d['config']['mean_loss'])"
done
