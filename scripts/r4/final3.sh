#!/bin/bash
# round 4 last check of the final tree: whole GPU suite, smoke, default bench
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/f3_tests.log 2>&1
rc=$?; tail -3 $O/f3_tests.log; [ $rc -eq 0 ] || grep -E "^E |FAILED|Error" $O/f3_tests.log | head -30; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/f3_smoke.log 2>&1; tail -2 $O/f3_smoke.log
timeout -k 10 300 python bench.py > $O/f3_bench.json 2> $O/f3_bench.err; python -c "import json; d=json.load(open('$O/f3_bench.json')); print('bench', d['value'], d['ms_per_step'], d.get('small_batch'))"
