#!/bin/bash
# round-3 full validation: every GPU test, smoke, headline bench
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tfull.log 2>&1
rc=$?; tail -4 $O/tfull.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" $O/tfull.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python bench.py > $O/b_final.json 2> $O/b_final.err || exit 1
cat $O/b_final.json
