#!/bin/bash
# round 4: whole GPU suite, smoke, default bench, per-kernel step profile of the final tree
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/fin_tests.log 2>&1
rc=$?; tail -3 $O/fin_tests.log; [ $rc -eq 0 ] || grep -E "^E |FAILED|Error" $O/fin_tests.log | head -30; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/fin_smoke.log 2>&1; tail -2 $O/fin_smoke.log
timeout -k 10 300 python bench.py > $O/fin_bench.json 2> $O/fin_bench.err; python -c "import json; d=json.load(open('$O/fin_bench.json')); print('bench', d['value'], d['ms_per_step'], d.get('small_batch'))"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/fin_tr -o k -- python3 $R/bench.py --steps 3 --warmup 2 --small-batch 0 > $R/$O/fin_tr.log 2>&1 || { echo "trace failed"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d $R/$O/fin_pmc -o p -- python3 $R/bench.py --steps 2 --warmup 1 --small-batch 0 > $R/$O/fin_pmc.log 2>&1 || { echo pmc failed; exit 1; }
cd $R
f=$(find $O/fin_tr -name "*kernel_trace.csv" | head -1)
python3 tools/step_breakdown.py $f 1 45 > $O/fin_break.txt
python3 tools/prof_sequence.py $f 1 > $O/fin_seq.txt
python3 tools/pmc_summary.py $(find $O/fin_pmc -name "*counter_collection.csv") > $O/fin_pmc_summary.txt
head -14 $O/fin_break.txt
find $O/fin_tr $O/fin_pmc -name "*.csv" -size +1M -delete
