#!/bin/bash
# round 4: BN link (fused bn1 backward reduction in conv2's halo dgrad) after the spill fix
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "halo or bnred" --timeout 120 --timeout-method thread > $O/r4_linkab_tests.log 2>&1
rc=$?; tail -3 $O/r4_linkab_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for L in 0 1; do
    MPA_BN_LINK=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/r4_link$L.$i.json 2> $O/r4_link$L.$i.err || { echo "bench L=$L failed"; tail -5 $O/r4_link$L.$i.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$O/r4_link$L.$i.json')); print('link=$L', d['value'], d['ms_per_step'])"
  done
done
R=$GRAFT_REPO_ROOT
cd /tmp
MPA_BN_LINK=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/seq_link1 -o r18 -- python3 $R/bench.py --steps 3 --warmup 2 > $R/$O/seq_link1.log 2>&1 || { echo seq failed; exit 1; }
cd $R
f=$(find $O/seq_link1 -name "*kernel_trace.csv" | head -1)
python3 tools/prof_sequence.py $f 1 > $O/seq_step_link1.txt
python3 tools/step_breakdown.py $f 1 30 > $O/break_link1.txt
rm -rf $O/seq_link1
head -14 $O/break_link1.txt
