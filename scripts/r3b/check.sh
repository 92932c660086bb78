#!/bin/bash
# re-entry check: smoke, headline bench, one-step kernel sequence at batch 1024
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
R=$(pwd)
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/b0.json 2> $O/b0.err || { tail -5 $O/b0.err; exit 1; }
cat $O/b0.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/seq -o r18 -- python3 $R/bench.py --steps 3 --warmup 2 --small-batch 0 > $R/$O/seq.log 2>&1 || exit 1
cd $R
f=$(find $O/seq -name "*kernel_trace.csv" | head -1)
python3 tools/prof_sequence.py $f 1 > $O/seq_step.txt && tail -1 $O/seq_step.txt
rm -f $f
timeout -k 10 300 python tools/bench_zoo_convs.py inception 256 5 > $O/zoo_inception.txt 2>&1 || { tail -5 $O/zoo_inception.txt; exit 1; }
timeout -k 10 300 python tools/bench_zoo_convs.py densenet 256 5 > $O/zoo_densenet.txt 2>&1 || { tail -5 $O/zoo_densenet.txt; exit 1; }
head -12 $O/zoo_inception.txt
