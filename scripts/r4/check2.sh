#!/bin/bash
# round 4 call 2: new GPU tests (learning, dropout graph replay, eval feeder), full-size
# learning record, headline bench + b1024 step breakdown, zoo graph-mode benches
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
R=$GRAFT_REPO_ROOT
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $T tests/test_determinism_gpu.py tests/test_learning_gpu.py tests/test_eval_pipeline_gpu.py > $O/r4c2_tests.log 2>&1
rc=$?; tail -5 $O/r4c2_tests.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED|passed|failed" $O/r4c2_tests.log | head -30; exit $rc; }
grep -E "losses|accs" $O/r4c2_tests.log | head -4
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/r4c2_bench.json 2> $O/r4c2_bench.err || { tail -5 $O/r4c2_bench.err; exit 1; }
cat $O/r4c2_bench.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/seq_c2 -o r18 -- python3 $R/bench.py --steps 3 --warmup 2 --small-batch 0 > $R/$O/seq_c2.log 2>&1 || { echo seq failed; exit 1; }
cd $R
f=$(find $O/seq_c2 -name "*kernel_trace.csv" | head -1)
python3 tools/prof_sequence.py $f 1 > $O/seq_step_c2.txt
python3 tools/step_breakdown.py $f 1 40 > $O/break_c2.txt
rm -rf $O/seq_c2
head -14 $O/break_c2.txt
timeout -k 10 600 python tools/learn_curve.py --synthetic_images 800 --image_size 224 --BATCH_SIZE 128 --NUM_CLASSES 64500 --NUM_EPOCHS 15 --resume_epochs 2 > $O/r4c2_curve.txt 2> $O/r4c2_curve.err || { tail -5 $O/r4c2_curve.err; exit 1; }
cat $O/r4c2_curve.txt
for g in off on; do
  timeout -k 10 300 python bench.py --model densenet --batch 256 --steps 10 --warmup 3 --small-batch 0 --graph $g > $O/r4c2_dense_$g.json 2> $O/r4c2_dense_$g.err || { tail -3 $O/r4c2_dense_$g.err; exit 1; }
  timeout -k 10 300 python bench.py --model inception --image-size 299 --batch 256 --steps 10 --warmup 3 --small-batch 0 --graph $g > $O/r4c2_inc_$g.json 2> $O/r4c2_inc_$g.err || { tail -3 $O/r4c2_inc_$g.err; exit 1; }
  python -c "import json; [print('$g', m, json.load(open('$O/r4c2_'+m+'_$g.json'))['value']) for m in ('dense','inc')]"
done
