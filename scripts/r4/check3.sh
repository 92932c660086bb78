#!/bin/bash
# round 4 call 3: tests of this round's kernels/paths, headline + A/B, zoo benches, eval, PMC
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
R=$GRAFT_REPO_ROOT
T="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $T tests/test_kernels_gpu.py -k "halo or bnred or stem_wgrad_fused or bn or dropout or dgrad" > $O/c3_t1.log 2>&1
rc=$?; tail -2 $O/c3_t1.log; [ $rc -eq 0 ] || grep -E "^E |FAILED|Error" $O/c3_t1.log | head -20; [ $rc -le 1 ] || exit $rc
timeout -k 10 900 $T tests/test_models_gpu.py tests/test_grouped_gpu.py tests/test_eval_pipeline_gpu.py tests/test_determinism_gpu.py > $O/c3_t2.log 2>&1
rc=$?; tail -2 $O/c3_t2.log; [ $rc -eq 0 ] || grep -E "^E |FAILED|Error" $O/c3_t2.log | head -20; [ $rc -le 1 ] || exit $rc
b() { local name=$1; shift; timeout -k 10 300 env "$@" > $O/c3_$name.json 2> $O/c3_$name.err || { echo "bench $name failed"; tail -4 $O/c3_$name.err; exit 1; }; python -c "import json; d=json.load(open('$O/c3_$name.json')); print('$name', d['value'], d['ms_per_step'])"; }
b head python bench.py --steps 20 --warmup 5
b nostemfuse MPA_FUSE_STEM_BWD=0 python bench.py --steps 20 --warmup 5 --small-batch 0
b nopair MPA_DGRAD_PAIR=0 python bench.py --steps 20 --warmup 5 --small-batch 0
b nolink MPA_BN_LINK=0 python bench.py --steps 20 --warmup 5 --small-batch 0
b head2 python bench.py --steps 20 --warmup 5 --small-batch 0
b vgg16 python bench.py --model vgg16 --batch 256 --steps 10 --warmup 3 --small-batch 0
b vgg16_nolink MPA_SEQ_LINK=0 python bench.py --model vgg16 --batch 256 --steps 10 --warmup 3 --small-batch 0
b inc python bench.py --model inception --image-size 299 --batch 256 --steps 10 --warmup 3 --small-batch 0
b inc_nocat MPA_CAT_INTO=0 MPA_INC_LINK=0 python bench.py --model inception --image-size 299 --batch 256 --steps 10 --warmup 3 --small-batch 0
b dense python bench.py --model densenet --batch 256 --steps 10 --warmup 3 --small-batch 0
for cfg in "resnet18 224 224" "inception 299 299"; do
  set -- $cfg
  MODEL=$1 HW=$2 timeout -k 10 300 python tools/bench_eval.py 20480 256 1,2,3 $3 >> $O/c3_eval.txt 2>> $O/c3_eval.err || { echo "eval $cfg failed"; tail -3 $O/c3_eval.err; exit 1; }
done
cat $O/c3_eval.txt
cd /tmp
B="python3 $R/bench.py --steps 2 --warmup 1 --small-batch 0"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d $R/$O/c3pmc1 -o p -- $B > $R/$O/c3pmc1.log 2>&1 || { echo pmc1 failed; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE TA_BUSY_avr --kernel-trace --output-format csv -d $R/$O/c3pmc3 -o p -- $B > $R/$O/c3pmc3.log 2>&1 || { echo pmc3 failed; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/c3seq -o r18 -- python3 $R/bench.py --steps 3 --warmup 2 --small-batch 0 > $R/$O/c3seq.log 2>&1 || { echo seq failed; exit 1; }
cd $R
python3 tools/pmc_summary.py $(find $O/c3pmc1 $O/c3pmc3 -name "*counter_collection.csv") > $O/c3_pmc_summary.txt
f=$(find $O/c3seq -name "*kernel_trace.csv" | head -1)
python3 tools/prof_sequence.py $f 1 > $O/c3_seq.txt
python3 tools/step_breakdown.py $f 1 40 > $O/c3_break.txt
find $O/c3pmc1 $O/c3pmc3 $O/c3seq -name "*.csv" -size +1M -delete
head -14 $O/c3_break.txt
