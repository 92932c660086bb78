#!/bin/bash
# round 4 call 9: valid-conv / 32-wide strip halo kernels, pipelined 2x2 pools; Inception + VGG A/B
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=gpurun_out
T="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_kernels_gpu.py -k "strip or halo or pool or conv_fwd or conv_dgrad or conv_wgrad" > $O/c9_t1.log 2>&1
rc=$?; tail -2 $O/c9_t1.log; [ $rc -eq 0 ] || grep -E "^E |FAILED|Error" $O/c9_t1.log | head -20; [ $rc -le 1 ] || exit $rc
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 $T tests/test_models_gpu.py tests/test_determinism_gpu.py -k "not dropout_models" > $O/c9_t2.log 2>&1
rc=$?; tail -2 $O/c9_t2.log; [ $rc -eq 0 ] || grep -E "^E |FAILED|Error" $O/c9_t2.log | head -20; [ $rc -le 1 ] || exit $rc
b() { local name=$1; shift; timeout -k 10 300 env "$@" > $O/c9_$name.json 2> $O/c9_$name.err || { echo "bench $name failed"; tail -4 $O/c9_$name.err; exit 1; }; python -c "import json; d=json.load(open('$O/c9_$name.json')); print('$name', d['value'], d['ms_per_step'])"; }
b inc python bench.py --model inception --image-size 299 --batch 256 --steps 10 --warmup 3 --small-batch 0
b inc_nokpad MPA_KPAD=0 python bench.py --model inception --image-size 299 --batch 256 --steps 10 --warmup 3 --small-batch 0
b inc_nostrip MPA_HALO_STRIP=0 python bench.py --model inception --image-size 299 --batch 256 --steps 10 --warmup 3 --small-batch 0
b vgg16 python bench.py --model vgg16 --batch 256 --steps 10 --warmup 3 --small-batch 0
b head python bench.py --steps 20 --warmup 5 --small-batch 0
b wgs MPA_WGRAD_STREAM=1 python bench.py --steps 20 --warmup 5 --small-batch 0
b nores MPA_RES_MASK=0 python bench.py --steps 20 --warmup 5 --small-batch 0
b head2 python bench.py --steps 20 --warmup 5 --small-batch 0
b wgs2 MPA_WGRAD_STREAM=1 python bench.py --steps 20 --warmup 5 --small-batch 0
b vgg16_wgs MPA_WGRAD_STREAM=1 python bench.py --model vgg16 --batch 256 --steps 10 --warmup 3 --small-batch 0
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/c9_inc -o k -- python3 $R/bench.py --model inception --image-size 299 --batch 256 --steps 3 --warmup 2 --small-batch 0 > $R/$O/c9_inc.log 2>&1 || { echo "inc trace failed"; exit 1; }
cd $R
f=$(find $O/c9_inc -name "*kernel_trace.csv" | head -1)
python3 tools/step_breakdown.py $f 1 50 > $O/c9_inc_break.txt
python3 tools/prof_sequence.py $f 1 > $O/c9_inc_seq.txt
head -30 $O/c9_inc_break.txt
find $O/c9_inc -name "*.csv" -size +1M -delete
