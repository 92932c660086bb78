#!/bin/bash
# round 4 call 8: 2x2 max-pool fast path + ReLU hand-off into the pool backward (VGG)
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=gpurun_out
T="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_kernels_gpu.py -k "maxpool or pool" tests/test_models_gpu.py > $O/c8_t1.log 2>&1
rc=$?; tail -2 $O/c8_t1.log; [ $rc -eq 0 ] || grep -E "^E |FAILED|Error" $O/c8_t1.log | head -20; [ $rc -le 1 ] || exit $rc
b() { local name=$1; shift; timeout -k 10 300 env "$@" > $O/c8_$name.json 2> $O/c8_$name.err || { echo "bench $name failed"; tail -4 $O/c8_$name.err; exit 1; }; python -c "import json; d=json.load(open('$O/c8_$name.json')); print('$name', d['value'], d['ms_per_step'])"; }
b vgg16 python bench.py --model vgg16 --batch 256 --steps 10 --warmup 3 --small-batch 0
b vgg16_nolink MPA_SEQ_LINK=0 python bench.py --model vgg16 --batch 256 --steps 10 --warmup 3 --small-batch 0
b vgg python bench.py --model vgg --batch 256 --steps 10 --warmup 3 --small-batch 0
b alexnet python bench.py --model alexnet --batch 256 --steps 10 --warmup 3 --small-batch 0
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/c8_vgg -o k -- python3 $R/bench.py --model vgg16 --batch 256 --steps 3 --warmup 2 --small-batch 0 > $R/$O/c8_vgg.log 2>&1 || { echo "vgg trace failed"; exit 1; }
cd $R
f=$(find $O/c8_vgg -name "*kernel_trace.csv" | head -1)
python3 tools/step_breakdown.py $f 1 40 > $O/c8_vgg_break.txt
head -34 $O/c8_vgg_break.txt
find $O/c8_vgg -name "*.csv" -size +1M -delete
