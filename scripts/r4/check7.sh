#!/bin/bash
# round 4 call 7: strip-tiled halo weight gradient (wide images) tests + VGG A/B + breakdown
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=gpurun_out
T="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_kernels_gpu.py -k "strip or halo" > $O/c7_t1.log 2>&1
rc=$?; tail -2 $O/c7_t1.log; [ $rc -eq 0 ] || grep -E "^E |FAILED|Error" $O/c7_t1.log | head -20; [ $rc -le 1 ] || exit $rc
[ $rc -eq 0 ] || exit 1
b() { local name=$1; shift; timeout -k 10 300 env "$@" > $O/c7_$name.json 2> $O/c7_$name.err || { echo "bench $name failed"; tail -4 $O/c7_$name.err; exit 1; }; python -c "import json; d=json.load(open('$O/c7_$name.json')); print('$name', d['value'], d['ms_per_step'])"; }
b vgg16 python bench.py --model vgg16 --batch 256 --steps 10 --warmup 3 --small-batch 0
b vgg16_nostrip MPA_HALO_STRIP=0 python bench.py --model vgg16 --batch 256 --steps 10 --warmup 3 --small-batch 0
b head python bench.py --steps 20 --warmup 5 --small-batch 0
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/c7_vgg -o k -- python3 $R/bench.py --model vgg16 --batch 256 --steps 3 --warmup 2 --small-batch 0 > $R/$O/c7_vgg.log 2>&1 || { echo "vgg trace failed"; exit 1; }
cd $R
f=$(find $O/c7_vgg -name "*kernel_trace.csv" | head -1)
python3 tools/step_breakdown.py $f 1 40 > $O/c7_vgg_break.txt
head -30 $O/c7_vgg_break.txt
find $O/c7_vgg -name "*.csv" -size +1M -delete
