#!/bin/bash
# round 4 call 4: fused stem backward (now eligible), model parity, headline A/B, LDS-DMA probe
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
T="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 120 ./tools/dma_probe > $O/c4_probe.txt 2>&1; rc=$?; cat $O/c4_probe.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 $T tests/test_kernels_gpu.py -k "stem_wgrad_fused" tests/test_models_gpu.py > $O/c4_t1.log 2>&1
rc=$?; tail -2 $O/c4_t1.log; [ $rc -eq 0 ] || grep -E "^E |FAILED|Error" $O/c4_t1.log | head -20; [ $rc -le 1 ] || exit $rc
b() { local name=$1; shift; timeout -k 10 300 env "$@" > $O/c4_$name.json 2> $O/c4_$name.err || { echo "bench $name failed"; tail -4 $O/c4_$name.err; exit 1; }; python -c "import json; d=json.load(open('$O/c4_$name.json')); print('$name', d['value'], d['ms_per_step'])"; }
b head python bench.py --steps 20 --warmup 5 --small-batch 0
b nostemfuse MPA_FUSE_STEM_BWD=0 python bench.py --steps 20 --warmup 5 --small-batch 0
b nobnpair MPA_BN_PAIR=0 python bench.py --steps 20 --warmup 5 --small-batch 0
b head2 python bench.py --steps 20 --warmup 5 --small-batch 0
