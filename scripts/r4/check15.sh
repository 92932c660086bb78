#!/bin/bash
# round 4 call 15: side / branch streams inside HIP-graph capture (replay == eager tests, A/B)
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
T="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $T tests/test_determinism_gpu.py > $O/c15_t1.log 2>&1
rc=$?; tail -3 $O/c15_t1.log; [ $rc -eq 0 ] || grep -E "^E |FAILED|Error" $O/c15_t1.log | head -30; [ $rc -le 1 ] || exit $rc
b() { local name=$1; shift; timeout -k 10 300 env "$@" > $O/c15_$name.json 2> $O/c15_$name.err || { echo "bench $name failed"; tail -4 $O/c15_$name.err; exit 1; }; python -c "import json; d=json.load(open('$O/c15_$name.json')); print('$name', d['value'], d['ms_per_step'], d.get('small_batch'))"; }
b dense_g python bench.py --model densenet --batch 256 --steps 10 --warmup 3 --small-batch 0 --graph on
b dense python bench.py --model densenet --batch 256 --steps 10 --warmup 3 --small-batch 0
b dense_g1 MPA_GRAPH_STREAMS=0 python bench.py --model densenet --batch 256 --steps 10 --warmup 3 --small-batch 0 --graph on
b inc_g python bench.py --model inception --image-size 299 --batch 256 --steps 10 --warmup 3 --small-batch 0 --graph on
b inc python bench.py --model inception --image-size 299 --batch 256 --steps 10 --warmup 3 --small-batch 0
b r18_g python bench.py --steps 20 --warmup 5 --graph on --small-batch 128
b r18 python bench.py --steps 20 --warmup 5
