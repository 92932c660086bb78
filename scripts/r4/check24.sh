#!/bin/bash
# round 4 call 24: cheaper side-stream switch (host time) - bitwise tests, small-batch and headline A/B vs the previous tree's numbers
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
T="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $T tests/test_determinism_gpu.py tests/test_multirank_gpu.py > $O/c24_t1.log 2>&1
rc=$?; tail -3 $O/c24_t1.log; [ $rc -eq 0 ] || grep -E "^E |FAILED|Error" $O/c24_t1.log | head -30; [ $rc -le 1 ] || exit $rc
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 300 python tools/host_profile.py resnet18 224 128 10 20 > $O/c24_hp.txt 2>&1 || { tail -5 $O/c24_hp.txt; exit 1; }
grep synchronized $O/c24_hp.txt
b() { local name=$1; shift; timeout -k 10 300 env "$@" > $O/c24_$name.json 2> $O/c24_$name.err || { echo "bench $name failed"; tail -4 $O/c24_$name.err; exit 1; }; python -c "import json; d=json.load(open('$O/c24_$name.json')); print('$name', d['value'], d['ms_per_step'], d.get('small_batch'))"; }
b r18 python bench.py --steps 20 --warmup 5
b r18b python bench.py --steps 20 --warmup 5
