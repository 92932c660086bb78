#!/bin/bash
# round 4 call 17: DenseNet direct layer walk (host time) - GPU tests + A/B
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
T="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $T tests/test_determinism_gpu.py tests/test_models_gpu.py tests/test_layer_parity_gpu.py -k "dense" > $O/c17_t1.log 2>&1
rc=$?; tail -3 $O/c17_t1.log; [ $rc -eq 0 ] || grep -E "^E |FAILED|Error" $O/c17_t1.log | head -30; [ $rc -le 1 ] || exit $rc
b() { local name=$1; shift; timeout -k 10 300 env "$@" > $O/c17_$name.json 2> $O/c17_$name.err || { echo "bench $name failed"; tail -4 $O/c17_$name.err; exit 1; }; python -c "import json; d=json.load(open('$O/c17_$name.json')); print('$name', d['value'], d['ms_per_step'])"; }
b dense python bench.py --model densenet --batch 256 --steps 10 --warmup 3 --small-batch 0
b dense_nowalk MPA_DENSE_WALK=0 python bench.py --model densenet --batch 256 --steps 10 --warmup 3 --small-batch 0
b dense2 python bench.py --model densenet --batch 256 --steps 10 --warmup 3 --small-batch 0
b dense_nowalk2 MPA_DENSE_WALK=0 python bench.py --model densenet --batch 256 --steps 10 --warmup 3 --small-batch 0
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 300 python tools/host_profile.py densenet 224 256 5 60 > $O/c17_hp.txt 2>&1 || { tail -5 $O/c17_hp.txt; exit 1; }
grep synchronized $O/c17_hp.txt
