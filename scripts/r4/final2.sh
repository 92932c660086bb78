#!/bin/bash
# round 4 end: whole GPU suite, smoke, default bench, model zoo table (after the stream / host-time changes)
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/f2_tests.log 2>&1
rc=$?; tail -3 $O/f2_tests.log; [ $rc -eq 0 ] || grep -E "^E |FAILED|Error" $O/f2_tests.log | head -30; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/f2_smoke.log 2>&1; tail -2 $O/f2_smoke.log
b() { local name=$1; shift; timeout -k 10 300 env "$@" > $O/f2_$name.json 2> $O/f2_$name.err || { echo "bench $name failed"; tail -4 $O/f2_$name.err; exit 1; }; python -c "import json; d=json.load(open('$O/f2_$name.json')); c=d['config']; print('%-11s %4s px batch %5s  %9.1f img/s  %6.2f ms/step' % ('$name', c.get('image_size'), c.get('global_batch'), d['value'], d['ms_per_step']), d.get('small_batch') or '')"; }
b resnet18 python bench.py
b resnet34 python bench.py --model resnet34 --batch 512 --steps 10 --warmup 3 --small-batch 0
b vgg16 python bench.py --model vgg16 --batch 256 --steps 10 --warmup 3 --small-batch 0
b inception python bench.py --model inception --image-size 299 --batch 256 --steps 10 --warmup 3 --small-batch 0
b densenet python bench.py --model densenet --batch 256 --steps 10 --warmup 3 --small-batch 0
b alexnet python bench.py --model alexnet --batch 512 --steps 10 --warmup 3 --small-batch 0
b squeezenet python bench.py --model squeezenet --batch 512 --steps 10 --warmup 3 --small-batch 0
b vgg python bench.py --model vgg --batch 256 --steps 10 --warmup 3 --small-batch 0
