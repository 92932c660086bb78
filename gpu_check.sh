#!/bin/bash
# GPU session runner: ./gpu_check.sh step1 step2 ...  Steps: kernels models smoke bench prof diag
# Stops at the first crash/timeout (pytest rc 1 = test failures only, continue).
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1; local t=$2; shift 2; timeout -k 10 "$t" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -4 gpurun_out/$name.log; return $rc; }
for step in "$@"; do
  case $step in
    kernels) run kernels 900 python -m pytest tests/test_kernels_gpu.py -q -p no:cacheprovider; rc=$? ;;
    models) run models 900 python -m pytest tests/test_models_gpu.py -q -p no:cacheprovider; rc=$? ;;
    gputests) run gputests 1200 python -m pytest tests -m gpu -q -p no:cacheprovider; rc=$? ;;
    smoke) run smoke 300 python __graft_entry__.py smoke; rc=$? ;;
    bench) run bench 600 python bench.py --steps 20 --warmup 5; rc=$? ;;
    bench128) run bench128 600 python bench.py --steps 20 --warmup 5 --batch 128; rc=$? ;;
    benchnog) run benchnog 600 python bench.py --steps 20 --warmup 5 --graph off; rc=$? ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o r18 --output-format csv -- python bench.py --steps 5 --warmup 2 --graph off; rc=$? ;;
    diag) run diag 600 python tools/diag_grads.py; rc=$? ;;
    diag2) run diag2 600 python tools/diag_grads.py twice; rc=$? ;;
    *) echo "unknown step $step"; rc=0 ;;
  esac
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $step rc=$rc"; exit $rc; fi
done
