#!/bin/bash
# One GPU session: kernel tests -> model tests -> smoke -> short bench.  Stops at the first
# crash/timeout (exit codes other than pytest's 0/1).
mkdir -p gpurun_out
run() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -5 gpurun_out/$name.log; return $rc; }
run kernels 900 python -m pytest tests/test_kernels_gpu.py -q -p no:cacheprovider; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
run models 900 python -m pytest tests/test_models_gpu.py -q -p no:cacheprovider; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
run smoke 300 python __graft_entry__.py smoke || exit $?
run bench 600 python bench.py --steps 10 --warmup 3 || exit $?
