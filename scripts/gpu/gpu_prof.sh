#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python tools/diag_grads.py > gpurun_out/diag2.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o r18 --output-format csv -- python bench.py --steps 5 --warmup 2 --graph off > gpurun_out/prof.log 2>&1 || exit $?
