#!/bin/bash
# round-3 GPU check: new GPU tests, graph bisect (deterministic and default), eval bench
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_determinism_gpu.py tests/test_preprocess_gpu.py tests/test_eval_pipeline_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t3.log 2>&1
rc=$?; tail -15 $O/t3.log; [ $rc -ne 0 ] && exit $rc
DET=1 timeout -k 10 300 python -u tools/graph_bisect.py 64 112 60 > $O/gb_det.log 2>&1 || exit $?
cat $O/gb_det.log
DET=0 timeout -k 10 300 python -u tools/graph_bisect.py 64 112 60 > $O/gb_nodet.log 2>&1 || exit $?
cat $O/gb_nodet.log
timeout -k 10 300 python -u tools/bench_eval.py 40000 256 1,2,4 256 > $O/bench_eval.log 2>&1 || exit $?
cat $O/bench_eval.log
