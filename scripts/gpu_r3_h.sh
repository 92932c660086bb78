#!/bin/bash
# round-3: DenseNet feature buffer + Inception commuted pool branch: kernel/model tests, then
# zoo bench + kernel traces for both
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "bn or chan or avgpool" tests/test_models_gpu.py tests/test_layer_parity_gpu.py -k "densenet or inception or bn or chan or avgpool" -x -q --timeout 300 --timeout-method thread > $O/t8.log 2>&1
rc=$?; tail -5 $O/t8.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r3_g.sh
