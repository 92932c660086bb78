#!/bin/bash
# round-3: zoo-model tests on the current tree, then DenseNet / Inception kernel traces
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_grouped_gpu.py tests/test_models_gpu.py tests/test_layer_parity_gpu.py tests/test_kernels_gpu.py -k "densenet or inception or grouped or channel or bn or avgpool" -x -q --timeout 300 --timeout-method thread > $O/t10.log 2>&1
rc=$?; tail -3 $O/t10.log; [ $rc -eq 0 ] || { grep -E "^E |Error" $O/t10.log | head -20; exit $rc; }
bash scripts/gpu_r3_g.sh
