#!/bin/bash
# round-3: fused Inception stem pools + helpers - tests, then zoo profiles
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_determinism_gpu.py tests/test_grouped_gpu.py tests/test_layer_parity_gpu.py -k "maxpool_fused or zero_cols or determinism or bitwise or grouped or feature_buffer or inception" -x -q --timeout 300 --timeout-method thread > $O/t12.log 2>&1
rc=$?; tail -3 $O/t12.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" $O/t12.log | head -20; exit $rc; }
bash scripts/gpu_r3_g.sh
