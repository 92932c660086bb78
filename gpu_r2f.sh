#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_models.log 2>&1 || { echo "model tests rc=$?"; tail -30 gpurun_out/t_models.log; exit 1; }
tail -2 gpurun_out/t_models.log
timeout -k 10 400 ./gpu_ab.sh - MPA_STEM_WFUSE=0 || exit 1
timeout -k 10 120 python __graft_entry__.py smoke 2>&1 | tail -1
