#!/bin/bash
# one-chunk wide halo wgrad: halo tests, Inception conv table + bench, zoo step breakdowns
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "halo" > $O/t_onech.log 2>&1
rc=$?; tail -1 $O/t_onech.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" $O/t_onech.log | head -20; exit $rc; }
ZOO_ONLY="147x147:32->64" timeout -k 10 300 python tools/bench_zoo_convs.py inception 256 5 2>&1 | grep -v amdgpu.ids
bash scripts/r3b/zoo_break.sh
