#!/bin/bash
# round 4 call 19: per-shape conv table, halo kernels on vs off (which shapes' halo wgrad loses to the GEMM)
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python tools/bench_zoo_convs.py inception 256 5 > $O/c19_inc.txt 2>&1 || { tail -5 $O/c19_inc.txt; exit 1; }
MPA_HALO=0 timeout -k 10 400 python tools/bench_zoo_convs.py inception 256 5 > $O/c19_inc_nohalo.txt 2>&1 || { tail -5 $O/c19_inc_nohalo.txt; exit 1; }
timeout -k 10 400 python tools/bench_zoo_convs.py densenet 256 5 > $O/c19_dense.txt 2>&1 || { tail -5 $O/c19_dense.txt; exit 1; }
MPA_HALO=0 timeout -k 10 400 python tools/bench_zoo_convs.py densenet 256 5 > $O/c19_dense_nohalo.txt 2>&1 || { tail -5 $O/c19_dense_nohalo.txt; exit 1; }
head -8 $O/c19_inc.txt; head -8 $O/c19_inc_nohalo.txt
