#!/bin/bash
# round 4 call 16: host-side cost of eager steps (cProfile) for DenseNet / Inception / ResNet-18
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python tools/host_profile.py densenet 224 256 5 70 > $O/c16_dense.txt 2>&1 || { tail -5 $O/c16_dense.txt; exit 1; }
head -1 $O/c16_dense.txt
timeout -k 10 300 python tools/host_profile.py inception 299 256 5 70 > $O/c16_inc.txt 2>&1 || { tail -5 $O/c16_inc.txt; exit 1; }
head -1 $O/c16_inc.txt


timeout -k 10 300 python tools/host_profile.py resnet18 224 128 10 70 > $O/c16_r18s.txt 2>&1 || { tail -5 $O/c16_r18s.txt; exit 1; }
head -1 $O/c16_r18s.txt
