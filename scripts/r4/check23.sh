#!/bin/bash
# round 4 call 23: host profile of the small-batch ResNet-18 step, backward on the calling thread
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 300 python tools/host_profile.py resnet18 224 128 10 60 > $O/c23_r18s.txt 2>&1 || { tail -5 $O/c23_r18s.txt; exit 1; }
grep synchronized $O/c23_r18s.txt
