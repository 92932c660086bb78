#!/bin/bash
# one-step kernel sequence: scripts/gpu/gpu_seq2.sh TAG [ENV=VAL ...]
mkdir -p gpurun_out
TAG=$1; shift
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/seq_$TAG -o r18 -- python3 $R/bench.py --steps 3 --warmup 2 $SEQ_ARGS > $R/gpurun_out/seq_$TAG.log 2>&1 || { echo seq failed; exit 1; }
cd $R
f=$(find gpurun_out/seq_$TAG -name "*kernel_trace.csv" | head -1)
python3 tools/prof_sequence.py $f 1 > gpurun_out/seq_step_$TAG.txt
rm -f $f
tail -1 gpurun_out/seq_step_$TAG.txt
