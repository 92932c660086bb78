#!/bin/bash
# per-kernel summary of one model's training step: scripts/gpu/gpu_zoo_prof.sh MODEL SIZE BATCH
mkdir -p gpurun_out
M=$1; S=$2; B=$3
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --model $M --image-size $S --batch $B --steps 10 --warmup 3 > gpurun_out/zoo_$M.log 2>&1 || { tail -5 gpurun_out/zoo_$M.log; exit 1; }
tail -1 gpurun_out/zoo_$M.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/zprof_$M -o z -- python3 $R/bench.py --model $M --image-size $S --batch $B --steps 3 --warmup 2 > $R/gpurun_out/zprof_$M.log 2>&1 || { echo prof failed; exit 1; }
cd $R
s=$(find gpurun_out/zprof_$M -name "*kernel_stats.csv" | head -1)
python3 tools/prof_summary.py $s 5 30 > gpurun_out/zprof_${M}_summary.txt 2>&1
rm -f $(find gpurun_out/zprof_$M -name "*kernel_trace.csv")
head -32 gpurun_out/zprof_${M}_summary.txt
