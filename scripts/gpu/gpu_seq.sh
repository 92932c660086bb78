set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/seq -o r18 -- python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/seq.log 2>&1
cd $R
f=$(find gpurun_out/seq -name "*kernel_trace.csv" | head -1)
python3 tools/prof_sequence.py $f 1 > gpurun_out/seq_step.txt
rm -f $f
