#!/bin/bash
# round-3: HIP-graph replay A/B at the round-2 failing size, graph vs eager at batch 128
export TMPDIR=/tmp
O=gpurun_out
DET=0 timeout -k 10 300 python -u tools/graph_bisect.py 256 224 80 > $O/gb_b256.log 2>&1 || exit $?
cat $O/gb_b256.log
MPA_DIAG_CE_MEMSET=1 DET=0 timeout -k 10 300 python -u tools/graph_bisect.py 256 224 80 > $O/gb_b256_memset.log 2>&1 || exit $?
cat $O/gb_b256_memset.log
for g in off on; do
  MPA_GRAPH_UNSAFE=1 timeout -k 10 200 python bench.py --batch 128 --steps 100 --warmup 10 --graph $g > $O/b128_$g.json 2>$O/b128_$g.err || exit $?
  cat $O/b128_$g.json
done
