#!/bin/bash
# round-3 A/B of halo / BN knobs on the headline step (batch 1024), then the conv sweep
export TMPDIR=/tmp
O=gpurun_out
run() { timeout -k 10 200 env "$@" python bench.py --steps 20 --warmup 5 --small-batch 0 2>/dev/null | python -c "import json,sys; r=json.loads(sys.stdin.readline()); print('%-30s %9.1f img/s %7.3f ms' % (sys.argv[1], r['value'], r['ms_per_step']))" "$*"; }
for i in 1 2; do
run MPA_X=default
run MPA_HALO_WRES=0
run MPA_BN_LINK=1
run MPA_HALO_PROD=0
done
timeout -k 10 300 python tools/bench_kernels.py 1024 10 > $O/kern_b1024.txt 2>&1 || exit $?
cat $O/kern_b1024.txt
