#!/bin/bash
# emulated-collective A/B at the default batch (1024): uncapped-RCCL proxy (32 CTAs x 1 ms,
# static grids) vs capped proxy (8 CTAs x 3 ms) with and without the grid reservation
mkdir -p gpurun_out
out=gpurun_out/comm_b1024.txt
: > $out
run() {
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 "$@" 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%-40s %8.1f img/s %7.3f ms' % ('$*' or '(none)', d['value'], d['ms_per_step']))" >> $out || exit 1
}
for rep in 1 2; do
  run
  run --emulate-comm 32:1000
  run --emulate-comm 8:3000
  run --emulate-comm 8:3000 --comm-reserve 8
  run --emulate-comm 8:6000 --comm-reserve 8
done
cat $out
