#!/bin/bash
# A/B runner: scripts/gpu/gpu_ab.sh "ENV=val ENV2=val" "ENV=val" ...  (each spec -> one bench run,
# whole list twice, alternating, so box drift shows up); "-" = no extra env.
mkdir -p gpurun_out
ARGS=${BENCH_ARGS:-"--steps 20 --warmup 5"}
for rep in 1 2; do
  for spec in "$@"; do
    [ "$spec" = "-" ] && spec=""
    out=$(env $spec timeout -k 10 240 python bench.py $ARGS 2>&1 | tail -1) || { echo "FAIL [$spec]"; echo "$out"; exit 1; }
    v=$(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])' 2>/dev/null || echo "$out")
    echo "rep$rep [$spec] $v" | tee -a gpurun_out/ab.log
  done
done
