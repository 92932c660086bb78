#!/bin/bash
# A/B runner with bench arguments: scripts/gpu/gpu_abx.sh "ENV=V ... | --bench-args ..." ...
# (either side of | may be empty; the list runs twice, alternating)
mkdir -p gpurun_out
BASE=${BENCH_ARGS:-"--steps 20 --warmup 5"}
for rep in 1 2; do
  for spec in "$@"; do
    envs=${spec%%|*}; args=""
    [[ "$spec" == *"|"* ]] && args=${spec#*|}
    out=$(env $envs timeout -k 10 240 python bench.py $BASE $args 2>&1 | tail -1) || { echo "FAIL [$spec]"; echo "$out"; exit 1; }
    v=$(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])' 2>/dev/null || echo "$out")
    echo "rep$rep [$spec] $v" | tee -a gpurun_out/abx.log
  done
done
