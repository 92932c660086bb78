#!/bin/bash
# One parameterised GPU-box runner (replaces the per-round one-off check scripts).
#
#   gpurun --timeout 1100 -- bash scripts/gpu/run.sh TAG STEP [STEP ...]
#
# Steps run in order, each under its own `timeout -k`; the script stops at the first step
# that fails (no GPU step runs after a fault, abort or time limit).  Results land in
# gpurun_out/TAG_*.
#
#   tests[=EXPR]     pytest -m gpu (optionally -k EXPR)          -> TAG_tests.log
#   smoke            __graft_entry__.smoke()                     -> TAG_smoke.log
#   bench[=ARGS]     python bench.py ARGS ("," separates args)   -> TAG_bench.json
#   seq[=ARGS]       rocprofv3 kernel trace of bench.py, one step's kernel sequence and
#                    the per-category breakdown                  -> TAG_seq.txt, TAG_breakdown.txt
#   stats[=ARGS]     rocprofv3 --kernel-trace --stats over bench.py -> TAG_stats/
#   ab=SPEC;SPEC..   bench A/B, two alternating repeats; SPEC = "ENV=V ... | --args"
#   kern[=ARGS]      tools/bench_kernels.py ARGS                 -> TAG_kern.txt
#   pmc=REGEX:CTRS   one rocprofv3 PMC pass over two bench steps, kernels matching REGEX
#                    (empty: all), counters CTRS (space separated) -> TAG_pmc_N/
#   trace            kernel trace of the pmc passes' run shape   -> TAG_trace/
#   gaps=ARGS        kernel trace of bench.py ARGS, inter-kernel gap distribution (tools/gap_stats.py)
#   (PMC_ARGS in the environment: extra bench.py arguments of pmc / trace)
#   py=SCRIPT,ARGS   python SCRIPT ARGS under a 300 s limit      -> TAG_py_N.log
#   env=NAME=VALUE   export NAME=VALUE for the steps after it
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG
n=0
args_of() { echo "${1//,/ }"; }

for step in "$@"; do
  n=$((n + 1))
  name=${step%%=*}; val=""
  [[ "$step" == *"="* ]] && val=${step#*=}
  echo "== [$n] $step ($(date +%T))"
  case $name in
    tests)
      k=(); [ -n "$val" ] && k=(-k "$val")
      timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 300 \
        --timeout-method thread -p no:cacheprovider "${k[@]}" > ${O}_tests.log 2>&1
      rc=$?; tail -3 ${O}_tests.log
      [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" ${O}_tests.log | head -30; exit $rc; } ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
        > ${O}_smoke.log 2>&1 || { tail -20 ${O}_smoke.log; exit 1; }
      tail -2 ${O}_smoke.log ;;
    bench)
      timeout -k 10 400 python bench.py $(args_of "$val") > ${O}_bench.json 2> ${O}_bench.err \
        || { tail -20 ${O}_bench.err; exit 1; }
      cp ${O}_bench.json ${O}_bench_$n.json
      python -c "import json; d=json.loads(open('${O}_bench.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'], d.get('small_batch'), d.get('phases_ms'), d.get('data_ring'), d.get('host'))" ;;
    seq)
      timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/${O}_seq -o r18 \
        -- python3 $R/bench.py --steps 3 --warmup 2 --small-batch 0 $(args_of "$val") \
        > ${O}_seq.log 2>&1 || { tail -20 ${O}_seq.log; exit 1; }
      f=$(find ${O}_seq -name "*kernel_trace.csv" | head -1)
      python3 tools/prof_sequence.py $f 1 > ${O}_seq.txt
      python3 tools/step_breakdown.py $f 1 40 > ${O}_breakdown.txt 2>&1 || true
      rm -f $f; tail -1 ${O}_seq.txt; head -14 ${O}_breakdown.txt ;;
    stats)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/${O}_stats -o s \
        -- python3 $R/bench.py --steps 10 --warmup 3 --small-batch 0 $(args_of "$val") \
        > ${O}_stats.log 2>&1 || { tail -20 ${O}_stats.log; exit 1; }
      find ${O}_stats -name "*kernel_trace.csv" -delete ;;
    ab)
      IFS=';' read -ra specs <<< "$val"
      for rep in 1 2; do
        for spec in "${specs[@]}"; do
          envs=${spec%%|*}; a=""
          [[ "$spec" == *"|"* ]] && a=${spec#*|}
          out=$(env $envs timeout -k 10 240 python bench.py --small-batch 0 $a 2>&1 | tail -1) \
            || { echo "FAIL [$spec]"; echo "$out"; exit 1; }
          v=$(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])' 2>/dev/null || echo "$out")
          echo "rep$rep [$spec] $v" | tee -a ${O}_ab.log
        done
      done ;;
    kern)
      timeout -k 10 400 python tools/bench_kernels.py $(args_of "$val") > ${O}_kern.txt 2>&1 \
        || { tail -20 ${O}_kern.txt; exit 1; }
      tail -12 ${O}_kern.txt ;;
    pmc)
      rx=${val%%:*}; ctrs=${val#*:}
      inc=(); [ -n "$rx" ] && inc=(--kernel-include-regex "$rx")
      timeout -s KILL 120 rocprofv3 --pmc $ctrs "${inc[@]}" \
        --output-format csv -d $R/${O}_pmc_$n -o p \
        -- python3 $R/bench.py --steps 2 --warmup 2 --small-batch 0 $PMC_ARGS \
        > ${O}_pmc_$n.log 2>&1 || { tail -20 ${O}_pmc_$n.log; exit 1; }
      echo "pmc pass $n done" ;;
    gaps)
      # inter-kernel gap distribution of bench.py ARGS (e.g. --batch,128,--graph,on)
      timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/${O}_gaps_$n -o g \
        -- python3 $R/bench.py --steps 8 --warmup 3 --small-batch 0 $(args_of "$val") \
        > ${O}_gaps_$n.log 2>&1 || { tail -20 ${O}_gaps_$n.log; exit 1; }
      f=$(find ${O}_gaps_$n -name "*kernel_trace.csv" | head -1)
      python3 tools/gap_stats.py $f 5 > ${O}_gaps_$n.txt; rm -f $f; tail -1 ${O}_gaps_$n.txt ;;
    trace)
      # kernel trace of the same run shape as the pmc passes (durations for pmc_dispatch.py)
      timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/${O}_trace -o t \
        -- python3 $R/bench.py --steps 2 --warmup 2 --small-batch 0 $PMC_ARGS \
        > ${O}_trace.log 2>&1 || { tail -20 ${O}_trace.log; exit 1; }
      echo "trace done" ;;
    py)
      s=${val%%,*}; a=""
      [[ "$val" == *","* ]] && a=${val#*,}
      timeout -k 10 300 python $s $(args_of "$a") > ${O}_py_$n.log 2>&1 \
        || { tail -30 ${O}_py_$n.log; exit 1; }
      tail -15 ${O}_py_$n.log ;;
    env) export "$val"; echo "export $val" ;;
    *) echo "unknown step $name"; exit 2 ;;
  esac
done
echo "== done ($(date +%T))"
