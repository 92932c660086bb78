#!/bin/bash
# comm-aware persistent grids: reserved-grid GPU tests, then bench A/B under an emulated
# overlapping collective (bench.py --emulate-comm BLOCKS:US [--comm-reserve BLOCKS])
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
out=gpurun_out/comm_reserve.txt
: > $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "comm_reserve" tests/test_models_gpu.py::test_step_phase_timers -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_reserve.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/t_reserve.log; exit 1; }
tail -1 gpurun_out/t_reserve.log
run() {
  echo "== $*" >> $out
  timeout -k 10 180 python bench.py --steps 20 --warmup 5 "$@" 2>/dev/null | tail -1 >> $out || exit 1
  tail -1 $out | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$*', d['ms_per_step'], d.get('phases_ms',''))"
}
run --timers on
run
for spec in "8:2000" "8:6000" "32:2000" "32:6000"; do
  b=${spec%%:*}
  run --emulate-comm $spec
  run --emulate-comm $spec --comm-reserve $b
done
run
