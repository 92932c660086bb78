#!/bin/bash
# Per-dispatch hardware counters of one ResNet-18 b1024 step (single stream): counter list,
# kernel trace (durations) and one rocprofv3 pass per counter group; summarised by
# tools/pmc_dispatch.py into gpurun_out/pmc_r18_summary.txt
set -e
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
export TMPDIR=/tmp PMC_ARGS="--wgrad-stream 0"
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc_counters_list.txt 2>&1 || true
bash scripts/gpu/run.sh pmc trace \
  "pmc=:SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
  "pmc=:FETCH_SIZE GRBM_GUI_ACTIVE" \
  "pmc=:WRITE_SIZE GRBM_GUI_ACTIVE" \
  "pmc=:SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
t=$(find gpurun_out/pmc_trace -name "*kernel_trace.csv" | head -1)
python3 tools/pmc_dispatch.py --trace $t $(find gpurun_out -path "*pmc_pmc_*" -name "*counter_collection.csv") > gpurun_out/pmc_r18_summary.txt
find gpurun_out -path "*pmc_pmc_*" -name "*.csv" -size +5M -delete
tail -5 gpurun_out/pmc_r18_summary.txt
