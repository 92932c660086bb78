set -o pipefail
bash scripts/gpu/pmc_tool.sh r6k_a "FETCH_SIZE GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" tools/bench_stem_bwd.py 1024 2 > /dev/null && \
bash scripts/gpu/pmc_tool.sh r6k_b "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum" tools/bench_stem_bwd.py 1024 2 > /dev/null && \
grep -A12 "stem_pool_wgrad\|stem_wgrad_kernel" gpurun_out/r6k_a_pmc.txt gpurun_out/r6k_b_pmc.txt
