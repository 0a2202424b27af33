#!/bin/bash
# r05p: apply timing probes on cfg2 (clean-row test, contexts, char-table reads),
# then the LDS counters of the per-base kernels on cfg2 and cfg4
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_r05_ab.sh r05p cfg2 "" "LIB=adam_amd/ab/libadam_bqsr_apply_no_badtest.so" \
  "LIB=adam_amd/ab/libadam_bqsr_apply_no_ctx.so" "LIB=adam_amd/ab/libadam_bqsr_apply_no_lut.so"
L="SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_LDS"
bash tools/pmc_sq.sh r05p_lds_cfg2 "$L" --config cfg2
bash tools/pmc_sq.sh r05p_lds_cfg4 "$L" --config cfg4
