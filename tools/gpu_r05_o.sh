#!/bin/bash
# r05o: GPU suite, observe load-order A/B (HEAD vs working tree), SQ instruction counts
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_r05_check_ab.sh r05o "LIB=adam_amd/ab/libadam_bqsr_prev.so" ""
bash tools/pmc_sq.sh r05o_sq "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_SMEM SQ_INSTS_BRANCH" --config cfg2
