#!/bin/bash
# SQ counters of the final tree's per-base kernels, cfg2 and cfg4: VALU,
# LDS bank-conflict / active cycles, waves, busy cycles (one PMC pass each).
# tools/gpu_r04_sq.sh TAG
set -e
TAG=$1
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
for c in cfg2 cfg4; do
  echo "== $c"
  bash tools/pmc_sq.sh "$TAG/$c" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES" --config $c
done
