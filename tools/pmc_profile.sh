#!/bin/bash
# PMC passes over a short bench run (one counter group per rocprofv3 run, as
# MI355X_MICROARCH.md's rocprofv3 section prescribes: <= 8 SQ, 4 TCC, 4 TCP,
# 2 TA, 2 TD, 2 GRBM per pass).  Usage (GPU box):
#   tools/pmc_profile.sh OUTDIR [bench args...]
set -e
OUT=$(mkdir -p "$1" && cd "$1" && pwd); shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
export TMPDIR=/tmp
mkdir -p "$OUT"
cd /tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
           "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d $OUT/pmc$i -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline "$@" > $OUT/pmc$i.log 2>&1
done
