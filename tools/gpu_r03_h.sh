#!/bin/bash
# GPU tests on a candidate library, its kernel stats against the in-tree one,
# SQ counters of cfg4, then the cfg3 / cfg4 measurement pass (tools/gpu_r03.sh):
# tools/gpu_r03_h.sh TAG CANDIDATE.so ["cfg3 cfg4"]
set -e
TAG=$1
LIB=$2
CONFIGS=${3:-"cfg3 cfg4"}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
case "$LIB" in /*) ;; *) LIB="$R/$LIB" ;; esac
rc=0
ADAM_BQSR_LIB="$LIB" timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$O/pytest_candidate.log" 2>&1 || rc=$?
if [ $rc = 0 ]; then
  echo "candidate tests: $(tail -1 "$O/pytest_candidate.log")"
elif [ $rc = 1 ]; then  # failed assertions only: the GPU is fine, measure on
  echo "candidate tests FAILED:"; tail -30 "$O/pytest_candidate.log"
else  # crash, abort or time limit: nothing more on the GPU in this call
  echo "candidate tests exit $rc:"; tail -30 "$O/pytest_candidate.log"; exit $rc
fi
bash tools/ab_lib.sh $TAG/ab "cfg2 cfg3" - "$LIB"
bash tools/pmc_sq.sh $TAG/sqa "SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVES SQ_WAVE_CYCLES" --config cfg4
bash tools/pmc_sq.sh $TAG/sqb "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_LDS_ADDR_CONFLICT SQ_WAIT_ANY" --config cfg4
bash tools/gpu_r03.sh $TAG "$CONFIGS" 0
