#!/bin/bash
# GPU suite, cfg4 A/B of the key-major records (the previous revision's
# library against the tree's), and one SQ stall-breakdown pass on cfg2
set -e
TAG=$1
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 \
  || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
bash tools/gpu_r05_ab.sh "$TAG" cfg4 "LIB=adam_amd/ab/libadam_bqsr_prev.so" ""
bash tools/pmc_sq.sh "$TAG/sq" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA" --config cfg2
