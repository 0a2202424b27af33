#!/bin/bash
# r05af: fold_hist counting pairs of quals -- GPU suite, then cfg4 HEAD against the tree
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/r05af"; mkdir -p "$O"; cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 \
  || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
bash tools/gpu_r05_ab.sh r05af cfg4 "LIB=adam_amd/ab/libadam_bqsr_head.so" ""
