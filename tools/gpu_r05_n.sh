#!/bin/bash
# GPU suite, prep A/B on cfg2, then the end-to-end gzip transform
set -e
TAG=$1
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 \
  || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
bash tools/gpu_r05_ab.sh "$TAG" cfg2 "" "LIB=adam_amd/ab/libadam_bqsr_pc4096.so" "LIB=adam_amd/ab/libadam_bqsr_pw5.so"
bash tools/gpu_r05_e2e.sh "$TAG/e2e" 10000000
