#!/bin/bash
# GPU suite, then an A/B of bench variants on cfg2:  tools/gpu_r05_check_ab.sh TAG "ARGS_A" "ARGS_B" ...
set -e
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 \
  || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
bash tools/gpu_r05_ab.sh "$TAG" cfg2 "$@"
