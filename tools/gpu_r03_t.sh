#!/bin/bash
# lean observe chunks-per-step A/B (gpurun): tools/gpu_r03_t.sh TAG LIB...
set -e
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity_more.py tests/test_gpu_staged.py -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 \
  || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
LIBS=()
for l in "$@"; do LIBS+=("$R/$l"); done
bash tools/ab_lib.sh $TAG "cfg2 cfg3" - "${LIBS[@]}"
echo done
