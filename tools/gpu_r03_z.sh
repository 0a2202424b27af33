#!/bin/bash
# kernel-form tests, then the arithmetic-context candidate (parity + cfg2 / cfg4 A/B) (gpurun)
set -e
TAG=$1; CAND=$2
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_forms.py -x -q --timeout 300 --timeout-method thread > "$O/pytest_forms.log" 2>&1 \
  || { tail -40 "$O/pytest_forms.log"; exit 1; }
tail -1 "$O/pytest_forms.log"
ADAM_BQSR_LIB="$R/$CAND" timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity_more.py -x -q --timeout 300 --timeout-method thread > "$O/pytest_cand.log" 2>&1 \
  || { tail -40 "$O/pytest_cand.log"; exit 1; }
tail -1 "$O/pytest_cand.log"
bash tools/ab_lib.sh $TAG "cfg2 cfg4" - "$R/$CAND"
echo done
