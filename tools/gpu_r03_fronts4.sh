#!/bin/bash
# lean observe on bucketed batches with fronts: parity, then cfg4 A/B against the chunk walk (gpurun)
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out/r03fr6
timeout -k 10 600 python -u -m pytest tests/test_gpu_forms.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03fr6/pytest_forms.log 2>&1 || { tail -30 gpurun_out/r03fr6/pytest_forms.log; exit 1; }
tail -1 gpurun_out/r03fr6/pytest_forms.log
bash tools/ab_env.sh r03fr6/ab4 cfg4 "ADAM_BQSR_OBSERVE=chunks" "ADAM_BQSR_OBSERVE=lean" "ADAM_BQSR_OBSERVE=chunks" "ADAM_BQSR_OBSERVE=lean"
