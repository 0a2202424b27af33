#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out/r02y
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r02y/pytest.log 2>&1 || { tail -30 gpurun_out/r02y/pytest.log; exit 1; }
tail -1 gpurun_out/r02y/pytest.log
bash tools/gpu_cfg.sh r02y cfg2 --no-cpu-baseline --no-parity 2>&1 | grep -E "^[0-9]|prep"
bash tools/gpu_cfg.sh r02y cfg3 --no-cpu-baseline --no-parity --steps 5 --warmup 1 2>&1 | grep -E "^[0-9]|prep"
