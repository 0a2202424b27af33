#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out/r02u
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity_more.py -m gpu -x -q --timeout 300 --timeout-method thread -k "sites" > gpurun_out/r02u/pytest.log 2>&1 || { tail -30 gpurun_out/r02u/pytest.log; exit 1; }
tail -2 gpurun_out/r02u/pytest.log
bash tools/gpu_cfg.sh r02u cfg3 --no-cpu-baseline --no-parity --steps 5 --warmup 1
