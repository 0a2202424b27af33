#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out/r02ac
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r02ac/all.log 2>&1 || { tail -30 gpurun_out/r02ac/all.log; exit 1; }
tail -2 gpurun_out/r02ac/all.log
bash tools/ab_cfg.sh r02ac cfg3 -
bash tools/ab_cfg.sh r02ac2 cfg2 -
