#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out/r02af
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r02af/all.log 2>&1 || { tail -30 gpurun_out/r02af/all.log; exit 1; }
tail -1 gpurun_out/r02af/all.log
bash tools/ab_env.sh r02af cfg2 "X=1"
bash tools/ab_env.sh r02af4 cfg4 "X=1"
