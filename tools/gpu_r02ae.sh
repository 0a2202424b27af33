#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out/r02ae
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r02ae/all.log 2>&1 || { tail -30 gpurun_out/r02ae/all.log; exit 1; }
tail -2 gpurun_out/r02ae/all.log
bash tools/ab_env.sh r02ae cfg2 "ADAM_BQSR_OBSERVE=chunk" "ADAM_BQSR_OBSERVE=read"
bash tools/ab_env.sh r02ae4 cfg4 "ADAM_BQSR_OBSERVE=chunk" "ADAM_BQSR_OBSERVE=read"
bash tools/ab_env.sh r02ae3 cfg3 "ADAM_BQSR_OBSERVE=chunk"
