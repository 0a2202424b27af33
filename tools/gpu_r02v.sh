#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_quick2.sh r02v
bash tools/gpu_cfg.sh r02v cfg3 --no-cpu-baseline --no-parity --steps 5 --warmup 1
