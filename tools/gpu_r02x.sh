#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_cfg.sh r02x cfg2 --no-cpu-baseline
bash tools/gpu_cfg.sh r02x cfg3 --no-cpu-baseline --no-parity --steps 5 --warmup 1
