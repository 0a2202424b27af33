#!/bin/bash
# r05at: apply at 5 chunks in flight a lane (42 spilled VGPRs) against the product (4) -- cfg2 twice, cfg4 once
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
A="LIB=adam_amd/ab/libadam_bqsr_apply5.so"
bash tools/gpu_r05_ab.sh r05at cfg2 "" "$A" "" "$A"
bash tools/gpu_r05_ab.sh r05at cfg4 "" "$A"
