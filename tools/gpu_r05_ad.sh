#!/bin/bash
# r05ad: GPU suite; the tree (prep's long form for listed reads) against HEAD on cfg2 / cfg4
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_r05_check_ab.sh r05ad "LIB=adam_amd/ab/libadam_bqsr_prev.so" ""
bash tools/gpu_r05_ab.sh r05ad cfg4 "LIB=adam_amd/ab/libadam_bqsr_prev.so" ""
