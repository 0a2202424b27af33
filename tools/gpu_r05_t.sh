#!/bin/bash
# r05t: GPU suite; cfg2 / cfg4: HEAD, the tree, the tree with offset-order table reads
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_r05_check_ab.sh r05t "LIB=adam_amd/ab/libadam_bqsr_prev.so" "" "LIB=adam_amd/ab/libadam_bqsr_korder.so"
bash tools/gpu_r05_ab.sh r05t cfg4 "LIB=adam_amd/ab/libadam_bqsr_prev.so" "" "LIB=adam_amd/ab/libadam_bqsr_korder.so"
