#!/bin/bash
# r05ai: the apply kernel clears the slot bitmap for the next prep (no fill pass) -- GPU suite, then cfg2 / cfg4 HEAD against the tree
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_r05_check_ab.sh r05ai "LIB=adam_amd/ab/libadam_bqsr_head.so" ""
bash tools/gpu_r05_ab.sh r05ai cfg4 "LIB=adam_amd/ab/libadam_bqsr_head.so" ""
bash tools/gpu_r05_ab.sh r05ai_red cfg2 "" "LIB=adam_amd/ab/libadam_bqsr_red4.so" "LIB=adam_amd/ab/libadam_bqsr_red32.so" "LIB=adam_amd/ab/libadam_bqsr_red64.so"
