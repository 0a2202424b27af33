#!/bin/bash
# r05ae: prep's long form for listed reads -- tree (prep_one outlined) / prep_one inline / without the long form / HEAD
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_r05_ab.sh r05ae cfg2 "LIB=adam_amd/ab/libadam_bqsr_no_long.so" "" "LIB=adam_amd/ab/libadam_bqsr_one_inline.so" "LIB=adam_amd/ab/libadam_bqsr_prev.so"
bash tools/gpu_r05_ab.sh r05ae cfg4 "LIB=adam_amd/ab/libadam_bqsr_no_long.so" "" "LIB=adam_amd/ab/libadam_bqsr_one_inline.so"
