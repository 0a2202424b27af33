#!/bin/bash
# r05aj: cfg2 -- HEAD (fill + atomic prep) / tree (the apply kernel clears the bitmap, final_groups by wavefronts) / tree with prep's word-store form without sites
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_r05_ab.sh r05aj cfg2 "LIB=adam_amd/ab/libadam_bqsr_head.so" "" "LIB=adam_amd/ab/libadam_bqsr_store.so" "LIB=adam_amd/ab/libadam_bqsr_head.so" "" "LIB=adam_amd/ab/libadam_bqsr_store.so"
