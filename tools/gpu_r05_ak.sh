#!/bin/bash
# r05ak: GPU suite; cfg2 -- HEAD (fill) / bitmap cleared by apply / by the fold chain's spare workgroups (tree) / tree with fused prep; cfg4 HEAD / tree
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_r05_check_ab.sh r05ak "LIB=adam_amd/ab/libadam_bqsr_head.so" "LIB=adam_amd/ab/libadam_bqsr_apply_zero.so" "" "--tune fused_prep=1" "LIB=adam_amd/ab/libadam_bqsr_head.so" "LIB=adam_amd/ab/libadam_bqsr_apply_zero.so" ""
bash tools/gpu_r05_ab.sh r05ak cfg4 "LIB=adam_amd/ab/libadam_bqsr_head.so" ""
