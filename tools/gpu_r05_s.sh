#!/bin/bash
# r05s: cfg4 apply slowdown hunt (HEAD / tree / offset-order addressing / test in every piece),
# then prep pipeline depth on cfg2
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_r05_ab.sh r05s cfg4 "LIB=adam_amd/ab/libadam_bqsr_prev.so" "" "LIB=adam_amd/ab/libadam_bqsr_korder.so" \
  "LIB=adam_amd/ab/libadam_bqsr_testall.so"
bash tools/gpu_r05_ab.sh r05s cfg2 "" "LIB=adam_amd/ab/libadam_bqsr_pw5.so" "LIB=adam_amd/ab/libadam_bqsr_prep_deep.so"
