#!/bin/bash
# r05x: GPU suite; prep's listed reads all in bqsr_prep_complex + the fold tiles' batched
# qual loads, against HEAD on cfg2 / cfg4; fold_segs at 1024 threads on cfg2
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_r05_check_ab.sh r05x "LIB=adam_amd/ab/libadam_bqsr_prev.so" "" "LIB=adam_amd/ab/libadam_bqsr_segs1024.so"
bash tools/gpu_r05_ab.sh r05x cfg4 "LIB=adam_amd/ab/libadam_bqsr_prev.so" ""
