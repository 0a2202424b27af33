#!/bin/bash
# r05y: GPU suite; prep_one through LDS-typed pointers (+ listed reads in bqsr_prep_complex,
# batched fold-tile loads, fold_segs at 1024 threads) against HEAD on cfg2 / cfg4
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_r05_check_ab.sh r05y "LIB=adam_amd/ab/libadam_bqsr_prev.so" ""
bash tools/gpu_r05_ab.sh r05y cfg4 "LIB=adam_amd/ab/libadam_bqsr_prev.so" ""
