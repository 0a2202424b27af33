#!/bin/bash
# r05w: GPU suite (long-MD edge cases); MD tags up to 32 bytes in prep's lock-step form, against HEAD on cfg2 / cfg4
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_r05_check_ab.sh r05w "LIB=adam_amd/ab/libadam_bqsr_prev.so" ""
bash tools/gpu_r05_ab.sh r05w cfg4 "LIB=adam_amd/ab/libadam_bqsr_prev.so" ""
