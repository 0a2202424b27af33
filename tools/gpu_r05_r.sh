#!/bin/bash
# r05r: GPU suite; apply's folded-clean skip against HEAD on cfg2 and cfg4
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_r05_check_ab.sh r05r "LIB=adam_amd/ab/libadam_bqsr_prev.so" ""
bash tools/gpu_r05_ab.sh r05r cfg4 "LIB=adam_amd/ab/libadam_bqsr_prev.so" ""
