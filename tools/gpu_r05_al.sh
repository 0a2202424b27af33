#!/bin/bash
# r05al: per-read event records (read order, no sites) -- GPU suite, then cfg2 HEAD / tree / tree with records off
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_r05_check_ab.sh r05al "LIB=adam_amd/ab/libadam_bqsr_head.so" "" "--tune records=0" "LIB=adam_amd/ab/libadam_bqsr_head.so" ""
