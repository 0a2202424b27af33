#!/bin/bash
# r05aq: deferred trims resolved from the lean observe step's own qual loads -- GPU suite, then cfg2 HEAD / tree twice, cfg3 HEAD / tree
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_r05_check_ab.sh r05aq "LIB=adam_amd/ab/libadam_bqsr_head.so" "" "LIB=adam_amd/ab/libadam_bqsr_head.so" ""
bash tools/gpu_r05_ab.sh r05aq cfg3 "LIB=adam_amd/ab/libadam_bqsr_head.so" ""
