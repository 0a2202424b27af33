#!/bin/bash
# r05ao: prep workgroups clear their own slots' bitmap words (no fill, no clear in apply) -- GPU suite, then cfg2 / cfg4 HEAD against the tree
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_r05_check_ab.sh r05ao "LIB=adam_amd/ab/libadam_bqsr_head.so" "" "LIB=adam_amd/ab/libadam_bqsr_head.so" ""
bash tools/gpu_r05_ab.sh r05ao cfg4 "LIB=adam_amd/ab/libadam_bqsr_head.so" ""
