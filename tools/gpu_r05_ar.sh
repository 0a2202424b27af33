#!/bin/bash
# r05ar: lean observe at 7 chunks a step (no VGPR spills); apply at 3 chunks in flight (no VGPR spills) on top --
# GPU suite, then cfg2 HEAD / tree / apply3 twice, cfg3 and cfg5 HEAD / tree
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
H="LIB=adam_amd/ab/libadam_bqsr_head.so"; A="LIB=adam_amd/ab/libadam_bqsr_apply3.so"
bash tools/gpu_r05_check_ab.sh r05ar "$H" "" "$A" "$H" "" "$A"
bash tools/gpu_r05_ab.sh r05ar cfg3 "$H" "" "$A"
bash tools/gpu_r05_ab.sh r05ar cfg5 "$H" ""
