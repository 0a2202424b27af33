#!/bin/bash
# r05z: GPU suite; the tree (prep listed reads in bqsr_prep_complex through LDS-typed pointers,
# fold tiles / segs / chain latency cuts) and the tree + 32-byte MD fast path, against HEAD
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_r05_check_ab.sh r05z "LIB=adam_amd/ab/libadam_bqsr_prev.so" "" "LIB=adam_amd/ab/libadam_bqsr_md32.so"
bash tools/gpu_r05_ab.sh r05z cfg4 "LIB=adam_amd/ab/libadam_bqsr_prev.so" "" "LIB=adam_amd/ab/libadam_bqsr_md32.so"
