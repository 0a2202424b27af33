#!/bin/bash
# Kernel stats of candidate libraries against the in-tree one, then one SQ
# LDS-counter pass per library on cfg2: tools/gpu_ab_libs.sh TAG "cfg2 cfg3" LIB.so ...
set -e
TAG=$1
CFGS=$2
shift 2
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
LIBS=()
for lib in "$@"; do
  case "$lib" in /*) ;; *) lib="$R/$lib" ;; esac
  LIBS+=("$lib")
done
bash tools/ab_lib.sh $TAG "$CFGS" - "${LIBS[@]}"
i=0
for lib in - "${LIBS[@]}"; do
  i=$((i+1))
  [ "$lib" = - ] && lib="$R/adam_amd/libadam_bqsr.so"
  echo "== SQ cfg2 $lib"
  ADAM_BQSR_LIB="$lib" bash tools/pmc_sq.sh $TAG/sq$i "SQ_INSTS_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY" --config cfg2 | grep observe_kernel
done
