#!/bin/bash
# The library as of a git revision, for an A/B on one box:
#   tools/build_rev.sh REV NAME  -> adam_amd/ab/libadam_bqsr_NAME.so
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
REV=$1; N=$2
T=$(mktemp -d /tmp/rev_XXXX)
git -C "$R" archive "$REV" adam_amd/csrc include | tar -x -C "$T"
mkdir -p "$R/adam_amd/ab"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -fPIC -shared \
  -x hip "$T/adam_amd/csrc/bqsr_capi.cpp" -o "$R/adam_amd/ab/libadam_bqsr_$N.so" -lpthread -lz -ldl
rm -rf "$T"
echo built adam_amd/ab/libadam_bqsr_$N.so from $REV
