#!/bin/bash
# A timing-probe or A/B build of the library from a patched copy of the
# sources (the product sources stay as they are):
#   tools/build_probe.sh NAME PATCH.py   -> adam_amd/ab/libadam_bqsr_NAME.so
# PATCH.py edits the copy in place: it gets the copy's csrc directory as argv[1].
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
N=$1; P=$2
T=$(mktemp -d /tmp/probe_XXXX)
mkdir -p "$T/adam_amd" "$T/include"
cp -r "$R/adam_amd/csrc" "$T/adam_amd/"
cp "$R"/include/*.h "$T/include/"
python3 "$P" "$T/adam_amd/csrc"
mkdir -p "$R/adam_amd/ab"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -fPIC -shared \
  -x hip "$T/adam_amd/csrc/bqsr_capi.cpp" -o "$R/adam_amd/ab/libadam_bqsr_$N.so" -lpthread -lz -ldl
rm -rf "$T"
echo built adam_amd/ab/libadam_bqsr_$N.so
