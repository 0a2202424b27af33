#!/bin/bash
# An A/B build of the library with extra defines (never the product library):
# tools/build_variant.sh NAME -DFLAG ...  ->  adam_amd/ab/libadam_bqsr_NAME.so
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
N=$1; shift
cd "$R"; mkdir -p adam_amd/ab
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -fPIC -shared "$@" \
  -x hip adam_amd/csrc/bqsr_capi.cpp -o adam_amd/ab/libadam_bqsr_$N.so -lpthread -lz -ldl
echo built adam_amd/ab/libadam_bqsr_$N.so
