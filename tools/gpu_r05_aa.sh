#!/bin/bash
# r05aa: what bqsr_prep_complex costs on cfg2 -- its launch alone, its blocks' list sizes; prep loads unconditional
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out/r05aa
ADAM_BQSR_LIB=$R/adam_amd/ab/libadam_bqsr_complex_count.so timeout -k 10 300 python3 bench.py --config cfg2 --no-cpu-baseline --no-parity --steps 1 --warmup 0 --event-steps 0 > gpurun_out/r05aa/count.log 2>&1 || true
grep -c COMPLEX gpurun_out/r05aa/count.log || true
grep COMPLEX gpurun_out/r05aa/count.log | head -20 || true
bash tools/gpu_r05_ab.sh r05aa cfg2 "" "LIB=adam_amd/ab/libadam_bqsr_complex_empty.so" "LIB=adam_amd/ab/libadam_bqsr_uncond.so"
