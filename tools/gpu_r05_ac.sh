#!/bin/bash
# r05ac: prep_one clock stamps (diagnostic build); GPU suite; the tree against HEAD on cfg2 / cfg4
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out/r05ac
ADAM_BQSR_LIB=$R/adam_amd/ab/libadam_bqsr_prep_clock.so timeout -k 10 300 python3 bench.py --config cfg2 --no-cpu-baseline --no-parity --steps 1 --warmup 0 --event-steps 0 > gpurun_out/r05ac/clock.log 2>&1 || true
grep PCLK gpurun_out/r05ac/clock.log | head -24 || true
bash tools/gpu_r05_check_ab.sh r05ac "LIB=adam_amd/ab/libadam_bqsr_prev.so" ""
bash tools/gpu_r05_ab.sh r05ac cfg4 "LIB=adam_amd/ab/libadam_bqsr_prev.so" ""
