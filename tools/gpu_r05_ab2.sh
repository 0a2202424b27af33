#!/bin/bash
# r05ab: the listed reads of cfg2's first prep blocks (device printf diagnostic build)
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out/r05ab
ADAM_BQSR_LIB=$R/adam_amd/ab/libadam_bqsr_complex_show.so timeout -k 10 300 python3 bench.py --config cfg2 --no-cpu-baseline --no-parity --steps 1 --warmup 0 --event-steps 0 > gpurun_out/r05ab/show.log 2>&1 || true
grep LISTED gpurun_out/r05ab/show.log | sort | uniq | head -60 || true
