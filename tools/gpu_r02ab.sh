#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out/r02ab
timeout -k 10 600 python -u -m pytest tests/test_gpu_sam.py -q --timeout 300 --timeout-method thread -k "sam or utf8 or transform or parse" > gpurun_out/r02ab/sam.log 2>&1 || { grep -E "^E " gpurun_out/r02ab/sam.log | head -20; }
tail -2 gpurun_out/r02ab/sam.log
timeout -k 10 300 python -u tools/bench_ingest.py --reads 2000000 > gpurun_out/r02ab/ingest.json 2> gpurun_out/r02ab/ingest.err
cat gpurun_out/r02ab/ingest.json
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r02ab/prof" -o run --output-format csv -- python3 "$R/tools/bench_ingest.py" --reads 2000000 --reps 2 > "$R/gpurun_out/r02ab/prof.log" 2>&1
find "$R/gpurun_out/r02ab/prof" -name "*kernel_stats.csv" -exec cat {} \;
