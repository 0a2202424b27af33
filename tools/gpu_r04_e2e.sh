#!/bin/bash
# tools/gpu_r04_e2e.sh TAG READS: the end-to-end transform -> ADAM throughput
# lines (tools/bench_adam.py) -- SAM with and without MarkDuplicates, BAM.
set -e
TAG=$1
READS=${2:-10000000}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/bench_adam.py --reads $READS --compression snappy > "$O/e2e_sam_md.json" 2> "$O/e2e_sam_md.log"
cat "$O/e2e_sam_md.json"
timeout -k 10 400 python -u tools/bench_adam.py --reads $READS --compression snappy --partition-bytes 8000000000 > "$O/e2e_sam_md_1p.json" 2> "$O/e2e_sam_md_1p.log"
cat "$O/e2e_sam_md_1p.json"
