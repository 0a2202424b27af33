#!/bin/bash
# tools/gpu_r04_e2e.sh TAG READS: the f1/f2 throughput lines -- transform SAM
# -> ADAM end to end (tools/bench_adam.py; snappy and the reference's gzip),
# and the ADAM Parquet read (tools/bench_parquet.py).
set -e
TAG=$1
READS=${2:-10000000}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/bench_adam.py --reads $READS --compression snappy > "$O/e2e_sam_snappy.json" 2> "$O/e2e_sam_snappy.log"
cat "$O/e2e_sam_snappy.json"
timeout -k 10 400 python -u tools/bench_adam.py --reads $READS --compression gzip > "$O/e2e_sam_gzip.json" 2> "$O/e2e_sam_gzip.log"
cat "$O/e2e_sam_gzip.json"
timeout -k 10 400 python -u tools/bench_parquet.py --reads 2000000 > "$O/parquet_read.json" 2> "$O/parquet_read.log"
cat "$O/parquet_read.json"
