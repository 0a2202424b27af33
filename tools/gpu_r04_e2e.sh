#!/bin/bash
# tools/gpu_r04_e2e.sh TAG READS [TESTS]: the f1/f2 throughput lines --
# transform SAM -> ADAM end to end (tools/bench_adam.py; snappy, and the
# reference's gzip), its kernel stats, and the ADAM Parquet read
# (tools/bench_parquet.py).  TESTS: pytest files to run first.
set -e
TAG=$1
READS=${2:-10000000}
TESTS=${3:-}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -v --timeout 300 --timeout-method thread > "$O/pytest_e2e.log" 2>&1 \
    || { rc=$?; tail -40 "$O/pytest_e2e.log"; exit $rc; }
  tail -1 "$O/pytest_e2e.log"
fi
timeout -k 10 400 python -u tools/bench_adam.py --reads $READS --compression snappy > "$O/e2e_sam_snappy.json" 2> "$O/e2e_sam_snappy.log"
cat "$O/e2e_sam_snappy.json"
timeout -k 10 400 python -u tools/bench_adam.py --reads $READS --compression snappy --bam > "$O/e2e_bam_snappy.json" 2> "$O/e2e_bam_snappy.log"
cat "$O/e2e_bam_snappy.json"
timeout -k 10 400 python -u tools/bench_adam.py --reads $READS --compression gzip > "$O/e2e_sam_gzip.json" 2> "$O/e2e_sam_gzip.log"
cat "$O/e2e_sam_gzip.json"
timeout -k 10 400 python -u tools/bench_parquet.py --reads 2000000 > "$O/parquet_read.json" 2> "$O/parquet_read.log"
cat "$O/parquet_read.json"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/e2e_stats" -o run --output-format csv -- \
  python3 "$R/tools/bench_adam.py" --reads $READS --compression snappy > "$O/e2e_stats.log" 2>&1
cd "$R"
KS=$(find "$O/e2e_stats" -name "*kernel_stats.csv" | head -1)
cp "$KS" "$O/e2e_kernel_stats.csv"
head -25 "$O/e2e_kernel_stats.csv"
