#!/bin/bash
# tools/gpu_e2e.sh TAG READS: transform SAM -> ADAM end to end at the
# reference's default gzip codec and at snappy (tools/bench_adam.py), the gzip
# run under rocprofv3 (kernel trace; its log is checked for signal / abort
# traces of the generator's process pool)
set -e
TAG=$1
READS=${2:-10000000}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/bench_adam.py --reads $READS --compression gzip > "$O/e2e_sam_gzip.json" 2> "$O/e2e_sam_gzip.log"
cat "$O/e2e_sam_gzip.json"
timeout -k 10 400 python -u tools/bench_adam.py --reads $READS --compression snappy > "$O/e2e_sam_snappy.json" 2> "$O/e2e_sam_snappy.log"
cat "$O/e2e_sam_snappy.json"
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$O/e2e_stats" -o run --output-format csv -- \
  python3 "$R/tools/bench_adam.py" --reads $READS --compression gzip > "$O/e2e_stats.json" 2> "$O/e2e_stats.log"
cd "$R"
cat "$O/e2e_stats.json"
if grep -n "SIGTERM\|Aborted\|caught signal" "$O/e2e_stats.log"; then echo "signal trace in the profiled run"; else echo "profiled run: no signal / abort trace"; fi
