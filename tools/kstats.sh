#!/bin/bash
# Kernel-trace statistics of a short bench run (GPU box):
#   tools/kstats.sh NAME [bench args...]  ->  gpurun_out/NAME/ (rocprofv3 csv) + gpurun_out/NAME.log
set -e
NAME=$1; shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/$NAME" -o run --output-format csv -- \
  python3 "$R/bench.py" --no-cpu-baseline "$@" > "$R/gpurun_out/$NAME.log" 2>&1
f=$(find "$R/gpurun_out/$NAME" -name '*kernel_stats.csv' | head -1)
cut -d, -f1-8 "$f" | cut -c1-160
