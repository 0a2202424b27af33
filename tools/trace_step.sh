#!/bin/bash
# kernel trace of bench steps (no stats), for gap analysis: tools/trace_step.sh TAG [bench args]
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1
shift
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$O/trace" -o run --output-format csv -- \
  python3 "$R/bench.py" --no-cpu-baseline --no-parity --steps 6 --warmup 1 --event-every 1000 "$@" > "$O/trace.log" 2>&1
echo traced
