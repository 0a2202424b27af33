#!/bin/bash
# One rocprofv3 --pmc pass for FETCH_SIZE and one for WRITE_SIZE over a short
# bench run (GPU box):  tools/fetch_profile.sh NAME [bench args...]
set -e
NAME=$1; shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
export TMPDIR=/tmp
mkdir -p "$R/gpurun_out/$NAME"
cd /tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/$NAME/pmc3" -o run --output-format csv -- \
  python3 "$R/bench.py" --no-cpu-baseline "$@" > "$R/gpurun_out/$NAME/pmc3.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/$NAME/pmc4" -o run --output-format csv -- \
  python3 "$R/bench.py" --no-cpu-baseline "$@" > "$R/gpurun_out/$NAME/pmc4.log" 2>&1
