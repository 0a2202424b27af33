#!/bin/bash
# tools/gpu_r04_cfgs.sh TAG: cfg4 profile + bench (tools/gpu_r04_prof.sh), the
# cfg5 bench line (streamed partitions, compacted outputs), cfg3 profile +
# bench.  Stops at the first failure.
set -e
TAG=$1
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
bash tools/gpu_r04_prof.sh "$TAG" cfg4 0
timeout -k 10 900 python -u bench.py --config cfg5 > "$O/bench_cfg5.json" 2> "$O/bench_cfg5.err"
cat "$O/bench_cfg5.json"
bash tools/gpu_r04_prof.sh "$TAG" cfg3 0
echo done
