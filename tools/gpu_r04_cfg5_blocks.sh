#!/bin/bash
# cfg5: workgroups of the D2H copy kernel (ADAM_BQSR_COPY_BLOCKS) on one box.
# tools/gpu_r04_cfg5_blocks.sh TAG "16 24 32 48"
set -e
TAG=$1
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
for b in $2; do
  ADAM_BQSR_COPY_BLOCKS=$b timeout -k 10 400 python -u bench.py --config cfg5 --no-cpu-baseline --no-parity --steps 6 --warmup 2 \
    > "$O/cfg5_b$b.json" 2> "$O/cfg5_b$b.err"
  python3 - "$O/cfg5_b$b.json" "$b" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        print("blocks", sys.argv[2], "ms/job", round(d["ms_per_step"], 2), "GB/s", round(d["pcie"]["achieved_GBps"], 1))
PY
done
