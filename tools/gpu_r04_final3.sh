#!/bin/bash
# tools/gpu_r04_final3.sh TAG: the cfg5 bench line, the f1/f2 throughput
# lines (tools/gpu_r04_e2e.sh) and the prep timing probe (listed reads
# skipped: their share of bqsr_prep_kernel) on cfg2.
set -e
TAG=$1
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py --config cfg5 > "$O/bench_cfg5.json" 2> "$O/bench_cfg5.err"
python3 - "$O/bench_cfg5.json" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        print("cfg5", round(d["ms_per_step"], 2), d["pcie"], d["roofline"]["kernel_ms"], round(d["roofline"]["frac"] or 0, 3), d["parity"]["ok"])
PY
bash tools/gpu_r04_e2e.sh "$TAG" 10000000
bash tools/ab_lib.sh "$TAG/probe" cfg2 - "$R/adam_amd/libadam_bqsr_prep_probe.so" > "$O/prep_probe.txt" 2>&1
cat "$O/prep_probe.txt"
echo done
