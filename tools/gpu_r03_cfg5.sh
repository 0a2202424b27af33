#!/bin/bash
# Round-3 pass (via gpurun): new GPU tests (BAM, MarkDuplicates), then the cfg5
# stream modes: tools/gpu_r03_cfg5.sh TAG
set -e
TAG=$1
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_sam.py -x -q --timeout 300 --timeout-method thread > "$O/pytest_sam.log" 2>&1 || { tail -40 "$O/pytest_sam.log"; exit 1; }
tail -1 "$O/pytest_sam.log"
for m in serial zerocopy pipe; do
  timeout -k 10 400 python -u bench.py --config cfg5 --steps 3 --warmup 1 --stream-mode $m --no-cpu-baseline --no-parity > "$O/cfg5_$m.json" 2> "$O/cfg5_$m.err"
  python3 -c "import json; d=json.load(open('$O/cfg5_$m.json')); print('$m', round(d['ms_per_step'],1), d['pcie'], d['roofline']['kernel_ms'])"
done
echo done
