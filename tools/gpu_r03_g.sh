#!/bin/bash
# GPU tests, the cfg5 line (pipelined, parity), then tools/gpu_r03.sh for CONFIGS
# tools/gpu_r03_g.sh TAG "cfg2"
set -e
TAG=$1
CONFIGS=${2:-cfg2}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
tail -1 "$O/smoke.log"
timeout -k 10 500 python -u bench.py --config cfg5 --steps 4 --warmup 1 > "$O/bench_cfg5.json" 2> "$O/bench_cfg5.err"
python3 -c "import json; d=json.load(open('$O/bench_cfg5.json')); print('cfg5', round(d['ms_per_step'],1), d['pcie'], d.get('parity',{}).get('ok'))"
bash tools/gpu_r03.sh $TAG "$CONFIGS" 0
