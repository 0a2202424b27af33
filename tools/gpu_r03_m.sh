#!/bin/bash
# Stream tests, then cfg5 with kernel-copy D2H (default) and DMA D2H:
# tools/gpu_r03_m.sh TAG
set -e
TAG=$1
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_multirank.py -x -q \
  --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
for m in kernel dma; do
  timeout -k 10 500 python -u bench.py --config cfg5 --steps 4 --warmup 1 --d2h $m > "$O/bench_cfg5_$m.json" 2> "$O/bench_cfg5_$m.err"
  python3 -c "import json; d=json.load(open('$O/bench_cfg5_$m.json')); print('cfg5 $m', round(d['ms_per_step'],1), d['pcie'], d.get('parity',{}).get('ok'))"
done
