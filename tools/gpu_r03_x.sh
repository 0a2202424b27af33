#!/bin/bash
# round-3 final: cfg5 (streamed, parity over the table / em of all partitions and the chars of two)
# and cfg4 bench lines with the final build (gpurun): tools/gpu_r03_x.sh TAG
set -e
TAG=$1
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
timeout -k 10 700 python -u bench.py --config cfg5 --steps 4 --warmup 1 --no-cpu-baseline > "$O/bench_cfg5.json" 2> "$O/bench_cfg5.err"
python3 -c "import json; d=json.load(open('$O/bench_cfg5.json')); print('cfg5', round(d['ms_per_step'],1), d['pcie'], d.get('parity',{}).get('ok'))"
timeout -k 10 600 python -u bench.py --config cfg4 > "$O/bench_cfg4.json" 2> "$O/bench_cfg4.err"
python3 -c "import json; d=json.load(open('$O/bench_cfg4.json')); print('cfg4', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['roofline']['kernel_ms'].items()}, d.get('parity',{}).get('ok'))"
echo done
