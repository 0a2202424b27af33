#!/bin/bash
# bench line + kernel stats of one config: tools/gpu_cfg.sh TAG CONFIG [bench args]
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1
CFG=$2
shift 2
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u bench.py --config "$CFG" "$@" > "$O/bench_$CFG.json" 2> "$O/bench_$CFG.err"
python -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['ms_per_step'],d['roofline']['kernel_ms'],d.get('parity',{}).get('ok'))" "$O/bench_$CFG.json"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/stats_$CFG" -o run --output-format csv -- \
  python3 "$R/bench.py" --config "$CFG" --no-cpu-baseline --no-parity --steps 5 --warmup 1 "$@" > "$O/stats_$CFG.log" 2>&1
find "$O/stats_$CFG" -name "*kernel_stats.csv" -exec head -14 {} \;
