#!/bin/bash
# Quick GPU pass: -m gpu suite, then the default bench line (parity check
# included) and a rocprofv3 kernel-stats run of the same workload.
#   tools/gpu_quick2.sh TAG [bench args...]
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1
shift
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -2 "$O/pytest.log"
timeout -k 10 500 python -u bench.py "$@" > "$O/bench.json" 2> "$O/bench.err"
python -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['ms_per_step'],d['roofline']['kernel_ms'],d.get('parity',{}).get('ok'))" "$O/bench.json"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/stats" -o run --output-format csv -- \
  python3 "$R/bench.py" --no-cpu-baseline --steps 10 --warmup 1 "$@" > "$O/stats.log" 2>&1
find "$O/stats" -name "*kernel_stats.csv" -exec head -14 {} \;
echo done
