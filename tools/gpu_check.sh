#!/bin/bash
# One GPU-box check of the current tree (run via gpurun):
#   tools/gpu_check.sh TAG [tests|notests] [configs...]
# -m gpu suite (unless notests), then per config a bench line without the CPU
# leg (cfg2 with it and its full-shard parity check), printing ms/job and the
# per-stage kernel times.  -> gpurun_out/TAG/{pytest.log, bench_<cfg>.json}
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1
MODE=${2:-tests}
shift 2 || true
CFGS=${*:-cfg2 cfg3 cfg4}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
if [ "$MODE" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 \
    || { tail -40 "$O/pytest.log"; exit 1; }
  tail -2 "$O/pytest.log"
fi
for c in $CFGS; do
  extra="--no-parity --no-cpu-baseline"
  [ "$c" = cfg2 ] && extra=""  # the parity check reuses the CPU leg's oracle run
  timeout -k 10 500 python -u bench.py --config "$c" --steps 10 $extra > "$O/bench_$c.json" 2> "$O/bench_$c.err"
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],round(d['ms_per_step'],3),{k:round(v,3) for k,v in d['roofline']['kernel_ms'].items()},d.get('parity',{}).get('ok'))" "$O/bench_$c.json" "$c"
done
echo done
