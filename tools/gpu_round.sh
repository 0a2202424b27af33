#!/bin/bash
# One GPU-box pass over the current tree (run via gpurun):
#   tools/gpu_round.sh TAG [tests|notests]
# -> gpurun_out/TAG/{pytest.log, smoke.log, bench.json, stats/, pmc3/, pmc4/}
# Every GPU step has its own time limit; the chain stops at the first failure.
set -e
TAG=$1
MODE=${2:-tests}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
if [ "$MODE" = tests ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$O/pytest.log" 2>&1
  tail -3 "$O/pytest.log"
  timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
  tail -1 "$O/smoke.log"
fi
timeout -k 10 400 python -u bench.py > "$O/bench.json" 2> "$O/bench.err"
cat "$O/bench.json"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/stats" -o run --output-format csv -- \
  python3 "$R/bench.py" --no-cpu-baseline --steps 10 --warmup 1 > "$O/stats.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc3" -o run --output-format csv -- \
  python3 "$R/bench.py" --no-cpu-baseline --steps 3 --warmup 1 > "$O/pmc3.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d "$O/pmc4" -o run --output-format csv -- \
  python3 "$R/bench.py" --no-cpu-baseline --steps 3 --warmup 1 > "$O/pmc4.log" 2>&1
echo done
