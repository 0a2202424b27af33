#!/bin/bash
# Round-3 pass (via gpurun): GPU tests, MarkDuplicates reads/s (device and host
# paths), the streamed cfg5 line with its parity check:
# tools/gpu_r03_misc.sh TAG [PYTEST]
set -e
TAG=$1
PYTEST=${2:-1}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
if [ "$PYTEST" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
  tail -1 "$O/pytest.log"
  timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
  tail -1 "$O/smoke.log"
fi
timeout -k 10 300 python -u tools/bench_markdup.py --reads 10000000 --reps 2 > "$O/markdup.json" 2> "$O/markdup.err"
cat "$O/markdup.json"
ADAM_BQSR_MARKDUP=host timeout -k 10 300 python -u tools/bench_markdup.py --reads 2000000 --reps 1 > "$O/markdup_host.json" 2> "$O/markdup_host.err"
cat "$O/markdup_host.json"
timeout -k 10 600 python -u bench.py --config cfg5 --steps 3 --warmup 1 > "$O/bench_cfg5.json" 2> "$O/bench_cfg5.err"
cat "$O/bench_cfg5.json"
echo done
