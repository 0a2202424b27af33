#!/bin/bash
# r05au: the final tree -- GPU suite, smoke, the default bench line (cfg2, N=1)
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/r05au"; mkdir -p "$O"; cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 \
  || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
tail -1 "$O/smoke.log"
timeout -k 10 600 python -u bench.py > "$O/bench.json" 2> "$O/bench.err"
cat "$O/bench.json"
