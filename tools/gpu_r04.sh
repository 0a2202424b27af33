#!/bin/bash
# round-4 check of the tree (gpurun): GPU suite, smoke, default bench line [+ extra bench args]
set -e
TAG=$1; shift || true
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=10 -v --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 \
  || { tail -60 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
tail -1 "$O/smoke.log"
timeout -k 10 600 python -u bench.py "$@" > "$O/bench.json" 2> "$O/bench.err"
python3 -c "import json; d=json.load(open('$O/bench.json')); print(round(d['ms_per_step'],3), '%.3g' % d['value'], {k: round(v,3) for k,v in d['roofline']['kernel_ms'].items()}, round(d['roofline']['frac'],3), d['parity']['ok'])"
echo done
