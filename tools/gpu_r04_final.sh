#!/bin/bash
# Round-end check of the committed tree: the GPU suite, smoke(), and the
# default bench line (what the driver runs).  tools/gpu_r04_final.sh TAG
set -e
TAG=$1
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 \
  || { rc=$?; tail -60 "$O/pytest.log"; exit $rc; }
tail -1 "$O/pytest.log"
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
tail -1 "$O/smoke.log"
timeout -k 10 600 python -u bench.py > "$O/bench.json" 2> "$O/bench.err"
python3 - "$O/bench.json" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        print("default bench", round(d["ms_per_step"], 4), "ms/job", "%.3e" % d["value"], d["unit"], "parity", d["parity"]["ok"],
              "frac", round(d["roofline"]["frac"], 3), d["roofline"]["kernel"])
PY
