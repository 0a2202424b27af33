#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out/r02ag
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r02ag/all.log 2>&1 || { tail -30 gpurun_out/r02ag/all.log; exit 1; }
tail -1 gpurun_out/r02ag/all.log
for e in 1 4 1000; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-parity --event-every $e > gpurun_out/r02ag/b$e.json 2>/dev/null
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],d['ms_per_step'],d['roofline']['kernel_ms'])" gpurun_out/r02ag/b$e.json $e
done
