#!/bin/bash
# Round-2 first GPU pass: the full -m gpu suite, smoke, the default bench
# line (with the parity check), and the fold kernel's phase profile
# (BQSR_FOLD_PROFILE build: tools/prof/libadam_bqsr_foldprof.so).
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$1"
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -3 "$O/pytest.log"
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
tail -1 "$O/smoke.log"
timeout -k 10 500 python -u bench.py > "$O/bench.json" 2> "$O/bench.err"
cat "$O/bench.json"
ADAM_BQSR_LIB="$R/tools/prof/libadam_bqsr_foldprof.so" timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$O/foldprof.log" 2>&1
grep FOLDPROF "$O/foldprof.log" | tail -2
echo done
