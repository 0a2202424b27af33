#!/bin/bash
# cfg4 A/B on one box: the key-major copy on / off (ADAM_BQSR_KEYMAJOR), the
# fold's block histograms by bqsr_fold_hist (default) or counted in the
# observe kernel (ADAM_BQSR_FOLD_HIST=observe), kernel stats + bench line
# each; then the cfg5 bench (compacted outputs, u16 lengths).
# tools/gpu_r04_fh.sh TAG [PYTEST_FILES]
set -e
TAG=$1
TESTS=${2:-}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -v --timeout 600 --timeout-method thread > "$O/pytest.log" 2>&1 \
    || { rc=$?; tail -40 "$O/pytest.log"; exit $rc; }
  tail -1 "$O/pytest.log"
fi
for v in pass:1 pass:0 observe:1; do
  fh=${v%:*}; km=${v#*:}
  (
    cd /tmp
    export ADAM_BQSR_FOLD_HIST=$fh ADAM_BQSR_KEYMAJOR=$km
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/cfg4_${fh}_km$km" -o run --output-format csv -- \
      python3 "$R/bench.py" --config cfg4 --no-cpu-baseline --no-parity --steps 10 --warmup 2 --event-steps 0 > "$O/cfg4_${fh}_km$km.log" 2>&1
  )
  (
    cd /tmp
    export ADAM_BQSR_FOLD_HIST=$fh ADAM_BQSR_KEYMAJOR=$km
    timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$O/cfg4_${fh}_km${km}_p/pmc_fetch" -o run --output-format csv -- \
      python3 "$R/bench.py" --config cfg4 --no-cpu-baseline --no-parity --steps 3 --warmup 1 --event-steps 0 > "$O/cfg4_${fh}_km${km}_fetch.log" 2>&1
  )
  echo "== fold_hist=$fh keymajor=$km"
  python3 tools/kstat_summary.py "$O/cfg4_${fh}_km$km" > "$O/cfg4_${fh}_km$km.txt" || true
  head -8 "$O/cfg4_${fh}_km$km.txt"
  python3 - "$O/cfg4_${fh}_km$km.log" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        print("ms/job", round(json.loads(line)["ms_per_step"], 3))
PY
  python3 tools/pmc_summary.py "$O/cfg4_${fh}_km${km}_p" "$O/cfg4_${fh}_km${km}_fetch.json" > "$O/cfg4_${fh}_km${km}_fetch.txt" || true
  grep -A2 -E "observe|apply_kernel|fold_hist" "$O/cfg4_${fh}_km${km}_fetch.txt" || true
done
timeout -k 10 900 python -u bench.py --config cfg5 > "$O/bench_cfg5.json" 2> "$O/bench_cfg5.err"
python3 - "$O/bench_cfg5.json" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        print("cfg5", round(d["ms_per_step"], 2), d["pcie"], d["parity"]["ok"])
PY
echo done
