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
  echo "== fold_hist=$fh keymajor=$km"; python3 tools/kstat_summary.py "$O/cfg4_${fh}_km$km" | head -12 || true
  tail -1 "$O/cfg4_${fh}_km$km.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms/job', round(d['ms_per_step'],3))"
done
timeout -k 10 900 python -u bench.py --config cfg5 > "$O/bench_cfg5.json" 2> "$O/bench_cfg5.err"
python3 -c "import json; d=json.load(open('$O/bench_cfg5.json')); print('cfg5', round(d['ms_per_step'],2), d['pcie'], d['parity']['ok'])"
echo done
