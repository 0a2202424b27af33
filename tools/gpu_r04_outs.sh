#!/bin/bash
# Bucketed apply: per-read outputs by bqsr_apply_outs in read order
# (ADAM_BQSR_APPLY_OUTS=apart) against the walk's stores, one box: the GPU
# tests with the switch on, cfg4 kernel stats both ways, then the switched
# cfg4 line with full-shard parity.  tools/gpu_r04_outs.sh TAG
set -e
TAG=$1
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
export TMPDIR=/tmp
ADAM_BQSR_APPLY_OUTS=apart timeout -k 10 600 python -u -m pytest tests/test_gpu_forms.py tests/test_gpu_parity.py tests/test_gpu_staged.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 || { rc=$?; tail -40 "$O/pytest.log"; exit $rc; }
tail -1 "$O/pytest.log"
for v in walk apart walk apart; do
  (cd /tmp && ADAM_BQSR_APPLY_OUTS=$v timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/$v" -o run --output-format csv -- \
    python3 "$R/bench.py" --config cfg4 --no-cpu-baseline --no-parity --steps 10 --warmup 1 --event-steps 0 > "$O/$v.log" 2>&1)
  echo "== $v"; python3 tools/kstat_summary.py "$O/$v" | grep -E "apply" || true
  python3 - "$O/$v.log" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        print("ms/job", round(json.loads(l)["ms_per_step"], 3))
PY
  rm -rf "$O/$v"
done
ADAM_BQSR_APPLY_OUTS=apart timeout -k 10 600 python -u bench.py --config cfg4 --no-cpu-baseline > "$O/bench_cfg4_apart.json" 2> "$O/bench_cfg4_apart.err"
python3 - "$O/bench_cfg4_apart.json" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        print("cfg4 apart", round(d["ms_per_step"], 3), "parity", d["parity"]["ok"], d["parity"]["reads_checked"])
PY
echo done
