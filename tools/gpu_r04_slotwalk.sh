#!/bin/bash
# Apply's chunk -> read map (slot_walk) against the chunk walk's mapping
# (ADAM_BQSR_SLOTWALK=0), one box: [the GPU suite,] rocprofv3 kernel stats of
# cfg2 and cfg3 both ways, then the default's cfg2 bench line with full-shard
# parity.  tools/gpu_r04_slotwalk.sh TAG [PYTEST]
set -e
TAG=$1
PYTEST=${2:-1}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
export TMPDIR=/tmp
if [ "$PYTEST" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 \
    || { rc=$?; tail -60 "$O/pytest.log"; exit $rc; }
  tail -1 "$O/pytest.log"
fi
run() {  # name config env...
  local name=$1 cfg=$2; shift 2
  (
    cd /tmp
    for kv in "$@"; do export "$kv"; done
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/$name" -o run --output-format csv -- \
      python3 "$R/bench.py" --config $cfg --no-cpu-baseline --no-parity --steps 10 --warmup 1 --event-steps 0 > "$O/$name.log" 2>&1
  )
  echo "== $name"; python3 tools/kstat_summary.py "$O/$name" | grep -E "prep|observe|apply|owner" || true
  python3 - "$O/$name.log" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        print("ms/job", round(json.loads(line)["ms_per_step"], 3))
PY
}
run cfg2_slot cfg2 X=1
run cfg2_walk cfg2 ADAM_BQSR_SLOTWALK=0
run cfg3_slot cfg3 X=1
run cfg3_walk cfg3 ADAM_BQSR_SLOTWALK=0
timeout -k 10 600 python -u bench.py --config cfg2 --no-cpu-baseline > "$O/bench_cfg2.json" 2> "$O/bench_cfg2.err"
python3 - "$O/bench_cfg2.json" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        print("cfg2", round(d["ms_per_step"], 3), "parity", d["parity"]["ok"], d["parity"]["reads_checked"])
PY
echo done
