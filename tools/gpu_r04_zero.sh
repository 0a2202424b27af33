#!/bin/bash
# Early (side-stream) zeroing of the slot bitmap against the prep's own
# memset (ADAM_BQSR_EARLY_ZERO=0), one box: the staged GPU tests, then cfg2
# and cfg4 bench lines both ways (no parity / CPU baseline), then the
# default's cfg2 line with full-shard parity.  tools/gpu_r04_zero.sh TAG
set -e
TAG=$1
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_staged.py tests/test_gpu_multirank.py tests/test_gpu_stream.py -x -v --timeout 300 \
  --timeout-method thread > "$O/pytest.log" 2>&1 || { rc=$?; tail -40 "$O/pytest.log"; exit $rc; }
tail -1 "$O/pytest.log"
line() {
  python3 - "$1" "$2" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        p = d.get("parity") or {}
        print(sys.argv[2], "ms/job", round(d["ms_per_step"], 4), "parity", p.get("ok"), p.get("reads_checked"))
PY
}
for rep in 1 2; do
  for c in cfg2 cfg4; do
    timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-parity --steps 40 --warmup 5 > "$O/${c}_early_$rep.json" 2>/dev/null
    line "$O/${c}_early_$rep.json" "$c early $rep"
    ADAM_BQSR_EARLY_ZERO=0 timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-parity --steps 40 --warmup 5 > "$O/${c}_memset_$rep.json" 2>/dev/null
    line "$O/${c}_memset_$rep.json" "$c memset $rep"
  done
done
timeout -k 10 600 python -u bench.py --config cfg2 --no-cpu-baseline > "$O/bench_cfg2.json" 2> "$O/bench_cfg2.err"
line "$O/bench_cfg2.json" "cfg2 default parity"
echo done
