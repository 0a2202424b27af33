#!/bin/bash
# GPU tests, then cfg4 with and without the bucket-major copies
# (ADAM_BQSR_GATHER=0), cfg2 kernel stats, and the cfg4 measurement pass:
# tools/gpu_r03_l.sh TAG
set -e
TAG=$1
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
export TMPDIR=/tmp
for v in "g1 cfg4 ADAM_BQSR_GATHER=1" "g0 cfg4 ADAM_BQSR_GATHER=0" "c2 cfg2 ADAM_BQSR_GATHER=1"; do
  set -- $v
  cd /tmp
  env $3 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/$1" -o run --output-format csv -- \
    python3 "$R/bench.py" --config $2 --no-cpu-baseline --no-parity --steps 5 --warmup 1 > "$O/$1.log" 2>&1
  cd "$R"
  echo "== $1 $2 $3 $(grep -o '"ms_per_step": [0-9.]*' "$O/$1.log")"
  python3 tools/kstat_summary.py "$O/$1" | head -8
done
bash tools/gpu_r03.sh $TAG cfg4 0
