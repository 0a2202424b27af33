#!/bin/bash
# cfg5 with the kernel-copy D2H at several copy grids, and cfg3 with / without
# the known-site bitmaps: tools/gpu_r03_n.sh TAG
set -e
TAG=$1
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
for nb in 32 128 512; do
  ADAM_BQSR_COPY_BLOCKS=$nb timeout -k 10 400 python -u bench.py --config cfg5 --steps 4 --warmup 1 --no-parity \
    --no-cpu-baseline > "$O/cfg5_b$nb.json" 2> "$O/cfg5_b$nb.err"
  python3 -c "import json; d=json.load(open('$O/cfg5_b$nb.json')); print('cfg5 blocks $nb', round(d['ms_per_step'],1), d['pcie']['achieved_GBps'])"
done
export TMPDIR=/tmp
for v in "s1 ADAM_BQSR_SITES_BITMAP=1" "s0 ADAM_BQSR_SITES_BITMAP=0"; do
  set -- $v
  cd /tmp
  env $2 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/$1" -o run --output-format csv -- \
    python3 "$R/bench.py" --config cfg3 --no-cpu-baseline --no-parity --steps 5 --warmup 1 > "$O/$1.log" 2>&1
  cd "$R"
  echo "== $1 $2 $(grep -o '"ms_per_step": [0-9.]*' "$O/$1.log")"
  cut -d, -f1,4 "$O/$1/run_kernel_stats.csv" | head -6
done
