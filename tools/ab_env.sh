#!/bin/bash
# A/B kernel stats of one config over environment settings: tools/ab_env.sh TAG CONFIG "VAR=val ..." ...
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1
CFG=$2
shift 2
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
export TMPDIR=/tmp
i=0
for envs in "$@"; do
  i=$((i+1))
  cd /tmp
  env $envs timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/s$i" -o run --output-format csv -- \
    python3 "$R/bench.py" --config "$CFG" --no-cpu-baseline --no-parity --steps 5 --warmup 1 > "$O/s$i.log" 2>&1
  echo "== $envs"
  find "$O/s$i" -name "*kernel_stats.csv" -exec grep -E "prep|observe|apply|reduce|fold_hist" {} \; | cut -d, -f1,4
done
