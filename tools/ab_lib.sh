#!/bin/bash
# A/B kernel stats of library builds on one box: tools/ab_lib.sh TAG "cfg2 cfg3" LIB1.so LIB2.so ...
# (LIB "-" = the in-tree library); per config and library a rocprofv3 --stats run.
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1
CFGS=$2
shift 2
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
export TMPDIR=/tmp
for c in $CFGS; do
  i=0
  for lib in "$@"; do
    i=$((i+1))
    [ "$lib" = - ] && lib="$R/adam_amd/libadam_bqsr.so"
    cd /tmp
    ADAM_BQSR_LIB="$lib" timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/${c}_$i" -o run --output-format csv -- \
      python3 "$R/bench.py" --config "$c" --no-cpu-baseline --no-parity --steps 5 --warmup 1 > "$O/${c}_$i.log" 2>&1
    echo "== $c $lib"
    python3 "$R/tools/kstat_summary.py" "$O/${c}_$i" | grep -E "observe|apply|prep_kernel|hist"
  done
done
