#!/bin/bash
# A/B of bench variants on one box, kernel stats per variant:
#   tools/gpu_ab.sh TAG CFG "VARIANT_A" "VARIANT_B" ...
# VARIANT: extra bench.py flags (e.g. "--tune fused_prep=0"), optionally led by
# LIB=path (a probe / A/B build of the library, tools/build_probe.sh).
set -e
TAG=$1; CFG=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"; mkdir -p "$O"
export TMPDIR=/tmp
i=0
for v in "$@"; do
  i=$((i+1))
  lib="$R/adam_amd/libadam_bqsr.so"; args="$v"
  case "$v" in LIB=*) lib="${v%% *}"; lib="$R/${lib#LIB=}"; args="${v#* }"; [ "$args" = "$v" ] && args="";; esac
  cd /tmp
  ADAM_BQSR_LIB="$lib" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/${CFG}_$i" -o run --output-format csv -- \
    python3 "$R/bench.py" --config "$CFG" --no-cpu-baseline --no-parity --steps 10 --warmup 2 $args > "$O/${CFG}_$i.log" 2>&1
  cd "$R"
  echo "== $CFG [$v]"
  python3 tools/kstat_summary.py "$O/${CFG}_$i" | head -14
  grep -h '^{' "$O/${CFG}_$i.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms/job', round(d['ms_per_step'],4))"
done
