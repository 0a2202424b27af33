#!/bin/bash
# Known sites on coordinate-sorted cfg3 (SnpTable.scala:15-23): the position
# bitmap (product), the sorted lists in global memory (ADAM_BQSR_SITES_BITMAP=0)
# and the LDS-staged sorted list (tools/build_variant.sh sites_lds
# -DADAM_BQSR_SITES_LDS), kernel stats on one box; the same on the random
# (unsorted) cfg3; then the LDS build's full-shard parity on sorted cfg3.
set -e
TAG=$1
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
export TMPDIR=/tmp
run() {  # name lib sorted env...
  local name=$1 lib=$2 sorted=$3; shift 3
  (
    cd /tmp
    for kv in "$@"; do export "$kv"; done
    export ADAM_BQSR_LIB="$lib"
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/$name" -o run --output-format csv -- \
      python3 "$R/bench.py" --config cfg3 $sorted --no-cpu-baseline --no-parity --steps 5 --warmup 1 > "$O/$name.log" 2>&1
  )
  echo "== $name"; python3 tools/kstat_summary.py "$O/$name" | grep -E "prep|observe|apply" || true
  python3 - "$O/$name.log" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        print("ms/job", round(json.loads(line)["ms_per_step"], 3))
PY
}
P="$R/adam_amd/libadam_bqsr.so"; V="$R/adam_amd/libadam_bqsr_sites_lds.so"
run sorted_bitmap "$P" --sorted X=1
run sorted_lists "$P" --sorted ADAM_BQSR_SITES_BITMAP=0
run sorted_lds "$V" --sorted X=1
run random_bitmap "$P" "" X=1
run random_lds "$V" "" X=1
ADAM_BQSR_LIB="$V" timeout -k 10 900 python -u bench.py --config cfg3 --sorted --steps 3 --no-cpu-baseline > "$O/bench_lds_sorted.json" 2> "$O/bench_lds_sorted.err"
python3 - "$O/bench_lds_sorted.json" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        print("lds sorted", round(d["ms_per_step"], 3), "parity", d["parity"]["ok"], d["parity"]["reads_checked"])
PY
echo done
