#!/bin/bash
# A/B kernel time + FETCH_SIZE of one config over libraries: tools/ab_pmc.sh TAG CONFIG lib1 lib2 ... ("-" = default)
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1
CFG=$2
shift 2
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
export TMPDIR=/tmp
i=0
for lib in "$@"; do
  i=$((i+1))
  if [ "$lib" = "-" ]; then unset ADAM_BQSR_LIB; else export ADAM_BQSR_LIB="$R/$lib"; fi
  cd "$R"
  timeout -k 10 300 python -u bench.py --config "$CFG" --no-cpu-baseline > "$O/b$i.json" 2> "$O/b$i.err"
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/s$i" -o run --output-format csv -- \
    python3 "$R/bench.py" --config "$CFG" --no-cpu-baseline --no-parity --steps 5 --warmup 1 > "$O/s$i.log" 2>&1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$O/f$i" -o run --output-format csv -- \
    python3 "$R/bench.py" --config "$CFG" --no-cpu-baseline --no-parity --steps 1 --warmup 0 > "$O/f$i.log" 2>&1
  echo "== $lib"
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['ms_per_step'],d['roofline']['kernel_ms'],d.get('parity',{}).get('ok'))" "$O/b$i.json"
  find "$O/s$i" -name "*kernel_stats.csv" -exec grep -E "prep|observe|apply" {} \; | cut -d, -f1,4
  python3 - "$O/f$i" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(list)
for row in csv.DictReader(open(f)):
    agg[row["Kernel_Name"][:48]].append(float(row["Counter_Value"]))
for k, v in agg.items():
    if any(s in k for s in ("prep", "observe", "apply")):
        print("FETCH", k, "%.4g KiB/launch" % (sum(v) / len(v)))
PY
done
