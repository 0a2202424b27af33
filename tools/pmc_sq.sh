#!/bin/bash
# One PMC pass of up to 8 SQ counters over a 1-step bench, summed per kernel:
# tools/pmc_sq.sh TAG "SQ_A SQ_B ..." [bench args]
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1
CTRS=$2
shift 2
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc $CTRS -d "$O/pmc" -o run --output-format csv -- \
  python3 "$R/bench.py" --no-cpu-baseline --no-parity --steps 1 --warmup 0 "$@" > "$O/pmc.log" 2>&1
python3 - "$O" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/pmc/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for row in csv.DictReader(open(f)):
    agg[row["Kernel_Name"][:40]][row["Counter_Name"]] += float(row["Counter_Value"])
for k, d in agg.items():
    if any(s in k for s in ("prep", "observe", "apply")):
        print(k, {c: "%.4g" % v for c, v in sorted(d.items())})
PY
