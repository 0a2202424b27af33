#!/bin/bash
# Dynamic instruction counts per kernel (one PMC pass): tools/pmc_insts.sh TAG [bench args]
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1
shift
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH \
  -d "$O/pmc" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --no-parity --steps 1 --warmup 0 "$@" > "$O/pmc.log" 2>&1
python3 - "$O" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/pmc/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for row in csv.DictReader(open(f)):
    agg[row["Kernel_Name"][:40]][row["Counter_Name"]] += float(row["Counter_Value"])
for k, d in agg.items():
    print(k, {c: "%.4g" % v for c, v in sorted(d.items())})
PY
