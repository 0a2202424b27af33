#!/bin/bash
# cfg4's chunk-walk observe: lane-rotated offset order (libadam_bqsr_rotate.so,
# -DADAM_BQSR_ROTATE) and the window row length mod 4 (ADAM_BQSR_WPAD) against
# the default, one box: the bucketed GPU tests on the variant, rocprofv3
# kernel stats per form, LDS bank-conflict counters for default and rotated,
# then the variant's cfg4 bench line with full-shard parity.
# tools/gpu_r04_rotate.sh TAG
set -e
TAG=$1
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
export TMPDIR=/tmp
P="$R/adam_amd/libadam_bqsr.so"; V="$R/adam_amd/libadam_bqsr_rotate.so"
ADAM_BQSR_LIB="$V" timeout -k 10 600 python -u -m pytest tests/test_gpu_forms.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 \
  --timeout-method thread > "$O/pytest_rotate.log" 2>&1 || { rc=$?; tail -40 "$O/pytest_rotate.log"; exit $rc; }
tail -1 "$O/pytest_rotate.log"
run() {  # name lib env...
  local name=$1 lib=$2; shift 2
  (
    cd /tmp
    for kv in "$@"; do export "$kv"; done
    export ADAM_BQSR_LIB="$lib"
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/$name" -o run --output-format csv -- \
      python3 "$R/bench.py" --config cfg4 --no-cpu-baseline --no-parity --steps 10 --warmup 1 --event-steps 0 > "$O/$name.log" 2>&1
  )
  echo "== $name"; python3 tools/kstat_summary.py "$O/$name" | grep -E "observe|apply|fold_hist" || true
  python3 - "$O/$name.log" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        print("ms/job", round(json.loads(line)["ms_per_step"], 3))
PY
}
run default "$P" X=1
run rotate "$V" X=1
run wpad1 "$P" ADAM_BQSR_WPAD=1
run wpad0 "$P" ADAM_BQSR_WPAD=0
run rotate_wpad1 "$V" ADAM_BQSR_WPAD=1
for v in default rotate; do
  lib=$P; [ $v = rotate ] && lib=$V
  (cd /tmp && ADAM_BQSR_LIB="$lib" timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAVES \
    -d "$O/sq_$v" -o run --output-format csv -- python3 "$R/bench.py" --config cfg4 --no-cpu-baseline --no-parity --steps 3 --warmup 1 \
    --event-steps 0 > "$O/sq_$v.log" 2>&1)
  python3 - "$O/sq_$v" "$v" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for row in csv.DictReader(open(f[0])):
    k = row["Kernel_Name"]
    if "observe_chunks" not in k: continue
    acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
for k, d in acc.items():
    print(sys.argv[2], "observe_chunks", {c: "%.3e" % v for c, v in d.items()},
          "conflict share %.3f" % (d["SQ_LDS_BANK_CONFLICT"] / max(1.0, d["SQ_LDS_IDX_ACTIVE"])))
PY
done
ADAM_BQSR_LIB="$V" timeout -k 10 600 python -u bench.py --config cfg4 --no-cpu-baseline > "$O/bench_cfg4_rotate.json" 2> "$O/bench_cfg4_rotate.err"
python3 - "$O/bench_cfg4_rotate.json" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        print("cfg4 rotate", round(d["ms_per_step"], 3), "parity", d["parity"]["ok"], d["parity"]["reads_checked"])
PY
echo done
