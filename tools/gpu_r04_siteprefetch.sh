#!/bin/bash
# cfg3 prep: the bitmap word at the next read's start loaded an iteration
# ahead (libadam_bqsr_siteprefetch.so) against the default, one box: kernel
# stats both ways (twice), then the variant's cfg3 line with full-shard parity.
# tools/gpu_r04_siteprefetch.sh TAG
set -e
TAG=$1
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
bash tools/ab_lib.sh "$TAG/ab" cfg3 - "$R/adam_amd/libadam_bqsr_siteprefetch.so" - "$R/adam_amd/libadam_bqsr_siteprefetch.so"
ADAM_BQSR_LIB="$R/adam_amd/libadam_bqsr_siteprefetch.so" timeout -k 10 600 python -u bench.py --config cfg3 --no-cpu-baseline \
  > "$O/bench_cfg3_pf.json" 2> "$O/bench_cfg3_pf.err"
python3 - "$O/bench_cfg3_pf.json" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        print("cfg3 prefetch", round(d["ms_per_step"], 3), "parity", d["parity"]["ok"], d["parity"]["reads_checked"])
PY
echo done
