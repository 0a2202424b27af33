#!/bin/bash
# A/B bench runs: tools/ab.sh TAG lib1 lib2 ... (default library when "-")
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1
shift
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
i=0
for lib in "$@"; do
  i=$((i+1))
  if [ "$lib" = "-" ]; then unset ADAM_BQSR_LIB; else export ADAM_BQSR_LIB="$R/$lib"; fi
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-parity > "$O/b$i.json" 2> "$O/b$i.err"
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],d['ms_per_step'],d['roofline']['kernel_ms'])" "$O/b$i.json" "$lib"
done
