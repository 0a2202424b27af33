#!/bin/bash
# lean observe on bucketed batches (cfg4) vs the chunk walk (gpurun): tools/gpu_r03_w.sh TAG
set -e
TAG=$1
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity_more.py tests/test_gpu_staged.py tests/test_gpu_stream.py -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 \
  || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
for f in lean chunks; do
  ADAM_BQSR_OBSERVE=$f timeout -k 10 300 python -u bench.py --config cfg4 --no-cpu-baseline --no-parity --steps 10 --warmup 2 > "$O/ab_cfg4_$f.json" 2> "$O/ab_cfg4_$f.err"
  python3 -c "import json; d=json.load(open('$O/ab_cfg4_$f.json')); print('cfg4 $f', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['roofline']['kernel_ms'].items()})"
done
echo done
