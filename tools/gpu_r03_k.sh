#!/bin/bash
# Streamed paths after a staging change: the stream / SAM / multi-rank GPU
# tests, the cfg5 line (pipelined, parity), then SAM and BAM ingest rates:
# tools/gpu_r03_k.sh TAG
set -e
TAG=$1
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_sam.py tests/test_gpu_multirank.py -x -q \
  --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
timeout -k 10 500 python -u bench.py --config cfg5 --steps 4 --warmup 1 > "$O/bench_cfg5.json" 2> "$O/bench_cfg5.err"
python3 -c "import json; d=json.load(open('$O/bench_cfg5.json')); print('cfg5', round(d['ms_per_step'],1), d['pcie'], d.get('parity',{}).get('ok'))"
timeout -k 10 300 python -u tools/bench_ingest.py --reads 2000000 > "$O/ingest_sam.json" 2> "$O/ingest_sam.err"
cat "$O/ingest_sam.json"
timeout -k 10 300 python -u tools/bench_ingest.py --reads 400000 --bam > "$O/ingest_bam.json" 2> "$O/ingest_bam.err"
cat "$O/ingest_bam.json"
