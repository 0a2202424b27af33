#!/bin/bash
# BAM ingest through the pinned ring (bgzf_inflate_device): the GPU suite,
# then the BAM -> ADAM transform line.  tools/gpu_r04_bam.sh TAG
set -e
TAG=$1
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 \
  || { rc=$?; tail -60 "$O/pytest.log"; exit $rc; }
tail -1 "$O/pytest.log"
timeout -k 10 400 python -u tools/bench_adam.py --reads 10000000 --compression snappy --bam > "$O/e2e_bam_snappy.json" 2> "$O/e2e_bam_snappy.log"
cat "$O/e2e_bam_snappy.json"
