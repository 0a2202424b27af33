#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out/r02aa
timeout -k 10 600 python -u -m pytest tests/test_gpu_sam.py -v -s --timeout 300 --timeout-method thread > gpurun_out/r02aa/sam.log 2>&1 || true
grep -E "PASS|FAIL|ERROR|ingest:" gpurun_out/r02aa/sam.log | tail -40
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_sam.py > gpurun_out/r02aa/all.log 2>&1 || true
tail -3 gpurun_out/r02aa/all.log
bash tools/ab_cfg.sh r02aa cfg3 - tools/prof/libadam_bqsr_STORE.so tools/prof/libadam_bqsr_NOSITES.so
