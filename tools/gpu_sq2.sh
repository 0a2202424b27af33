#!/bin/bash
# GPU tests, then two SQ counter passes over one cfg2 bench step (tools/pmc_sq.sh):
# tools/gpu_sq2.sh TAG [CONFIG] [PYTEST]
set -e
TAG=$1
CFG=${2:-cfg2}
PYTEST=${3:-1}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
if [ "$PYTEST" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
  tail -1 "$O/pytest.log"
fi
timeout -k 10 300 python -u bench.py --config $CFG --no-cpu-baseline --no-parity --steps 10 --warmup 2 > "$O/bench.json" 2> "$O/bench.err"
python3 -c "import json; d=json.load(open('$O/bench.json')); print(round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['roofline']['kernel_ms'].items()})"
bash tools/pmc_sq.sh $TAG/a "SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVES SQ_WAVE_CYCLES" --config $CFG
bash tools/pmc_sq.sh $TAG/b "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_LDS_ADDR_CONFLICT SQ_WAIT_ANY" --config $CFG
echo done
