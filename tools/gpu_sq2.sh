#!/bin/bash
# GPU tests, A/B timings of the per-base kernel forms, then two SQ counter
# passes over one bench step (tools/pmc_sq.sh): tools/gpu_sq2.sh TAG [CONFIG] [PYTEST]
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
ab() {  # ab NAME CONFIG [ENV=VAL ...]
  local name=$1 c=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-parity --steps 10 --warmup 2 > "$O/ab_$name.json" 2> "$O/ab_$name.err"
  python3 -c "import json; d=json.load(open('$O/ab_$name.json')); print('$name', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['roofline']['kernel_ms'].items()})"
}
ab cfg2_new cfg2
ab cfg2_oldobs cfg2 ADAM_BQSR_OBSERVE=read
ab cfg2_oldapp cfg2 ADAM_BQSR_APPLY=chunk
ab cfg4_new cfg4
ab cfg4_oldapp cfg4 ADAM_BQSR_APPLY=chunk
bash tools/pmc_sq.sh $TAG/a "SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVES SQ_WAVE_CYCLES" --config $CFG
bash tools/pmc_sq.sh $TAG/b "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_LDS_ADDR_CONFLICT SQ_WAIT_ANY" --config $CFG
bash tools/pmc_sq.sh $TAG/c "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" --config $CFG || true
echo done
