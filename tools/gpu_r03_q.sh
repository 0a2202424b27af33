#!/bin/bash
# lean observe: counter copies A/B (gpurun): tools/gpu_r03_q.sh TAG
set -e
TAG=$1
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity_more.py -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 \
  || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
run() {  # name env... 
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline --no-parity --steps 10 --warmup 2 > "$O/ab_${C}_$n.json" 2> "$O/ab_${C}_$n.err"
  python3 -c "import json,sys; d=json.load(open('$O/ab_${C}_$n.json')); print('$C $n', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['roofline']['kernel_ms'].items()})"
}
for C in cfg2 cfg3; do
  run read ADAM_BQSR_OBSERVE=read
  for nc in 1 2 3 4; do run c$nc ADAM_BQSR_LEAN_COPIES=$nc; done
done
for nc in 1 4; do
  ADAM_BQSR_LEAN_COPIES=$nc bash tools/pmc_sq.sh $TAG/sq2_c$nc "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE" --config cfg2
  ADAM_BQSR_LEAN_COPIES=$nc bash tools/pmc_sq.sh $TAG/sq3_c$nc "SQ_LDS_ADDR_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES" --config cfg2
done
echo done
