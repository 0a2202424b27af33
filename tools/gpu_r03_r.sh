#!/bin/bash
# lean apply A/B (gpurun): tools/gpu_r03_r.sh TAG
set -e
TAG=$1
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 \
  || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
timeout -k 10 500 python -u bench.py --config cfg2 --steps 20 > "$O/bench_cfg2.json" 2> "$O/bench_cfg2.err"
python -c "import json,sys;d=json.load(open(sys.argv[1]));print('cfg2',round(d['ms_per_step'],3),{k:round(v,3) for k,v in d['roofline']['kernel_ms'].items()},d.get('parity',{}).get('ok'))" "$O/bench_cfg2.json"
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline --no-parity --steps 10 --warmup 2 > "$O/ab_${C}_$n.json" 2> "$O/ab_${C}_$n.err"
  python3 -c "import json,sys; d=json.load(open('$O/ab_${C}_$n.json')); print('$C $n', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['roofline']['kernel_ms'].items()})"
}
for C in cfg2 cfg3; do
  run walk ADAM_BQSR_APPLY=walk
  run lean ADAM_BQSR_APPLY=lean
done
for f in lean walk; do
  ADAM_BQSR_APPLY=$f bash tools/pmc_sq.sh $TAG/sq_$f "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_SALU" --config cfg2
done
echo done
