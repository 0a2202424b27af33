#!/bin/bash
# observe A/B + SQ counters of the lean kernel (gpurun): tools/gpu_r03_p.sh TAG [tests]
set -e
TAG=$1
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
if [ "${2:-tests}" = tests ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity_more.py -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 \
    || { tail -40 "$O/pytest.log"; exit 1; }
  tail -1 "$O/pytest.log"
fi
for c in cfg2 cfg3; do
  for f in lean read; do
    ADAM_BQSR_OBSERVE=$f timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-parity --steps 10 --warmup 2 \
      > "$O/ab_${c}_$f.json" 2> "$O/ab_${c}_$f.err"
    python3 -c "import json,sys; d=json.load(open('$O/ab_${c}_$f.json')); print('$c $f', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['roofline']['kernel_ms'].items()})"
  done
done
for f in lean read; do
  ADAM_BQSR_OBSERVE=$f bash tools/pmc_sq.sh $TAG/sq1_$f "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM" --config cfg2
  ADAM_BQSR_OBSERVE=$f bash tools/pmc_sq.sh $TAG/sq2_$f "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE" --config cfg2
  ADAM_BQSR_OBSERVE=$f bash tools/pmc_sq.sh $TAG/sq3_$f "SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD" --config cfg2
done
echo done
