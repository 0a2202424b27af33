#!/bin/bash
# A/B of the wavefront-aggregation build (tools/build_variant.sh agg
# -DADAM_BQSR_WAVE_AGG) against the product library on one box: kernel stats
# and SQ counters on cfg2 (lean observe) and cfg4 (chunk-walk observe), and
# the variant's full-shard parity on cfg2.  tools/gpu_r04_agg.sh TAG
set -e
TAG=$1
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"; mkdir -p "$O"; cd "$R"
AGG="$R/adam_amd/libadam_bqsr_agg.so"
bash tools/ab_lib.sh "$TAG/stats" "cfg2 cfg4" - "$AGG" > "$O/stats.txt" 2>&1
cat "$O/stats.txt"
for lib in - "$AGG"; do
  [ "$lib" = - ] && L="$R/adam_amd/libadam_bqsr.so" || L="$lib"
  n=$(basename "$L" .so)
  for c in cfg2 cfg4; do
    ADAM_BQSR_LIB="$L" bash tools/pmc_sq.sh "$TAG/sq_${n}_${c}_a" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU" --config $c > "$O/sq_${n}_${c}_a.txt" 2>&1
    ADAM_BQSR_LIB="$L" bash tools/pmc_sq.sh "$TAG/sq_${n}_${c}_b" "SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES" --config $c > "$O/sq_${n}_${c}_b.txt" 2>&1
    echo "== $n $c"; cat "$O/sq_${n}_${c}_a.txt" "$O/sq_${n}_${c}_b.txt" | grep -E "observe|apply" || true
  done
done
ADAM_BQSR_LIB="$AGG" timeout -k 10 600 python -u bench.py --steps 5 --no-cpu-baseline > "$O/bench_agg_cfg2.json" 2> "$O/bench_agg_cfg2.err"
python3 -c "import json; d=json.load(open('$O/bench_agg_cfg2.json')); print('agg cfg2', round(d['ms_per_step'],3), d['parity']['ok'])"
echo done
