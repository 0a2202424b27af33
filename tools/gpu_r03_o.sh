#!/bin/bash
# Lean observe (bqsr_observe_lean) on the GPU box: tools/gpu_r03_o.sh TAG [full]
#   GPU suite (-x), cfg2 with its full-shard parity check, then cfg2 / cfg3
#   A/B lean (default) against the previous lane-per-read kernel
#   (ADAM_BQSR_OBSERVE=read), then a rocprofv3 kernel-trace of cfg2.
set -e
TAG=$1
MODE=${2:-full}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 \
  || { tail -40 "$O/pytest.log"; exit 1; }
tail -2 "$O/pytest.log"
timeout -k 10 500 python -u bench.py --config cfg2 --steps 20 > "$O/bench_cfg2.json" 2> "$O/bench_cfg2.err"
python -c "import json,sys;d=json.load(open(sys.argv[1]));print('cfg2 lean',round(d['ms_per_step'],3),{k:round(v,3) for k,v in d['roofline']['kernel_ms'].items()},d.get('parity'))" "$O/bench_cfg2.json"
for c in cfg2 cfg3; do
  for f in lean read; do
    ADAM_BQSR_OBSERVE=$f timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-parity --steps 10 --warmup 2 \
      > "$O/ab_${c}_$f.json" 2> "$O/ab_${c}_$f.err"
    python3 -c "import json,sys; d=json.load(open('$O/ab_${c}_$f.json')); print('$c $f', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['roofline']['kernel_ms'].items()})"
  done
done
[ "$MODE" = full ] || exit 0
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_cfg2" -o run --output-format csv -- \
  python3 "$R/bench.py" --config cfg2 --no-cpu-baseline --no-parity --steps 10 > "$O/prof_cfg2.log" 2>&1
cut -d, -f1-8 "$O/prof_cfg2/run_kernel_stats.csv" | head -12 | cut -c1-150
echo done
