#!/bin/bash
# A/B of observe forms (run via gpurun): tools/ab_observe.sh TAG [PYTEST]
# -> gpurun_out/TAG/{pytest.log, ab_CFG_FORM.json}
set -e
TAG=$1
PYTEST=${2:-1}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
if [ "$PYTEST" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
  tail -1 "$O/pytest.log"
fi
for c in cfg2 cfg3 cfg4; do
  for f in rows old; do
    if [ $f = old ]; then
      if [ $c = cfg4 ]; then export ADAM_BQSR_OBSERVE=chunk; else export ADAM_BQSR_OBSERVE=read; fi
    else
      unset ADAM_BQSR_OBSERVE
    fi
    timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-parity --steps 10 --warmup 2 --event-steps 3 > "$O/ab_${c}_$f.json" 2> "$O/ab_${c}_$f.err"
    python3 -c "import json,sys; d=json.load(open('$O/ab_${c}_$f.json')); print('$c $f', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['roofline']['kernel_ms'].items()})"
  done
done
unset ADAM_BQSR_OBSERVE
echo done
