#!/bin/bash
# front-ordered pieces for bucketed batches: parity, cfg4 bench with full-shard parity, A/B (gpurun)
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/r03fr; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity_more.py tests/test_gpu_forms.py tests/test_gpu_staged.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python bench.py --config cfg4 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_cfg4.json 2> $O/bench_cfg4.err
python3 -c "import json; d=json.load(open('$O/bench_cfg4.json')); print(round(d['ms_per_step'],3), '%.3g' % d['value'], {k: round(v,3) for k,v in d['roofline']['kernel_ms'].items()}, round(d['roofline']['frac'],3), d['parity']['ok'], d['parity']['reads_checked'])"
bash tools/ab_env.sh r03fr/ab4 cfg4 "ADAM_BQSR_FRONTS=0" "ADAM_BQSR_FRONTS=4" "ADAM_BQSR_FRONTS=0" "ADAM_BQSR_FRONTS=4" "ADAM_BQSR_FRONTS=8"
