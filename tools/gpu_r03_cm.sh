#!/bin/bash
# cell-major char tables: parity, then A/B against row-major on cfg2 / cfg4 (gpurun)
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out/r03cm
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_forms.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03cm/pytest.log 2>&1
tail -3 gpurun_out/r03cm/pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r03cm/bench_cfg2.json 2> gpurun_out/r03cm/bench_cfg2.err
cat gpurun_out/r03cm/bench_cfg2.json
bash tools/ab_env.sh r03cm/ab2 cfg2 "ADAM_BQSR_CHARS=row" "ADAM_BQSR_CHARS=cell" "ADAM_BQSR_CHARS=row" "ADAM_BQSR_CHARS=cell"
bash tools/ab_env.sh r03cm/ab4 cfg4 "ADAM_BQSR_CHARS=row" "ADAM_BQSR_CHARS=cell"
