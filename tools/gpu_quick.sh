#!/bin/bash
# GPU tests + quick cfg2 / cfg4 bench lines (gpurun):  tools/gpu_quick.sh TAG
set -e
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_cfg2.json 2> $O/bench_cfg2.err
cut -c1-200 $O/bench_cfg2.json; grep -o '"kernel_ms[^}]*}' $O/bench_cfg2.json
timeout -k 10 300 python -u bench.py --config cfg4 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_cfg4.json 2> $O/bench_cfg4.err
cut -c1-200 $O/bench_cfg4.json; grep -o '"kernel_ms[^}]*}' $O/bench_cfg4.json
