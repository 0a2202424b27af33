set -e
mkdir -p gpurun_out/r01_s3b
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r01_s3b/pytest.log 2>&1 || { tail -40 gpurun_out/r01_s3b/pytest.log; exit 1; }
tail -3 gpurun_out/r01_s3b/pytest.log
timeout -k 10 600 python -u bench.py --config cfg5 --steps 5 --warmup 1 > gpurun_out/r01_s3b/bench_cfg5.json 2> gpurun_out/r01_s3b/bench_cfg5.err
cat gpurun_out/r01_s3b/bench_cfg5.json
timeout -k 10 300 python -u bench.py --config cfg4 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r01_s3b/bench_cfg4.json 2> gpurun_out/r01_s3b/bench_cfg4.err
cat gpurun_out/r01_s3b/bench_cfg4.json
timeout -k 10 300 python -u bench.py --config cfg3 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r01_s3b/bench_cfg3.json 2> gpurun_out/r01_s3b/bench_cfg3.err
cat gpurun_out/r01_s3b/bench_cfg3.json
