set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04c
timeout -k 10 600 python -u -m pytest tests/test_gpu_adam_out.py tests/test_bench_launch.py tests/test_gpu_copy.py tests/test_gpu_sam.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r04c/pytest.log 2>&1 || { tail -80 gpurun_out/r04c/pytest.log; exit 1; }
tail -3 gpurun_out/r04c/pytest.log
