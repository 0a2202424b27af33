#!/bin/bash
# fronts with the chunk walk adding into base-key slabs: parity, cfg4 bench (full-shard parity), kernel stats (gpurun)
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/r03fr7; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_forms.py tests/test_gpu_parity.py tests/test_gpu_parity_more.py tests/test_gpu_staged.py tests/test_gpu_stream.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu_r03.sh r03fr7 cfg4 0
