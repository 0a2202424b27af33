#!/bin/bash
# observe lean revisions A/B against a library build of the previous commit (gpurun):
#   tools/gpu_r03_s.sh TAG OTHER.so
set -e
TAG=$1
OTHER=$2
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity_more.py tests/test_gpu_staged.py -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 \
  || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
bash tools/ab_lib.sh $TAG "cfg2 cfg3" - "$R/$OTHER"
for lib in - "$OTHER"; do
  [ "$lib" = - ] && L="$R/adam_amd/libadam_bqsr.so" || L="$R/$lib"
  echo "== SQ cfg2 $lib"
  ADAM_BQSR_LIB="$L" bash tools/pmc_sq.sh $TAG/sq_$(basename $L .so) "SQ_INSTS_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY" --config cfg2 | grep observe
done
echo done
