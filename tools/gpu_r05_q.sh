#!/bin/bash
# r05q: load-pattern microbenchmark; LDS counters of the product observe on cfg2
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out/r05q
timeout -k 10 120 ./tools/ubench_stride | tee gpurun_out/r05q/ubench_stride.txt
L="SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_LDS"
bash tools/pmc_sq.sh r05q_lds_cfg2 "$L" --config cfg2
