#!/bin/bash
# SQ counter passes over a short cfg2 bench (gpurun): tools/gpu_sq.sh TAG
set -e
R=$(pwd); O=$R/gpurun_out/$1; mkdir -p $O
export TMPDIR=/tmp; cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/p1 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $O/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE -d $O/p2 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $O/p2.log 2>&1
echo ok
