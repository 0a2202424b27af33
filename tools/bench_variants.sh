#!/bin/bash
# cfg2 bench under the library's layout / lane switches (gpurun): tools/bench_variants.sh [VAR=VALUE ...]
set -e
O=gpurun_out/r01_var; mkdir -p $O
for v in "X=0" "$@"; do
  env $v timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 20 --warmup 3 > $O/b.json 2>/dev/null
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' $O/b.json) $(grep -o '"kernel_ms[^}]*}' $O/b.json)"
done
