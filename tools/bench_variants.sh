set -e
O=gpurun_out/r01_var; mkdir -p $O
for v in "X=0" "ADAM_BQSR_OBSERVE_ROTATE=1" "ADAM_BQSR_LANES=chunk" "ADAM_BQSR_ORDER=group"; do
  env $v timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 --warmup 2 > $O/b.json 2>/dev/null
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' $O/b.json) $(grep -o '"kernel_ms[^}]*}' $O/b.json)"
done
