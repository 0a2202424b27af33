cd $GRAFT_REPO_ROOT
for pr in 0 1 4 8 13; do
  ADAM_BQSR_LIB=$GRAFT_REPO_ROOT/tools/probe/lib_probe.so ADAM_BQSR_PROBE=$pr timeout -k 10 300 python -u bench.py --config cfg2 --no-cpu-baseline --no-parity --steps 10 --warmup 2 > gpurun_out/pr$pr.json 2>/dev/null
  python3 -c "import json; d=json.load(open('gpurun_out/pr$pr.json')); print('probe $pr', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['roofline']['kernel_ms'].items()})"
done
