set -e
R=$(pwd); O=$R/gpurun_out/r01_ks; mkdir -p $O
export TMPDIR=/tmp; cd /tmp
for c in cfg3 cfg4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$c -o run --output-format csv -- python3 $R/bench.py --config $c --no-cpu-baseline --steps 5 --warmup 1 > $O/$c.log 2>&1
done
echo ok
