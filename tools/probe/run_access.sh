set -e
R=$(pwd); O=$R/gpurun_out/probe; mkdir -p $O
timeout -k 10 120 ./tools/probe/access | tee $O/access.txt
export TMPDIR=/tmp; cd /tmp
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/w -o run --output-format csv -- $R/tools/probe/access > $O/w.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/f -o run --output-format csv -- $R/tools/probe/access > $O/f.log 2>&1
echo ok
