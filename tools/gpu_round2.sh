#!/bin/bash
# Round-2 measurement pass (run via gpurun): tools/gpu_round2.sh TAG
# -> gpurun_out/TAG/{pytest.log, smoke.log, bench_cfg{2,3,4}.json, stats_cfg{2,3,4}/, pmc_fetch/, pmc_write/, ingest.json}
set -e
TAG=$1
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
tail -1 "$O/pytest.log"
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
tail -1 "$O/smoke.log"
timeout -k 10 500 python -u bench.py > "$O/bench_cfg2.json" 2> "$O/bench_cfg2.err"
cat "$O/bench_cfg2.json"
timeout -k 10 500 python -u bench.py --config cfg3 --no-parity --no-cpu-baseline --steps 10 > "$O/bench_cfg3.json" 2> "$O/bench_cfg3.err"
timeout -k 10 500 python -u bench.py --config cfg4 --no-parity --no-cpu-baseline --steps 10 > "$O/bench_cfg4.json" 2> "$O/bench_cfg4.err"
timeout -k 10 300 python -u tools/bench_ingest.py --reads 2000000 > "$O/ingest.json" 2> "$O/ingest.err"
export TMPDIR=/tmp
cd /tmp
for c in cfg2 cfg3 cfg4; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/stats_$c" -o run --output-format csv -- \
    python3 "$R/bench.py" --config $c --no-cpu-baseline --no-parity --steps 10 --warmup 1 > "$O/stats_$c.log" 2>&1
done
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_fetch" -o run --output-format csv -- \
  python3 "$R/bench.py" --no-cpu-baseline --no-parity --steps 3 --warmup 1 > "$O/pmc_fetch.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d "$O/pmc_write" -o run --output-format csv -- \
  python3 "$R/bench.py" --no-cpu-baseline --no-parity --steps 3 --warmup 1 > "$O/pmc_write.log" 2>&1
echo done
