#!/bin/bash
# Round measurement pass (run via gpurun): tools/gpu_round3.sh TAG
# -> gpurun_out/TAG/{pytest.log, smoke.log, pmc_fetch/, pmc_write/, pmc_summary.json, pmc_traffic.json,
#    bench_cfg{2,3,4}.json, stats_cfg{2,3,4}/, ingest.json}
# PMC passes first, so the cfg2 bench line carries this tree's traffic.
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
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_fetch" -o run --output-format csv -- \
  python3 "$R/bench.py" --no-cpu-baseline --no-parity --steps 3 --warmup 1 > "$O/pmc_fetch.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d "$O/pmc_write" -o run --output-format csv -- \
  python3 "$R/bench.py" --no-cpu-baseline --no-parity --steps 3 --warmup 1 > "$O/pmc_write.log" 2>&1
python3 "$R/tools/pmc_summary.py" "$O" "$O/pmc_summary.json" > /dev/null
python3 "$R/tools/make_traffic.py" "$O/pmc_summary.json" "$O/pmc_traffic.json" cfg2 "gpurun_out/$TAG" > /dev/null
for c in cfg2 cfg3 cfg4; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/stats_$c" -o run --output-format csv -- \
    python3 "$R/bench.py" --config $c --no-cpu-baseline --no-parity --steps 10 --warmup 1 > "$O/stats_$c.log" 2>&1
done
cd "$R"
timeout -k 10 500 python -u bench.py --traffic "$O/pmc_traffic.json" > "$O/bench_cfg2.json" 2> "$O/bench_cfg2.err"
cat "$O/bench_cfg2.json"
timeout -k 10 500 python -u bench.py --config cfg3 --no-parity --no-cpu-baseline --steps 10 > "$O/bench_cfg3.json" 2> "$O/bench_cfg3.err"
timeout -k 10 500 python -u bench.py --config cfg4 --no-parity --no-cpu-baseline --steps 10 > "$O/bench_cfg4.json" 2> "$O/bench_cfg4.err"
timeout -k 10 300 python -u tools/bench_ingest.py --reads 2000000 > "$O/ingest.json" 2> "$O/ingest.err"
echo done
