#!/bin/bash
# Measurement pass (run via gpurun): tools/gpu_prof.sh TAG [CONFIGS] [PYTEST]
# Per config: FETCH_SIZE and WRITE_SIZE in separate --pmc passes, a
# --kernel-trace --stats pass, the summaries bench.py reads
# (gpurun_out/TAG/CFG/{pmc_traffic,kernel_stats}.json), then the bench line.
# Every GPU step has its own limit; the script stops at the first failure.
set -e
TAG=$1
CONFIGS=${2:-"cfg2"}
PYTEST=${3:-0}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
COMMIT=$(cat "$R/.commit" 2>/dev/null || echo unknown)
if [ "$PYTEST" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=10 -v --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 \
    || { rc=$?; tail -60 "$O/pytest.log"; exit $rc; }
  tail -1 "$O/pytest.log"
  timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
  tail -1 "$O/smoke.log"
fi
export TMPDIR=/tmp
for c in $CONFIGS; do
  mkdir -p "$O/$c"
  cd /tmp
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$O/$c/pmc_fetch" -o run --output-format csv -- \
    python3 "$R/bench.py" --config $c --no-cpu-baseline --no-parity --steps 3 --warmup 1 --event-steps 0 > "$O/$c/pmc_fetch.log" 2>&1
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$O/$c/pmc_write" -o run --output-format csv -- \
    python3 "$R/bench.py" --config $c --no-cpu-baseline --no-parity --steps 3 --warmup 1 --event-steps 0 > "$O/$c/pmc_write.log" 2>&1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/$c/stats" -o run --output-format csv -- \
    python3 "$R/bench.py" --config $c --no-cpu-baseline --no-parity --steps 10 --warmup 1 --event-steps 0 > "$O/$c/stats.log" 2>&1
  cd "$R"
  python3 tools/pmc_summary.py "$O/$c" "$O/$c/pmc_summary.json" > /dev/null
  READS=$(python3 -c "from adam_amd import synth; c=synth.CONFIGS['$c']; print(c['n_reads'] if '$c' != 'cfg5' else c['n_reads']//8)")
  python3 tools/make_traffic.py "$O/$c/pmc_summary.json" "$O/$c/pmc_traffic.json" $c "gpurun_out/$TAG/$c" $READS > /dev/null
  KS=$(find "$O/$c/stats" -name "*kernel_stats.csv" | head -1)
  cp "$KS" "$O/$c/kernel_stats.csv"
  python3 tools/make_kstats.py "$KS" "$O/$c/kernel_stats.json" $c $READS "gpurun_out/$TAG/$c" $COMMIT
  cp "$O/$c/pmc_traffic.json" profiles/pmc_traffic_$c.json
  cp "$O/$c/kernel_stats.json" profiles/kernel_stats_$c.json
  timeout -k 10 600 python -u bench.py --config $c > "$O/bench_$c.json" 2> "$O/bench_$c.err"
  cat "$O/bench_$c.json"
done
echo done
