"""bench.py --gpus N: the launcher starts N ranks itself (the driver's
command form `python bench.py --gpus N`, without torch.distributed.run).

CPU tests cover the launcher with stand-in rank programs (success relays
rank 0's line; a failing rank ends the job with its exit status and the
others are terminated) and the real bench on a host without a GPU (every
rank fails, no result line).  The GPU tests run the real multi-rank bench
with two gloo ranks sharing device 0: cfg3 (resident, known sites) and cfg5
(streamed), each with its multi-rank oracle parity."""
import io
import json
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    sys.path.insert(0, ROOT)
    import bench
    return bench


def test_launch_relays_rank0_line():
    bench = _bench()
    prog = ("import os, json; r = int(os.environ['RANK']); "
            "assert os.environ['WORLD_SIZE'] == '3' and os.environ['MASTER_ADDR'] == '127.0.0.1'; "
            "print(json.dumps({'rank': r, 'port': os.environ['MASTER_PORT']}) if r == 0 else 'rank %d' % r)")
    out = io.StringIO()
    rc = bench.launch(3, [sys.executable, "-c", prog], out=out)
    assert rc == 0
    line = json.loads(out.getvalue().strip())
    assert line["rank"] == 0 and int(line["port"]) > 0


def test_launch_failing_rank_ends_the_job():
    bench = _bench()
    # rank 1 fails at once; rank 0 would wait (as in a collective) for a minute
    prog = "import os, sys, time; r = int(os.environ['RANK']); (sys.exit(3) if r == 1 else time.sleep(60))"
    out = io.StringIO()
    t = time.time()
    rc = bench.launch(2, [sys.executable, "-c", prog], out=out)
    assert rc == 3
    assert time.time() - t < 30
    assert out.getvalue() == ""


def test_bench_multi_rank_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
                        "--reads", "1000", "--steps", "1", "--warmup", "0"], capture_output=True, text=True,
                       timeout=300, cwd=ROOT)
    assert p.returncode != 0
    assert p.stdout.strip() == ""
    assert "no HIP device" in p.stderr


def _run_gpu_bench(extra):
    p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
                        "--steps", "2", "--warmup", "1", "--event-steps", "1", "--no-cpu-baseline"] + extra,
                       capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_bench_two_ranks_cfg3_gloo():
    d = _run_gpu_bench(["--config", "cfg3", "--reads", "400000"])
    assert d["n_gpus"] == 2
    assert d["parity"]["ranks"] == 2 and d["parity"]["ok"], d["parity"]
    assert d["parity"]["reads_checked"] == 400000
    assert d["value"] > 0


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_bench_two_ranks_cfg5_gloo():
    d = _run_gpu_bench(["--config", "cfg5", "--reads", "300000", "--part-reads", "100000"])
    assert d["n_gpus"] == 2
    p = d["parity"]
    assert p["ranks"] == 2 and p["ok"], p
    assert p["table_words_equal"] and p["expected_mismatch_equal"]
    assert p["reads_checked"] == 2 * 200000  # first + last partition of each rank
