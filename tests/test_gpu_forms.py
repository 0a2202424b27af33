"""GPU parity of the bucketed passes' piece orders that the default sizes do
not reach (the library reads ADAM_BQSR_FRONTS once per process, so each runs
in a child process): the chunk walk on bucketed batches with front-ordered
pieces forced on (5 fronts; the default picks fronts only from 8192 reads per
piece, cfg4's ~11) and off.  Each child checks a read-order and two bucketed
jobs against the oracle (tests/_parity.check: table words, expectedMismatch
bits, every output char)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import os, sys
sys.path.insert(0, {root!r}); sys.path.insert(0, os.path.join({root!r}, "tests")); sys.path.insert(0, os.path.join({root!r}, "oracle"))
from _parity import check
from adam_amd import synth
b = synth.generate(12000, (100,), 1, seed=61)
check([b.slice(0, 5000), b.slice(5000, 12000)], synth.known_sites(2_000_000, seed=5))
os.environ["ADAM_BQSR_ORDER"] = "group"
b = synth.generate(6000, (150, 250), 8, seed=62)
check([b.slice(0, 2000), b.slice(2000, 6000)], synth.known_sites(2_000_000, seed=5))
os.environ["ADAM_BQSR_ORDER"] = "read"
b = synth.generate(6000, (60, 100, 140), 3, seed=63)
check([b])
print("forms ok")
"""


@pytest.mark.gpu
@pytest.mark.timeout(300)
@pytest.mark.parametrize("fronts,fold_hist,key_major", [("5", "pass", "1"), ("5", "observe", "1"), ("0", "pass", "1"),
                                                        ("5", "pass", "0"), ("0", "pass", "0")])
def test_piece_orders(fronts, fold_hist, key_major):
    # front-ordered pieces of the bucketed jobs forced on / off (bqsr_capi.cpp
    # fronts()); with fronts, the fold's block histograms by bqsr_fold_hist or
    # counted in the observe kernel (ADAM_BQSR_FOLD_HIST); the bucketed passes
    # on the key-major copy or the batch's own layout (ADAM_BQSR_KEYMAJOR)
    env = dict(os.environ, ADAM_BQSR_FRONTS=fronts, ADAM_BQSR_FOLD_HIST=fold_hist, ADAM_BQSR_KEYMAJOR=key_major)
    r = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT)], env=env, capture_output=True, text=True,
                       timeout=280)
    assert r.returncode == 0 and "forms ok" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_default_fronts_full_parity():
    # the default front split on a bucketed batch large enough for it
    # (bqsr_capi.cpp fronts(): 8 read groups -> 16 base keys; 2.4M reads give
    # min(ceil(8 * 256 / 16), 2.4M / (8192 * 16)) = 18 fronts, 288 pieces >= 256
    # CUs), no environment override: one job against the oracle over the
    # whole batch -- table words, expectedMismatch bits, every char
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle as O
    from adam_amd import bqsr, synth
    from adam_amd.job import ResidentJob
    b = synth.generate(2_400_000, (150, 250), 8, seed=71)
    dims = bqsr.dims_of([b])
    job = ResidentJob(b, dims, None, 0)
    try:
        job.step()
        words, em, q, st, ln, exc = job.results()
    finally:
        job.close()
    ow, oem, out, out_len = O.bqsr(b, None, O.Dims(dims.n_rg, dims.max_len), n_parts=1, nthreads=16, fold1=True)
    assert np.array_equal(words, ow)
    assert np.float64(em).tobytes() == np.float64(oem).tobytes()
    bad, first = O.compare_device_output(b, out, out_len, q, st, ln, exc)
    assert bad == 0, first
