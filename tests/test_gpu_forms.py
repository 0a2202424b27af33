"""GPU parity of the bucketed passes' piece orders that the default sizes do
not reach: the chunk walk on bucketed batches with front-ordered pieces forced
on (5 fronts; the default picks fronts only from 8192 reads per piece, cfg4's
~11) and off, on the key-major copy and on the batch's own layout
(bqsr_context_tune).  Each case checks a read-order and two bucketed jobs
against the oracle (tests/_parity.check: table words, expectedMismatch bits,
every output char)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


@pytest.mark.gpu
@pytest.mark.timeout(300)
@pytest.mark.parametrize("fronts,key_major", [(5, 1), (0, 1), (5, 0), (0, 0)])
def test_piece_orders(fronts, key_major):
    from _parity import check
    from adam_amd import bqsr, synth
    ctx = bqsr.Context.get(0)
    with ctx.tuned(fronts=fronts, key_major=key_major):
        b = synth.generate(12000, (100,), 1, seed=61)
        check([b.slice(0, 5000), b.slice(5000, 12000)], synth.known_sites(2_000_000, seed=5))
        with ctx.tuned(order="group"):
            b = synth.generate(6000, (150, 250), 8, seed=62)
            check([b.slice(0, 2000), b.slice(2000, 6000)], synth.known_sites(2_000_000, seed=5))
        with ctx.tuned(order="read"):
            b = synth.generate(6000, (60, 100, 140), 3, seed=63)
            check([b])


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


@pytest.mark.gpu
@pytest.mark.timeout(600)
@pytest.mark.parametrize("n_rg,lens", [(1, (100,)), (6, (150, 250))])
def test_repeated_jobs_bitmap_cleared(n_rg, lens):
    # each atomic-form prep workgroup clears its own slots' bitmap words
    # before its ORs (no fill pass, nothing carried between jobs).  One
    # resident batch, jobs with known sites, without, with again: site bits
    # left in a word from one job would mask bases of the next.  (100 bp: the
    # sites jobs store whole words, the others clear; 150/250 bp: every job
    # atomic.)  Each job against the oracle.
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle as O
    from adam_amd import bqsr, synth
    from adam_amd.job import ResidentJob
    b = synth.generate(300_000, lens, n_rg, seed=77)
    sites = synth.known_sites(400_000, seed=78)
    snp = bqsr.SnpTable(sites)
    dims = bqsr.dims_of([b])
    od = O.Dims(dims.n_rg, dims.max_len)
    want = {True: O.bqsr(b, O.Sites(sites), od, n_parts=1, nthreads=16, fold1=True),
            False: O.bqsr(b, None, od, n_parts=1, nthreads=16, fold1=True)}
    job = ResidentJob(b, dims, snp, 0)
    sites_h = job.sites_h
    try:
        for with_sites in (True, False, True, False):
            job.sites_h = sites_h if with_sites else None
            job.step()
            words, em, q, st, ln, exc = job.results()
            ow, oem, out, out_len = want[with_sites]
            assert np.array_equal(words, ow), with_sites
            assert np.float64(em).tobytes() == np.float64(oem).tobytes()
            bad, first = O.compare_device_output(b, out, out_len, q, st, ln, exc)
            assert bad == 0, first
    finally:
        job.close()
