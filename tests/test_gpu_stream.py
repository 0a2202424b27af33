"""Streamed partitions (BASELINE cfg5 path, adam_amd/stream.py): pinned host
partitions uploaded on a copy stream, observed as they land, merged in
partition order, applied from HBM with results copied back -- against the CPU
oracle over the same partitions merged in the same order, bit for bit: table
words, per-partition and merged expectedMismatch, recalibrated qualities."""
import ctypes

import numpy as np
import pytest

from _parity import run_oracle
from adam_amd import _capi, bqsr, synth
from adam_amd.records import F_HAS_QUAL, F_HAS_SEQ

pytestmark = pytest.mark.gpu


def _slots(batch):
    f = batch.flags
    lq = np.where(f & F_HAS_QUAL, np.diff(batch.qual_offset.astype(np.int64)), 0)
    ls = np.where(f & F_HAS_SEQ, np.diff(batch.seq_offset.astype(np.int64)), 0)
    span = (np.maximum(lq, ls) + 15) // 16 * 16
    return np.concatenate([[0], np.cumsum(span)])[:-1]


def _odd_bases(b):
    """Forward reads with lowercase / non-ACGTN bytes (context index -1, Q10):
    the staged 2-bit codes' exception list carries them.  And quals the
    staged 16-slot qual chunks cannot code (a chunk spanning more than 14
    values, qual 0): their exception list and zero code carry them."""
    from adam_amd.records import F_NEG_STRAND
    for r in range(0, b.n_reads, 37):
        if not b.flags[r] & F_NEG_STRAND and b.seq_offset[r + 1] - b.seq_offset[r] > 10:
            a = int(b.seq_offset[r])
            b.seq[a + 3] = ord("x")
            b.seq[a + 7] = ord("a")
            b.seq[a + 8] = ord("N")
    for r in range(5, b.n_reads, 29):
        a, e = int(b.qual_offset[r]), int(b.qual_offset[r + 1])
        if e - a > 40:
            # (SAM chars: phred + 33)
            b.qual[a + 17: a + 33: 2] = 33 + 4   # alternating with ~38: a chunk spanning 35 values
            b.qual[a + 20] = 33                  # '!' (phred 0): the zero code
            b.qual[a + 35] = 33 + 59
            b.qual[a + 36: a + 40] = np.array([33 + 45, 33 + 58, 33 + 3, 33 + 50], np.uint8)
    return b


@pytest.mark.parametrize("sizes,lens,n_rg,with_sites,odd,zero_copy,d2h,compact", [
    ((7000, 5000, 9000), (150,), 1, True, False, False, "kernel", None),
    ((3000, 1, 4000), (100, 250), 4, False, False, False, "kernel", None),
    ((4000, 6000), (101,), 2, False, True, False, "dma", None),
    ((4000, 6001), (101,), 2, False, True, False, "kernel", None),
    ((4000, 6001), (101,), 2, False, True, False, "kernel", False),
    ((5000, 3000), (150,), 1, True, True, True, "kernel", None)])
def test_streamed_partitions(sizes, lens, n_rg, with_sites, odd, zero_copy, d2h, compact):
    import torch
    from adam_amd.stream import StreamedShard
    dev = torch.device("cuda", 0)
    torch.zeros(1, device=dev)  # torch's HIP runtime first, as bench.py does
    parts = [synth.generate(n, lens, n_rg, 900 + i) for i, n in enumerate(sizes)]
    if odd:
        parts = [_odd_bases(p) for p in parts]
    sites = synth.known_sites(200_000) if with_sites else None
    snp = bqsr.SnpTable(sites) if sites else None
    d = bqsr.dims_of(parts)
    ctx = bqsr.Context.get(0)
    L = _capi.lib()
    words_t = torch.zeros(int(L.bqsr_table_words(d)), dtype=torch.int64, device=dev)
    th = ctypes.c_void_p()
    _capi.check(L.bqsr_table_create(ctx.handle, d, ctypes.c_void_p(words_t.data_ptr()), ctypes.byref(th)))
    sh = StreamedShard(ctx, parts, d, snp.handle(ctx) if snp else None, 0,
                       site_contigs=snp.contigs if snp else None, zero_copy=zero_copy, d2h=d2h, compact=compact)
    assert sh.compact == (compact is not False and not zero_copy and d2h == "kernel")
    try:
        for _ in range(2):  # the second job re-uploads over the resident partitions
            em_t = sh.run(th)
            assert sh.finish() == 0
        o = run_oracle(parts, sites)
        assert np.array_equal(words_t.cpu().numpy(), o.words)
        assert sh.em.cpu().numpy()[:len(parts)].tolist() == o.parts_em
        assert float(em_t.cpu()[0]) == o.em
        for i, p in enumerate(parts):
            ref_out, ref_len = o.outs[i]
            slots = _slots(p)
            for r in range(p.n_reads):
                a = int(p.qual_offset[r])
                got = sh.qual_chars(i, int(slots[r]), r)
                assert np.array_equal(got, ref_out[a:a + int(ref_len[r])]), (i, r)
            assert sh.outputs(i)[0] == ("compact" if sh.compact else "slots")
    finally:
        sh.close()
        L.bqsr_table_destroy(th)


def test_upload_refuses_another_staged_partition():
    """A batch uploads only the staged partition it was created from: its
    quality window and histogram came from that partition, so another one --
    even of the same shape, here the same reads staged twice -- is refused."""
    import torch
    L = _capi.lib()
    ctx = bqsr.Context.get(0)
    part = synth.generate(3000, (100,), 1, 4321)
    s, keep = part.c_struct(None)
    a, b = ctypes.c_void_p(), ctypes.c_void_p()
    _capi.check(L.bqsr_stage_records(ctx.handle, ctypes.byref(s), ctypes.byref(a)))
    _capi.check(L.bqsr_stage_records(ctx.handle, ctypes.byref(s), ctypes.byref(b)))
    bh = ctypes.c_void_p()
    try:
        _capi.check(L.bqsr_batch_create_staged(ctx.handle, a, ctypes.byref(bh)))
        sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        _capi.check(L.bqsr_batch_upload_async(bh, a, sp))
        assert L.bqsr_batch_upload_async(bh, b, sp) == _capi.INVALID_ARG
        torch.cuda.synchronize()
    finally:
        if bh:
            L.bqsr_batch_destroy(bh)
        L.bqsr_staged_destroy(a)
        L.bqsr_staged_destroy(b)
