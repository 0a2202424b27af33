"""More HIP-vs-oracle parity cases (bit for bit, through the C ABI):

* quals 60..127 across three read groups: the qualByRG key aliasing of
  `q + 60 * rg` (rg0/q61 == rg1/q1), q = 0 attributed to group rg - 1 and
  q >= 61 to rg + 1 by finalize's `(key - 1) / 60` (RecalTable.scala:121,129;
  StandardCovariate.scala:25-32), and the apply path for quals above the LDS
  char-table rows;
* a crafted table (bqsr_table_upload) whose shifts drive apply to Java chars
  above 0xFF (Q < -33) and to non-ASCII codes 128..255 (Q > 94)
  (RecalUtil.scala:37-40, quirk Q14);
* known sites loaded by SnpTable.from_vcf from the reference's own
  small.vcf (SnpTable.scala:32-47, raw 1-based POS, quirk Q7);
* a 1M-read partition (1e8 bases): the expectedMismatch fold's block / tile /
  element descent at scale.
"""
import ctypes
import os

import numpy as np
import pytest

import oracle as O
from _parity import check
from adam_amd import _capi, bqsr, synth
from adam_amd.records import ADAMRecord, RecordBatch

pytestmark = pytest.mark.gpu


@pytest.fixture
def read_order(request):
    """BQSR_TUNE_ORDER (bqsr_context_tune): 'read' = the per-base passes walk
    reads in batch order, 'group' = bucketed by read group (device counting
    sort, pieces per read group); the library picks 'group' for several read
    groups by default."""
    from adam_amd import bqsr as _b
    with _b.Context.get(0).tuned(order=request.param):
        yield request.param

GOLD = os.path.join(os.path.dirname(__file__), "golden", "reference_resources")


def high_qual_batch(n_reads, n_rg, seed, frac=0.5):
    """Synthetic reads whose interior quals are redrawn uniformly from 0..127
    (chars '!'..0xA0) in a fraction of the reads."""
    b = synth.generate(n_reads, (100,), n_rg, seed)
    rng = np.random.default_rng(seed)
    q = b.qual.copy()
    for r in np.nonzero(rng.random(b.n_reads) < frac)[0]:
        a, e = int(b.qual_offset[r]), int(b.qual_offset[r + 1])
        if e - a > 4:
            q[a + 2:e - 2] = rng.integers(0, 128, e - a - 4) + 33
    b.qual = q
    return b


def test_quals_60_to_127_three_read_groups():
    b = high_qual_batch(20000, 3, 41)
    g, o = check([b.slice(0, 7000), b.slice(7000, 20000)])
    K = 60 * 2 + 128
    touched = g.words[:K]
    assert touched[0] > 0 and touched[61] > 0 and touched[127 + 120] > 0  # q=0, aliased 61, rg2/q127


def test_quals_60_to_127_one_read_group_edges():
    # rg0 keys 0..127: key 0 and keys 1..60 are group 0, keys 61..120 group 1,
    # 121..127 group 2 -- groups that exist only through aliasing
    b = high_qual_batch(6000, 1, 43, frac=1.0)
    check([b])


# ---- crafted table: chars above 0xFF and non-ASCII ---------------------------

L10 = 10


def crafted_table(seed):
    """Dense table words (2 read groups, max_len 10) and the quals each read
    group's reads use.  Read group 1's keys take random bins whose mismatch
    count may exceed the observations (possible only through the C ABI, not
    from reads): E = mm/obs far above 1 makes the recalibrated error
    probability huge, Q very negative, (Q + 33).toChar above 0xFF.  Read group
    0's 'near-cancel' keys have qualScore error ~= cycle error + context
    error, so newP is a rounding residue: Q 95..200, chars 128..255 (group 0
    is kept apart so group 1's huge error rates do not swamp the residue)."""
    d = O.Dims(2, L10)
    K, C = 60 + 128, 2 * L10 + 1
    cells = C + 21
    w = np.zeros(K + 2 * K * cells, np.int64)
    t = w[:K]
    obs = w[K:K + K * cells].reshape(K, cells)
    mm = w[K + K * cells:].reshape(K, cells)
    rng = np.random.default_rng(seed)
    pairs = [(1, 0), (3, 1), (1000, 0), (10 ** 6, 1), (10 ** 9, 2000), (10 ** 6, 2), (1, 10 ** 6), (1000, 10 ** 15),
             (7, 7)]
    rand_q = [5, 20, 40, 41, 60]   # read group 1: keys 65..120, group 1
    near_q = [3, 10, 30, 38, 45, 59]  # read group 0: keys 3..59, group 0
    for q in rand_q:
        k = q + 60
        t[k] = rng.integers(1, 1000)
        for c in range(cells):
            if rng.random() < 0.8:
                obs[k, c], mm[k, c] = pairs[rng.integers(0, len(pairs))]
    for i, k in enumerate(near_q):
        t[k] = 5
        obs[k, :C], mm[k, :C] = 1, 0
        obs[k, L10 + 1], mm[k, L10 + 1] = 10 ** 9 + 12345 * i, 2000 + i
        obs[k, C:], mm[k, C:] = 10 ** 6, 1
    return d, w, {0: near_q, 1: rand_q}


def reads_for_keys(quals_by_rg, n, seed):
    rng = np.random.default_rng(seed)
    recs = []
    for i in range(n):
        rg = i % 2
        q = rng.choice(quals_by_rg[rg], L10)
        seq = "".join(rng.choice(list("ACGTN"), L10, p=[0.24, 0.24, 0.24, 0.24, 0.04]))
        recs.append(ADAMRecord(record_group_id=rg, read_mapped=True, primary_alignment=True, start=1000 + i,
                               reference_name="1", cigar="10M", mismatching_positions="10", sequence=seq,
                               qual="".join(chr(int(v) + 33) for v in q),
                               read_negative_strand=bool(i & 2), read_paired=bool(i & 4),
                               second_of_pair=bool(i & 8)))
    return RecordBatch.from_records(recs)


@pytest.mark.parametrize("seed,em", [(7, 0.0), (8, 123.456), (9, 1e5)])
def test_crafted_table_chars_above_0xff(seed, em):
    d, w, keys = crafted_table(seed)
    batch = reads_for_keys(keys, 3000, seed)
    # oracle
    fin = O.Final(d, w, em)
    ref, ref_len = O.apply(batch, fin)
    # HIP path: upload the same words, finalize with the same expectedMismatch, apply
    ctx = bqsr.Context.get(0)
    tab = bqsr.RecalTable(_capi.Dims(2, L10), ctx, expected_mismatch=em)
    tab.set_words(w)
    gfin = tab.finalize_table()
    chars = np.zeros(int(batch.qual_offset[-1]), dtype=np.uint16)
    out_len = np.zeros(batch.n_reads, dtype=np.uint32)
    s, keep = batch.c_struct()
    _capi.check(_capi.lib().bqsr_apply_records(ctx.handle, ctypes.byref(s), gfin.handle, chars.ctypes.data,
                                               out_len.ctypes.data))
    assert np.array_equal(out_len, ref_len[:batch.n_reads])
    n = int(batch.qual_offset[-1])
    bad = np.nonzero(chars[:n] != ref[:n])[0]
    assert bad.size == 0, (bad[:10], chars[bad[:10]], ref[bad[:10]])
    assert (ref[:n] > 0xFF).sum() > 100          # the exception list path
    assert ((ref[:n] >= 128) & (ref[:n] <= 0xFF)).sum() > 10  # non-ASCII bytes in the fast path


def test_crafted_table_compacted_outputs():
    """The streamed path's compacted outputs (bqsr_compact_outputs_async):
    chars at u32 offsets per read, the exception list's entries rewritten to
    positions in the chars -- on the crafted table whose chars go above 0xFF."""
    import torch
    d, w, keys = crafted_table(8)
    batch = reads_for_keys(keys, 3000, 8)
    fin = O.Final(d, w, 123.456)
    ref, ref_len = O.apply(batch, fin)
    ctx = bqsr.Context.get(0)
    tab = bqsr.RecalTable(_capi.Dims(2, L10), ctx, expected_mismatch=123.456)
    tab.set_words(w)
    gfin = tab.finalize_table()
    L = _capi.lib()
    s, keep = batch.c_struct()
    bh = ctypes.c_void_p()
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    _capi.check(L.bqsr_batch_create(ctx.handle, ctypes.byref(s), sp, ctypes.byref(bh)))
    try:
        ns, n = int(L.bqsr_batch_slots(bh)), batch.n_reads
        dev = torch.device("cuda", 0)
        oq = torch.empty(ns + 64, dtype=torch.uint8, device=dev)
        ost, oln = (torch.empty(n, dtype=torch.int32, device=dev) for _ in range(2))
        exc = torch.empty(1 << 16, dtype=torch.int64, device=dev)
        chars = torch.empty(ns + 64, dtype=torch.uint8, device=dev)
        off = torch.empty(n + 1, dtype=torch.int32, device=dev)
        lens = torch.empty(n, dtype=torch.int16, device=dev)
        p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        _capi.check(L.bqsr_apply_stage(ctx.handle, bh, gfin.handle, p(oq), p(ost), p(oln), p(exc), 1 << 16,
                                       _capi.STAGE_RESET | _capi.STAGE_KERNEL, sp))
        _capi.check(L.bqsr_compact_outputs_async(ctx.handle, bh, p(oq), p(ost), p(oln), p(exc), 1 << 16, p(chars),
                                                 p(off), p(lens), sp))
        nexc = ctypes.c_int64()
        _capi.check(L.bqsr_apply_result(bh, ctypes.byref(nexc), sp))
        torch.cuda.synchronize()
        assert nexc.value > 100
        offs = off.cpu().numpy()
        assert np.array_equal(np.diff(offs.astype(np.int64)), ref_len[:n].astype(np.int64))
        assert np.array_equal(lens.cpu().numpy().view(np.uint16).astype(np.int64), ref_len[:n].astype(np.int64))
        bad, first = O.compare_compact_output(batch, ref, ref_len, chars.cpu().numpy()[:int(offs[n])], offs,
                                              exc.cpu().numpy()[:nexc.value])
        assert bad == 0, first
    finally:
        L.bqsr_batch_destroy(bh)


# ---- known sites from the reference's VCF -------------------------------------

def test_sites_from_small_vcf():
    snp = bqsr.SnpTable.from_vcf(os.path.join(GOLD, "small.vcf"))
    assert "20" in snp.table and 14370 in snp.table["20"].tolist()
    sites = {k: v.tolist() for k, v in snp.table.items()}
    # reads on contig "20" around the VCF positions (0-based refPos == raw POS masks, Q7)
    b = synth.generate(30000, (100,), 1, 51, contig_len=1_300_000, contig="20")
    g_sites, o_sites = check([b], sites)
    g_none, _ = check([b], None)
    assert not np.array_equal(g_sites.words, g_none.words)  # some bases were masked by the VCF sites


@pytest.mark.parametrize("lens", [(101,), (150, 250)])
def test_sites_bitmap_dense(lens):
    """Dense sites (the prep kernel's position bitmap): runs where every
    position is a site, so reads of 101-250 bases take several 64-offset
    steps with bits in all three sbits words of a step, plus a sparse contig
    (no bitmap: the linear scan) on the same batch."""
    rng = np.random.default_rng(7)
    dense = np.unique(np.concatenate([np.arange(5_000, 9_000), np.arange(40_001, 40_600, 3),
                                      rng.integers(1, 200_000, size=20_000)]))
    b = synth.generate(20000, lens, 1, 71, contig_len=200_000, contig="chr20")
    sites = {"chr20": dense.tolist(), "chr7": [5, 90_000_000]}
    g_sites, o_sites = check([b], sites)
    g_none, _ = check([b], None)
    assert not np.array_equal(g_sites.words, g_none.words)


@pytest.mark.parametrize("lens,seed", [((1, 3, 7, 15, 16, 17, 31), 81), ((5, 33, 64, 100, 128), 82),
                                       ((101,), 83)])
def test_sites_word_stores(lens, seed):
    """Known sites with reads of <= 128 bases: prep's pass 1 stores every
    bitmap word (PrepParams::store_words) -- several short reads per word,
    reads starting mid-word, words shared across wavefronts (the boundary
    shares pass 2 ORs in), complex reads (indels) whose bits pass 2 adds on
    the stored words -- against the oracle, with dense and sparse sites."""
    rng = np.random.default_rng(seed)
    dense = np.unique(np.concatenate([np.arange(2_000, 6_000), rng.integers(1, 60_000, size=8_000)]))
    b = synth.generate(30000, lens, 1, seed, contig_len=60_000, contig="chr20", p_indel=0.1, p_softclip=0.2)
    check([b], {"chr20": dense.tolist()})
    check([b.slice(0, 12345), b.slice(12345, 30000)], {"chr20": dense.tolist(), "chr7": [5, 90_000_000]})


# ---- the fold at scale --------------------------------------------------------

def test_fold_one_million_reads():
    b = synth.generate(1_000_000, (100,), 1, 61)
    g, o = check([b])
    assert g.em == o.em


# ---- prep's lock-step path ([S]M[S] CIGAR, MD <= 16 bytes) and its borders ----

S32 = "ACGTACGTACGTACGTACGTACGTACGTACGT"
Q32 = "IIIIHHHHGGGGFFFF" * 2


def rec32(**kw):
    base = dict(record_group_id=0, read_mapped=True, primary_alignment=True, start=20000, reference_name="1",
                cigar="32M", mismatching_positions="32", sequence=S32, qual=Q32)
    base.update(kw)
    return ADAMRecord(**base)


EDGE32 = [
    rec32(),
    rec32(mismatching_positions="0A31"), rec32(mismatching_positions="31A0"), rec32(mismatching_positions="31"),
    rec32(mismatching_positions="5a26"), rec32(mismatching_positions="10AC20"),
    rec32(mismatching_positions="1A1A1A1A1A1A1A21"), rec32(mismatching_positions="1A1A1A1A1A1A1A1A1"),
    rec32(mismatching_positions="40"), rec32(mismatching_positions="3G3^T25"), rec32(mismatching_positions="0"),
    rec32(cigar="2S30M", mismatching_positions="29C0"), rec32(cigar="30M2S", mismatching_positions="0T29"),
    rec32(cigar="1S30M1S", mismatching_positions="30"), rec32(cigar="5S27M", mismatching_positions="12"),
    rec32(cigar="16S16M", start=15), rec32(cigar="32M", start=0),
    rec32(cigar="3H29M", sequence=S32[:29], qual=Q32[:29]), rec32(cigar="30M2H", sequence=S32[:30], qual=Q32[:30]),
    rec32(cigar="10M1I21M", mismatching_positions="31"), rec32(cigar="10M2D22M", mismatching_positions="10^AA22"),
    rec32(qual="#" * 16 + "I" * 16), rec32(qual="#" * 15 + "I" * 17), rec32(qual="I" * 17 + "#" * 15),
    rec32(qual="I" * 16 + "#" * 16), rec32(qual="#" * 32),
    rec32(read_negative_strand=True, cigar="2S30M", mismatching_positions="7T22"),
    rec32(read_paired=True, second_of_pair=True, cigar="30M2S", mismatching_positions="30"),
    rec32(mismatching_positions=None), rec32(mismatching_positions=None, cigar="2S30M"),
    rec32(sequence=S32[:31] + "N"), rec32(sequence="acgt" * 8),
    rec32(record_group_id=1, qual="5" * 32, mismatching_positions="16T15"),
]


@pytest.mark.parametrize("read_order", ["read", "group"], indirect=True)
def test_prep_fast_path_borders(read_order):
    check([RecordBatch.from_records(EDGE32 * 2)], sites={"1": [20003, 20010, 20031, 20032, 15, 20]})


@pytest.mark.parametrize("bad,err", [
    (rec32(mismatching_positions="A31"), "MD_PARSE"), (rec32(mismatching_positions="31A"), "MD_PARSE"),
    (rec32(mismatching_positions="99999999999"), "MD_PARSE"), (rec32(mismatching_positions="3Z28"), "MD_PARSE"),
    (rec32(cigar="20M"), "CIGAR_SHORT"), (rec32(cigar="0S32M"), "CIGAR_INVALID"),
    (rec32(cigar="32M0S"), "CIGAR_INVALID"), (rec32(sequence=S32[:20]), "SEQ_SHORT"),
    (rec32(reference_name=None), "NULL_FIELD"), (rec32(start=None), "NULL_FIELD"),
    (rec32(read_negative_strand=True, sequence=S32[:31] + "x"), "BAD_REVCOMP_BASE"),
])
def test_prep_fast_path_errors(bad, err):
    ok = [rec32(), rec32(qual="H" * 32)]
    check([RecordBatch.from_records(ok + [bad] + ok)], expect_error=err)


@pytest.mark.parametrize("read_order", ["read", "group"], indirect=True)
def test_char_table_row_gap(read_order):
    """Quals drawn from 5..14 and 30..41 only: the char-table rows 15..29 of
    the window hold no key (0 entries), so apply's clean rows are one side of
    the gap and the other side's offsets take the checked path -- every char
    must still match the oracle."""
    b = synth.generate(12000, (100,), 2, 77)
    rng = np.random.default_rng(77)
    q = b.qual.copy()
    lo = rng.integers(5, 15, q.size)
    hi = rng.integers(30, 42, q.size)
    pick = np.where(rng.random(q.size) < 0.35, lo, hi) + 33
    keep = q <= 33 + 2  # leave the Q2 tails (trimming) as they are
    b.qual = np.where(keep, q, pick).astype(q.dtype)
    check([b.slice(0, 5000), b.slice(5000, 12000)])
