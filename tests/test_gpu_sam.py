"""SAM ingest (§8 f1), the output path (§8 f2) and the transform harness on
the device, against records.read_sam (the SAMRecordConverter restatement) and
the CPU oracle."""
import os
import time

import numpy as np
import pytest

import markdup as M  # oracle/markdup.py
import oracle as O
from _parity import run_oracle
from adam_amd import _capi, bqsr, synth
from adam_amd import records as R
from adam_amd.records import read_sam
from adam_amd.sam import SamText
from adam_amd.samgen import sam_text
from adam_amd.transform import sam_partitions, transform

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden", "reference_resources")
FIXTURES = ["artificial.realigned.sam", "artificial.sam", "reads12.sam", "small.sam",
            "small_realignment_targets.sam", "unmapped.sam"]
COLS = ["flags", "rg_id", "ref_index", "start", "seq_offset", "seq", "qual_offset", "qual", "cigar_offset", "cigar",
        "md_offset", "md"]


def assert_same_columns(a: R.RecordBatch, b: R.RecordBatch):
    assert a.n_reads == b.n_reads
    assert a.ref_names == b.ref_names
    for c in COLS:
        x, y = getattr(a, c), getattr(b, c)
        assert x.dtype == y.dtype and np.array_equal(x, y), c


@pytest.mark.parametrize("name", FIXTURES)
def test_parse_reference_fixtures(name):
    path = os.path.join(GOLD, name)
    assert_same_columns(SamText.read(path).batch(), read_sam(path))


EDGE = (b"@HD\tVN:1.4\r\n"
        b"@SQ\tSN:chrA\tLN:1000\n@SQ\tSN:chrB\tLN:1000\n\n"
        b"@RG\tID:zeta\tLB:l1\n@RG\tID:alpha\n@RG\tID:mid\tLB:l2\n"
        b"q1\t0\tchrA\t10\t60\t5M\t*\t0\t0\tACGTN\tIIIII\tMD:Z:5\tRG:Z:mid\r\n"
        b"\n"
        b"q2\t16\tchrB\t0\t60\t2S3M\t*\t0\t0\tAC\xe9GT\t#\xa0I!~\tMD:Z:1A1\tMD:i:3\tXX:Z:a:b:c\n"
        b"q3\t4\t*\t0\t0\t*\t*\t0\t0\t*\t*\n"
        b"q4\t1107\tchrZ\t77\t60\t1M1I1D1N1S1H1P1=1X\t*\t0\t0\tAAAAAAA\tBBBBBBB\tRG:Z:nope\tRG:Z:alpha\n"
        b"q5\t+3\tchrA\t 5 \t60\t4M\t*\t0\t0\tGGGG\t????\n"
        b"q6\t-1\tchrB\t1\t60\t3M\t*\t0\t0\tTTT\t@@@\tMD:Z:\n"
        b"q7\t256\tchrA\t99\t60\t2M\t*\t0\t0\tCC\tDD")  # no final newline


def test_parse_edge_cases(tmp_path):
    p = tmp_path / "edge.sam"
    p.write_bytes(EDGE)
    got = SamText(EDGE).batch()
    want = read_sam(str(p))
    assert got.n_reads == 7
    assert_same_columns(got, want)


@pytest.mark.parametrize("line,status", [
    (b"q\t0\tchrA\t1\t60\t3M\t*\t0\t0\tAAA\n", "SAM_PARSE"),                      # 10 fields
    (b"q\t0\tchrA\t1\t60\t3M\t*\t0\t0\tAAA\tIII\tMD5\n", "SAM_PARSE"),            # tag without two ':'
    (b"q\t0\tchrA\t1\t60\t3M\t*\t0\t0\tAAA\tIII\t\n", "SAM_PARSE"),               # empty optional field
    (b"q\tx1\tchrA\t1\t60\t3M\t*\t0\t0\tAAA\tIII\n", "SAM_PARSE"),                # FLAG
    (b"q\t0\tchrA\tx\t60\t3M\t*\t0\t0\tAAA\tIII\n", "SAM_PARSE"),                 # POS of a known RNAME
    (b"q\t0\tchrA\t1\t60\t3Q\t*\t0\t0\tAAA\tIII\n", "SAM_PARSE"),                 # CIGAR op
    (b"q\t0\tchrA\t1\t60\tM\t*\t0\t0\tAAA\tIII\n", "SAM_PARSE"),                  # CIGAR without length
    (b"q\t0\tchrA\t1\t60\t3\t*\t0\t0\tAAA\tIII\n", "SAM_PARSE"),                  # trailing number
    (b"q\t0\tchrA\t1\t60\t3M\t*\t0\t0\tAAA\tIII\n@CO\tlate\n", "UNSUPPORTED"),  # header after a record
])
def test_parse_errors(tmp_path, line, status):
    text = b"@SQ\tSN:chrA\tLN:10\n" + line
    with pytest.raises(_capi.BQSRError) as e:
        SamText(text)
    assert e.value.name == status
    if status == "SAM_PARSE":  # the Python restatement throws on the same text
        p = tmp_path / "bad.sam"
        p.write_bytes(text)
        with pytest.raises(Exception):
            read_sam(str(p))


def test_parse_unknown_rname_ignores_pos(tmp_path):
    # int(pos) is only evaluated for a header RNAME (records.py:331-335)
    text = b"@SQ\tSN:chrA\tLN:10\nq\t0\tchrQ\tx\t60\t3M\t*\t0\t0\tAAA\tIII\n"
    p = tmp_path / "u.sam"
    p.write_bytes(text)
    assert_same_columns(SamText(text).batch(), read_sam(str(p)))


def test_parse_synthetic_reads(tmp_path):
    b = synth.generate(60000, (100, 150), 3, 97, contig_len=2_000_000)
    text = sam_text(b, n_rg=3)
    p = tmp_path / "syn.sam"
    p.write_bytes(text)
    t0 = time.perf_counter()
    s = SamText(text)
    dt = time.perf_counter() - t0
    got = s.batch()
    assert_same_columns(got, read_sam(str(p)))
    print("ingest: %d reads, %.1f MB in %.3f s (incl. H2D)" % (got.n_reads, len(text) / 1e6, dt))


def _oracle_quals(batch, sites):
    o = run_oracle([batch], sites)
    assert o.error is None, o.error
    chars, out_len = o.outs[0]
    return o, [chars[int(batch.qual_offset[r]):int(batch.qual_offset[r]) + int(out_len[r])]
               for r in range(batch.n_reads)]


def _records(text: bytes):
    return [l.split(b"\t") for l in text.split(b"\n") if l and not l.startswith(b"@")]


def test_transform_recalibrate_round_trip(tmp_path):
    src = os.path.join(GOLD, "artificial.realigned.sam")
    vcf = os.path.join(GOLD, "small.vcf")
    out = tmp_path / "out.sam"
    transform(src, str(out), recalibrate=True, dbsnp=vcf)
    batch = read_sam(src)
    snp = bqsr.SnpTable.from_vcf(vcf)
    o, quals = _oracle_quals(batch, {k: v.tolist() for k, v in snp.table.items()})
    before, after = _records(open(src, "rb").read()), _records(out.read_bytes())
    assert len(before) == len(after) == batch.n_reads
    eligible = 0
    for r, (a, b) in enumerate(zip(before, after)):
        assert a[:10] == b[:10] and a[11:] == b[11:]  # every field but QUAL kept
        f = int(batch.flags[r])
        if (f & R.F_MAPPED) and (f & R.F_PRIMARY) and not (f & R.F_DUPLICATE):
            eligible += 1
            assert b[10] == "".join(map(chr, quals[r])).encode("utf-8"), r
        else:
            assert b[10] == a[10]
    assert eligible > 0


def test_transform_empty_table_and_null_rg(tmp_path):
    with pytest.raises(_capi.BQSRError) as e:
        transform(os.path.join(GOLD, "small.sam"), str(tmp_path / "o.sam"), recalibrate=True)
    assert e.value.name == "EMPTY_TABLE"
    with pytest.raises(_capi.BQSRError) as e:
        transform(os.path.join(GOLD, "artificial.sam"), str(tmp_path / "o.sam"), recalibrate=True)
    assert e.value.name == "NULL_RG"


def test_transform_synthetic_reads(tmp_path):
    b = synth.generate(20000, (100,), 2, 5, contig_len=500_000)
    text = sam_text(b, n_rg=2)
    src, out = tmp_path / "in.sam", tmp_path / "out.sam"
    src.write_bytes(text)
    sites = synth.known_sites(5000, contig_len=500_000)
    vcf = tmp_path / "s.vcf"
    vcf.write_text("".join("chr20\t%d\t.\tA\tC\n" % p for p in sites["chr20"]))
    transform(str(src), str(out), recalibrate=True, dbsnp=str(vcf))
    batch = read_sam(str(src))
    o, quals = _oracle_quals(batch, {"chr20": sites["chr20"].tolist()})
    before, after = _records(text), _records(out.read_bytes())
    for r, (a, c) in enumerate(zip(before, after)):
        f = int(batch.flags[r])
        assert a[:10] == c[:10] and a[11:] == c[11:]
        if (f & R.F_MAPPED) and (f & R.F_PRIMARY) and not (f & R.F_DUPLICATE):
            assert c[10] == "".join(map(chr, quals[r])).encode("utf-8"), r
        else:
            assert c[10] == a[10]


def _partition_batches(tmp_path, text: bytes, partition_bytes: int):
    header, ranges = sam_partitions(text, partition_bytes)
    parts = []
    for i, (a, b) in enumerate(ranges):
        f = tmp_path / ("part%d.sam" % i)
        f.write_bytes(header + text[a:b])
        parts.append(read_sam(str(f)))
    return parts


@pytest.mark.parametrize("n_parts", [2, 7])
def test_transform_partitions(tmp_path, n_parts):
    # an input larger than one partition: cut at line boundaries, every
    # partition observed into one table, expectedMismatch folded in partition
    # order, applied and rewritten partition by partition -- against the
    # oracle over the same partitions (the reference's RDD of those splits)
    b = synth.generate(30000, (100, 151), 3, 11, contig_len=500_000)
    text = sam_text(b, n_rg=3)
    src, out = tmp_path / "in.sam", tmp_path / "out.sam"
    src.write_bytes(text)
    sites = synth.known_sites(5000, contig_len=500_000)
    vcf = tmp_path / "s.vcf"
    vcf.write_text("".join("chr20\t%d\t.\tA\tC\n" % p for p in sites["chr20"]))
    pb = len(text) // n_parts + 1
    st = transform(str(src), str(out), recalibrate=True, dbsnp=str(vcf), partition_bytes=pb)
    parts = _partition_batches(tmp_path, text, pb)
    assert st["partitions"] == len(parts) >= n_parts
    o = run_oracle(parts, {"chr20": sites["chr20"].tolist()})
    assert o.error is None, o.error
    quals = []
    for p, (chars, out_len) in zip(parts, o.outs):
        quals += [chars[int(p.qual_offset[r]):int(p.qual_offset[r]) + int(out_len[r])] for r in range(p.n_reads)]
    flags = np.concatenate([p.flags for p in parts])
    res = out.read_bytes()
    assert res.startswith(sam_partitions(text, pb)[0])
    before, after = _records(text), _records(res)
    assert len(before) == len(after) == len(quals) == b.n_reads
    for r, (a, c) in enumerate(zip(before, after)):
        f = int(flags[r])
        assert a[:10] == c[:10] and a[11:] == c[11:]
        if (f & R.F_MAPPED) and (f & R.F_PRIMARY) and not (f & R.F_DUPLICATE):
            assert c[10] == "".join(map(chr, quals[r])).encode("utf-8"), r
        else:
            assert c[10] == a[10]


def test_transform_partitions_error_order(tmp_path):
    # a read without a read group in the third partition: the job raises
    # NULL_RG (computeTable's error, before any apply) and writes no output
    b = synth.generate(6000, (100,), 1, 12, contig_len=500_000)
    text = sam_text(b, n_rg=1)
    lines = text.split(b"\n")
    body = [i for i, l in enumerate(lines) if l and not l.startswith(b"@")]
    k = body[len(body) // 2]
    lines[k] = b"\t".join(f for f in lines[k].split(b"\t") if not f.startswith(b"RG:Z:"))
    text = b"\n".join(lines)
    src, out = tmp_path / "in.sam", tmp_path / "out.sam"
    src.write_bytes(text)
    pb = len(text) // 4 + 1
    parts = _partition_batches(tmp_path, text, pb)
    o = run_oracle(parts)
    assert o.error == "NULL_RG"
    with pytest.raises(_capi.BQSRError) as e:
        transform(str(src), str(out), recalibrate=True, partition_bytes=pb)
    assert e.value.name == o.error
    assert not out.exists() and not (tmp_path / "out.sam.partial").exists()


def test_rewrite_java_chars_as_utf8():
    # the output path's encoding (Q14): the apply buffers of a job, overwritten
    # with chars of every UTF-8 length (u8 slots plus exceptions above 0xFF)
    from adam_amd.job import ResidentJob
    import torch
    src = os.path.join(GOLD, "artificial.realigned.sam")
    sam = SamText.read(src)
    batch = sam.batch()
    job = ResidentJob(batch, bqsr.dims_of([batch]), None, 0)
    try:
        job.step()
        L = _capi.lib()
        n = batch.n_reads
        slots = np.zeros(n, np.int64)
        # the batch's slot of each read: consecutive 16-aligned spans (bqsr_capi.cpp slot_span)
        lq = np.diff(batch.qual_offset.astype(np.int64))
        ls = np.diff(batch.seq_offset.astype(np.int64))
        span = ((np.maximum(lq, ls) + 15) // 16) * 16
        slots[1:] = np.cumsum(span)[:-1]
        assert int(L.bqsr_batch_slots(job.bh)) == int(span.sum())
        oq = np.zeros(job.out_qual.numel(), np.uint8)
        ost = np.zeros(n, np.int32)
        oln = np.zeros(n, np.int32)
        exc = []
        want = {}
        for r in range(n):
            k = int(min(lq[r], 12))
            chars = [0x41 + ((r * 7 + j * 29) % 0xBE) for j in range(k)]
            if k > 3:
                chars[2] = 0x100 + r * 97
                chars[3] = 0x7FF + r
            for j, c in enumerate(chars):
                oq[slots[r] + 1 + j] = c & 0xFF
                if c > 0xFF:
                    exc.append(((int(slots[r]) + 1 + j) << 16) | c)
            ost[r], oln[r] = 1, k
            want[r] = "".join(map(chr, chars)).encode("utf-8")
        job.out_qual.copy_(torch.from_numpy(oq))
        job.out_start[:n].copy_(torch.from_numpy(ost))
        job.out_len[:n].copy_(torch.from_numpy(oln))
        job.exc[:len(exc)].copy_(torch.from_numpy(np.asarray(exc[::-1], np.int64)))
        job.n_exc = len(exc)
        torch.cuda.synchronize()
        sam.rewrite(job)
        after = _records(sam.text())
        before = _records(open(src, "rb").read())
        for r in range(n):
            f = int(batch.flags[r])
            if (f & R.F_MAPPED) and (f & R.F_PRIMARY) and not (f & R.F_DUPLICATE):
                assert after[r][10] == want[r], r
            else:
                assert after[r][10] == before[r][10]
    finally:
        job.close()
        sam.close()


def _dup_text(n: int, far: bool = False) -> bytes:
    """pairs and fragments stacked on few positions: mates share a QNAME --
    read 2k+1 with read 2k, or (far) read k + n/2 with read k, so mates
    land in different partitions"""
    b = synth.generate(n, (60,), 2, 11, contig_len=3000, p_duplicate=0.0)
    text = sam_text(b, n_rg=2, qname="p")
    lines = text.split(b"\n")
    body = [l for l in lines if l and not l.startswith(b"@")]
    h = len(body) // 2
    pairs = [(k + h, k) for k in range(0, h, 3)] if far else [(k, k - 1) for k in range(1, len(body), 2)]
    for k, m in pairs:
        f = body[k].split(b"\t")
        f[0] = body[m].split(b"\t")[0]
        body[k] = b"\t".join(f)
    return b"\n".join([l for l in lines if l.startswith(b"@")] + body) + b"\n"


def _dup_want(src):
    """MarkDuplicates' restatement (oracle/markdup.py) over the records of src"""
    text = open(src, "rb").read()
    batch = read_sam(str(src))
    recs = _records(text)
    rg_lib = {i: "lib%d" % (i % 2) for i in range(2)}
    reads = []
    for r, f in enumerate(recs):
        fl = int(batch.flags[r])
        flag = int(f[1])
        cig = R.parse_cigar(f[5].decode())
        reads.append(dict(name=f[0].decode(), library=rg_lib[int(batch.rg_id[r])] if fl & R.F_HAS_RG else None,
                          rg=int(batch.rg_id[r]) if fl & R.F_HAS_RG else None, mapped=bool(fl & R.F_MAPPED),
                          primary=bool(fl & R.F_PRIMARY), paired=bool(fl & R.F_PAIRED),
                          mate_mapped=flag != 0 and bool(flag & 1) and not flag & 8, neg=bool(fl & R.F_NEG_STRAND),
                          ref=0, start=int(batch.start[r]), qual=f[10].decode("latin-1"),
                          cigar=[(int(e) >> 4, "MIDNSHP=X"[int(e) & 15]) for e in cig]))
    return M.mark_duplicates(reads)


def test_transform_mark_duplicates(tmp_path):
    text = _dup_text(4000)
    src, out = tmp_path / "in.sam", tmp_path / "out.sam"
    src.write_bytes(text)
    st = transform(str(src), str(out), mark_duplicates=True)
    recs = _records(text)
    want = _dup_want(src)
    assert st["duplicates"] == sum(want) > 0
    after = _records(out.read_bytes())
    for r, (a, c) in enumerate(zip(recs, after)):
        flag = int(a[1])
        assert int(c[1]) == ((flag | 0x400) if want[r] else (flag & ~0x400)), r
        assert a[2:] == c[2:]


def test_compare_baseqs_transform_output(tmp_path):
    # compare -baseqs (§8 f4) between the input and its recalibrated output
    from adam_amd.compare import compare_baseqs
    src = os.path.join(GOLD, "small_realignment_targets.sam")
    out = tmp_path / "out.sam"
    transform(src, str(out), recalibrate=True)
    r = compare_baseqs(src, str(out), "latin-1", "utf-8")
    assert r["unique1"] == r["unique2"] == 0
    assert r["count"] > 0 and r["identity"] < r["count"]


@pytest.mark.parametrize("name,count", [("unmapped.sam", 200), ("small.sam", 20), ("reads12.sam", 200)])
def test_device_parse_reference_fixture_counts(name, count):
    """AdamContextSuite.scala:32-43 / AdamRDDFunctionsSuite.scala:539-547:
    the reference loads 200, 20 and 200 records from these files."""
    assert SamText.read(os.path.join(GOLD, name)).batch().n_reads == count


def _dup_sam(n_reads, seed, contig_len, n_rg=2):
    """Synthetic SAM with pairs (mates share a QNAME) and fragments stacked on
    few positions, secondary and unmapped reads included."""
    b = synth.generate(n_reads, (60, 80), n_rg, seed, contig_len=contig_len, p_duplicate=0.0, p_secondary=0.05,
                       p_unmapped=0.05)
    text = sam_text(b, n_rg=n_rg, qname="q")
    lines = text.split(b"\n")
    head = [l for l in lines if l.startswith(b"@")]
    body = [l for l in lines if l and not l.startswith(b"@")]
    for k in range(1, len(body), 3):  # two reads of every three share a QNAME
        f = body[k].split(b"\t")
        f[0] = body[k - 1].split(b"\t")[0]
        body[k] = b"\t".join(f)
    return b"\n".join(head + body) + b"\n"


def _host_markdup(text, n_rg):
    """bqsr_mark_duplicates (the host path) over the same records' columns."""
    from adam_amd import sam as S
    s = SamText(text)
    try:
        batch = s.batch()
    finally:
        s.close()
    recs = _records(text)
    n = batch.n_reads
    names = [f[0].decode("latin-1") for f in recs]
    libs = [("lib%d" % (int(batch.rg_id[r]) % 2)) if int(batch.flags[r]) & R.F_HAS_RG else None for r in range(n)]
    mate = [int(f[1]) != 0 and bool(int(f[1]) & 1) and not int(f[1]) & 8 for f in recs]
    return S.mark_duplicates(names, libs, batch.flags, mate, batch.rg_id, batch.ref_index, batch.start,
                             batch.qual_offset, batch.qual, batch.cigar_offset, batch.cigar)


@pytest.mark.parametrize("n_reads,contig_len", [(3000, 2000), (60000, 20000), (200000, 1_000_000)])
def test_mark_duplicates_device_equals_host(n_reads, contig_len):
    """The device MarkDuplicates (sorts + segmented passes) flags exactly the
    reads the host path flags (MarkDuplicates.scala:24-111, ties by first
    appearance in both)."""
    text = _dup_sam(n_reads, 700 + n_reads, contig_len)
    want = _host_markdup(text, 2)
    s = SamText(text)
    try:
        nd = s.mark_duplicates()
        got = (s.batch().flags & R.F_DUPLICATE) != 0
    finally:
        s.close()
    assert nd == int(want.sum()) > 0
    assert np.array_equal(got, want), int(np.nonzero(got != want)[0][0])


@pytest.mark.parametrize("name", FIXTURES)
def test_bam_ingest_reference_fixtures(name):
    """The reference's SAM fixtures converted to BAM (adam_amd/bam_writer.py)
    ingest to the same columns as their SAM text (AdamContext.scala:122-137
    adamBamLoad, SAMRecordConverter semantics)."""
    from adam_amd.bam_writer import sam_to_bam
    path = os.path.join(GOLD, name)
    with open(path, "rb") as fh:
        text = fh.read()
    s = SamText(sam_to_bam(text), bam=True)
    try:
        got = s.batch()
    finally:
        s.close()
    assert_same_columns(got, read_sam(path))


def test_bam_ingest_synthetic_and_mark_duplicates(tmp_path):
    """60k synthetic reads (pairs, fragments, 2 read groups): BAM columns equal
    the SAM text's, and MarkDuplicates flags the same reads from either."""
    from adam_amd.bam_writer import sam_to_bam
    text = _dup_sam(60000, 4242, 30000)
    bam = sam_to_bam(text)
    p = tmp_path / "x.bam"
    p.write_bytes(bam)
    a, b = SamText(text), SamText.read(str(p))
    try:
        assert b.bam
        assert_same_columns(b.batch(), a.batch())
        na, nb = a.mark_duplicates(), b.mark_duplicates()
        assert na == nb > 0
        assert np.array_equal(a.batch().flags, b.batch().flags)
        # the BAM's records are SAM lines on the device: the FLAG rewrite works as for SAM input
        a.rewrite()
        b.rewrite()
        fa = [int(f[1]) for f in _records(a.text())]
        fb = [int(f[1]) for f in _records(b.text())]
        assert fa == fb
    finally:
        a.close()
        b.close()


def _bgzf_corruptions(bam):
    """Damaged copies of a BAM's first BGZF block (an untrusted file): each
    must fail with SAM_PARSE, never read outside the input or allocate from
    a forged size."""
    import struct
    xlen = bam[10] | (bam[11] << 8)
    bsize = bam[16] | (bam[17] << 8)
    out = {"truncated_header": bam[:14], "truncated_block": bam[:bsize // 2]}
    b = bytearray(bam)
    b[10:12] = struct.pack("<H", 60000)  # XLEN past the end of the block / file
    out["xlen_overrun"] = bytes(b[:200])
    b = bytearray(bam)
    b[14:16] = struct.pack("<H", 5000)  # the BC subfield's SLEN overruns the extra field
    out["subfield_overrun"] = bytes(b)
    b = bytearray(bam)
    b[16:18] = struct.pack("<H", 1)  # BSIZE smaller than the header: negative compressed size
    out["bsize_small"] = bytes(b)
    b = bytearray(bam)
    blen = bsize + 1
    b[blen - 4:blen] = struct.pack("<I", 1 << 31)  # forged ISIZE: a multi-GB output buffer
    out["isize_huge"] = bytes(b)
    b = bytearray(bam)
    b[12 + xlen + 2] ^= 0xFF  # compressed bytes damaged
    out["deflate_damaged"] = bytes(b)
    return out


def test_bam_ingest_rejects_damaged_bgzf():
    from adam_amd.bam_writer import sam_to_bam
    with open(os.path.join(GOLD, FIXTURES[0]), "rb") as fh:
        bam = sam_to_bam(fh.read())
    assert bam[12:14] == b"BC"
    for name, data in _bgzf_corruptions(bam).items():
        with pytest.raises(_capi.BQSRError) as e:
            SamText(data, bam=True).close()
        assert e.value.status == _capi.SAM_PARSE, (name, e.value)


@pytest.mark.parametrize("n_parts,recal", [(3, False), (8, False), (5, True)])
def test_transform_mark_duplicates_partitions(tmp_path, n_parts, recal):
    # MarkDuplicates across partitions (bqsr_dup_set): mates in different
    # partitions still form one bucket; the duplicate bits are the whole
    # input's, then BQSR streams the partitions with those bits set
    text = _dup_text(6000, far=True)
    src, out = tmp_path / "in.sam", tmp_path / "out.sam"
    src.write_bytes(text)
    pb = len(text) // n_parts + 1
    st = transform(str(src), str(out), mark_duplicates=True, recalibrate=recal, partition_bytes=pb)
    assert st["partitions"] >= n_parts
    recs = _records(text)
    want = _dup_want(src)
    assert st["duplicates"] == sum(want) > 0
    after = _records(out.read_bytes())
    assert len(after) == len(recs)
    for r, (a, c) in enumerate(zip(recs, after)):
        flag = int(a[1])
        assert int(c[1]) == ((flag | 0x400) if want[r] else (flag & ~0x400)), r
        assert a[2:10] == c[2:10] and a[11:] == c[11:]
    if not recal:
        assert [a[10] for a in recs] == [c[10] for c in after]
        return
    # BQSR over the same partitions, duplicates flagged, through the oracle
    parts = _partition_batches(tmp_path, text, pb)
    base = 0
    for p in parts:
        d = np.asarray(want[base:base + p.n_reads], bool)
        p.flags = np.where(d, p.flags | R.F_DUPLICATE, p.flags & ~np.uint32(R.F_DUPLICATE)).astype(np.uint32)
        base += p.n_reads
    o = run_oracle(parts)
    assert o.error is None, o.error
    quals = []
    for p, (chars, out_len) in zip(parts, o.outs):
        quals += [chars[int(p.qual_offset[r]):int(p.qual_offset[r]) + int(out_len[r])] for r in range(p.n_reads)]
    flags = np.concatenate([p.flags for p in parts])
    for r, (a, c) in enumerate(zip(recs, after)):
        f = int(flags[r])
        if (f & R.F_MAPPED) and (f & R.F_PRIMARY) and not (f & R.F_DUPLICATE):
            assert c[10] == "".join(map(chr, quals[r])).encode("utf-8"), r
        else:
            assert c[10] == a[10]


def test_dup_set_refusals():
    # apply before finish, a parse of another size, an unknown partition
    from adam_amd.sam import DupSet
    text = _dup_text(400)
    s1 = SamText(text)
    d = DupSet()
    try:
        d.add(s1)
        with pytest.raises(_capi.BQSRError):
            d.apply(0, s1)
        assert d.finish() >= 0
        with pytest.raises(_capi.BQSRError):
            d.add(s1)
        with pytest.raises(_capi.BQSRError):
            d.apply(1, s1)
        hdr = b"".join(l + b"\n" for l in text.split(b"\n") if l.startswith(b"@"))
        body = [l for l in text.split(b"\n") if l and not l.startswith(b"@")]
        s2 = SamText(hdr + b"\n".join(body[:10]) + b"\n")
        try:
            with pytest.raises(_capi.BQSRError):
                d.apply(0, s2)
        finally:
            s2.close()
        d.apply(0, s1)
    finally:
        d.close()
        s1.close()


def _job_outcome(job):
    """(error name, results) of one step"""
    try:
        job.step()
    except _capi.BQSRError as e:
        return e.name, None
    return None, job.results()


@pytest.mark.parametrize("name", FIXTURES + ["EDGE", "synthetic", "synthetic-sites"])
def test_device_batch_matches_host_batch(tmp_path, name):
    # bqsr_sam_batch_create (the parse packed on the device) against
    # bqsr_batch_create over the same parse's downloaded columns: the same
    # slots, dims, and one job step's table, expectedMismatch, outputs and
    # errors bit for bit
    from adam_amd.job import ResidentJob
    snp = None
    if name == "EDGE":
        text = EDGE
    elif name.startswith("synthetic"):
        b = synth.generate(30000, (76, 100, 151), 3, 5, contig_len=400_000)
        text = sam_text(b, n_rg=3)
        if name == "synthetic-sites":
            sites = synth.known_sites(4000, contig_len=400_000)
            snp = bqsr.SnpTable({"chr20": sites["chr20"].tolist()})
    else:
        text = open(os.path.join(GOLD, name), "rb").read()
    sam = SamText(text)
    try:
        rb = sam.batch()
        j1 = ResidentJob(rb, bqsr.dims_of([rb]), snp, 0)
        j2 = ResidentJob(None, None, snp, 0, sam=sam)
        try:
            L = _capi.lib()
            assert int(L.bqsr_batch_slots(j1.bh)) == int(L.bqsr_batch_slots(j2.bh))
            assert int(L.bqsr_batch_reads(j2.bh)) == rb.n_reads
            assert int(L.bqsr_batch_bases(j2.bh)) == rb.n_bases
            d1, d2 = L.bqsr_batch_dims(j1.bh), L.bqsr_batch_dims(j2.bh)
            assert (d1.n_rg, d1.max_len) == (d2.n_rg, d2.max_len)
            assert (j2.dims.n_rg, j2.dims.max_len) == (j1.dims.n_rg, j1.dims.max_len)
            for j in (j1, j2):  # slots apply leaves unwritten compare equal
                for t in (j.out_qual, j.out_start, j.out_len, j.exc):
                    t.zero_()
            e1, r1 = _job_outcome(j1)
            e2, r2 = _job_outcome(j2)
            assert e1 == e2
            if r1 is not None:
                from _parity import apply_written
                assert np.array_equal(r1[0], r2[0])
                assert np.float64(r1[1]).tobytes() == np.float64(r2[1]).tobytes()
                for x, y in zip(r1[3:], r2[3:]):
                    assert np.array_equal(x, y)
                # (a bucketed batch's piece order comes from an atomic counting sort: the scratch
                # bytes of a read's last chunk may differ between two batches, its chars may not)
                assert np.array_equal(apply_written(rb, r1[2], r1[3], r1[4]), apply_written(rb, r2[2], r2[3], r2[4]))
        finally:
            j1.close()
            j2.close()
    finally:
        sam.close()


def test_transform_mark_duplicates_large_against_restatement(tmp_path):
    # 60k reads (pairs half the input apart, fragments, two libraries) through
    # the device MarkDuplicates against oracle/markdup.py directly
    text = _dup_text(60000, far=True)
    src, out = tmp_path / "in.sam", tmp_path / "out.sam"
    src.write_bytes(text)
    st = transform(str(src), str(out), mark_duplicates=True)
    want = _dup_want(src)
    assert st["duplicates"] == sum(want) > 1000
    after = _records(out.read_bytes())
    got = [bool(int(c[1]) & 0x400) for c in after]
    assert got == list(want)
