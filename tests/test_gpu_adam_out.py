"""ADAM Parquet out of the device path: `transform
IN.{sam,bam} OUT.adam [-mark_duplicate_reads] [-recalibrate_base_qualities]`
(cli/Transform.scala:62-97 ending in adamSave, AdamRDDFunctions.scala:37-56).

* the device's ADAMRecord columns against tests/_adam_ref.py (a per-record
  restatement of SAMRecordConverter.scala:26-144 over htsjdk's SAMRecord) on
  the reference's SAM fixtures and on edge texts covering every field and
  tag rule;
* BAM input: the records become SAM lines on the device; their ADAM
  columns equal the SAM text's; float tags come out as Java's
  Float.toString;
* the recalibrated qual column against the CPU oracle's chars on the
  fixtures (+ small.vcf) and on 200k synthetic reads through BAM;
* MarkDuplicates' duplicateRead through BAM -> ADAM against the SAM path;
* part files: adamSave's directory, rows in input order.
"""
import os
import struct
import sys

import numpy as np
import pytest

pa = pytest.importorskip("pyarrow")
import pyarrow.parquet as pq  # noqa: E402

from _adam_ref import convert_sam, java_float_str  # noqa: E402
from adam_amd import _capi, synth  # noqa: E402
from adam_amd import adam_save as A  # noqa: E402
from adam_amd import records as R  # noqa: E402
from adam_amd.bam_writer import sam_to_bam  # noqa: E402
from adam_amd.sam import SamText  # noqa: E402
from adam_amd.samgen import sam_text  # noqa: E402
from adam_amd.transform import transform  # noqa: E402
from test_gpu_sam import FIXTURES, GOLD, _oracle_quals, _records  # noqa: E402

pytestmark = pytest.mark.gpu


def _table(data: bytes, bam: bool = False):
    s = SamText(data, bam=bam)
    try:
        t = A.adam_table(s, 0, s.counts().n_reads, A.header_info(s))
        # header-derived columns are dictionary arrays over the header's values
        for f in t.schema:
            want = A.schema().field(f.name).type
            assert f.type == want or (pa.types.is_dictionary(f.type) and f.type.value_type == want), f
        return t.cast(A.schema())
    finally:
        s.close()


def _assert_rows(t, want):
    got = t.to_pylist()
    assert len(got) == len(want)
    for r, (g, w) in enumerate(zip(got, want)):
        for k, v in w.items():
            assert g[k] == v, (r, k, g[k], v)


@pytest.mark.parametrize("name", FIXTURES)
def test_adam_columns_reference_fixtures(name):
    text = open(os.path.join(GOLD, name), "rb").read()
    t = _table(text)
    assert t.schema == A.schema()
    _assert_rows(t, convert_sam(text, A._iso8601_epoch_ms))
    # the same records as BAM (records -> SAM lines on the device): the same table
    assert _table(sam_to_bam(text), bam=True).equals(t)


EDGE = (b"@HD\tVN:1.4\n"
        b"@SQ\tSN:chrA\tLN:1000\tUR:file:/a.fa\n@SQ\tSN:chrB\tLN:2000\n"
        b"@RG\tID:zeta\tLB:l1\tSM:s1\tPL:ILLUMINA\tPU:u1\tCN:ctr\tDS:desc\tPI:250\tFO:TACG\tKS:GATC\t"
        b"DT:2013-06-01T12:30:00Z\n"
        b"@RG\tID:alpha\tDT:2012-01-02\tPI:x\n@RG\tID:mid\tLB:l2\n"
        b"q1\t99\tchrA\t10\t60\t5M\t=\t200\t195\tACGTN\tIIIII\tMD:Z:5\tRG:Z:mid\tNM:i:+0\tAS:i:-12\tXA:A:c\n"
        b"q2\t147\tchrB\t0\t255\t2S3M\tchrA\t7\t0\tACGGT\t#II!~\tXS:f:1.50\tXF:f:-0.000015\tMD:Z:1A1\tMD:i:3\n"
        b"q3\t4\t*\t0\t0\t*\t*\t0\t0\t*\t*\n"
        b"q4\t1107\tchrZ\t77\t60\t01M1I1D1N1S1H1P1=1X\t*\t0\t0\tAAAAAAA\tBBBBBBB\tRG:Z:nope\tRG:Z:alpha\tZZ:Z:x:y\n"
        b"q5\t0\tchrA\t5\t3\t4M\tchrB\t0\t0\tGGGG\t????\tYF:f:12345678\tYG:f:1e-3\tYH:f:1.0E7\tRG:Z:zeta\n"
        b"q6\t513\tchrB\t1\t60\t3M\t*\t9\t0\tTTT\t@@@\tMD:Z:\tNM:i:2147483647\n")


def test_adam_columns_edge_fields():
    t = _table(EDGE)
    want = convert_sam(EDGE, A._iso8601_epoch_ms)
    _assert_rows(t, want)
    rows = t.to_pylist()
    # spot checks of the rules the restatement encodes
    assert rows[0]["attributes"] == "AS:i:-12\tNM:i:0\tRG:Z:mid\tXA:A:c"  # descending binary tag, MD apart
    assert rows[1]["attributes"] == "XS:f:1.5\tXF:f:-1.5E-5"
    assert rows[1]["mismatchingPositions"] == "3"  # the last MD wins
    assert rows[1]["mapq"] is None and rows[1]["mateReference"] == "chrA" and rows[1]["mateAlignmentStart"] == 6
    assert rows[2]["attributes"] == "" and rows[2]["referenceId"] is None and not rows[2]["readMapped"]
    assert rows[3]["cigar"] == "1M1I1D1N1S1H1P1=1X" and rows[3]["recordGroupName"] == "alpha"
    assert rows[3]["recordGroupPredictedMedianInsertSize"] is None  # PI:x does not parse
    assert rows[4]["attributes"] == "YH:f:1.0E7\tYG:f:0.001\tRG:Z:zeta\tYF:f:1.2345678E7"
    assert rows[3]["attributes"] == "ZZ:Z:x:y\tRG:Z:alpha"
    assert not any(rows[4][k] for k in A.BOOL_COLS)  # FLAG 0: every flag false (Q2)
    assert rows[4]["recordGroupRunDateEpoch"] == 1370089800000 and rows[4]["recordGroupPlatformUnit"] == "u1"
    assert rows[0]["referenceUrl"] == "file:/a.fa" and rows[0]["referenceLength"] == 1000
    assert rows[5]["failedVendorQualityChecks"] and rows[5]["mismatchingPositions"] == ""


@pytest.mark.parametrize("tag", [b"XB:B:c,1,2", b"XH:H:1AE3", b"XI:i:2147483648"])
def test_adam_columns_refuse_what_the_reference_cannot_convert(tag):
    text = b"@SQ\tSN:chrA\tLN:10\nq\t0\tchrA\t1\t60\t3M\t*\t0\t0\tAAA\tIII\t" + tag + b"\n"
    s = SamText(text)
    try:
        with pytest.raises(_capi.BQSRError) as e:
            A.adam_table(s, 0, 1, A.header_info(s))
        assert e.value.name == "UNSUPPORTED"
    finally:
        s.close()


def _bam_with_floats(vals):
    """A one-record-per-value BAM whose records carry an 'f' tag each (and a
    B:f array on the first), written directly in the BAM layout."""
    import zlib
    hdr = b"@SQ\tSN:c\tLN:100\n"
    body = b"BAM\1" + struct.pack("<i", len(hdr)) + hdr + struct.pack("<i", 1) + struct.pack("<i", 2) + b"c\0" + \
        struct.pack("<i", 100)
    for i, v in enumerate(vals):
        name = b"r%d\0" % i
        tags = b"XFf" + struct.pack("<f", v)
        if i == 0:
            tags += b"XBBf" + struct.pack("<i", 2) + struct.pack("<ff", 0.5, -3.25)
        rec = struct.pack("<iiBBHHHiiii", 0, 0, len(name), 60, 4680, 1, 0, 1, -1, -1, 0) + name + \
            struct.pack("<I", (1 << 4) | 0) + bytes([0x10]) + bytes([30]) + tags
        body += struct.pack("<i", len(rec)) + rec
    out = b""
    for k in range(0, len(body), 60000):
        chunk = body[k:k + 60000]
        c = zlib.compressobj(6, zlib.DEFLATED, -15)
        cdata = c.compress(chunk) + c.flush()
        out += (b"\x1f\x8b\x08\x04\0\0\0\0\0\xff\x06\0BC\x02\0" + struct.pack("<H", len(cdata) + 25) + cdata +
                struct.pack("<II", zlib.crc32(chunk) & 0xFFFFFFFF, len(chunk)))
    return out + b"\x1f\x8b\x08\x04\0\0\0\0\0\xff\x06\0BC\x02\0\x1b\0\x03\0\0\0\0\0\0\0\0\0"


def test_bam_float_tags_as_java_text():
    vals = [1.5, 1e-5, 100.0, 0.001, 1e7, 123456.7, 3.4028235e38, 0.1, 9999999.0, -2.5, 0.0,
            float("inf"), 1.0 / 3.0, 2.0 ** -20]
    s = SamText(_bam_with_floats(vals), bam=True)
    try:
        lines = [l.split(b"\t") for l in s.text().split(b"\n") if l and not l.startswith(b"@")]
    finally:
        s.close()
    assert len(lines) == len(vals)
    for v, f in zip(vals, lines):
        tag = [x for x in f[11:] if x.startswith(b"XF:f:")][0]
        assert tag[5:].decode() == java_float_str(v), (v, tag)
    arr = [x for x in lines[0][11:] if x.startswith(b"XB:")][0]
    assert arr == b"XB:B:f,0.5,-3.25"


def _pass_through(b, r):
    f = int(b.flags[r])
    return not ((f & R.F_MAPPED) and (f & R.F_PRIMARY) and not (f & R.F_DUPLICATE))


def _check_quals(table_or_path, batch, quals):
    t = pq.read_table(table_or_path) if isinstance(table_or_path, str) else table_or_path
    got = t.column("qual").to_pylist()
    assert len(got) == batch.n_reads
    for r in range(batch.n_reads):
        if _pass_through(batch, r):
            q = batch.qual[int(batch.qual_offset[r]):int(batch.qual_offset[r + 1])]
            assert got[r] == (bytes(q).decode("latin-1") if batch.flags[r] & R.F_HAS_QUAL else "*"), r
        else:
            assert got[r] == "".join(map(chr, quals[r])), r


@pytest.mark.parametrize("fmt", ["sam", "bam"])
def test_transform_to_adam_fixture_quals_against_oracle(tmp_path, fmt):
    src = os.path.join(GOLD, "artificial.realigned.sam")
    vcf = os.path.join(GOLD, "small.vcf")
    text = open(src, "rb").read()
    inp = tmp_path / ("in." + fmt)
    inp.write_bytes(text if fmt == "sam" else sam_to_bam(text))
    out = str(tmp_path / "o.adam")
    st = transform(str(inp), out, recalibrate=True, dbsnp=vcf)
    assert os.path.isdir(out) and os.path.exists(os.path.join(out, "_SUCCESS"))
    batch = R.read_sam(src)
    sites = {}
    for line in open(vcf):
        if not line.startswith("#"):
            f = line.split("\t")
            sites.setdefault(f[0], []).append(int(f[1]))
    _, quals = _oracle_quals(batch, sites)
    _check_quals(out, batch, quals)
    assert st["reads"] == batch.n_reads
    # every other column as the converter writes it for the input records
    t = pq.read_table(out)
    want = convert_sam(text, A._iso8601_epoch_ms)
    for k in ("readName", "sequence", "cigar", "start", "attributes", "recordGroupName", "readNegativeStrand"):
        assert t.column(k).to_pylist() == [w[k] for w in want], k


def test_transform_bam_to_adam_200k_against_oracle(tmp_path):
    b = synth.generate(200_000, (100, 150), 3, 2024, contig_len=5_000_000)
    text = sam_text(b, n_rg=3)
    inp = tmp_path / "in.bam"
    inp.write_bytes(sam_to_bam(text))
    sites = synth.known_sites(100_000, contig_len=5_000_000, seed=9)
    vcf = tmp_path / "s.vcf"
    vcf.write_text("".join("chr20\t%d\t.\tA\tC\n" % p for p in sites["chr20"]))
    out = str(tmp_path / "o.adam")
    st = transform(str(inp), out, recalibrate=True, dbsnp=str(vcf), part_reads=60_000, compression="snappy")
    assert st["parts"] == 4
    assert sorted(f for f in os.listdir(out) if f.endswith(".parquet")) == ["part-r-%05d.parquet" % i for i in range(4)]
    s = SamText(text)
    batch = s.batch()
    s.close()
    _, quals = _oracle_quals(batch, {"chr20": sites["chr20"].tolist()})
    _check_quals(out, batch, quals)
    # SAM input gives the same files' rows
    inp2 = tmp_path / "in.sam"
    inp2.write_bytes(text)
    out2 = str(tmp_path / "o2.adam")
    transform(str(inp2), out2, recalibrate=True, dbsnp=str(vcf), part_reads=60_000)
    assert pq.read_table(out2).equals(pq.read_table(out))


def test_transform_bam_to_adam_mark_duplicates(tmp_path):
    b = synth.generate(4000, (60,), 2, 11, contig_len=3000, p_duplicate=0.0)
    text = sam_text(b, n_rg=2, qname="p")
    lines = text.split(b"\n")
    body = [l for l in lines if l and not l.startswith(b"@")]
    for k in range(1, len(body), 2):  # mates share a QNAME
        f = body[k].split(b"\t")
        f[0] = body[k - 1].split(b"\t")[0]
        body[k] = b"\t".join(f)
    text = b"\n".join([l for l in lines if l.startswith(b"@")] + body) + b"\n"
    src, out_sam = tmp_path / "in.sam", tmp_path / "o.sam"
    src.write_bytes(text)
    st = transform(str(src), str(out_sam), mark_duplicates=True, recalibrate=True)
    want_dup = [bool(int(f[1]) & 0x400) for f in _records(out_sam.read_bytes())]
    want_q = [f[10].decode("latin-1") for f in _records(out_sam.read_bytes())]
    bam = tmp_path / "in.bam"
    bam.write_bytes(sam_to_bam(text))
    out = str(tmp_path / "o.adam")
    st2 = transform(str(bam), out, mark_duplicates=True, recalibrate=True)
    t = pq.read_table(out)
    assert st2["duplicates"] == st["duplicates"] == sum(want_dup) > 0
    assert t.column("duplicateRead").to_pylist() == want_dup
    assert t.column("qual").to_pylist() == want_q


def test_bam_rewrite_to_sam(tmp_path):
    """BAM input, SAM output: the records' lines with the recalibrated QUAL
    (the rewrite a BAM parse could not do before its records became text)."""
    src = os.path.join(GOLD, "artificial.realigned.sam")
    vcf = os.path.join(GOLD, "small.vcf")
    a, b2 = tmp_path / "a.sam", tmp_path / "b.sam"
    bam = tmp_path / "in.bam"
    bam.write_bytes(sam_to_bam(open(src, "rb").read()))
    transform(src, str(a), recalibrate=True, dbsnp=vcf)
    transform(str(bam), str(b2), recalibrate=True, dbsnp=vcf)
    assert [f[10] for f in _records(a.read_bytes())] == [f[10] for f in _records(b2.read_bytes())]
