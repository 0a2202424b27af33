"""`transform` with ADAMRecord Parquet in / out (adamLoad / adamSave; SURVEY.md §8
f1/f2) on the device: the recalibrated qual column against the CPU oracle and
against the SAM path's QUAL fields; MarkDuplicates' duplicateRead column
against the SAM path's FLAG 0x400."""
import os

import numpy as np
import pytest

pa = pytest.importorskip("pyarrow")
import pyarrow.parquet as pq  # noqa: E402

from adam_amd import bqsr, synth  # noqa: E402
from adam_amd import parquet as P  # noqa: E402
from adam_amd import records as R  # noqa: E402
from adam_amd.samgen import sam_text  # noqa: E402
from adam_amd.transform import transform  # noqa: E402
from test_gpu_sam import GOLD, _oracle_quals, _records  # noqa: E402

pytestmark = pytest.mark.gpu


def _sam_quals(path):
    return [f[10] for f in _records(open(path, "rb").read())]


@pytest.mark.parametrize("via", ["sam", "adam"])
def test_transform_to_adam_matches_sam_path(tmp_path, via):
    src = os.path.join(GOLD, "artificial.realigned.sam")
    vcf = os.path.join(GOLD, "small.vcf")
    inp = src
    if via == "adam":  # the fixture stored as ADAM first, then transformed ADAM -> ADAM
        recs = R.read_sam_records(src)
        inp = str(tmp_path / "in.adam")
        P.write_parquet(R.RecordBatch.from_records(recs), inp, [r.read_name for r in recs])
    out_sam, out_adam = str(tmp_path / "o.sam"), str(tmp_path / "o.adam")
    transform(src, out_sam, recalibrate=True, dbsnp=vcf)
    st = transform(inp, out_adam, recalibrate=True, dbsnp=vcf)
    t = pq.read_table(out_adam)
    assert st["reads"] == t.num_rows == len(_sam_quals(out_sam))
    got = [None if q is None else q.encode("utf-8") for q in t.column("qual").to_pylist()]
    assert got == _sam_quals(out_sam)
    # every other column is written back as read
    assert t.column("readName").to_pylist() == [f[0].decode() for f in _records(open(src, "rb").read())]


def test_transform_adam_synthetic_against_oracle(tmp_path):
    b = synth.generate(20000, (100, 150), 2, 17, contig_len=500_000)
    inp, out = str(tmp_path / "in.parquet"), str(tmp_path / "out.parquet")
    P.write_parquet(b, inp)
    sites = synth.known_sites(5000, contig_len=500_000)
    vcf = tmp_path / "s.vcf"
    vcf.write_text("".join("chr20\t%d\t.\tA\tC\n" % p for p in sites["chr20"]))
    transform(inp, out, recalibrate=True, dbsnp=str(vcf))
    _, quals = _oracle_quals(b, {"chr20": sites["chr20"].tolist()})
    got = pq.read_table(out).column("qual").to_pylist()
    for r in range(b.n_reads):
        f = int(b.flags[r])
        if (f & R.F_MAPPED) and (f & R.F_PRIMARY) and not (f & R.F_DUPLICATE):
            assert got[r] == "".join(map(chr, quals[r])), r
        else:  # passed through
            q = b.qual[int(b.qual_offset[r]):int(b.qual_offset[r + 1])]
            assert got[r] == bytes(q).decode("latin-1"), r


def test_transform_adam_mark_duplicates_matches_sam_path(tmp_path):
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
    st = transform(str(src), str(out_sam), mark_duplicates=True)
    want = [bool(int(f[1]) & 0x400) for f in _records(out_sam.read_bytes())]
    # the same reads as ADAM records: readName, recordGroupLibrary (the @RG LB), mateMapped (FLAG 0x1, not 0x8)
    recs = R.read_sam_records(str(src))
    batch = R.RecordBatch.from_records(recs)
    flags = [int(f[1]) for f in _records(text)]
    t = P.batch_to_table(batch, [r.read_name for r in recs])
    lib = ["lib%d" % (int(batch.rg_id[r]) % 2) if batch.flags[r] & R.F_HAS_RG else None for r in range(batch.n_reads)]
    t = t.append_column("recordGroupLibrary", pa.array(lib, pa.string()))
    t = t.append_column("mateMapped", pa.array([fl != 0 and bool(fl & 1) and not fl & 8 for fl in flags], pa.bool_()))
    inp, out = str(tmp_path / "in.adam"), str(tmp_path / "o.adam")
    pq.write_table(t, inp)
    st2 = transform(inp, out, mark_duplicates=True)
    got = pq.read_table(out).column("duplicateRead").to_pylist()
    assert st2["duplicates"] == st["duplicates"] == sum(want) > 0
    assert got == want
