"""ADAMRecord Parquet on the device (bqsr_arrow_*, parquet.ArrowReads; SURVEY.md
§8 f1/f2): the batch packed from Arrow's buffers on the device against the
host conversion (parquet.table_to_batch + bqsr_batch_create) -- one job step
bit for bit -- and the qual column rebuilt on the device against the host
path's (recalibrated_qual_column)."""
import numpy as np
import pytest

pa = pytest.importorskip("pyarrow")
import pyarrow.parquet as pq  # noqa: E402

from adam_amd import _capi, bqsr, synth  # noqa: E402
from adam_amd import parquet as P  # noqa: E402
from adam_amd import records as R  # noqa: E402
from adam_amd.job import ResidentJob  # noqa: E402

pytestmark = pytest.mark.gpu


def _edge_table():
    """nulls in every nullable column, chars of every UTF-8 length in
    sequence / qual / MD (a surrogate pair among them), empty strings, "*"
    CIGAR, null booleans, two referenceNames and one unknown"""
    q = lambda n, c="I": c * n  # noqa: E731
    rows = [
        dict(referenceName="chr20", start=100, sequence="ACGTACGTAC", qual=q(10), cigar="10M", recordGroupId=0,
             mismatchingPositions="10", readMapped=True, primaryAlignment=True),
        dict(referenceName="chr20", start=200, sequence="ACGTNCGTAC", qual="IIéIIIIĀII", cigar="2S8M",
             recordGroupId=1, mismatchingPositions="3A6", readMapped=True, primaryAlignment=True,
             readNegativeStrand=True),
        dict(referenceName="chrX", start=5, sequence="ACéGT", qual="I\U0001F600II", cigar="5M", recordGroupId=0,
             mismatchingPositions="5", readMapped=True, primaryAlignment=True),
        dict(referenceName=None, start=None, sequence=None, qual=None, cigar=None, recordGroupId=None,
             mismatchingPositions=None, readMapped=None, primaryAlignment=None),
        dict(referenceName="chr1", start=0, sequence="", qual="", cigar="*", recordGroupId=2,
             mismatchingPositions="", readMapped=False, primaryAlignment=True),
        dict(referenceName="chr20", start=300, sequence="ACGTACGTACGT", qual="(((((((((((☃", cigar="4M1I7M",
             recordGroupId=1, mismatchingPositions="11☃", readMapped=True, primaryAlignment=True,
             duplicateRead=None, readPaired=True, secondOfPair=True),
    ]
    cols = {}
    types = dict(referenceName=pa.string(), start=pa.int64(), sequence=pa.string(), qual=pa.string(),
                 cigar=pa.string(), recordGroupId=pa.int32(), mismatchingPositions=pa.string(),
                 readPaired=pa.bool_(), readMapped=pa.bool_(), readNegativeStrand=pa.bool_(),
                 secondOfPair=pa.bool_(), primaryAlignment=pa.bool_(), duplicateRead=pa.bool_())
    for k, t in types.items():
        cols[k] = pa.array([r.get(k) for r in rows], t)
    return pa.table(cols)


def _synthetic_table(tmp_path, n=40000, row_group=7000):
    b = synth.generate(n, (76, 100, 151), 3, 23, contig_len=400_000)
    path = str(tmp_path / "s.parquet")
    pq.write_table(P.batch_to_table(b), path, row_group_size=row_group)
    return P.read_table(path, P.BQSR_PROJECTION)


def _outcome(job):
    try:
        job.step()
    except _capi.BQSRError as e:
        return e.name, None
    return None, job.results()


def _same_jobs(table, snp=None):
    batch = P.table_to_batch(table)
    A = P.ArrowReads(table)
    try:
        j1 = ResidentJob(batch, bqsr.dims_of([batch]), snp, 0)
        j2 = ResidentJob(None, None, snp, 0, handle=A.device_batch(snp.contigs if snp else None))
        try:
            L = _capi.lib()
            assert int(L.bqsr_batch_slots(j1.bh)) == int(L.bqsr_batch_slots(j2.bh))
            assert int(L.bqsr_batch_reads(j2.bh)) == batch.n_reads
            assert int(L.bqsr_batch_bases(j2.bh)) == batch.n_bases
            assert (j1.dims.n_rg, j1.dims.max_len) == (j2.dims.n_rg, j2.dims.max_len)
            for j in (j1, j2):  # slots apply leaves unwritten compare equal
                for t in (j.out_qual, j.out_start, j.out_len, j.exc):
                    t.zero_()
            e1, r1 = _outcome(j1)
            e2, r2 = _outcome(j2)
            assert e1 == e2
            if r1 is not None:
                from _parity import apply_written
                assert np.array_equal(r1[0], r2[0])
                assert np.float64(r1[1]).tobytes() == np.float64(r2[1]).tobytes()
                for x, y in zip(r1[3:], r2[3:]):
                    assert np.array_equal(x, y)
                # (the chars a read owns; the scratch bytes of its last chunk follow the piece order)
                assert np.array_equal(apply_written(batch, r1[2], r1[3], r1[4]),
                                      apply_written(batch, r2[2], r2[3], r2[4]))
            return e1, batch, A, j2
        except Exception:
            j2.close()
            raise
        finally:
            j1.close()
    except Exception:
        A.close()
        raise


def test_arrow_edge_batch_matches_host():
    e, batch, A, job = _same_jobs(_edge_table())
    try:
        pass
    finally:
        job.close()
        A.close()


@pytest.mark.parametrize("sites", [False, True])
def test_arrow_synthetic_batch_and_qual_column(tmp_path, sites):
    table = _synthetic_table(tmp_path)
    assert table.column("qual").num_chunks > 1  # several Arrow chunks
    snp = None
    if sites:
        s = synth.known_sites(4000, contig_len=400_000)
        snp = bqsr.SnpTable({"chr20": s["chr20"].tolist()})
    err, batch, A, job = _same_jobs(table, snp)
    try:
        assert err is None
        got = A.qual_column(job).to_pylist()
        parts = bqsr.adam_bqsr([batch], snp, bqsr.Context.get(0))
        want = P.recalibrated_qual_column(parts, batch.n_reads).to_pylist()
        assert got == want
    finally:
        job.close()
        A.close()


def test_arrow_qual_column_pass_through_keeps_input():
    # a read BQSR passes through keeps its input string (the device path), and
    # recalibrated reads' chars are UTF-8; no job: every input string kept
    t = _edge_table()
    A = P.ArrowReads(t)
    try:
        assert A.qual_column().to_pylist() == t.column("qual").to_pylist()
    finally:
        A.close()


@pytest.mark.parametrize("cigar", ["10Q", "M", "5M5", "1" * 12 + "M"])
def test_arrow_malformed_cigar(cigar):
    t = _edge_table()
    c = t.column("cigar").to_pylist()
    c[0] = cigar
    t = t.set_column(t.column_names.index("cigar"), "cigar", pa.array(c, pa.string()))
    with pytest.raises(_capi.BQSRError) as e:
        P.ArrowReads(t)
    assert e.value.name == "SAM_PARSE"
    if cigar != "1" * 12 + "M":  # (over 2^28: the host restatement raises too)
        with pytest.raises(R.CigarParseError):
            P.table_to_batch(t)


def test_arrow_empty_table():
    t = _edge_table().slice(0, 0)
    A = P.ArrowReads(t)
    try:
        assert A.n_reads == 0
        assert A.qual_column().to_pylist() == []
    finally:
        A.close()


def _dup_table(n=6000, seed=11):
    """pairs and fragments stacked on few positions (mates share a readName),
    libraries per read (some null), a few null readNames, referenceId set"""
    b = synth.generate(n, (60,), 3, seed, contig_len=3000, p_duplicate=0.0)
    t = P.batch_to_table(b)
    rng = np.random.default_rng(seed)
    names = ["r%d" % (r // 2 if r % 4 < 2 else r) for r in range(n)]  # half the reads in pairs
    for r in rng.choice(n, 20, replace=False):
        names[r] = None
    libs = ["lib%d" % (int(b.rg_id[r]) % 2) if r % 13 else None for r in range(n)]
    t = t.set_column(t.column_names.index("readName"), "readName", pa.array(names, pa.string()))
    t = t.append_column("recordGroupLibrary", pa.array(libs, pa.string()))
    t = t.append_column("referenceId", pa.array([0 if b.flags[r] & R.F_HAS_REFNAME else None for r in range(n)],
                                                pa.int32()))
    t = t.append_column("mateMapped", pa.array([bool(r % 3) for r in range(n)], pa.bool_()))
    return t


def test_arrow_mark_duplicates_matches_host_form():
    # the device MarkDuplicates over Arrow columns against bqsr_mark_duplicates
    # (the host form, itself checked against oracle/markdup.py)
    from adam_amd import sam as S
    t = _dup_table()
    batch = P.table_to_batch(t.select([c for c in P.BQSR_PROJECTION if c in t.column_names]))
    col = lambda name: t.column(name).to_pylist()  # noqa: E731
    want = S.mark_duplicates(col("readName"), col("recordGroupLibrary"), batch.flags,
                             np.asarray(col("mateMapped"), np.uint8), batch.rg_id,
                             np.asarray([-1 if v is None else v for v in col("referenceId")], np.int32), batch.start,
                             batch.qual_offset, batch.qual, batch.cigar_offset, batch.cigar)
    assert want.sum() > 0
    A = P.ArrowReads(t, markdup=True)
    try:
        nd = A.mark_duplicates()
        got = np.asarray(A.flag_column(R.F_DUPLICATE).to_pylist(), bool)
        assert nd == int(want.sum())
        assert np.array_equal(got, want)
        # the batch built after carries the bits
        bh = A.device_batch()
        _capi.lib().bqsr_batch_destroy(bh)
    finally:
        A.close()


def test_transform_adam_markdup_recal_device(tmp_path):
    # Parquet in -> MarkDuplicates + BQSR on the device -> Parquet out, against
    # the host form's duplicate bits and the oracle-backed host BQSR path
    from adam_amd import sam as S
    from adam_amd.transform import transform
    t = _dup_table(8000, 5)
    inp, out = str(tmp_path / "in.parquet"), str(tmp_path / "out.parquet")
    pq.write_table(t, inp)
    st = transform(inp, out, mark_duplicates=True, recalibrate=True)
    o = pq.read_table(out)
    batch = P.table_to_batch(t.select([c for c in P.BQSR_PROJECTION if c in t.column_names]))
    col = lambda name: t.column(name).to_pylist()  # noqa: E731
    want = S.mark_duplicates(col("readName"), col("recordGroupLibrary"), batch.flags,
                             np.asarray(col("mateMapped"), np.uint8), batch.rg_id,
                             np.asarray([-1 if v is None else v for v in col("referenceId")], np.int32), batch.start,
                             batch.qual_offset, batch.qual, batch.cigar_offset, batch.cigar)
    assert st["duplicates"] == int(want.sum())
    assert o.column("duplicateRead").to_pylist() == list(want)
    batch.flags = np.where(want, batch.flags | R.F_DUPLICATE, batch.flags & ~np.uint32(R.F_DUPLICATE)).astype(np.uint32)
    parts = bqsr.adam_bqsr([batch], None, bqsr.Context.get(0))
    assert o.column("qual").to_pylist() == P.recalibrated_qual_column(parts, batch.n_reads).to_pylist()
    assert o.column("readName").to_pylist() == col("readName")
