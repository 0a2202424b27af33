"""ADAMRecord Parquet (adam.avdl:4-68; adamLoad / adamSave, AdamContext.scala:139-161,318-331,
AdamRDDFunctions.scala:37-56): the reader against the SAM fixtures' columns through the
in-tree writer, the vectorized CIGAR parse against records.parse_cigar (TextCigarCodec
rules), nulls and non-ASCII strings.  Parity unpinned against files ADAM itself wrote
(the reference cannot run here)."""
import os

import numpy as np
import pytest

pa = pytest.importorskip("pyarrow")

from adam_amd import parquet as P
from adam_amd import records as R
from adam_amd import synth

GOLD = os.path.join(os.path.dirname(__file__), "golden", "reference_resources")
FIXTURES = ["artificial.realigned.sam", "artificial.sam", "reads12.sam", "small.sam",
            "small_realignment_targets.sam", "unmapped.sam"]
COLS = ["flags", "rg_id", "ref_index", "start", "seq_offset", "seq", "qual_offset", "qual", "cigar_offset", "cigar",
        "md_offset", "md"]


def same(a: R.RecordBatch, b: R.RecordBatch):
    assert a.n_reads == b.n_reads and a.ref_names == b.ref_names
    for c in COLS:
        assert np.array_equal(getattr(a, c), getattr(b, c)), c


@pytest.mark.parametrize("name", FIXTURES)
def test_fixture_round_trip(tmp_path, name):
    recs = R.read_sam_records(os.path.join(GOLD, name))
    b = R.RecordBatch.from_records(recs)
    path = str(tmp_path / "x.parquet")
    P.write_parquet(b, path, [r.read_name for r in recs])
    same(b, P.read_parquet(path))
    t = P.read_table(path)
    assert t.num_rows == len(recs) and t.column("readName").to_pylist() == [r.read_name for r in recs]
    # the reference's own fixture counts (AdamContextSuite.scala:32-43)
    if name == "unmapped.sam":
        assert t.num_rows == 200
    if name == "small.sam":
        assert t.num_rows == 20


def test_projection_reads_only_bqsr_columns(tmp_path):
    b = synth.generate(500, (50,), 2, 3)
    path = str(tmp_path / "x.parquet")
    P.write_parquet(b, path)
    t = P.read_table(path, P.BQSR_PROJECTION)
    assert set(t.column_names) == set(P.BQSR_PROJECTION)


def test_cigar_parse_matches_textcigarcodec():
    rng = np.random.default_rng(5)
    cig = []
    for _ in range(3000):
        k = int(rng.integers(0, 6))
        cig.append("".join("%d%s" % (int(rng.integers(0, 300)), "MIDNSHP=X"[int(rng.integers(0, 9))])
                           for _ in range(k)) or "*")
    cig += ["*", "", "0M", "123456789M", "1M1I1D1N1S1H1P1=1X"]
    present = np.ones(len(cig), bool)
    present[5] = False
    data = "".join(c if p else "" for c, p in zip(cig, present)).encode()
    lens = np.asarray([len(c) if p else 0 for c, p in zip(cig, present)], np.uint64)
    off = np.zeros(len(cig) + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    coff, el = P.parse_cigars(present, off, np.frombuffer(data, np.uint8))
    for r, (c, p) in enumerate(zip(cig, present)):
        want = R.parse_cigar(c) if p else np.zeros(0, np.uint32)
        assert np.array_equal(el[int(coff[r]):int(coff[r + 1])], want), c


@pytest.mark.parametrize("bad", ["5", "M", "5Q", "1234567890M", "5M3", "3M M"])
def test_cigar_parse_rejects_malformed(bad):
    with pytest.raises(R.CigarParseError):
        R.parse_cigar(bad)
    d = np.frombuffer(bad.encode(), np.uint8)
    with pytest.raises(R.CigarParseError):
        P.parse_cigars(np.ones(1, bool), np.asarray([0, len(bad)], np.uint64), d)


def test_nulls_and_non_ascii(tmp_path):
    recs = [R.ADAMRecord(), R.ADAMRecord(sequence="ACGN", qual="\u00a0!#\u0141", cigar="4M", start=7,
                                         reference_name="c1", record_group_id=0, mismatching_positions="4",
                                         read_mapped=True, primary_alignment=True),
            R.ADAMRecord(sequence="A\u0141GT", qual=None, cigar=None, start=None, reference_name=None,
                         read_paired=True, second_of_pair=True, duplicate_read=True)]
    t = pa.table({"sequence": [r.sequence for r in recs], "qual": [r.qual for r in recs],
                  "cigar": [r.cigar for r in recs], "start": pa.array([r.start for r in recs], pa.int64()),
                  "referenceName": [r.reference_name for r in recs],
                  "recordGroupId": pa.array([r.record_group_id for r in recs], pa.int32()),
                  "mismatchingPositions": [r.mismatching_positions for r in recs],
                  "readMapped": [r.read_mapped for r in recs], "primaryAlignment": [r.primary_alignment for r in recs],
                  "readPaired": [r.read_paired for r in recs], "secondOfPair": [r.second_of_pair for r in recs],
                  "duplicateRead": pa.array([None, False, True], pa.bool_())})
    b = P.table_to_batch(t)
    assert list(b.flags & R.F_HAS_QUAL) == [0, R.F_HAS_QUAL, 0]
    assert list(b.flags & R.F_HAS_START) == [0, R.F_HAS_START, 0]
    assert list(b.flags & R.F_DUPLICATE) == [0, 0, R.F_DUPLICATE]
    # qual chars as c & 0xFF ((c - 33).toByte sees 8 bits), other chars above 0xFF as 0xFF
    assert bytes(b.qual[int(b.qual_offset[1]):int(b.qual_offset[2])]) == bytes([0xA0, 0x21, 0x23, 0x41])
    assert bytes(b.seq[int(b.seq_offset[2]):int(b.seq_offset[3])]) == b"A\xffGT"
    assert b.ref_names == ["c1"] and list(b.ref_index) == [-1, 0, -1]


def test_synthetic_round_trip_high_quals(tmp_path):
    b = synth.generate(3000, (100, 150), 3, 9)
    q = b.qual.copy()
    q[::7] = 0xA0  # Latin-1 chars: two UTF-8 bytes in Parquet
    b = R.RecordBatch(b.flags, b.rg_id, b.ref_index, b.ref_names, b.start, b.seq_offset, b.seq, b.qual_offset, q,
                      b.cigar_offset, b.cigar, b.md_offset, b.md)
    path = str(tmp_path / "x.parquet")
    P.write_parquet(b, path)
    same(b, P.read_parquet(path))


def test_chars_beyond_the_bmp_are_surrogate_pairs():
    # a Java String holds U+1F600 as two chars (0xD83D 0xDE00): two quals
    # (their low bytes), two sequence bytes 0xFF
    t = pa.table({"sequence": ["A\U0001F600C"], "qual": ["I\U0001F600I"], "cigar": ["4M"],
                  "start": pa.array([3], pa.int64()), "readMapped": [True], "primaryAlignment": [True]})
    b = P.table_to_batch(t)
    assert bytes(b.qual[:4]) == bytes([0x49, 0x3D, 0x00, 0x49])
    assert bytes(b.seq[:4]) == b"A\xff\xffC"
