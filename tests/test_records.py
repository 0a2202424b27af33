"""Host-side ingest: SAM -> ADAMRecord columns with SAMRecordConverter
semantics (converters/SAMRecordConverter.scala:26-144,
models/RecordGroupDictionary.scala:36-43), and the RecordBatch round trip the
C ABI consumes."""
import os

import numpy as np
import pytest

from adam_amd import records as R
from adam_amd.records import (ADAMRecord, RecordBatch, characterize_tags, cigar_to_text, parse_cigar, read_sam,
                              read_sam_records)

GOLD = os.path.join(os.path.dirname(__file__), "golden", "reference_resources")


def recs(name):
    return read_sam(os.path.join(GOLD, name)).to_records()


def test_flag_zero_reads_are_unmapped_and_non_primary():
    # Q2: the converter sets flags only when flags != 0 (SAMRecordConverter.scala:74)
    rs = recs("small.sam")
    zero = [r for r in rs if not (r.read_mapped or r.read_negative_strand or r.read_paired)]
    assert zero and all(not r.read_mapped and not r.primary_alignment for r in zero)
    rev = [r for r in rs if r.read_negative_strand]
    assert rev and all(r.read_mapped and r.primary_alignment for r in rev)


def test_start_is_zero_based_and_qual_star_kept():
    r = recs("small.sam")[0]
    assert r.start == 26472784 - 1
    assert r.qual == "*"  # getBaseQualityString is "*" and is stored as is
    assert r.mismatching_positions is None


def test_record_group_index_is_sorted_name_order():
    rs = recs("artificial.realigned.sam")
    assert {r.record_group_id for r in rs} == {0}
    rs = recs("artificial.sam")  # MD but no RG header entry -> null recordGroupId (Q1)
    assert all(r.record_group_id is None for r in rs)
    assert any(r.mismatching_positions is not None for r in rs)


def test_flags_of_realigned_pairs():
    rs = recs("artificial.realigned.sam")
    first = [r for r in rs if r.read_paired and not r.second_of_pair]
    second = [r for r in rs if r.second_of_pair]
    assert len(first) == 5 and len(second) == 5
    assert sum(r.mismatching_positions is not None for r in first) == 3


@pytest.mark.parametrize("text", ["10M", "3H2S5M4S", "1S28M1D32M1I15M1D23M", "3M1P2N7M", "5=2X"])
def test_cigar_round_trip(text):
    assert cigar_to_text(parse_cigar(text)) == text


def test_batch_round_trip_and_offsets():
    b = read_sam(os.path.join(GOLD, "small_realignment_targets.sam"))
    rs = b.to_records()
    b2 = RecordBatch.from_records(rs)
    assert b2.n_reads == b.n_reads
    assert np.array_equal(b2.flags, b.flags)
    assert np.array_equal(b2.qual_offset, b.qual_offset)
    assert b.n_bases == int(sum(len(r.sequence) for r in rs))
    assert [r.flag_bits & R.F_HAS_MD != 0 for r in rs] == [r.mismatching_positions is not None for r in rs]


# The reference's own facts about its fixtures (AdamContextSuite.scala:32-43,
# AdamRDDFunctionsSuite.scala:539-547).
REF_COUNTS = {"unmapped.sam": 200, "small.sam": 20, "reads12.sam": 200}


@pytest.mark.parametrize("name,count", sorted(REF_COUNTS.items()))
def test_reference_fixture_read_counts(name, count):
    path = os.path.join(GOLD, name)
    assert read_sam(path).n_reads == count
    assert len(read_sam_records(path)) == count


def test_reference_reads12_tag_counts():
    # adamCharacterizeTags over reads12.sam: NM, AS and XS on all 200 reads
    counts = characterize_tags(read_sam_records(os.path.join(GOLD, "reads12.sam")))
    assert counts["NM"] == 200 and counts["AS"] == 200 and counts["XS"] == 200
    assert "MD" not in counts  # MD becomes mismatchingPositions, not an attribute


def test_synth_slice_is_the_same_reads_of_the_bigger_set():
    """A rank's shard (first_read = r0) equals reads [r0, r1) of one generation."""
    from adam_amd import synth
    whole = synth.generate(3000, (100, 150), 3, 99)
    part = synth.generate(1200, (100, 150), 3, 99, first_read=1100)
    ref = whole.slice(1100, 2300)
    for c in ("flags", "rg_id", "start", "seq", "qual", "cigar", "md", "seq_offset", "qual_offset", "cigar_offset",
              "md_offset"):
        assert np.array_equal(getattr(part, c), getattr(ref, c)), c


def test_bam_writer_bgzf_structure():
    """The in-tree BAM writer's output is BGZF (gzip members with a BC
    subfield) holding BAM\\1, the header text and one record per SAM line."""
    import gzip
    import struct
    from adam_amd.bam_writer import sam_to_bam
    path = os.path.join(GOLD, "small_realignment_targets.sam")
    text = open(path, "rb").read()
    bam = sam_to_bam(text)
    assert bam[:4] == b"\x1f\x8b\x08\x04" and bam[12:14] == b"BC"
    raw = gzip.decompress(bam)
    assert raw[:4] == b"BAM\x01"
    l_text = struct.unpack("<i", raw[4:8])[0]
    assert raw[8:8 + l_text].startswith(b"@")
    p = 8 + l_text
    n_ref = struct.unpack("<i", raw[p:p + 4])[0]
    p += 4
    for _ in range(n_ref):
        ln = struct.unpack("<i", raw[p:p + 4])[0]
        p += 4 + ln + 4
    n = 0
    while p < len(raw):
        p += 4 + struct.unpack("<i", raw[p:p + 4])[0]
        n += 1
    assert p == len(raw)
    assert n == sum(1 for l in text.split(b"\n") if l and not l.startswith(b"@"))


def test_bam_writer_parallel_same_stream():
    # the pool form (tools/bench_adam.py --bam): the same decompressed BAM
    # stream as the serial writer, block boundaries aside
    import gzip
    from adam_amd import synth
    from adam_amd.bam_writer import sam_to_bam, sam_to_bam_parallel
    from adam_amd.samgen import sam_text
    text = sam_text(synth.generate(3000, (100,), 2, 5), n_rg=2)
    par = sam_to_bam_parallel(text, 3)
    assert gzip.decompress(par) == gzip.decompress(sam_to_bam(text))
    assert par.endswith(bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000"))


def test_sam_partitions_cut_at_records():
    # transform's streamed partitions: the header once, the records cut after
    # a newline, every record in exactly one range, ranges in file order
    from adam_amd.transform import sam_partitions
    text = open(os.path.join(GOLD, "artificial.realigned.sam"), "rb").read()
    body = text[len(sam_partitions(text, 1 << 30)[0]):]
    for pb in (1, 57, 500, 4096, 1 << 30):
        header, ranges = sam_partitions(text, pb)
        assert not header or header.endswith(b"\n")
        assert all(l.startswith(b"@") for l in header.split(b"\n") if l)
        assert b"".join(text[a:b] for a, b in ranges) == body
        assert all(text[b - 1:b] == b"\n" for a, b in ranges[:-1])
        assert all(b - a >= min(pb, len(body)) or i == len(ranges) - 1 for i, (a, b) in enumerate(ranges))
    assert sam_partitions(b"", 10) == (b"", [])
    assert sam_partitions(b"@HD\tVN:1.4\n", 10) == (b"@HD\tVN:1.4\n", [])
    assert sam_partitions(b"r\t0\n", 10) == (b"", [(0, 4)])
