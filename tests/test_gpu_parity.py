"""HIP path vs the CPU oracle, bit for bit: covariate tables (int64),
per-partition expectedMismatch (double, exact), recalibrated qualities
(Java chars) and the exception class of failing inputs."""
import os

import numpy as np
import pytest

from _parity import check, run_gpu, run_oracle, assert_same
from adam_amd import bqsr, synth
from adam_amd.records import ADAMRecord, RecordBatch, read_sam

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden", "reference_resources")


def rec(**kw):
    base = dict(record_group_id=0, read_mapped=True, primary_alignment=True, start=10000, reference_name="1",
                cigar="10M", mismatching_positions="10", sequence="ACGTACGTAC", qual="IIIIIIIIII")
    base.update(kw)
    return ADAMRecord(**base)


# ---- reference fixtures ------------------------------------------------------

def test_g1_read_covariates_suite_read():
    # ReadCovariatesSuite.scala:27-35
    r = rec(mismatching_positions="5C4", sequence="CTACCCTAAC", qual="##LKLPPQ##")
    g, o = check([RecordBatch.from_records([r])])
    touched = g.words[:128]
    assert {k: int(touched[k]) for k in np.nonzero(touched)[0]} == {42: 1, 43: 2, 47: 2, 48: 1}


def test_g2_artificial_realigned_sam():
    b = read_sam(os.path.join(GOLD, "artificial.realigned.sam"))
    g, o = check([b])
    assert g.words[40] == 480


def test_small_realignment_targets_sam():
    check([read_sam(os.path.join(GOLD, "small_realignment_targets.sam"))])


def test_small_sam_is_empty_table():
    # no MD tags -> no usable read -> finalizeTable's reduce throws
    check([read_sam(os.path.join(GOLD, "small.sam"))], expect_error="EMPTY_TABLE")


def test_artificial_sam_null_rg():
    check([read_sam(os.path.join(GOLD, "artificial.sam"))], expect_error="NULL_RG")


@pytest.mark.parametrize("name", ["reads12.sam", "unmapped.sam"])
def test_other_sams(name):
    # no MD: nothing usable -> EMPTY_TABLE, same as the reference
    check([read_sam(os.path.join(GOLD, name))])


# ---- synthetic ----------------------------------------------------------------

def test_synthetic_one_partition():
    check([synth.generate(3000, (100,), 1, seed=11)])


def test_synthetic_partitions_and_sites():
    b = synth.generate(9000, (101,), 1, seed=12)
    sites = synth.known_sites(2_000_000, seed=3)
    parts = [b.slice(0, 3000), b.slice(3000, 3001), b.slice(3001, 9000)]
    check(parts, sites)


def test_synthetic_many_read_groups_mixed_lengths():
    # 96 read groups, 150/250 bp: most keys fall outside the LDS window
    b = synth.generate(6000, (150, 250), 96, seed=13)
    check([b])


@pytest.fixture
def read_order(request):
    """BQSR_TUNE_ORDER (bqsr_context_tune): 'read' = the per-base passes walk
    reads in batch order, 'group' = bucketed by read group (device counting
    sort, pieces per read group); the library picks 'group' for several read
    groups by default."""
    from adam_amd import bqsr as _b
    with _b.Context.get(0).tuned(order=request.param):
        yield request.param


@pytest.mark.parametrize("read_order", ["read", "group"], indirect=True)
@pytest.mark.parametrize("n_reads,n_rg,lens,seed", [
    (6000, 96, (150, 250), 21),    # many groups, a few reads per workgroup and group
    (40000, 8, (100,), 22),        # few groups, each spread over many workgroups
    (20000, 1, (101,), 23),        # one group
    (3000, 3, (60, 100, 140), 24),
])
def test_read_orders(read_order, n_reads, n_rg, lens, seed):
    b = synth.generate(n_reads, lens, n_rg, seed=seed)
    check([b.slice(0, n_reads // 3), b.slice(n_reads // 3, n_reads)], synth.known_sites(2_000_000, seed=5))


@pytest.mark.parametrize("read_order", ["read", "group"], indirect=True)
def test_read_orders_edge_cases(read_order):
    check([RecordBatch.from_records(EDGE * 3)], sites={"1": [10002, 10005, 40, 44, 10013]})


def test_fold_many_binades():
    # 3M bases: the expectedMismatch fold crosses many binades and uses the
    # block / tile / exact levels
    b = synth.generate(30000, (100,), 1, seed=14)
    check([b])


def test_empty_partition():
    b = synth.generate(2000, (100,), 1, seed=15)
    check([b.slice(0, 0), b, b.slice(0, 0)])


# ---- edge cases ----------------------------------------------------------------

EDGE = [
    rec(),  # plain
    rec(cigar="3H2S5M3S", start=42, mismatching_positions="1A3"),  # Q4: hard clip shifts, soft clips in window
    rec(cigar="2S6M2S", mismatching_positions="3C2", sequence="CTACCCTAAC", qual="##LKLPPQ##"),  # ReadCovariatesSuite 2
    rec(cigar="4M2I4M", mismatching_positions="2T5"),  # insertion masked
    rec(cigar="4M2D6M", mismatching_positions="4^GG6"),  # deletion
    rec(cigar="3M1P2N7M", mismatching_positions="3^AC0G6"),  # P advances (Q5)
    rec(cigar="5=5X", mismatching_positions="5ACGTA0"),
    rec(mismatching_positions=""),  # empty MD: every window base mismatches
    rec(mismatching_positions="4"),  # MD shorter than the span
    rec(mismatching_positions="3a6"),  # lower case MD
    rec(sequence="ANGTNCGTAN"),  # N bases
    rec(sequence="ANGTNCGTAN", read_negative_strand=True),
    rec(sequence="acgtACGTac"),  # lower case: idx -1 contexts (forward only)
    rec(read_negative_strand=True, read_paired=True, second_of_pair=True),
    rec(read_paired=True, second_of_pair=True),
    rec(second_of_pair=True),  # secondOfPair without readPaired: not negated
    rec(qual="#IIIIIII##"),
    rec(qual="##########"),  # nothing left after trimming
    rec(qual="I#I#I#I#II"),  # interior Q2 kept
    rec(qual="*", sequence="ACGTACGTAC"),  # Lq < Ls
    rec(start=5, cigar="10S10M", sequence="ACGTACGTACACGTACGTAC", qual="IIIIIIIIIIIIIIIIIIII"),
    rec(duplicate_read=True),
    rec(primary_alignment=False),
    rec(read_mapped=False),
    rec(mismatching_positions=None, record_group_id=0),  # not usable, recalibrated in apply
    rec(record_group_id=1, qual="JJJJJJJJJJ"),
    rec(record_group_id=2, qual="5555555555", mismatching_positions="0A0C0G0T6"),
    # one insertion or deletion: the prep's lock-step form (S? M (I|D) M S?)
    rec(cigar="1S3M2I3M1S", mismatching_positions="1A1T2"),  # clips both sides, letters either side of the I
    rec(cigar="3M2D7M", mismatching_positions="1A1^GC2T4"),  # letter before, deletion, letter after
    rec(cigar="2S4M1D4M", mismatching_positions="4^A0C3"),  # mismatch right after the deletion
    rec(cigar="10M", mismatching_positions="4^AC6"),  # an MD deletion the CIGAR has not: positions of M
    rec(cigar="4M2I4M", mismatching_positions="4^A4"),  # MD deletion over an insertion read
    rec(cigar="5M3D5M", mismatching_positions="5^ACG2"),  # MD shorter than the span past the deletion
    rec(cigar="2M3I5M", mismatching_positions="7", read_negative_strand=True),
    rec(cigar="6M1I3M", mismatching_positions="0T8", read_paired=True, second_of_pair=True),
    rec(cigar="3M0I7M", mismatching_positions="10"),  # zero-length insertion: the per-read path
    rec(start=10000, cigar="9M1D1M", mismatching_positions="9^T1", sequence="ACGTACGTAC"),
    # MD tags of 17..32 bytes: the lock-step form's second 16 bytes (fast_md)
    rec(cigar="40M", sequence="ACGT" * 10, qual="I" * 40, mismatching_positions="3A3C3G3T3A3C3G3T6"),  # 8 letters
    rec(cigar="40M", sequence="ACGT" * 10, qual="I" * 40, mismatching_positions="1A1C1G1T1A1C1G1T1A21"),  # 9: per-read path
    rec(cigar="10M14D10M", sequence="ACGTACGTAC" * 2, qual="I" * 20, mismatching_positions="10^ACGTACGTACGTAC10"),
    rec(cigar="2S36M2S", sequence="ACGT" * 10, qual="I" * 40, mismatching_positions="0A0C0G0T0A0C0G0T4A19",
        read_negative_strand=True),
    rec(cigar="40M", sequence="ACGT" * 10, qual="I" * 40, mismatching_positions="0" * 29 + "40"),  # 31 digits
    rec(cigar="40M", sequence="ACGT" * 10, qual="I" * 40, mismatching_positions="20A" + "0" * 29 + "19"),  # 33 bytes
    # Q2 tails: every trimmed base a mismatch, the tag longer than 16 bytes --
    # listed in pass 1, then prep's long form (only the letters inside the
    # trimmed window count)
    rec(cigar="40M", sequence="ACGT" * 10, qual="I" * 30 + "#" * 10,
        mismatching_positions="30A0C0G0T0A0C0G0T0A0C0"),
    rec(cigar="40M", sequence="ACGT" * 10, qual="I" * 30 + "#" * 10, read_negative_strand=True,
        mismatching_positions="5G24A0C0G0T0A0C0G0T0A0C0"),
    rec(cigar="3S37M", sequence="ACGT" * 10, qual="#" * 4 + "I" * 26 + "#" * 10,
        mismatching_positions="0T26A0C0G0T0A0C0G0T0A0"),
    rec(cigar="40M", sequence="ACGT" * 10, qual="#" * 40, mismatching_positions="30A0C0G0T0A0C0G0T0A0C0"),
    rec(cigar="40M", sequence="ACGT" * 10, qual="I" * 36 + "#" * 4,
        mismatching_positions="1A1C1G1T1A1C1G1T1A1C16A0C0G0T0"),  # 10 letters in the window
    rec(cigar="20M2I18M", sequence="ACGT" * 10, qual="I" * 30 + "#" * 10,
        mismatching_positions="28A0C0G0T0A0C0G0T0A0C0"),
]


def test_edge_cases_one_partition():
    check([RecordBatch.from_records(EDGE)], sites={"1": [10002, 10005, 40, 44, 10013]})


def test_edge_cases_split():
    b = RecordBatch.from_records(EDGE)
    check([b.slice(0, 7), b.slice(7, 20), b.slice(20, b.n_reads)])


@pytest.mark.parametrize("bad,err", [
    (rec(record_group_id=None), "NULL_RG"),
    (rec(mismatching_positions="5Z4"), "MD_PARSE"),
    (rec(mismatching_positions="A5"), "MD_PARSE"),
    (rec(mismatching_positions="5A"), "MD_PARSE"),
    (rec(mismatching_positions="2147483648"), "MD_PARSE"),  # Integer.parseInt overflow
    (rec(mismatching_positions="5^4"), "MD_PARSE"),  # '^' without letters
    (rec(mismatching_positions="5^^A4"), "MD_PARSE"),
    (rec(cigar="4M2I4M", mismatching_positions="3AZ4"), "MD_PARSE"),
    (rec(cigar="40M", sequence="ACGT" * 10, qual="I" * 40, mismatching_positions="3A3C3G3T3A3C3G3Z6"), "MD_PARSE"),
    (rec(cigar="40M", sequence="ACGT" * 10, qual="I" * 40, mismatching_positions="3A3C3G3T3A3C3G3T6^"), "MD_PARSE"),
    (rec(cigar="6M"), "CIGAR_SHORT"),
    (rec(cigar="*"), "CIGAR_SHORT"),
    (rec(cigar="0M10M"), "CIGAR_INVALID"),
    (rec(read_negative_strand=True, sequence="ACGTAxGTAC"), "BAD_REVCOMP_BASE"),
    (rec(qual="IIII\xc0IIIII"), "QUAL_RANGE"),
    (rec(reference_name=None), "NULL_FIELD"),
    (rec(qual=None), "NULL_FIELD"),
    (rec(sequence="ACGTA", cigar="10M"), "SEQ_SHORT"),
])
def test_errors(bad, err):
    ok = [rec(), rec(qual="HHHHHHHHHH")]
    check([RecordBatch.from_records(ok + [bad] + ok)], expect_error=err)


def test_missing_key_in_apply():
    # a read without MD (not observed) whose key never appears in the table
    recs = [rec(), rec(mismatching_positions=None, qual="++++++++++")]
    check([RecordBatch.from_records(recs)], expect_error="MISSING_KEY")


def test_all_masked():
    # every observed base is an insertion: avg = em / 0 -> NaN shifts -> Q0
    recs = [rec(cigar="10I", mismatching_positions="0"), rec(mismatching_positions=None)]
    check([RecordBatch.from_records(recs)])


# ---- committed golden fixtures (tests/golden/g1_g2.json) ------------------------

@pytest.mark.parametrize("name", ["g1", "g2"])
def test_golden_fixture(name):
    import json
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from make_golden import g1_batch, g2_batch
    with open(os.path.join(os.path.dirname(__file__), "golden", "g1_g2.json")) as fh:
        fx = json.load(fh)[name]
    b = g1_batch() if name == "g1" else g2_batch()
    g = run_gpu([b])
    assert g.error is None
    nz = np.nonzero(g.words)[0]
    assert {str(int(i)): int(g.words[i]) for i in nz} == fx["table_nonzero"]
    assert float(g.em).hex() == fx["expected_mismatch"]
    chars, out_len = g.outs[0]
    got = [[int(c) for c in chars[int(b.qual_offset[r]):int(b.qual_offset[r]) + int(out_len[r])]]
           for r in range(b.n_reads)]
    assert got == fx["chars"]
