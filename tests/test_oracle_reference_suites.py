"""The reference's own BQSR-relevant ScalaTest suites, ported against the CPU
oracle (which pins the oracle before it is trusted as the GPU's checker).

Sources (adam-core/src/test/scala/edu/berkeley/cs/amplab/adam/):
  rdd/recalibration/ReadCovariatesSuite.scala:25-71
  rich/RichADAMRecordSuite.scala:25-55,83-126
  util/MdTagSuite.scala:27-114
  rdd/AdamContextSuite.scala:133-142
  rdd/RecalibrateBaseQualitiesSuite.scala:33-402 (ErrorCount / table / finalize parts)
"""
import math

import numpy as np
import pytest

import oracle as O
from adam_amd.records import ADAMRecord, RecordBatch, parse_cigar


def cov(rec, sites=None):
    return O.read_covariates(RecordBatch.from_records([rec]), 0, O.Sites(sites) if sites else None)


# ---- ReadCovariatesSuite ----------------------------------------------------

@pytest.mark.parametrize("cigar,md", [("10M", "5C4"), ("2S6M2S", "3C2")])
def test_read_covariates_quality_offset_and_softclip(cigar, md):
    # "Test Quality Offset" / "Test ReadCovar on SoftClipped Read"
    r = ADAMRecord(record_group_id=0, read_mapped=True, start=10000, reference_name="1", cigar=cigar,
                   mismatching_positions=md, sequence="CTACCCTAAC", qual="##LKLPPQ##")
    bases = cov(r)
    assert bases[0][3] == 43  # firstBaseCovar.qual
    assert all(b[3] == b[0] for b in bases)  # qual == qualByRG for rg 0
    mism = bases[3]  # drop(3).next
    assert mism[3] == 47
    assert mism[4] is True


# ---- RichADAMRecordSuite ----------------------------------------------------

def refpos(cigar, start):
    return O.reference_positions(parse_cigar(cigar), start)


@pytest.mark.parametrize("cigar,start,unclipped", [("10M", 42, 42), ("2S8M", 42, 40), ("3H2S5M4S", 42, 37)])
def test_unclipped_start(cigar, start, unclipped):
    # unclippedStart is where referencePositions begins (H emits no position)
    assert refpos(cigar, start)[0] == unclipped


@pytest.mark.parametrize("cigar,start,end", [("10M", 10, 20), ("8M2S", 10, 18), ("6M2S2H", 10, 16)])
def test_reference_end(cigar, start, end):
    assert O.reference_end(parse_cigar(cigar), start) == end


def test_cigar_clipping_sequence():
    assert refpos("10S90M", 100)[0] == 90


def test_reference_positions():
    p = refpos("90M10H", 1000)
    assert len(p) == 90 and p[0] == 1000
    p = refpos("10S90M", 1000)
    assert len(p) == 100 and p[0] == 990 and p[10] == 1000
    p = refpos("10M10M", 1000)
    assert all(p[i] == 1000 + i for i in range(20))
    p = refpos("5M5D10M", 1000)
    assert len(p) == 15 and p[0] == 1000 and p[5] == 1010
    p = refpos("10M2I10M", 1000)
    assert len(p) == 22 and p[0] == 1000 and p[10] is None and p[12] == 1010
    p = refpos("10M3D10M2I", 1000)
    assert len(p) == 22 and p[0] == 1000 and p[10] == 1013 and p[20] is None
    p = refpos("1S28M1D32M1I15M1D23M", 1000)
    assert len(p) == 100
    assert (p[0], p[1], p[29], p[61], p[62], p[78], p[99]) == (999, 1000, 1029, None, 1061, 1078, 1099)


# ---- MdTagSuite ----------------------------------------------------------------

def is_match(runs, p):
    return any(lo <= p < hi for lo, hi in runs)


def test_md_null_and_empty():
    assert O.md_runs("", 0) == []  # MdTag("", 0L) parses; null is "no MD" (mdEvent None)


@pytest.mark.parametrize("md", ["ACTG0", "0ACTZ", "0ACTG"])
def test_md_invalid(md):
    with pytest.raises(O.OracleError) as e:
        O.md_runs(md, 0)
    assert e.value.code == 2  # MD_PARSE (IllegalArgumentException)


def test_md_valid():
    assert not is_match(O.md_runs("0A0", 0), 0)
    r = O.md_runs("100", 0)
    assert all(is_match(r, i) for i in range(100)) and not is_match(r, -1)
    r = O.md_runs("100C2", 0)
    assert all(is_match(r, i) for i in range(100)) and not is_match(r, 100)
    assert all(is_match(r, i) for i in range(101, 103))
    r = O.md_runs("100C0^C20", 0)
    assert all(is_match(r, i) for i in range(100)) and not is_match(r, 100) and not is_match(r, 101)
    assert all(is_match(r, i) for i in range(102, 122))
    r = O.md_runs("0^ACGTACGTACGT10", 0)
    assert not any(is_match(r, i) for i in range(12))
    r = O.md_runs("22^A79", 0)
    assert all(is_match(r, i) for i in range(22)) and not is_match(r, 22)
    assert all(is_match(r, i) for i in range(23, 23 + 79))
    r = O.md_runs("39r36c23", 0)  # lower case (seen in 1000G)
    assert all(is_match(r, i) for i in range(39)) and not is_match(r, 39)
    assert all(is_match(r, i) for i in range(40, 76)) and not is_match(r, 76)
    assert all(is_match(r, i) for i in range(77, 100))
    r = O.md_runs("34Y18G46", 0)
    assert not is_match(r, 34)


def test_md_start_offset():
    assert O.md_runs("60", 1) == [(1, 61)]


# ---- AdamContextSuite (phred) ----------------------------------------------------

def test_phred_conversions():
    # successProbabilityToPhred(p) = probabilityToPhred(1.0 - p)
    assert O.error_prob_to_phred(1.0 - 0.9) == 10
    assert O.error_prob_to_phred(1.0 - 0.99999) == 50
    assert 0.89 < 1.0 - O.pow10cache(10) < 0.91
    assert 0.99998 < 1.0 - O.pow10cache(50) < 0.999999


# ---- RecalibrateBaseQualitiesSuite (table semantics on the dense table) ----------

def dims(n_rg=3, max_len=10):
    return O.Dims(n_rg, max_len)


def test_error_prob_clamp_and_merge_symmetry():
    # ErrorCount ++ / getErrorProb (RecalTable.scala:203-214) through finalize:
    # one key, counts on the cycle covariate
    d = dims(1, 10)
    rng = np.random.default_rng(1)
    for base_sum, mm_sum in [(10000, 0), (100000, 1), (1000000, 10), (10000000, 100)]:
        b1 = int(rng.integers(0, base_sum))
        m1 = min(b1, int(rng.integers(0, mm_sum))) if mm_sum else 0
        w1 = np.zeros(O.table_words(d), np.int64)
        w2 = np.zeros(O.table_words(d), np.int64)
        t1, o1, x1 = O.split_table(d, w1)
        t2, o2, x2 = O.split_table(d, w2)
        t1[30] = t2[30] = 1
        o1[30, 10] = b1
        x1[30, 10] = m1
        o2[30, 10] = base_sum - b1
        x2[30, 10] = mm_sum - m1
        left, right = w1 + w2, w2 + w1
        assert np.array_equal(left, right)
        fin = O.Final(d, left, 0.0)
        assert fin.global_counts() == (base_sum, mm_sum)
        # readGroupDelta = max(1e-6, mm/obs) - avg, avg = em/obs = 0 here
        sh, _ = fin.shifts(30, 30, 1, 0)
        assert sh[0] == max(1e-6, mm_sum / base_sum)


P10 = [O.pow10cache(q) for q in range(256)]


def test_finalization_and_deltas_large_scale():
    # "Util :: RecalTable :: Finalization and Deltas :: LargeScale" (:323-378):
    # 10 tables of keys 1..120, 3 covariates of values 0..2, 1000 obs / 1 mm each
    d = O.Dims(3, 10)
    total = None
    em = 0.0
    for _ in range(10):
        w = np.zeros(O.table_words(d), np.int64)
        t, o, x = O.split_table(d, w)
        em_t = 0.0
        for qual in range(1, 121):
            rg = qual // 61
            quality = qual - 60 * rg
            t[qual] = 1000
            for c in range(3):  # the cycle covariate carries values 0..2
                o[qual, 10 + c] = 1000
                x[qual, 10 + c] = 1
            inc = P10[quality] * 3
            for _b in range(1000):
                em_t += inc
        total = w if total is None else total + w
        em = em + em_t
    fin = O.Final(d, total, em)
    expected_counts = sum(10000 * 3 * 2 for _ in range(1, 61))
    expected_mm = sum(30000 * 2 * O.pow10cache(t) for t in range(1, 61))
    rate = expected_mm / expected_counts
    assert fin.global_counts()[0] == expected_counts
    assert fin.group_counts(0)[0] == 30000 * 60
    assert fin.group_counts(1)[1] == 30 * 60
    for qual in range(1, 121):
        sh, _ = fin.shifts(qual, qual % 60 if qual % 60 else 60, 1, 0)
        assert abs((10.0 / 10000 - rate) - sh[0]) < 1e-12


def test_qual_by_rg_example():
    # "Covariate :: QualByRg :: Example" (:380-402): key = q + 60 * rg
    quals = {
        0: [2, 2, 2, 2, 2, 2, 25, 32, 27, 22, 33, 35, 37, 33, 37, 38, 32, 26, 28, 24, 23, 22, 37, 38, 33, 33, 33,
            33, 33, 33],
        1: [25, 25, 25, 25, 25, 26, 26, 26, 26, 25, 26, 26, 26, 27, 27, 27, 27, 27, 27, 27, 29, 29, 2, 2, 2, 2,
            2, 2, 2, 2],
        2: [32, 32, 32, 33, 33, 33, 33, 35, 35, 32, 33, 28, 29, 29, 29, 29, 29, 29, 29, 29, 2, 2, 2, 2, 2, 2, 2,
            2, 2, 2],
    }
    for rg, q in quals.items():
        r = ADAMRecord(record_group_id=rg, read_mapped=True, start=100, reference_name="1", cigar="30M",
                       mismatching_positions="30", sequence="A" * 30, qual="".join(chr(v + 33) for v in q))
        got = [b[0] for b in cov(r)]
        kept = [v for v in q]
        st = next(i for i, v in enumerate(kept) if v > 2)
        en = len(kept) - next(i for i, v in enumerate(reversed(kept)) if v > 2)
        assert got == [v + 60 * rg for v in kept[st:en]]


def test_known_site_mask_raw_vcf_pos():
    # SnpTable compares 0-based positions with raw VCF POS (quirk Q7)
    r = ADAMRecord(record_group_id=0, read_mapped=True, start=100, reference_name="c", cigar="5M",
                   mismatching_positions="5", sequence="ACGTA", qual="IIIII")
    masked = [b[5] for b in cov(r, {"c": [102]})]
    assert masked == [False, False, True, False, False]
    masked = [b[5] for b in cov(r, {"other": [102]})]  # unknown contig: not masked
    assert masked == [False] * 5
