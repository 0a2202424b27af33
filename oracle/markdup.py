"""MarkDuplicates restated in plain Python.  TEST INFRASTRUCTURE ONLY.

Only tests/ import this module, as the checker of the library's
bqsr_mark_duplicates (adam_amd/csrc/mark_duplicates.cpp).  It follows:

  core/rdd/MarkDuplicates.scala:24-111           markReads, score, scoreAndMarkReads, apply
  core/models/SingleReadBucket.scala:27-37       buckets by (recordGroupId, readName)
  core/models/ReferencePositionPair.scala:27-63  the bucket's (left, right) 5' positions
  core/models/ReferencePosition.scala             ReferencePositionWithOrientation ordering
  core/rich/RichADAMRecord.scala:77-118           end, unclippedStart/End, fivePrimePosition

Pinned by the cases of core/.../rdd/MarkDuplicatesSuite.scala (ported in
tests/test_markdup.py).  Group iteration order in Spark is its shuffle's; here
buckets keep first-appearance order, and sortBy is stable as Scala's is.  So
which of several equally scored best buckets stays unmarked is unpinned
against the reference: `equivalent_marks` accepts any choice among them.

A read is a dict: name, library, rg (None = no recordGroupId), mapped,
primary, paired, mate_mapped, neg, ref, start, qual (str), cigar (list of
(length, op char)).
"""
from typing import Dict, List, Optional, Tuple

CONSUMES_REF = set("MDN=X")
CLIPPED = set("SH")


def five_prime(r) -> int:
    """RichADAMRecord.fivePrimePosition (:112-118)."""
    if not r["neg"]:
        p = r["start"]
        for length, op in r["cigar"]:  # unclippedStart: takeWhile(isClipped)
            if op not in CLIPPED:
                break
            p -= length
        return p
    end = r["start"] + sum(length for length, op in r["cigar"] if op in CONSUMES_REF)
    for length, op in reversed(r["cigar"]):  # unclippedEnd
        if op not in CLIPPED:
            break
        end += length
    return end


def rpos(r) -> Tuple[int, int, bool]:
    """ReferencePositionWithOrientation: (refId, pos) then negativeStrand (false < true)."""
    return (r["ref"], five_prime(r), r["neg"])


def score(r) -> int:
    """MarkDuplicates.score (:37-39): Σ of (char - 33).toByte values >= 15."""
    s = 0
    for ch in r["qual"]:
        v = (ord(ch) - 33) & 0xFF
        v = v - 256 if v >= 128 else v
        if v >= 15:
            s += v
    return s


def mark_duplicates(reads: List[dict], ties: Optional[list] = None) -> List[bool]:
    """MarkDuplicates.apply (:100-111).  `ties`, when a list, receives per
    scoreAndMarkReads call whose best score is shared the primary-read index
    lists of the tied best buckets (the first of them kept here)."""
    dup = [False] * len(reads)
    # SingleReadBucket.apply: groupBy (recordGroupId, readName); partition mapped / primary
    buckets: Dict[tuple, dict] = {}
    for i, r in enumerate(reads):
        b = buckets.setdefault((r["rg"], r["name"]), {"prim": [], "sec": [], "unm": []})
        if not r["mapped"]:
            b["unm"].append(i)
        elif r["primary"]:
            b["prim"].append(i)
        else:
            b["sec"].append(i)
    # ReferencePositionPair.apply
    keyed = []
    for b in buckets.values():
        left = right = None
        if b["prim"]:
            p1 = rpos(reads[b["prim"][0]])
            if len(b["prim"]) > 1:  # lift(1) defined, with or without the mate flags
                p2 = rpos(reads[b["prim"][1]])
                left, right = (p1, p2) if p1 < p2 else (p2, p1)
            else:
                left = p1
        first = (b["prim"] + b["sec"] + b["unm"])[0]
        keyed.append((left, right, reads[first]["library"], b))

    def mark(b, are_dups):  # markReads
        for i in b["prim"] + b["sec"]:
            dup[i] = are_dups
        for i in b["unm"]:
            dup[i] = False

    def score_and_mark(bs):  # scoreAndMarkReads
        scored = sorted(((sum(score(reads[i]) for i in b["prim"]), b) for b in bs), key=lambda t: -t[0])
        best = [b["prim"] for s, b in scored if s == scored[0][0]]
        if ties is not None and len(best) > 1:
            ties.append(best)
        for k, (_, b) in enumerate(scored):
            for i in b["prim"]:
                dup[i] = k != 0
            for i in b["sec"]:
                dup[i] = True
            for i in b["unm"]:
                dup[i] = False

    groups: Dict[tuple, List[tuple]] = {}
    for left, right, lib, b in keyed:  # groupBy(leftPositionAndLibrary)
        groups.setdefault((left, lib), []).append((right, b))
    for (left, lib), members in groups.items():
        if left is None:
            for _, b in members:
                mark(b, False)
            continue
        by_right: Dict[Optional[tuple], list] = {}
        for right, b in members:
            by_right.setdefault(right, []).append(b)
        fragments = by_right.get(None)
        has_pairs = any(k is not None for k in by_right)
        if has_pairs:
            for b in fragments or []:
                mark(b, True)
            for k, bs in by_right.items():
                if k is not None:
                    score_and_mark(bs)
        elif fragments:
            score_and_mark(fragments)
    return dup


def equivalent_marks(reads: List[dict], got) -> Tuple[bool, str]:
    """Whether a marking equals mark_duplicates' up to the choice among tied
    best buckets: reads outside the ties must match exactly; in each tie
    exactly one bucket's primaries are all unmarked and every other tied
    bucket's primaries are all marked."""
    ties: list = []
    want = mark_duplicates(reads, ties)
    got = [bool(x) for x in got]
    tied = {i for t in ties for b in t for i in b}
    for i, (g, w) in enumerate(zip(got, want)):
        if g != w and i not in tied:
            return False, "read %d: %s, expected %s (not in a tie)" % (i, g, w)
    for t in ties:
        kept = [b for b in t if not any(got[i] for i in b)]
        if len(kept) != 1 or any(not all(got[i] for i in b) for b in t if b is not kept[0]):
            return False, "tie of %d buckets: %d kept" % (len(t), len(kept))
    return True, ""
