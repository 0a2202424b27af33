"""`adam compare -baseqs` (§8 f4): per-base quality concordance of two read
sets, e.g. a reference run's recalibrated reads against this build's.

Restates adam-cli/.../cli/CompareAdam.scala:139-172 (printSummary) over
core/rdd/comparisons/ComparisonTraversalEngine.scala (reads in
SingleReadBuckets keyed by readName, the two inputs joined by name),
core/models/ReadBucket.scala:97-110 (a bucket's reads split into unpaired /
first / second of pair, primary / secondary) and
core/metrics/AvailableComparisons.scala:149-177 (BaseQualityScores: for each
of five categories holding exactly one read on both sides, the pairs
(q1, q2) of the two reads' qualityScores zipped; the histogram's count and
identity, diff% = 100 (count - identity) / count).  qualityScores are
(char - 33).toByte values (RichADAMRecord.scala:43).

Inputs are SAM files read with SAMRecordConverter's flag semantics (flags
only when the FLAG word is non-zero); ``encoding`` is how QUAL bytes map to
Java chars: latin-1 for plain SAM, utf-8 for this build's transform output
(which writes chars above 0x7F as UTF-8).  A validation tool: host Python.
"""
from __future__ import annotations

import argparse
import sys
from collections import Counter, defaultdict
from typing import Dict, List, Optional, Tuple

CATS = ("unpairedPrimary", "pairedFirstPrimary", "pairedSecondPrimary", "unpairedSecondary", "pairedFirstSecondary",
        "pairedSecondSecondary", "unmapped")
# the categories BaseQualityScores.matchedByName visits (:172-177): not unpairedSecondary, not unmapped
BASEQ_CATS = ("unpairedPrimary", "pairedFirstPrimary", "pairedSecondPrimary", "pairedFirstSecondary",
              "pairedSecondSecondary")


def quality_scores(qual: str) -> List[int]:
    """RichADAMRecord.qualityScores: (char - 33).toByte, as Int."""
    out = []
    for ch in qual:
        v = (ord(ch) - 33) & 0xFF
        out.append(v - 256 if v >= 128 else v)
    return out


def load_buckets(path: str, encoding: str = "latin-1") -> Dict[str, List[Dict[str, List[List[int]]]]]:
    """readName -> its ReadBuckets (one per recordGroupId), each category a
    list of the reads' qualityScores in input order."""
    rg_names = set()
    body = []
    with open(path, "rb") as fh:
        for raw in fh.read().split(b"\n"):
            line = raw[:-1] if raw.endswith(b"\r") else raw
            if not line:
                continue
            if line.startswith(b"@"):
                f = line.split(b"\t")
                if f[0] == b"@RG":
                    for t in f[1:]:
                        if t.startswith(b"ID:"):
                            rg_names.add(t[3:])
                continue
            body.append(line)
    buckets: Dict[Tuple[Optional[bytes], bytes], Dict[str, List[List[int]]]] = {}
    for line in body:
        f = line.split(b"\t")
        name, flag, qual = f[0], int(f[1]), f[10]
        rg = None
        for t in f[11:]:
            k = t.split(b":", 2)
            if len(k) == 3 and k[0] == b"RG":
                rg = k[2]
        if rg is not None and rg not in rg_names:
            rg = None
        mapped = primary = paired = first = False
        if flag != 0:  # SAMRecordConverter.scala:72-108
            paired = bool(flag & 0x1)
            first = paired and bool(flag & 0x40)
            primary = not flag & 0x100
            mapped = not flag & 0x4
        b = buckets.setdefault((rg, name), {c: [] for c in CATS})
        q = quality_scores(qual.decode(encoding))
        if not mapped:
            cat = "unmapped"
        elif primary:
            cat = "pairedFirstPrimary" if first else ("pairedSecondPrimary" if paired else "unpairedPrimary")
        else:
            cat = "pairedFirstSecondary" if first else ("pairedSecondSecondary" if paired else "unpairedSecondary")
        b[cat].append(q)
    named: Dict[str, list] = defaultdict(list)
    for (rg, name), b in buckets.items():  # keyBy(_.allReads.head.getReadName)
        named[name.decode("latin-1")].append(b)
    return named


def base_quality_points(b1, b2) -> List[Tuple[int, int]]:
    """BaseQualityScores.matchedByName (AvailableComparisons.scala:149-177)."""
    pts: List[Tuple[int, int]] = []
    for c in BASEQ_CATS:
        r1, r2 = b1[c], b2[c]
        if len(r1) == len(r2) == 1:
            pts.extend(zip(r1[0], r2[0]))
    return pts


def compare_baseqs(path1: str, path2: str, encoding1: str = "latin-1", encoding2: str = "latin-1") -> dict:
    n1, n2 = load_buckets(path1, encoding1), load_buckets(path2, encoding2)
    hist: Counter = Counter()
    for name, bs1 in n1.items():  # named1.join(named2): every pair of buckets sharing the name
        for b1 in bs1:
            for b2 in n2.get(name, ()):
                hist.update(base_quality_points(b1, b2))
    count = sum(hist.values())
    identity = sum(v for (a, b), v in hist.items() if a == b)
    return dict(total1=sum(len(v) for v in n1.values()), unique1=sum(len(v) for k, v in n1.items() if k not in n2),
                total2=sum(len(v) for v in n2.values()), unique2=sum(len(v) for k, v in n2.items() if k not in n1),
                count=count, identity=identity, diff_pct=100.0 * (count - identity) / count if count else float("nan"),
                histogram=hist)


def summary(path1: str, path2: str, r: dict) -> str:
    """CompareAdam.printSummary's text."""
    out = ["%15s: %s" % ("INPUT1", path1), "\t%15s: %d" % ("total-reads", r["total1"]),
           "\t%15s: %d" % ("unique-reads", r["unique1"]), "%15s: %s" % ("INPUT2", path2),
           "\t%15s: %d" % ("total-reads", r["total2"]), "\t%15s: %d" % ("unique-reads", r["unique2"]), "",
           "baseqs", "\t%15s: %d" % ("count", r["count"]), "\t%15s: %d" % ("identity", r["identity"]),
           "\t%15s: %.5f" % ("diff%", r["diff_pct"])]
    return "\n".join(out)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="adam_amd.compare", description="compare -baseqs of two SAM files")
    ap.add_argument("input1")
    ap.add_argument("input2")
    ap.add_argument("-comparisons", default="baseqs")
    ap.add_argument("-encoding1", default="latin-1")
    ap.add_argument("-encoding2", default="latin-1")
    ap.add_argument("-output", default=None, help="also write the histogram (value\\tcount) here")
    a = ap.parse_args(argv)
    if a.comparisons != "baseqs":
        ap.error("only the baseqs comparison is in this build")
    r = compare_baseqs(a.input1, a.input2, a.encoding1, a.encoding2)
    print(summary(a.input1, a.input2, r))
    if a.output:
        with open(a.output, "w") as fh:  # Histogram.write
            fh.write("value\tcount\n")
            for (x, y), c in sorted(r["histogram"].items()):
                fh.write("(%d,%d)\t%d\n" % (x, y, c))
    return 0


if __name__ == "__main__":
    sys.exit(main())
