"""Test infrastructure: a per-record Python restatement of the ADAMRecords
`transform` saves for SAM text input -- SAMRecordConverter.convert
(adam-core/.../converters/SAMRecordConverter.scala:26-144) over htsjdk's
SAMRecord of each line -- to check the device's ADAM columns
(adam_amd/csrc/adam_out.hip) field by field.  Not used by the product.

htsjdk behaviour restated (picard/samtools 1.93, as the reference pins it):
getAttributes returns the tags sorted by binary tag (second char << 8 |
first char), a repeated tag replacing the earlier value; 'i' values are
Integer (a Long outside Int), 'f' Float (Float.parseFloat), 'A' Character,
'Z' String; getCigarString re-encodes the parsed CIGAR; getReadGroup is the
header @RG of the RG tag's value (null when not in the header).
"""
from __future__ import annotations

import re
from typing import Dict, List, Optional

import numpy as np

OPS = "MIDNSHP=X"


def java_float_str(v) -> str:
    """java.lang.Float.toString of a float32 value (shortest round-trip
    digits, Java's layout)."""
    f = np.float32(v)
    if np.isnan(f):
        return "NaN"
    if np.isinf(f):
        return "Infinity" if f > 0 else "-Infinity"
    sign = "-" if np.signbit(f) else ""
    if f == 0:
        return sign + "0.0"
    s = np.format_float_scientific(abs(f), unique=True, trim="-")  # e.g. 1.5e+00, 1e-05
    mant, exp = s.split("e")
    digits = mant.replace(".", "").rstrip("0") or "0"
    e = int(exp)
    if -3 <= e < 7:
        if e >= 0:
            ip = digits[:e + 1].ljust(e + 1, "0")
            fp = digits[e + 1:] or "0"
            return sign + ip + "." + fp
        return sign + "0." + "0" * (-e - 1) + digits
    return sign + digits[0] + "." + (digits[1:] or "0") + "E" + str(e)


def _header(text: str):
    rg: Dict[str, Dict[str, str]] = {}
    rg_ids: List[str] = []
    sq: List[Dict[str, str]] = []
    for line in text.split("\n"):
        line = line.rstrip("\r")
        if not line.startswith("@"):
            continue
        f = line.split("\t")
        kv = dict(t.split(":", 1) for t in f[1:] if ":" in t)
        if f[0] == "@RG":
            rg_ids.append(kv["ID"])
            rg[kv["ID"]] = kv
        elif f[0] == "@SQ":
            sq.append(kv)
    names = sorted(rg_ids)
    rg_index = {nm: i for i, nm in enumerate(names)}  # toMap: the last index of a repeated name
    sq_index: Dict[str, int] = {}
    for i, r in enumerate(sq):
        sq_index.setdefault(r["SN"], i)
    return rg, rg_index, sq, sq_index


def _int_or_none(v):
    try:
        return int(v)
    except (TypeError, ValueError):
        return None


def _cigar_canonical(c: str) -> str:
    if c == "*" or c == "":
        return "*"
    return "".join("%d%s" % (int(n), op) for n, op in re.findall(r"(\d+)([%s])" % re.escape(OPS), c))


def convert_sam(text: bytes, run_date=None) -> List[dict]:
    """Every record of a SAM text as the dict of ADAMRecord fields
    (adam.avdl names; None = null)."""
    t = text.decode("latin-1")
    rg, rg_index, sq, sq_index = _header(t)
    out = []
    for line in t.split("\n"):
        line = line.rstrip("\r")
        if not line or line.startswith("@"):
            continue
        f = line.split("\t")
        qname, flag, rname, pos, mapq, cigar, rnext, pnext, tlen, seq, qual = f[:11]
        flag = int(flag)
        rec = dict.fromkeys(["referenceName", "referenceId", "start", "mapq", "mateReference", "mateAlignmentStart",
                             "recordGroupName", "recordGroupId", "mismatchingPositions",
                             "recordGroupSequencingCenter", "recordGroupDescription", "recordGroupRunDateEpoch",
                             "recordGroupFlowOrder", "recordGroupKeySequence", "recordGroupLibrary",
                             "recordGroupPredictedMedianInsertSize", "recordGroupPlatform",
                             "recordGroupPlatformUnit", "recordGroupSample", "mateReferenceId", "referenceLength",
                             "referenceUrl", "mateReferenceLength", "mateReferenceUrl"])
        rec.update(readName=qname, sequence=seq, cigar=_cigar_canonical(cigar), qual=qual)
        ref = sq_index.get(rname, -1) if rname != "*" else -1
        if ref >= 0:
            rec.update(referenceId=ref, referenceName=rname, referenceLength=_int_or_none(sq[ref].get("LN")),
                       referenceUrl=sq[ref].get("UR"))
            if int(pos) != 0:
                rec["start"] = int(pos) - 1
            if int(mapq) != 255:
                rec["mapq"] = int(mapq)
        mref = ref if rnext == "=" else (sq_index.get(rnext, -1) if rnext != "*" else -1)
        if mref >= 0:
            rec.update(mateReferenceId=mref, mateReference=sq[mref]["SN"],
                       mateReferenceLength=_int_or_none(sq[mref].get("LN")), mateReferenceUrl=sq[mref].get("UR"))
            if int(pnext) > 0:
                rec["mateAlignmentStart"] = int(pnext) - 1
        b = dict(readPaired=False, properPair=False, readMapped=False, mateMapped=False, readNegativeStrand=False,
                 mateNegativeStrand=False, firstOfPair=False, secondOfPair=False, primaryAlignment=False,
                 failedVendorQualityChecks=False, duplicateRead=False)
        if flag != 0:
            if flag & 1:
                b["readPaired"] = True
                b["mateNegativeStrand"] = bool(flag & 0x20)
                b["mateMapped"] = not flag & 0x8
                b["properPair"] = bool(flag & 0x2)
                b["firstOfPair"] = bool(flag & 0x40)
                b["secondOfPair"] = bool(flag & 0x80)
            b["duplicateRead"] = bool(flag & 0x400)
            b["readNegativeStrand"] = bool(flag & 0x10)
            b["primaryAlignment"] = not flag & 0x100
            b["failedVendorQualityChecks"] = bool(flag & 0x200)
            b["readMapped"] = not flag & 0x4
        rec.update(b)
        # attributes: htsjdk's sorted list, then `tags ::= attr` (descending), MD apart
        tags: Dict[int, tuple] = {}
        for tg in f[11:]:
            name, typ, val = tg[:2], tg[3], tg[5:]
            tags[ord(name[0]) | ord(name[1]) << 8] = (name, typ, val)
        parts = []
        rgv = None
        for key in sorted(tags, reverse=True):
            name, typ, val = tags[key]
            if name == "MD":
                rec["mismatchingPositions"] = val
                continue
            if name == "RG":
                rgv = val
            if typ == "i":
                v = int(val)
                assert -2 ** 31 <= v < 2 ** 31
                val = str(v)
            elif typ == "f":
                val = java_float_str(float(val))
            else:
                assert typ in "AZ", typ
            parts.append("%s:%s:%s" % (name, typ, val))
        rec["attributes"] = "\t".join(parts)
        if rgv is not None and rgv in rg:
            g = rg[rgv]
            rec.update(recordGroupId=rg_index[rgv], recordGroupName=rgv,
                       recordGroupSequencingCenter=g.get("CN"), recordGroupDescription=g.get("DS"),
                       recordGroupFlowOrder=g.get("FO"), recordGroupKeySequence=g.get("KS"),
                       recordGroupLibrary=g.get("LB"), recordGroupPredictedMedianInsertSize=_int_or_none(g.get("PI")),
                       recordGroupPlatform=g.get("PL"), recordGroupPlatformUnit=g.get("PU"),
                       recordGroupSample=g.get("SM"))
            if "DT" in g and run_date is not None:
                rec["recordGroupRunDateEpoch"] = run_date(g["DT"])
        out.append(rec)
    return out
