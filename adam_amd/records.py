"""ADAMRecord columns: the host-side flattening in front of the C ABI.

A partition of ``ADAMRecord``s (adam-format/src/main/resources/avro/adam.avdl:4-68)
is flattened into the ``bqsr_records`` column layout of ``include/adam_bqsr.h``.
Only the fields BQSR reads are kept: the boolean flags, recordGroupId, start,
referenceName, sequence, qual, cigar and mismatchingPositions (MD).

``read_sam`` reproduces the ingest semantics BQSR depends on
(adam-core/.../converters/SAMRecordConverter.scala:26-144 and
models/RecordGroupDictionary.scala:36-43): start = POS - 1, flags are only set
when the SAM flag word is non-zero (quirk Q2), MD:Z becomes
mismatchingPositions, the RG id is the index of the read group in the sorted
header read-group names.
"""
from __future__ import annotations

import ctypes
import dataclasses
from typing import Iterable, List, Optional, Sequence

import numpy as np

# flag bits, include/adam_bqsr.h
F_PAIRED = 1 << 0
F_MAPPED = 1 << 1
F_NEG_STRAND = 1 << 2
F_SECOND_OF_PAIR = 1 << 3
F_PRIMARY = 1 << 4
F_DUPLICATE = 1 << 5
F_HAS_RG = 1 << 8
F_HAS_MD = 1 << 9
F_HAS_QUAL = 1 << 10
F_HAS_SEQ = 1 << 11
F_HAS_CIGAR = 1 << 12
F_HAS_START = 1 << 13
F_HAS_REFNAME = 1 << 14

CONTIG_UNKNOWN = -1

_CIGAR_OPS = "MIDNSHP=X"


class CigarParseError(ValueError):
    """samtools TextCigarCodec.decode rejected the string (malformed CIGAR)."""


def parse_cigar(text: Optional[str]) -> np.ndarray:
    """CIGAR text -> BAM u32 elements (len << 4 | op), as samtools
    TextCigarCodec.decode (RichADAMRecord.samtoolsCigar, rich/RichADAMRecord.scala:58-60).
    ``"*"`` is the empty CIGAR."""
    if text is None:
        raise ValueError("null cigar")
    if text == "*" or text == "":
        return np.zeros(0, dtype=np.uint32)
    out = []
    num = None
    for ch in text:
        if "0" <= ch <= "9":
            num = (0 if num is None else num) * 10 + (ord(ch) - 48)
        else:
            op = _CIGAR_OPS.find(ch)
            if op < 0 or num is None:
                raise CigarParseError("Malformed CIGAR string: " + text)
            if num >= (1 << 28):
                raise CigarParseError("CIGAR element too long: " + text)
            out.append((num << 4) | op)
            num = None
    if num is not None:
        raise CigarParseError("Malformed CIGAR string: " + text)
    return np.asarray(out, dtype=np.uint32)


def cigar_to_text(ops: Sequence[int]) -> str:
    if len(ops) == 0:
        return "*"
    return "".join("%d%s" % (int(e) >> 4, _CIGAR_OPS[int(e) & 0xF]) for e in ops)


@dataclasses.dataclass
class ADAMRecord:
    """The ADAMRecord fields BQSR touches (adam.avdl:4-68).  ``None`` = Avro null."""

    sequence: Optional[str] = None
    qual: Optional[str] = None
    cigar: Optional[str] = None
    start: Optional[int] = None
    reference_name: Optional[str] = None
    record_group_id: Optional[int] = None
    mismatching_positions: Optional[str] = None
    read_paired: bool = False
    read_mapped: bool = False
    read_negative_strand: bool = False
    second_of_pair: bool = False
    primary_alignment: bool = False
    duplicate_read: bool = False
    read_name: Optional[str] = None
    # optional fields other than MD, "TAG:TYPE:VALUE" joined by tabs in the
    # converter's order (SAMRecordConverter.scala:110-121 prepends each: the
    # reverse of the SAM line's order); not read by BQSR
    attributes: Optional[str] = None

    @property
    def flag_bits(self) -> int:
        f = 0
        f |= F_PAIRED if self.read_paired else 0
        f |= F_MAPPED if self.read_mapped else 0
        f |= F_NEG_STRAND if self.read_negative_strand else 0
        f |= F_SECOND_OF_PAIR if self.second_of_pair else 0
        f |= F_PRIMARY if self.primary_alignment else 0
        f |= F_DUPLICATE if self.duplicate_read else 0
        f |= F_HAS_RG if self.record_group_id is not None else 0
        f |= F_HAS_MD if self.mismatching_positions is not None else 0
        f |= F_HAS_QUAL if self.qual is not None else 0
        f |= F_HAS_SEQ if self.sequence is not None else 0
        f |= F_HAS_CIGAR if self.cigar is not None else 0
        f |= F_HAS_START if self.start is not None else 0
        f |= F_HAS_REFNAME if self.reference_name is not None else 0
        return f


class _CRecords(ctypes.Structure):
    _fields_ = [
        ("n_reads", ctypes.c_int64),
        ("flags", ctypes.c_void_p),
        ("rg_id", ctypes.c_void_p),
        ("contig_id", ctypes.c_void_p),
        ("start", ctypes.c_void_p),
        ("seq_offset", ctypes.c_void_p),
        ("seq", ctypes.c_void_p),
        ("qual_offset", ctypes.c_void_p),
        ("qual", ctypes.c_void_p),
        ("cigar_offset", ctypes.c_void_p),
        ("cigar", ctypes.c_void_p),
        ("md_offset", ctypes.c_void_p),
        ("md", ctypes.c_void_p),
    ]


def _offsets(lengths: np.ndarray) -> np.ndarray:
    off = np.zeros(len(lengths) + 1, dtype=np.uint64)
    np.cumsum(lengths, out=off[1:])
    return off


class RecordBatch:
    """One partition of ADAMRecords in ``bqsr_records`` column form.

    ``ref_names`` lists the distinct reference names; ``ref_index[r]`` is the
    read's index in it (-1 when referenceName is null).  The contig ids the C
    ABI wants are resolved against a SnpTable by :meth:`contig_ids_for`.
    """

    def __init__(self, flags, rg_id, ref_index, ref_names, start, seq_offset, seq, qual_offset, qual,
                 cigar_offset, cigar, md_offset, md):
        self.flags = np.ascontiguousarray(flags, dtype=np.uint32)
        self.rg_id = np.ascontiguousarray(rg_id, dtype=np.int32)
        self.ref_index = np.ascontiguousarray(ref_index, dtype=np.int32)
        self.ref_names = list(ref_names)
        self.start = np.ascontiguousarray(start, dtype=np.int64)
        self.seq_offset = np.ascontiguousarray(seq_offset, dtype=np.uint64)
        self.seq = np.ascontiguousarray(seq, dtype=np.uint8)
        self.qual_offset = np.ascontiguousarray(qual_offset, dtype=np.uint64)
        self.qual = np.ascontiguousarray(qual, dtype=np.uint8)
        self.cigar_offset = np.ascontiguousarray(cigar_offset, dtype=np.uint64)
        self.cigar = np.ascontiguousarray(cigar, dtype=np.uint32)
        self.md_offset = np.ascontiguousarray(md_offset, dtype=np.uint64)
        self.md = np.ascontiguousarray(md, dtype=np.uint8)
        n = len(self.flags)
        for name in ("rg_id", "ref_index", "start"):
            if len(getattr(self, name)) != n:
                raise ValueError("column %s has the wrong length" % name)
        for name in ("seq_offset", "qual_offset", "cigar_offset", "md_offset"):
            if len(getattr(self, name)) != n + 1:
                raise ValueError("offsets %s must have n_reads + 1 entries" % name)

    @property
    def n_reads(self) -> int:
        return len(self.flags)

    @property
    def n_bases(self) -> int:
        """Sum of read (sequence) lengths: the `bases` of the benchmark metric."""
        return int(self.seq_offset[-1])

    def max_len(self) -> int:
        if self.n_reads == 0:
            return 1
        return max(1, int(np.max(np.diff(self.seq_offset.astype(np.int64)))))

    def n_rg(self) -> int:
        has = (self.flags & F_HAS_RG) != 0
        return int(self.rg_id[has].max()) + 1 if has.any() else 1

    def contig_ids_for(self, contig_names: Optional[Sequence[str]]) -> np.ndarray:
        """referenceName -> index into a SnpTable contig list (BQSR_CONTIG_UNKNOWN when absent)."""
        lut = np.full(len(self.ref_names) + 1, CONTIG_UNKNOWN, dtype=np.int32)
        if contig_names:
            pos = {c: i for i, c in enumerate(contig_names)}
            for i, name in enumerate(self.ref_names):
                lut[i] = pos.get(name, CONTIG_UNKNOWN)
        return lut[self.ref_index]  # ref_index -1 -> last entry (unknown); null names carry no HAS_REFNAME bit

    def c_struct(self, contig_ids: Optional[np.ndarray] = None):
        """ctypes ``bqsr_records`` viewing this batch (keep the returned tuple alive)."""
        cid = self.contig_ids_for(None) if contig_ids is None else np.ascontiguousarray(contig_ids, dtype=np.int32)
        keep = [cid]
        s = _CRecords()
        s.n_reads = self.n_reads

        def p(a):
            if a.size == 0:
                a = np.zeros(1, dtype=a.dtype)
            keep.append(a)
            return a.ctypes.data

        s.flags = p(self.flags)
        s.rg_id = p(self.rg_id)
        s.contig_id = p(cid)
        s.start = p(self.start)
        s.seq_offset = p(self.seq_offset)
        s.seq = p(self.seq)
        s.qual_offset = p(self.qual_offset)
        s.qual = p(self.qual)
        s.cigar_offset = p(self.cigar_offset)
        s.cigar = p(self.cigar)
        s.md_offset = p(self.md_offset)
        s.md = p(self.md)
        return s, keep

    def slice(self, r0: int, r1: int) -> "RecordBatch":
        """Reads [r0, r1) as their own partition."""
        def sub(off, col):
            a, b = int(off[r0]), int(off[r1])
            return (off[r0:r1 + 1] - off[r0]).astype(np.uint64), col[a:b]
        so, s = sub(self.seq_offset, self.seq)
        qo, q = sub(self.qual_offset, self.qual)
        co, c = sub(self.cigar_offset, self.cigar)
        mo, m = sub(self.md_offset, self.md)
        return RecordBatch(self.flags[r0:r1], self.rg_id[r0:r1], self.ref_index[r0:r1], self.ref_names,
                           self.start[r0:r1], so, s, qo, q, co, c, mo, m)

    @staticmethod
    def from_records(recs: Iterable[ADAMRecord]) -> "RecordBatch":
        recs = list(recs)
        names: List[str] = []
        name_idx = {}
        flags, rg, ridx, start = [], [], [], []
        seqs, quals, cigs, mds = [], [], [], []
        for r in recs:
            flags.append(r.flag_bits)
            rg.append(r.record_group_id if r.record_group_id is not None else 0)
            if r.reference_name is None:
                ridx.append(-1)
            else:
                if r.reference_name not in name_idx:
                    name_idx[r.reference_name] = len(names)
                    names.append(r.reference_name)
                ridx.append(name_idx[r.reference_name])
            start.append(r.start if r.start is not None else 0)
            seqs.append((r.sequence or "").encode("latin-1"))
            quals.append((r.qual or "").encode("latin-1"))
            cigs.append(parse_cigar(r.cigar) if r.cigar is not None else np.zeros(0, dtype=np.uint32))
            mds.append((r.mismatching_positions or "").encode("latin-1"))

        def cat(chunks, dtype):
            if not chunks:
                return np.zeros(0, dtype=dtype)
            return np.concatenate([np.frombuffer(c, dtype=dtype) if isinstance(c, bytes) else c.astype(dtype)
                                   for c in chunks]) if chunks else np.zeros(0, dtype)

        lens = lambda chunks: np.asarray([len(c) for c in chunks], dtype=np.uint64)
        return RecordBatch(np.asarray(flags, np.uint32), np.asarray(rg, np.int32), np.asarray(ridx, np.int32),
                           names, np.asarray(start, np.int64), _offsets(lens(seqs)), cat(seqs, np.uint8),
                           _offsets(lens(quals)), cat(quals, np.uint8), _offsets(lens(cigs)),
                           cat(cigs, np.uint32), _offsets(lens(mds)), cat(mds, np.uint8))

    def to_records(self) -> List[ADAMRecord]:
        out = []
        for r in range(self.n_reads):
            f = int(self.flags[r])

            def s(off, col):
                return bytes(col[int(off[r]):int(off[r + 1])]).decode("latin-1")

            out.append(ADAMRecord(
                sequence=s(self.seq_offset, self.seq) if f & F_HAS_SEQ else None,
                qual=s(self.qual_offset, self.qual) if f & F_HAS_QUAL else None,
                cigar=cigar_to_text(self.cigar[int(self.cigar_offset[r]):int(self.cigar_offset[r + 1])])
                if f & F_HAS_CIGAR else None,
                start=int(self.start[r]) if f & F_HAS_START else None,
                reference_name=self.ref_names[self.ref_index[r]] if f & F_HAS_REFNAME else None,
                record_group_id=int(self.rg_id[r]) if f & F_HAS_RG else None,
                mismatching_positions=s(self.md_offset, self.md) if f & F_HAS_MD else None,
                read_paired=bool(f & F_PAIRED), read_mapped=bool(f & F_MAPPED),
                read_negative_strand=bool(f & F_NEG_STRAND), second_of_pair=bool(f & F_SECOND_OF_PAIR),
                primary_alignment=bool(f & F_PRIMARY), duplicate_read=bool(f & F_DUPLICATE)))
        return out


# --- SAM ingest (SAMRecordConverter semantics) --------------------------------

def read_sam(path: str) -> RecordBatch:
    """Load a SAM text file the way ``sc.adamLoad`` + ``SAMRecordConverter.convert``
    would (core/rdd/AdamContext.scala:122-137, converters/SAMRecordConverter.scala:26-144)."""
    return RecordBatch.from_records(read_sam_records(path))


def characterize_tags(recs: Iterable[ADAMRecord]) -> dict:
    """Records carrying each optional-field tag, MD excluded
    (AdamRDDFunctions.scala:200-202 adamCharacterizeTags over the converter's
    attributes)."""
    counts: dict = {}
    for r in recs:
        for t in (r.attributes or "").split("\t"):
            if t:
                k = t.split(":", 1)[0]
                counts[k] = counts.get(k, 0) + 1
    return counts


def read_sam_records(path: str) -> List[ADAMRecord]:
    """The ADAMRecords of a SAM text file (SAMRecordConverter semantics)."""
    rg_names: List[str] = []
    sq_names: List[str] = []
    body: List[List[str]] = []
    with open(path, "r", encoding="latin-1") as fh:
        for line in fh:
            line = line.rstrip("\n")
            if not line:
                continue
            if line.startswith("@"):
                f = line.split("\t")
                tags = dict(t.split(":", 1) for t in f[1:] if ":" in t)
                if f[0] == "@RG":
                    rg_names.append(tags["ID"])
                elif f[0] == "@SQ":
                    sq_names.append(tags["SN"])
                continue
            body.append(line.split("\t"))
    # RecordGroupDictionary: readGroupNames.sorted.zipWithIndex
    rg_index = {n: i for i, n in enumerate(sorted(rg_names))}
    recs = []
    for f in body:
        qname, flag, rname, pos, _mapq, cigar, _rnext, _pnext, _tlen, seq, qual = f[:11]
        flag = int(flag)
        tags = {}
        attrs = []
        for t in f[11:]:
            k, typ, v = t.split(":", 2)
            tags[k] = v
            if k != "MD":
                attrs.insert(0, t)
        # getReadString / getBaseQualityString / getCigarString return "*" when
        # absent, and the converter stores those strings as they are
        r = ADAMRecord(read_name=qname, sequence=seq, qual=qual, cigar=cigar)
        if rname != "*" and rname in sq_names:
            r.reference_name = rname
            p = int(pos)
            if p != 0:
                r.start = p - 1
        if flag != 0:  # "We only need to set the flags that are true" (Q2)
            if flag & 0x1:
                r.read_paired = True
                if flag & 0x80:
                    r.second_of_pair = True
            if flag & 0x400:
                r.duplicate_read = True
            if flag & 0x10:
                r.read_negative_strand = True
            if not flag & 0x100:
                r.primary_alignment = True
            if not flag & 0x4:
                r.read_mapped = True
        if "MD" in tags:
            r.mismatching_positions = tags["MD"]
        if "RG" in tags and tags["RG"] in rg_index:
            r.record_group_id = rg_index[tags["RG"]]
        if len(f) > 11:  # samRecord.getAttributes is null without optional fields
            r.attributes = "\t".join(attrs)
        recs.append(r)
    return recs
