"""ADAM's own storage: ADAMRecord Parquet in and out.

The reference stores reads as Avro-Parquet ADAMRecords
(adam-format/src/main/resources/avro/adam.avdl:4-68) and loads them with
``adamLoad`` -> ``adamParquetLoad`` (core/rdd/AdamContext.scala:139-161,
318-331), optionally with an Avro projection (AvroParquetInputFormat.
setRequestedProjection, :150; core/projections/Projection.scala:10-34 over
ADAMRecordField.scala:28-71); ``adamSave`` writes them back
(core/rdd/AdamRDDFunctions.scala:37-56).

Here the Parquet pages are decoded by Arrow's C++ reader on host threads --
they come out columnar already: a string column is an offsets buffer and one
byte buffer, the ``bqsr_records`` layout itself -- and only the columns BQSR
reads are requested (:data:`BQSR_PROJECTION`).  The conversion to a
:class:`RecordBatch` is vectorized (flags from the boolean columns, CIGAR
strings to BAM elements with TextCigarCodec's rules in numpy); the batch then
goes to the device like a SAM or BAM parse.

Semantics kept: an Avro null is "field absent" (the HAS_* bits, the
reference's NPEs / NullPointer paths); strings are UTF-8 in Parquet and Java
strings in the reference (UTF-16 code units: a char beyond the BMP is a
surrogate pair), so a qual char c enters as the byte c & 0xFF (BQSR uses
``(c - 33).toByte``, which only sees those 8 bits) and a sequence or MD char
above 0xFF as the byte 0xFF (no base, no MD digit or letter).  A null
boolean is read as false (the reference unboxes it: an NPE -- parity
unpinned, as is every comparison against files ADAM itself wrote: the
reference cannot run here, so the reader is checked against its own writer
and the SAM fixtures' columns).
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .records import (CigarParseError, F_DUPLICATE, F_HAS_CIGAR, F_HAS_MD, F_HAS_QUAL, F_HAS_REFNAME, F_HAS_RG,
                      F_HAS_SEQ, F_HAS_START, F_MAPPED, F_NEG_STRAND, F_PAIRED, F_PRIMARY, F_SECOND_OF_PAIR,
                      RecordBatch, cigar_to_text)

# the ADAMRecord fields BQSR reads (RecalibrateBaseQualities, ReadCovariates, RichADAMRecord, MdTag)
BQSR_PROJECTION = ("referenceName", "start", "sequence", "qual", "cigar", "recordGroupId", "mismatchingPositions",
                   "readPaired", "readMapped", "readNegativeStrand", "secondOfPair", "primaryAlignment",
                   "duplicateRead")
# ... and MarkDuplicates (MarkDuplicates.scala:24-111, SingleReadBucket, ReferencePositionPair)
MARKDUP_PROJECTION = ("readName", "recordGroupLibrary", "mateMapped", "referenceId")

_BOOL_BITS = (("readPaired", F_PAIRED), ("readMapped", F_MAPPED), ("readNegativeStrand", F_NEG_STRAND),
              ("secondOfPair", F_SECOND_OF_PAIR), ("primaryAlignment", F_PRIMARY), ("duplicateRead", F_DUPLICATE))

_CIGAR_OP = np.full(256, -1, dtype=np.int64)
for _i, _c in enumerate("MIDNSHP=X"):
    _CIGAR_OP[ord(_c)] = _i


def _pa():
    import pyarrow as pa
    import pyarrow.compute as pc
    import pyarrow.parquet as pq
    return pa, pc, pq


def _string_column(col, kind: str) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """(present, offsets u64 [n+1], bytes u8) of a nullable string column;
    kind 'qual' / 'seq' / 'md' decides how chars above 0x7F become bytes."""
    pa, pc, _ = _pa()
    present = np.asarray(pc.is_valid(col).to_numpy(zero_copy_only=False), dtype=bool)
    arr = pc.fill_null(col, "").cast(pa.large_binary())
    if isinstance(arr, pa.ChunkedArray):
        arr = arr.combine_chunks()
    n = len(arr)
    bufs = arr.buffers()
    off = np.frombuffer(bufs[1], dtype=np.int64, count=arr.offset + n + 1)[arr.offset:] if n else np.zeros(1, np.int64)
    data = np.frombuffer(bufs[2], dtype=np.uint8) if bufs[2] is not None else np.zeros(0, np.uint8)
    data = data[int(off[0]):int(off[-1])]
    off = (off - off[0]).astype(np.uint64)
    if data.size and int(data.max()) >= 0x80:  # UTF-8 beyond ASCII: one byte per Java char, rebuilt per string
        units = [np.frombuffer(bytes(data[int(off[r]):int(off[r + 1])]).decode("utf-8").encode("utf-16-le"), "<u2")
                 for r in range(n)]  # Java chars: UTF-16 code units (surrogate pairs beyond the BMP)
        if kind == "qual":
            enc = [(u & 0xFF).astype(np.uint8).tobytes() for u in units]
        else:
            enc = [np.minimum(u, 0xFF).astype(np.uint8).tobytes() for u in units]
        lens = np.fromiter((len(b) for b in enc), dtype=np.uint64, count=n)
        off = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum(lens, out=off[1:])
        data = np.frombuffer(b"".join(enc), dtype=np.uint8)
    return present, off, np.ascontiguousarray(data)


def parse_cigars(present: np.ndarray, off: np.ndarray, data: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """CIGAR strings (offsets / bytes) -> (element offsets [n+1], BAM elements
    len << 4 | op), samtools TextCigarCodec.decode's rules vectorized: "*" is
    the empty CIGAR, every op is preceded by 1..9 digits (a length below
    2^28), a string ends with an op, ops are MIDNSHP=X.  Raises
    CigarParseError as records.parse_cigar does."""
    n = len(off) - 1
    lens = np.diff(off.astype(np.int64))
    first = data[np.minimum(off[:-1].astype(np.int64), data.size - 1)] if data.size else np.zeros(n, np.uint8)
    star = (lens == 1) & (first == ord("*"))
    use = present & ~star & (lens > 0)
    d = data.astype(np.int64)
    isdig = (d >= 48) & (d <= 57)
    owner = np.repeat(np.arange(n), lens)  # read of each byte
    keep = use[owner] if owner.size else np.zeros(0, bool)
    pos = np.nonzero(~isdig & keep)[0]  # op bytes of the parsed strings
    if np.any(_CIGAR_OP[d[pos]] < 0):
        raise CigarParseError("Malformed CIGAR string (bad op)")
    rd = owner[pos]
    seg0 = np.maximum(np.concatenate([[-1], pos[:-1]]) + 1, off[:-1].astype(np.int64)[rd]) if pos.size else pos
    nd = pos - seg0
    if np.any(nd < 1) or np.any(nd > 9):
        raise CigarParseError("Malformed CIGAR string (op without a length, or length too long)")
    # every parsed string ends with an op
    last = off[1:].astype(np.int64) - 1
    if np.any(isdig[last[use]]):
        raise CigarParseError("Malformed CIGAR string (ends in a digit)")
    val = np.zeros(pos.size, dtype=np.int64)
    for k in range(1, 10):
        m = nd >= k
        val[m] += (d[pos[m] - k] - 48) * (10 ** (k - 1))
    if np.any(val >= (1 << 28)):
        raise CigarParseError("CIGAR element too long")
    elems = ((val << 4) | _CIGAR_OP[d[pos]]).astype(np.uint32)
    counts = np.bincount(rd, minlength=n).astype(np.uint64) if n else np.zeros(0, np.uint64)
    coff = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(counts, out=coff[1:])
    return coff, elems


def table_to_batch(t) -> RecordBatch:
    """An Arrow table of ADAMRecord columns (BQSR_PROJECTION) -> RecordBatch."""
    pa, pc, _ = _pa()
    n = t.num_rows
    names = set(t.column_names)

    def col(name, typ):
        return t.column(name) if name in names else pa.nulls(n, typ)

    flags = np.zeros(n, dtype=np.uint32)
    for name, bit in _BOOL_BITS:
        v = pc.fill_null(col(name, pa.bool_()), False).to_numpy(zero_copy_only=False)
        flags |= np.where(np.asarray(v, dtype=bool), np.uint32(bit), np.uint32(0))
    s_present, s_off, s_data = _string_column(col("sequence", pa.string()), "seq")
    q_present, q_off, q_data = _string_column(col("qual", pa.string()), "qual")
    m_present, m_off, m_data = _string_column(col("mismatchingPositions", pa.string()), "md")
    c_present, c_off, c_data = _string_column(col("cigar", pa.string()), "cigar")
    cig_off, cig = parse_cigars(c_present, c_off, c_data)
    rgc = col("recordGroupId", pa.int32())
    rg_present = np.asarray(pc.is_valid(rgc).to_numpy(zero_copy_only=False), bool)
    rg = np.asarray(pc.fill_null(rgc, 0).to_numpy(zero_copy_only=False), dtype=np.int32)
    stc = col("start", pa.int64())
    st_present = np.asarray(pc.is_valid(stc).to_numpy(zero_copy_only=False), bool)
    start = np.asarray(pc.fill_null(stc, 0).to_numpy(zero_copy_only=False), dtype=np.int64)
    refc = col("referenceName", pa.string())
    ref_present = np.asarray(pc.is_valid(refc).to_numpy(zero_copy_only=False), bool)
    # referenceName -> index in first-appearance order (RecordBatch.ref_names)
    enc = pc.fill_null(refc, "").combine_chunks() if isinstance(refc, pa.ChunkedArray) else pc.fill_null(refc, "")
    dic = enc.dictionary_encode()
    codes = np.asarray(dic.indices.to_numpy(zero_copy_only=False), dtype=np.int64)
    dict_names = dic.dictionary.to_pylist()
    order: Dict[int, int] = {}
    ref_names: List[str] = []
    for c in codes[ref_present]:
        if int(c) not in order:
            order[int(c)] = len(ref_names)
            ref_names.append(dict_names[int(c)])
    remap = np.full(max(1, len(dict_names)), -1, dtype=np.int32)
    for c, i in order.items():
        remap[c] = i
    ref_index = np.where(ref_present, remap[codes] if codes.size else codes, -1).astype(np.int32)
    for present, bit in ((rg_present, F_HAS_RG), (m_present, F_HAS_MD), (q_present, F_HAS_QUAL),
                         (s_present, F_HAS_SEQ), (c_present, F_HAS_CIGAR), (st_present, F_HAS_START),
                         (ref_present, F_HAS_REFNAME)):
        flags |= np.where(present, np.uint32(bit), np.uint32(0))
    return RecordBatch(flags, rg, ref_index, ref_names, start, s_off, s_data, q_off, q_data, cig_off, cig, m_off,
                       m_data)


class _Strings(ctypes.Structure):
    _fields_ = [("offsets", ctypes.c_void_p), ("data", ctypes.c_void_p), ("validity", ctypes.c_void_p)]


class _Chunk(ctypes.Structure):
    _fields_ = [("n_reads", ctypes.c_int64), ("sequence", _Strings), ("qual", _Strings), ("cigar", _Strings),
                ("md", _Strings), ("reference", ctypes.c_void_p), ("reference_validity", ctypes.c_void_p),
                ("start", ctypes.c_void_p), ("start_validity", ctypes.c_void_p), ("record_group", ctypes.c_void_p),
                ("record_group_validity", ctypes.c_void_p), ("bools", ctypes.c_void_p * 6),
                ("bools_validity", ctypes.c_void_p * 6), ("read_name", _Strings), ("reference_id", ctypes.c_void_p),
                ("reference_id_validity", ctypes.c_void_p), ("library", ctypes.c_void_p)]


_arrow_bound = False


def _arrow_lib():
    global _arrow_bound
    from . import _capi
    L = _capi.lib()
    if not _arrow_bound:
        vp, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
        pp = ctypes.POINTER(ctypes.c_void_p)
        sig = {
            "bqsr_arrow_load": (ctypes.c_int, [vp, ctypes.POINTER(_Chunk), i32, vp, pp]),
            "bqsr_arrow_destroy": (None, [vp]),
            "bqsr_arrow_reads": (i64, [vp]),
            "bqsr_arrow_batch_create": (ctypes.c_int, [vp, vp, vp, i32, vp, pp]),
            "bqsr_arrow_qual_prepare": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, i64, vp, ctypes.POINTER(i64)]),
            "bqsr_arrow_qual_column": (ctypes.c_int, [vp, vp, vp, vp]),
            "bqsr_arrow_mark_duplicates": (ctypes.c_int, [vp, vp, ctypes.POINTER(i64)]),
            "bqsr_arrow_flag_bitmap": (ctypes.c_int, [vp, ctypes.c_uint32, vp]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _arrow_bound = True
    return L


class ArrowReads:
    """ADAMRecord columns of an Arrow table on the device (bqsr_arrow,
    include/adam_sam.h): Arrow's buffers uploaded as they are, the parse
    layout built on the device; ``device_batch`` packs them into a BQSR batch
    and ``qual_column`` rebuilds the qual column after apply -- no per-read
    host work on either side."""

    def __init__(self, table, ctx=None, stream=None, markdup: bool = False):
        """markdup: also load MarkDuplicates' columns (readName, referenceId,
        recordGroupLibrary) for ``mark_duplicates``."""
        from . import bqsr
        from ._capi import check
        pa, pc, _ = _pa()
        self.L = _arrow_lib()
        self.ctx = ctx or bqsr.Context.get(0)
        n = table.num_rows
        names = set(table.column_names)
        # referenceName -> indices into one dictionary (its distinct names)
        if "referenceName" in names:
            refc = table.column("referenceName")
            self.ref_names = [v for v in pc.unique(refc).to_pylist() if v is not None]
        else:
            self.ref_names = []
        value_set = pa.array(self.ref_names, pa.string())
        libs = None
        if markdup and "recordGroupLibrary" in names:
            libs = pa.array(sorted(v for v in pc.unique(table.column("recordGroupLibrary")).to_pylist()
                                   if v is not None), pa.string())
        keep = []

        def flat(a):
            if a.offset:
                a = pa.concat_arrays([a])
            keep.append(a)
            return a

        def addr(b):
            return None if b is None else b.address

        chunks = []
        for rb in table.to_batches():
            m = rb.num_rows
            if m == 0:
                continue
            C = _Chunk()
            C.n_reads = m
            for fld, attr in (("sequence", "sequence"), ("qual", "qual"), ("cigar", "cigar"),
                              ("mismatchingPositions", "md")):
                if fld not in names:
                    continue
                a = rb.column(rb.schema.get_field_index(fld))
                if a.type != pa.string():
                    a = a.cast(pa.string())
                a = flat(a)
                b = a.buffers()
                setattr(C, attr, _Strings(addr(b[1]), addr(b[2]) or addr(b[1]), addr(b[0])))
            if "referenceName" in names:
                a = rb.column(rb.schema.get_field_index("referenceName"))
                idx = flat(pc.index_in(a, value_set=value_set).cast(pa.int32()))
                b = idx.buffers()
                C.reference, C.reference_validity = addr(b[1]), addr(b[0])
            for fld, typ, v, vv in (("start", pa.int64(), "start", "start_validity"),
                                    ("recordGroupId", pa.int32(), "record_group", "record_group_validity")):
                if fld in names:
                    a = rb.column(rb.schema.get_field_index(fld))
                    a = flat(a if a.type == typ else a.cast(typ))
                    b = a.buffers()
                    setattr(C, v, addr(b[1]))
                    setattr(C, vv, addr(b[0]))
            for k, (fld, _bit) in enumerate(_BOOL_BITS):
                if fld in names:
                    a = flat(rb.column(rb.schema.get_field_index(fld)))
                    b = a.buffers()
                    C.bools[k], C.bools_validity[k] = addr(b[1]), addr(b[0])
            if markdup:
                if "readName" in names:
                    a = rb.column(rb.schema.get_field_index("readName"))
                    a = flat(a if a.type == pa.string() else a.cast(pa.string()))
                    b = a.buffers()
                    C.read_name = _Strings(addr(b[1]), addr(b[2]) or addr(b[1]), addr(b[0]))
                if "referenceId" in names:
                    a = rb.column(rb.schema.get_field_index("referenceId"))
                    a = flat(a if a.type == pa.int32() else a.cast(pa.int32()))
                    b = a.buffers()
                    C.reference_id, C.reference_id_validity = addr(b[1]), addr(b[0])
                if libs is not None:
                    a = rb.column(rb.schema.get_field_index("recordGroupLibrary"))
                    rank = pc.add(pc.fill_null(pc.index_in(a, value_set=libs), -1).cast(pa.int32()), 1)
                    a = flat(rank.cast(pa.int32()))
                    C.library = addr(a.buffers()[1])
            chunks.append(C)
        arr = (_Chunk * max(1, len(chunks)))(*chunks)
        self.h = ctypes.c_void_p()
        check(self.L.bqsr_arrow_load(self.ctx.handle, arr, len(chunks), stream, ctypes.byref(self.h)))
        del keep
        self.n_reads = n

    def device_batch(self, contigs: Optional[Sequence[str]] = None, stream=None) -> ctypes.c_void_p:
        """A BQSR batch of the reads (the caller owns it)."""
        from ._capi import check
        from .records import CONTIG_UNKNOWN
        lut = np.full(max(1, len(self.ref_names)), CONTIG_UNKNOWN, np.int32)
        if contigs:
            pos = {c: i for i, c in enumerate(contigs)}
            for i, nm in enumerate(self.ref_names):
                lut[i] = pos.get(nm, CONTIG_UNKNOWN)
        bh = ctypes.c_void_p()
        check(self.L.bqsr_arrow_batch_create(self.ctx.handle, self.h, lut.ctypes.data, len(self.ref_names), stream,
                                             ctypes.byref(bh)))
        return bh

    def mark_duplicates(self) -> int:
        """MarkDuplicates over the reads (bqsr_arrow_mark_duplicates; load
        with markdup=True): their duplicateRead bits updated; the count."""
        from ._capi import check
        nd = ctypes.c_int64()
        check(self.L.bqsr_arrow_mark_duplicates(self.ctx.handle, self.h, ctypes.byref(nd)))
        return int(nd.value)

    def flag_column(self, bit: int):
        """The reads' flag bit as a pa.BooleanArray (no nulls)."""
        from ._capi import check
        pa, _, _ = _pa()
        n = self.n_reads
        bm = np.zeros(max(1, (n + 7) // 8), np.uint8)
        check(self.L.bqsr_arrow_flag_bitmap(self.h, int(bit), bm.ctypes.data))
        return pa.Array.from_buffers(pa.bool_(), n, [None, pa.py_buffer(bm)])

    def qual_column(self, job=None):
        """The qual column (pa.StringArray) after a ResidentJob's step over
        this object's batch (job None: the input strings)."""
        from ._capi import check
        pa, _, _ = _pa()
        nb = ctypes.c_int64()
        if job is None:
            check(self.L.bqsr_arrow_qual_prepare(self.ctx.handle, self.h, None, None, None, None, None, 0, None,
                                                 ctypes.byref(nb)))
        else:
            p = job._ptr
            check(self.L.bqsr_arrow_qual_prepare(self.ctx.handle, self.h, job.bh, p(job.out_qual), p(job.out_start),
                                                 p(job.out_len), p(job.exc), job.n_exc, job.sp, ctypes.byref(nb)))
        n = self.n_reads
        off = np.empty(n + 1, np.int32)
        data = np.empty(max(1, nb.value), np.uint8)
        valid = np.empty(max(1, (n + 7) // 8), np.uint8)
        check(self.L.bqsr_arrow_qual_column(self.h, off.ctypes.data, data.ctypes.data, valid.ctypes.data))
        return pa.StringArray.from_buffers(n, pa.py_buffer(off), pa.py_buffer(data[:nb.value]), pa.py_buffer(valid))

    def close(self):
        if self.h:
            self.L.bqsr_arrow_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def read_table(path: str, columns: Optional[Sequence[str]] = None):
    """The ADAMRecord Parquet file (or directory of part files) at `path`, the
    requested columns only (those the file lacks are left out)."""
    _, _, pq = _pa()
    f = pq.ParquetDataset(path)
    have = set(f.schema.names)
    cols = None if columns is None else [c for c in columns if c in have]
    return f.read(columns=cols, use_threads=True)


def read_parquet(path: str) -> RecordBatch:
    """adamLoad with a BQSR projection: the reads of `path` as one RecordBatch."""
    return table_to_batch(read_table(path, BQSR_PROJECTION))


def _strings_of(present: np.ndarray, off: np.ndarray, data: np.ndarray):
    pa, _, _ = _pa()
    n = len(present)
    if n == 0:
        return pa.array([], pa.string())
    arr = pa.LargeStringArray.from_buffers(n, pa.py_buffer(off.astype(np.int64)), pa.py_buffer(data.tobytes()),
                                           pa.py_buffer(np.packbits(present, bitorder="little").tobytes()))
    return arr.cast(pa.string())


def batch_to_table(b: RecordBatch, read_name: Optional[Sequence[Optional[str]]] = None):
    """RecordBatch -> Arrow table of ADAMRecord columns (adam.avdl field names and
    types; HAS_* bits off = null).  Strings are the batch's bytes as Latin-1."""
    pa, _, _ = _pa()
    f = b.flags
    has = lambda bit: (f & bit) != 0

    def strcol(present, off, data):
        if data.size and int(data.max()) >= 0x80:
            strs = [bytes(data[int(off[r]):int(off[r + 1])]).decode("latin-1") if present[r] else None
                    for r in range(len(present))]
            return pa.array(strs, pa.string())
        return _strings_of(present, off, data)

    has_cig = has(F_HAS_CIGAR)
    co = b.cigar_offset.astype(np.int64)
    cig = [cigar_to_text(b.cigar[co[r]:co[r + 1]]) if has_cig[r] else None for r in range(b.n_reads)]
    cols = {
        "referenceName": pa.DictionaryArray.from_arrays(
            pa.array(np.where(has(F_HAS_REFNAME), b.ref_index, 0).astype(np.int32), mask=~has(F_HAS_REFNAME)),
            pa.array(b.ref_names if b.ref_names else [""], pa.string())).cast(pa.string()),
        "start": pa.array(b.start, pa.int64(), mask=~has(F_HAS_START)),
        "readName": pa.array(list(read_name) if read_name is not None else [None] * b.n_reads, pa.string()),
        "sequence": strcol(has(F_HAS_SEQ), b.seq_offset, b.seq),
        "cigar": pa.array(cig, pa.string()),
        "qual": strcol(has(F_HAS_QUAL), b.qual_offset, b.qual),
        "recordGroupId": pa.array(b.rg_id, pa.int32(), mask=~has(F_HAS_RG)),
    }
    for name, bit in _BOOL_BITS:
        cols[name] = pa.array(has(bit), pa.bool_())
    cols["mismatchingPositions"] = strcol(has(F_HAS_MD), b.md_offset, b.md)
    return pa.table(cols)


def write_parquet(b: RecordBatch, path: str, read_name: Optional[Sequence[Optional[str]]] = None) -> None:
    """adamSave of a RecordBatch's ADAMRecord fields (one Parquet file)."""
    _, _, pq = _pa()
    pq.write_table(batch_to_table(b, read_name), path)


def recalibrated_qual_column(parts, n_reads: int):
    """The qual column after BQSR: per read the recalibrated Java chars
    (bqsr.Partition: chars[qo[r] : qo[r] + out_len[r]]), null where the input
    had none; UTF-8 as Avro writes Java strings (chars above 0x7F take 2-3
    bytes, RecalUtil's `toChar` of values beyond Latin-1 included)."""
    pa, _, _ = _pa()
    out: List[Optional[str]] = []
    for p in parts:
        b = p.batch
        has_q = (b.flags & F_HAS_QUAL) != 0
        ch = p.chars
        ascii_only = not ch.size or int(ch.max()) < 0x80
        for r in range(b.n_reads):
            if not has_q[r] and not p.out_len[r]:
                out.append(None)
                continue
            o, ln = int(b.qual_offset[r]), int(p.out_len[r])
            seg = ch[o:o + ln]
            out.append(seg.astype(np.uint8).tobytes().decode("ascii") if ascii_only else "".join(map(chr, seg)))
    assert len(out) == n_reads
    return pa.array(out, pa.string())
