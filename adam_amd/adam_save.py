"""adamSave from the device: ADAMRecord Parquet part files built from a SAM /
BAM parse on the GPU.

The reference's `transform` always ends in ``adamSave``
(adam-cli/.../cli/Transform.scala:95-96 -> core/rdd/AdamRDDFunctions.scala:
37-56): Avro-Parquet ADAMRecords (adam-format/.../avro/adam.avdl:4-68), one
part file per RDD partition, GZIP-compressed by default, dictionary encoding
on.  The records are SAMRecordConverter's (core/converters/
SAMRecordConverter.scala:26-144).

Here the record-level columns come from the device (``bqsr_sam_adam_prepare``
/ ``bqsr_sam_adam_columns``, adam_amd/csrc/adam_out.hip): Arrow offsets,
bytes, validity and flag bitmaps, copied to host memory and wrapped by
pyarrow without a per-record step.  The columns that depend only on the read
group or the @SQ entry are looked up by index from the header
(:class:`HeaderInfo`).  Part files are written by a pool of host threads
while the device builds the next one.
"""
from __future__ import annotations

import ctypes
import os
import re
import shutil
from concurrent.futures import ThreadPoolExecutor
from datetime import datetime, timedelta, timezone
from typing import Dict, List, Optional, Tuple

import numpy as np

from ._capi import check

# adam.avdl:4-68, in order: (name, arrow type name)
ADAM_FIELDS: List[Tuple[str, str]] = [
    ("referenceName", "string"), ("referenceId", "int32"), ("start", "int64"), ("mapq", "int32"),
    ("readName", "string"), ("sequence", "string"), ("mateReference", "string"), ("mateAlignmentStart", "int64"),
    ("cigar", "string"), ("qual", "string"), ("recordGroupName", "string"), ("recordGroupId", "int32"),
    ("readPaired", "bool"), ("properPair", "bool"), ("readMapped", "bool"), ("mateMapped", "bool"),
    ("readNegativeStrand", "bool"), ("mateNegativeStrand", "bool"), ("firstOfPair", "bool"),
    ("secondOfPair", "bool"), ("primaryAlignment", "bool"), ("failedVendorQualityChecks", "bool"),
    ("duplicateRead", "bool"), ("mismatchingPositions", "string"), ("attributes", "string"),
    ("recordGroupSequencingCenter", "string"), ("recordGroupDescription", "string"),
    ("recordGroupRunDateEpoch", "int64"), ("recordGroupFlowOrder", "string"), ("recordGroupKeySequence", "string"),
    ("recordGroupLibrary", "string"), ("recordGroupPredictedMedianInsertSize", "int32"),
    ("recordGroupPlatform", "string"), ("recordGroupPlatformUnit", "string"), ("recordGroupSample", "string"),
    ("mateReferenceId", "int32"), ("referenceLength", "int64"), ("referenceUrl", "string"),
    ("mateReferenceLength", "int64"), ("mateReferenceUrl", "string"),
]
STR_COLS = ("readName", "sequence", "cigar", "qual", "mismatchingPositions", "attributes")  # bqsr_adam_host order
I32_COLS = ("referenceId", "mapq", "mateReferenceId", "recordGroupId")
I64_COLS = ("start", "mateAlignmentStart")
BOOL_COLS = ("readPaired", "properPair", "readMapped", "mateMapped", "readNegativeStrand", "mateNegativeStrand",
             "firstOfPair", "secondOfPair", "primaryAlignment", "failedVendorQualityChecks", "duplicateRead")
# the read group's header fields (SAMReadGroupRecord getters, SAMRecordConverter.scala:123-141)
RG_TAGS = (("recordGroupSequencingCenter", "CN"), ("recordGroupDescription", "DS"), ("recordGroupFlowOrder", "FO"),
           ("recordGroupKeySequence", "KS"), ("recordGroupLibrary", "LB"), ("recordGroupPlatform", "PL"),
           ("recordGroupPlatformUnit", "PU"), ("recordGroupSample", "SM"))


PER_READ_STRINGS = ("readName", "sequence", "qual", "attributes", "mismatchingPositions")
DICT_COLS = [n for n, k in ADAM_FIELDS if n not in PER_READ_STRINGS]
# gzip part files: the per-base strings as literal-only Huffman DEFLATE blocks
# (parquet_gzip.cpp: their letter frequencies are their redundancy)
HUFFMAN_COLS = ("sequence", "qual")
STATS_COLS = [n for n, k in ADAM_FIELDS if n not in PER_READ_STRINGS]


class AdamSizes(ctypes.Structure):
    _fields_ = [("n_reads", ctypes.c_int64), ("str_bytes", ctypes.c_int64 * 6), ("bitmap_words", ctypes.c_int64)]


class AdamHost(ctypes.Structure):
    _fields_ = [("str_offsets", ctypes.c_void_p * 6), ("str_bytes", ctypes.c_void_p * 6),
                ("str_valid", ctypes.c_void_p * 6), ("i32", ctypes.c_void_p * 4), ("i64", ctypes.c_void_p * 2),
                ("int_valid", ctypes.c_void_p * 6), ("bools", ctypes.c_void_p * 11)]


_bound = False


def _lib():
    global _bound
    from . import sam as S
    L = S._lib()
    if not _bound:
        vp, i64 = ctypes.c_void_p, ctypes.c_int64
        L.bqsr_sam_adam_set_quals.restype = ctypes.c_int
        L.bqsr_sam_adam_set_quals.argtypes = [vp, vp, vp, vp, vp, vp, vp, i64, vp]
        L.bqsr_sam_adam_prepare.restype = ctypes.c_int
        L.bqsr_sam_adam_prepare.argtypes = [vp, vp, i64, i64, vp, ctypes.POINTER(AdamSizes)]
        L.bqsr_sam_adam_columns.restype = ctypes.c_int
        L.bqsr_sam_adam_columns.argtypes = [vp, vp, ctypes.POINTER(AdamHost), vp]
        L.bqsr_sam_header_text.restype = ctypes.c_int
        L.bqsr_sam_header_text.argtypes = [vp, ctypes.c_char_p, i64, ctypes.POINTER(i64)]
        L.bqsr_parquet_gzip.restype = ctypes.c_int
        L.bqsr_parquet_gzip.argtypes = [vp, i64, ctypes.c_char_p, ctypes.c_int32, ctypes.c_char_p, ctypes.c_int32,
                                        ctypes.POINTER(i64)]
        L.bqsr_gzip_bytes.restype = ctypes.c_int
        L.bqsr_gzip_bytes.argtypes = [vp, i64, ctypes.c_int32, ctypes.c_int32, vp, i64, ctypes.POINTER(i64)]
        _bound = True
    return L


def _iso8601_epoch_ms(v: str) -> Optional[int]:
    """SAMReadGroupRecord.getRunDate (ISO 8601) -> epoch milliseconds; a
    value without a zone is read as UTC (htsjdk takes the JVM's zone: parity
    unpinned); None when it does not parse."""
    m = re.fullmatch(r"(\d{4})-(\d{2})-(\d{2})(?:[T ](\d{2}):(\d{2})(?::(\d{2})(?:\.(\d{1,3})\d*)?)?"
                     r"(Z|[+-]\d{2}:?\d{2})?)?", v.strip())
    if not m:
        return None
    y, mo, d, hh, mi, ss, ms, tz = m.groups()
    try:
        dt = datetime(int(y), int(mo), int(d), int(hh or 0), int(mi or 0), int(ss or 0),
                      int((ms or "0").ljust(3, "0")) * 1000, tzinfo=timezone.utc)
    except ValueError:
        return None
    if tz and tz != "Z":
        sign = 1 if tz[0] == "+" else -1
        t = tz[1:].replace(":", "")
        dt -= sign * timedelta(hours=int(t[:2]), minutes=int(t[2:]))
    return int(dt.timestamp() * 1000)


class HeaderInfo:
    """The header's @RG and @SQ records, by the ids the device columns carry:
    recordGroupId = the index in the sorted @RG IDs (RecordGroupDictionary.
    scala:36-43, a repeated ID taking its last index), referenceId = the @SQ
    line index (the first line of a name)."""

    def __init__(self, text: str):
        rg_lines: Dict[str, Dict[str, str]] = {}
        rg_ids: List[str] = []
        self.sq: List[Dict[str, str]] = []
        for line in text.split("\n"):
            line = line.rstrip("\r")
            if not line.startswith("@"):
                continue
            f = line.split("\t")
            kv = dict(t.split(":", 1) for t in f[1:] if ":" in t)
            if f[0] == "@RG" and "ID" in kv:
                rg_ids.append(kv["ID"])
                rg_lines[kv["ID"]] = kv  # the last line of an ID
            elif f[0] == "@SQ" and "SN" in kv:
                self.sq.append(kv)
        names = sorted(rg_ids)
        self.rg: List[Optional[Dict[str, str]]] = [None] * len(names)
        for i, nm in enumerate(names):
            if i + 1 < len(names) and names[i + 1] == nm:
                continue
            self.rg[i] = dict(rg_lines[nm], ID=nm)

    def rg_column(self, key: str, kind: str = "str"):
        vals = []
        for r in self.rg:
            v = None if r is None else r.get(key)
            if v is not None and kind == "int":
                try:
                    v = int(v)
                except ValueError:
                    v = None
            elif v is not None and kind == "date":
                v = _iso8601_epoch_ms(v)
            vals.append(v)
        return vals

    def sq_column(self, key: str, kind: str = "str"):
        out = []
        for r in self.sq:
            v = r.get(key)
            if v is not None and kind == "int":
                try:
                    v = int(v)
                except ValueError:
                    v = None
            out.append(v)
        return out


def set_quals(sam, bh=None, out_qual=None, out_start=None, out_len=None, exc=None, n_exc: int = 0, stream=None):
    """The ADAM qual column of `sam` from an apply's device outputs for batch
    bh (bqsr_sam_adam_set_quals: no text rewrite); bh None: the text's."""
    check(_lib().bqsr_sam_adam_set_quals(sam.ctx.handle, sam.h, bh, out_qual, out_start, out_len, exc, n_exc,
                                         stream))


def header_info(sam) -> HeaderInfo:
    L = _lib()
    n = ctypes.c_int64()
    check(L.bqsr_sam_header_text(sam.h, None, 0, ctypes.byref(n)))
    buf = ctypes.create_string_buffer(max(1, n.value))
    check(L.bqsr_sam_header_text(sam.h, buf, n.value, ctypes.byref(n)))
    return HeaderInfo(buf.raw[:n.value].decode("latin-1"))


def schema():
    import pyarrow as pa
    t = {"string": pa.string(), "int32": pa.int32(), "int64": pa.int64(), "bool": pa.bool_()}
    return pa.schema([pa.field(n, t[k], nullable=True) for n, k in ADAM_FIELDS])


def _pinned(nbytes: int) -> np.ndarray:
    """a pinned host block (numpy view of a torch pinned tensor; the view
    keeps the tensor alive)"""
    import torch
    t = torch.empty(max(64, int(nbytes)), dtype=torch.uint8, pin_memory=True)
    return t.numpy()


def adam_table(sam, r0: int, n: int, hdr: HeaderInfo, stream=None):
    """The ADAMRecord table of records [r0, r0 + n) of a parse (SamText), from
    its current text (after ``rewrite``: recalibrated qual, MarkDuplicates'
    flag)."""
    import pyarrow as pa
    L = _lib()
    ctx = sam.ctx
    sz = AdamSizes()
    check(L.bqsr_sam_adam_prepare(ctx.handle, sam.h, r0, n, stream, ctypes.byref(sz)))
    W = sz.bitmap_words
    # every host buffer carved from one pinned block (the D2H copies run at
    # the link's rate; torch's host allocator recycles the block once the
    # part file is written and the table dropped)
    plan = ([(n + 1, np.int32)] * 6 + [(sz.str_bytes[c], np.uint8) for c in range(6)] + [(W, np.uint64)] * 6 +
            [(n, np.int32)] * 4 + [(n, np.int64)] * 2 + [(W, np.uint64)] * 6 + [(W, np.uint64)] * 11)
    sizes = [((max(1, cnt) * np.dtype(dt).itemsize + 63) // 64) * 64 for cnt, dt in plan]
    block = _pinned(sum(sizes))
    pos = [0]

    def buf(count, dtype):
        nb = ((max(1, count) * np.dtype(dtype).itemsize + 63) // 64) * 64
        a = block[pos[0]:pos[0] + nb].view(dtype)[:max(1, count)]
        pos[0] += nb
        return a

    soff = [buf(n + 1, np.int32) for _ in range(6)]
    sbytes = [buf(sz.str_bytes[c], np.uint8) for c in range(6)]
    svalid = [buf(W, np.uint64) for _ in range(6)]
    i32 = [buf(n, np.int32) for _ in range(4)]
    i64 = [buf(n, np.int64) for _ in range(2)]
    ivalid = [buf(W, np.uint64) for _ in range(6)]
    bools = [buf(W, np.uint64) for _ in range(11)]
    H = AdamHost()
    for c in range(6):
        H.str_offsets[c] = soff[c].ctypes.data
        H.str_bytes[c] = sbytes[c].ctypes.data if sz.str_bytes[c] else None
        H.str_valid[c] = svalid[c].ctypes.data
        H.int_valid[c] = ivalid[c].ctypes.data
    for c in range(4):
        H.i32[c] = i32[c].ctypes.data
    for c in range(2):
        H.i64[c] = i64[c].ctypes.data
    for c in range(11):
        H.bools[c] = bools[c].ctypes.data
    check(L.bqsr_sam_adam_columns(ctx.handle, sam.h, ctypes.byref(H), stream))
    pb = lambda a: pa.py_buffer(a)  # noqa: E731 (zero-copy views of the host buffers)
    cols = {}
    for c, name in enumerate(STR_COLS):
        cols[name] = pa.StringArray.from_buffers(n, pb(soff[c]), pb(sbytes[c][:sz.str_bytes[c]]), pb(svalid[c]))
    ints = {}
    for c, name in enumerate(I32_COLS):
        ints[name] = pa.Array.from_buffers(pa.int32(), n, [pb(ivalid[c]), pb(i32[c][:n])])
    for c, name in enumerate(I64_COLS):
        ints[name] = pa.Array.from_buffers(pa.int64(), n, [pb(ivalid[4 + c]), pb(i64[c][:n])])
    cols.update(ints)
    for c, name in enumerate(BOOL_COLS):
        cols[name] = pa.Array.from_buffers(pa.bool_(), n, [None, pb(bools[c])])
    # by index: the @SQ entry of referenceId / mateReferenceId, the @RG record
    # of recordGroupId -- dictionary arrays over the header's values with the
    # index columns as their indices (no per-record copy; Parquet stores them
    # as plain string / int columns, dictionary-encoded)
    src = {"ref": (i32[0], ivalid[0]), "mref": (i32[2], ivalid[2]), "rg": (i32[3], ivalid[3])}
    masks: Dict[Tuple[str, bytes], object] = {}

    def lookup(values, which, typ):
        idx, valid = src[which]
        has = np.asarray([v is not None for v in values], bool)
        if not has.any():
            return pa.nulls(n, typ)
        dic = pa.array([v if v is not None else (0 if typ != pa.string() else "") for v in values], typ)
        if has.all():
            vbuf = pb(valid)
        else:  # entries without the value: null
            key = (which, has.tobytes())
            if key not in masks:
                vb = np.unpackbits(valid.view(np.uint8), count=n, bitorder="little").astype(bool)
                ok = vb & has[np.clip(idx[:n], 0, len(values) - 1)]
                masks[key] = pa.py_buffer(np.packbits(ok, bitorder="little"))
            vbuf = masks[key]
        ind = pa.Array.from_buffers(pa.int32(), n, [vbuf, pb(idx[:n])])
        return pa.DictionaryArray.from_arrays(ind, dic, safe=False)

    sq_name = [r["SN"] for r in hdr.sq]
    sq_len, sq_url = hdr.sq_column("LN", "int"), hdr.sq_column("UR")
    cols["referenceName"] = lookup(sq_name, "ref", pa.string())
    cols["referenceLength"] = lookup(sq_len, "ref", pa.int64())
    cols["referenceUrl"] = lookup(sq_url, "ref", pa.string())
    cols["mateReference"] = lookup(sq_name, "mref", pa.string())
    cols["mateReferenceLength"] = lookup(sq_len, "mref", pa.int64())
    cols["mateReferenceUrl"] = lookup(sq_url, "mref", pa.string())
    cols["recordGroupName"] = lookup(hdr.rg_column("ID"), "rg", pa.string())
    for name, key in RG_TAGS:
        cols[name] = lookup(hdr.rg_column(key), "rg", pa.string())
    cols["recordGroupRunDateEpoch"] = lookup(hdr.rg_column("DT", "date"), "rg", pa.int64())
    cols["recordGroupPredictedMedianInsertSize"] = lookup(hdr.rg_column("PI", "int"), "rg", pa.int32())
    # (the arrays hold their host buffers: pa.py_buffer keeps each numpy array alive)
    return pa.table([cols[name] for name, _ in ADAM_FIELDS], names=[name for name, _ in ADAM_FIELDS])


_PART_FILE = re.compile(r"^(part-r-\d{5}\.parquet|_SUCCESS|\.?part-r-\d{5}\.parquet\.crc|\._SUCCESS\.crc)$")


def is_adam_output(path: str) -> bool:
    """A directory holding nothing but adamSave part files (and _SUCCESS):
    what AdamWriter may replace when asked to overwrite."""
    if os.path.islink(path) or not os.path.isdir(path):
        return False
    for e in os.scandir(path):
        if not (e.is_file(follow_symlinks=False) and _PART_FILE.match(e.name)):
            return False
    return True


class AdamWriter:
    """adamSave's output: a directory of part files, written by host threads
    as the tables arrive (``OUT.partial`` renamed to ``OUT`` on ``close``)."""

    def __init__(self, path: str, compression: str = "gzip", threads: Optional[int] = None,
                 overwrite: bool = False, native_gzip: bool = True):
        self.path = path
        self.tmp = path + ".partial"
        # adamSave goes through Hadoop's FileOutputFormat, which refuses an
        # existing output path (FileAlreadyExistsException).  overwrite=True
        # replaces only what looks like an earlier adamSave output.
        for p in (path, self.tmp):
            if os.path.lexists(p):
                if not overwrite:
                    raise FileExistsError("output path %s already exists" % p)
                if not is_adam_output(p):
                    raise FileExistsError("refusing to replace %s: not an ADAM part-file directory" % p)
        if os.path.exists(self.tmp):
            shutil.rmtree(self.tmp)
        os.makedirs(self.tmp)
        self.overwrite = overwrite
        self.compression = None if compression in (None, "none") else compression
        # gzip at zlib's default level 6 (parquet-mr's GzipCodec through Hadoop;
        # Arrow's own default is 9)
        self.level = 6 if self.compression == "gzip" else None
        # (native_gzip False: Arrow's own zlib writer, for comparisons)
        self.native_gzip = native_gzip
        self.gzip_threads = 2
        nth = threads or max(1, min(16, len(os.sched_getaffinity(0))))
        self.pool = ThreadPoolExecutor(max_workers=nth)
        self.futures = []
        self.parts = 0
        self.rows = 0

    def _write(self, table, name):
        import pyarrow as pa
        import pyarrow.parquet as pq
        # dictionary pages and statistics where they pay: not for the
        # per-read strings (names, bases, quals, tags), whose dictionaries
        # overflow and whose min / max no reader filters on
        path = os.path.join(self.tmp, name)
        if self.compression != "gzip" or not self.native_gzip:
            pq.write_table(table, path, compression=self.compression, compression_level=self.level,
                           use_dictionary=DICT_COLS, write_statistics=STATS_COLS, store_schema=False)
            return
        # gzip: Arrow encodes the pages uncompressed in memory, the library
        # writes them gzip-compressed (bqsr_parquet_gzip: quals and bases as
        # literal-only Huffman blocks, the rest at zlib's level 6)
        buf = pa.BufferOutputStream()
        pq.write_table(table, buf, compression="none", use_dictionary=DICT_COLS, write_statistics=STATS_COLS,
                       store_schema=False)
        data = buf.getvalue()
        n = ctypes.c_int64()
        check(_lib().bqsr_parquet_gzip(ctypes.c_void_p(data.address), data.size, path.encode(), self.level,
                                       b",".join(c.encode() for c in HUFFMAN_COLS), self.gzip_threads,
                                       ctypes.byref(n)))

    def add(self, table):
        name = "part-r-%05d.parquet" % self.parts
        self.parts += 1
        self.rows += table.num_rows
        self.futures.append(self.pool.submit(self._write, table, name))
        if len(self.futures) > 64:  # bound the tables held in memory
            self.futures.pop(0).result()

    def emit(self, sam, part_reads: int = 1 << 20, stream=None):
        """Every record of a parse, part_reads records per part file."""
        hdr = header_info(sam)
        n = sam.counts().n_reads
        for r0 in range(0, max(n, 1), max(1, part_reads)):
            self.add(adam_table(sam, r0, min(part_reads, n - r0) if n else 0, hdr, stream))

    def close(self, ok: bool = True):
        try:
            for f in self.futures:
                f.result()
        finally:
            self.pool.shutdown(wait=True)
        if ok:
            open(os.path.join(self.tmp, "_SUCCESS"), "wb").close()
            if os.path.lexists(self.path):
                # (checked at __init__; checked again: the path may have appeared since)
                if not (self.overwrite and is_adam_output(self.path)):
                    shutil.rmtree(self.tmp, ignore_errors=True)
                    raise FileExistsError("output path %s already exists" % self.path)
                shutil.rmtree(self.path)
            os.replace(self.tmp, self.path)
        else:
            shutil.rmtree(self.tmp, ignore_errors=True)
