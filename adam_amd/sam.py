"""SAM text through the device (include/adam_sam.h): ingest, MarkDuplicates,
and the recalibrated text back out.

``SamText(data)`` parses a whole SAM file on the device with the
SAMRecordConverter semantics ``records.read_sam`` restates
(core/converters/SAMRecordConverter.scala:26-144); ``.batch()`` returns the
columns as a RecordBatch (byte-identical to ``read_sam``);
``.mark_duplicates()`` runs MarkDuplicates (core/rdd/MarkDuplicates.scala:24-111)
over the records and updates their duplicateRead bits; ``.rewrite(job)``
puts a ResidentJob's recalibrated quality strings into the records' QUAL
fields (the output path, core/rdd/AdamRDDFunctions.scala:37-56, as SAM text).
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence

import numpy as np

from . import _capi, bqsr
from ._capi import check
from .records import RecordBatch


class SamCounts(ctypes.Structure):
    _fields_ = [("n_reads", ctypes.c_int64), ("seq_bytes", ctypes.c_int64), ("qual_bytes", ctypes.c_int64),
                ("cigar_ops", ctypes.c_int64), ("md_bytes", ctypes.c_int64), ("text_bytes", ctypes.c_int64),
                ("n_ref_names", ctypes.c_int32), ("n_read_groups", ctypes.c_int32)]


class SamColumns(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("flags", "rg_id", "ref_index", "start", "seq_offset", "seq",
                                               "qual_offset", "qual", "cigar_offset", "cigar", "md_offset", "md")]


class DupReads(ctypes.Structure):
    _fields_ = [("n_reads", ctypes.c_int64), ("read_name", ctypes.c_void_p), ("library", ctypes.c_void_p),
                ("flags", ctypes.c_void_p), ("mate_mapped", ctypes.c_void_p), ("rg_id", ctypes.c_void_p),
                ("reference_id", ctypes.c_void_p), ("start", ctypes.c_void_p), ("qual_offset", ctypes.c_void_p),
                ("qual", ctypes.c_void_p), ("cigar_offset", ctypes.c_void_p), ("cigar", ctypes.c_void_p)]


_bound = False


def _lib():
    global _bound
    L = _capi.lib()
    if not _bound:
        vp, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
        pp = ctypes.POINTER(ctypes.c_void_p)
        sig = {
            "bqsr_sam_parse": (ctypes.c_int, [vp, ctypes.c_char_p, i64, vp, pp]),
            "bqsr_bam_parse": (ctypes.c_int, [vp, ctypes.c_char_p, i64, vp, pp]),
            "bqsr_sam_destroy": (None, [vp]),
            "bqsr_sam_get_counts": (ctypes.c_int, [vp, ctypes.POINTER(SamCounts)]),
            "bqsr_sam_ref_name": (ctypes.c_char_p, [vp, i32]),
            "bqsr_sam_device_columns": (ctypes.c_int, [vp, ctypes.POINTER(SamColumns)]),
            "bqsr_sam_download": (ctypes.c_int, [vp, ctypes.POINTER(SamColumns)]),
            "bqsr_sam_rewrite_quals": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, i64, vp]),
            "bqsr_sam_text_download": (ctypes.c_int, [vp, ctypes.c_char_p]),
            "bqsr_mark_duplicates": (ctypes.c_int, [ctypes.POINTER(DupReads), vp]),
            "bqsr_sam_mark_duplicates": (ctypes.c_int, [vp, ctypes.POINTER(i64)]),
            "bqsr_sam_batch_create": (ctypes.c_int, [vp, vp, vp, i32, vp, pp]),
            "bqsr_dup_set_create": (ctypes.c_int, [vp, i64, pp]),
            "bqsr_dup_set_add": (ctypes.c_int, [vp, vp]),
            "bqsr_dup_set_finish": (ctypes.c_int, [vp, ctypes.POINTER(i64)]),
            "bqsr_dup_set_apply": (ctypes.c_int, [vp, i64, vp, ctypes.POINTER(i64)]),
            "bqsr_dup_set_destroy": (None, [vp]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _bound = True
    return L


class SamText:
    """A SAM file parsed into device columns (bqsr_sam)."""

    def __init__(self, data: bytes, ctx: Optional[bqsr.Context] = None, stream=None, bam: bool = False):
        """data: SAM text, or BAM bytes (BGZF) with bam=True -- the same
        columns either way (bqsr_bam_parse; a BAM has no text to rewrite)."""
        self.L = _lib()
        self.ctx = ctx or bqsr.Context.get(0)
        self.h = ctypes.c_void_p()
        self.bam = bam
        parse = self.L.bqsr_bam_parse if bam else self.L.bqsr_sam_parse
        # a uint8 numpy array (e.g. a view of an mmap) is passed by address
        src = ctypes.c_char_p(data.ctypes.data) if isinstance(data, np.ndarray) and data.size else data
        if isinstance(src, np.ndarray):
            src = b""
        check(parse(self.ctx.handle, src, len(data), stream, ctypes.byref(self.h)))

    @classmethod
    def read(cls, path: str, ctx: Optional[bqsr.Context] = None) -> "SamText":
        """A .sam or .bam file (BAM by its BGZF magic)."""
        with open(path, "rb") as fh:
            data = fh.read()
        return cls(data, ctx, bam=data[:4] == b"\x1f\x8b\x08\x04")

    def counts(self) -> SamCounts:
        c = SamCounts()
        check(self.L.bqsr_sam_get_counts(self.h, ctypes.byref(c)))
        return c

    def ref_names(self) -> List[str]:
        c = self.counts()
        return [self.L.bqsr_sam_ref_name(self.h, i).decode("latin-1") for i in range(c.n_ref_names)]

    def batch(self) -> RecordBatch:
        """The columns on the host, as records.read_sam builds them."""
        c = self.counts()
        n = c.n_reads
        a = dict(flags=np.zeros(n, np.uint32), rg_id=np.zeros(n, np.int32), ref_index=np.zeros(n, np.int32),
                 start=np.zeros(n, np.int64), seq_offset=np.zeros(n + 1, np.uint64),
                 seq=np.zeros(c.seq_bytes, np.uint8), qual_offset=np.zeros(n + 1, np.uint64),
                 qual=np.zeros(c.qual_bytes, np.uint8), cigar_offset=np.zeros(n + 1, np.uint64),
                 cigar=np.zeros(c.cigar_ops, np.uint32), md_offset=np.zeros(n + 1, np.uint64),
                 md=np.zeros(c.md_bytes, np.uint8))
        cols = SamColumns(**{k: (v.ctypes.data if v.size else None) for k, v in a.items()})
        check(self.L.bqsr_sam_download(self.h, ctypes.byref(cols)))
        return RecordBatch(a["flags"], a["rg_id"], a["ref_index"], self.ref_names(), a["start"], a["seq_offset"],
                           a["seq"], a["qual_offset"], a["qual"], a["cigar_offset"], a["cigar"], a["md_offset"],
                           a["md"])

    def device_batch(self, contigs: Optional[Sequence[str]] = None, stream=None) -> ctypes.c_void_p:
        """The records as a BQSR batch packed on the device
        (bqsr_sam_batch_create; the caller owns the returned bqsr_batch*).
        contigs: the SnpTable's contig names (None: no known sites)."""
        names = self.ref_names()
        from .records import CONTIG_UNKNOWN
        lut = np.full(max(1, len(names)), CONTIG_UNKNOWN, np.int32)
        if contigs:
            pos = {c: i for i, c in enumerate(contigs)}
            for i, nm in enumerate(names):
                lut[i] = pos.get(nm, lut[i])
        bh = ctypes.c_void_p()
        check(self.L.bqsr_sam_batch_create(self.ctx.handle, self.h, lut.ctypes.data, len(names), stream,
                                           ctypes.byref(bh)))
        return bh

    def mark_duplicates(self) -> int:
        """MarkDuplicates over the records (their duplicateRead bits updated); returns the duplicate count."""
        n = ctypes.c_int64()
        check(self.L.bqsr_sam_mark_duplicates(self.h, ctypes.byref(n)))
        return int(n.value)

    def rewrite(self, job=None) -> None:
        """The output text: every record's QUAL field replaced by the
        recalibrated string a ResidentJob (adam_amd/job.py) built from this
        parse's batch() (kept when job is None); FLAG 0x400 following
        MarkDuplicates when it ran."""
        if job is None:
            check(self.L.bqsr_sam_rewrite_quals(self.ctx.handle, self.h, None, None, None, None, None, 0, None))
            return
        p = job._ptr
        check(self.L.bqsr_sam_rewrite_quals(self.ctx.handle, self.h, job.bh, p(job.out_qual), p(job.out_start),
                                            p(job.out_len), p(job.exc), job.n_exc, job.sp))

    def text(self) -> bytes:
        n = self.counts().text_bytes
        buf = ctypes.create_string_buffer(max(1, n))
        check(self.L.bqsr_sam_text_download(self.h, buf))
        return buf.raw[:n]

    def close(self):
        if self.h:
            self.L.bqsr_sam_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DupSet:
    """MarkDuplicates across the partitions of one input (bqsr_dup_set):
    add() every partition's parse in input order, finish(), then apply(i,
    parse) to a re-parse of partition i."""

    def __init__(self, ctx: Optional[bqsr.Context] = None, reads_hint: int = 0):
        self.L = _lib()
        self.ctx = ctx or bqsr.Context.get(0)
        self.h = ctypes.c_void_p()
        check(self.L.bqsr_dup_set_create(self.ctx.handle, int(reads_hint), ctypes.byref(self.h)))
        self.parts = 0

    def add(self, sam: SamText) -> int:
        check(self.L.bqsr_dup_set_add(self.h, sam.h))
        self.parts += 1
        return self.parts - 1

    def finish(self) -> int:
        n = ctypes.c_int64()
        check(self.L.bqsr_dup_set_finish(self.h, ctypes.byref(n)))
        return int(n.value)

    def apply(self, part: int, sam: SamText) -> int:
        n = ctypes.c_int64()
        check(self.L.bqsr_dup_set_apply(self.h, int(part), sam.h, ctypes.byref(n)))
        return int(n.value)

    def close(self):
        if self.h:
            self.L.bqsr_dup_set_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def mark_duplicates(read_name: Sequence[Optional[str]], library: Sequence[Optional[str]], flags, mate_mapped,
                    rg_id, reference_id, start, qual_offset, qual, cigar_offset, cigar) -> np.ndarray:
    """bqsr_mark_duplicates over host columns (no device needed): the
    duplicateRead value MarkDuplicates gives each read."""
    L = _lib()
    n = len(flags)
    names = [None if s is None else s.encode("latin-1") for s in read_name]
    libs = [None if s is None else s.encode("latin-1") for s in library]
    name_a = (ctypes.c_char_p * max(1, n))(*names) if n else (ctypes.c_char_p * 1)()
    lib_a = (ctypes.c_char_p * max(1, n))(*libs) if n else (ctypes.c_char_p * 1)()
    arrs = dict(flags=np.ascontiguousarray(flags, np.uint32), mate_mapped=np.ascontiguousarray(mate_mapped, np.uint8),
                rg_id=np.ascontiguousarray(rg_id, np.int32), reference_id=np.ascontiguousarray(reference_id, np.int32),
                start=np.ascontiguousarray(start, np.int64), qual_offset=np.ascontiguousarray(qual_offset, np.uint64),
                qual=np.ascontiguousarray(qual, np.uint8), cigar_offset=np.ascontiguousarray(cigar_offset, np.uint64),
                cigar=np.ascontiguousarray(cigar, np.uint32))
    keep = {k: (v if v.size else np.zeros(1, v.dtype)) for k, v in arrs.items()}
    R = DupReads(n, ctypes.cast(name_a, ctypes.c_void_p), ctypes.cast(lib_a, ctypes.c_void_p),
                 *[keep[k].ctypes.data for k in ("flags", "mate_mapped", "rg_id", "reference_id", "start",
                                                  "qual_offset", "qual", "cigar_offset", "cigar")])
    dup = np.zeros(max(1, n), np.uint8)
    check(L.bqsr_mark_duplicates(ctypes.byref(R), dup.ctypes.data))
    return dup[:n].astype(bool)
