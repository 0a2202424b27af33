"""Host-side mirror of ADAM's BQSR interface over the MI355X C ABI.

Same names, argument meaning and error behaviour as the reference:

  RecalibrateBaseQualities.apply(rdd, dbsnp)   core/rdd/RecalibrateBaseQualities.scala:34-46
  RecalibrateBaseQualities.usable_read         :29-32
  RecalibrateBaseQualities.compute_table       :52-64   (observe, one C call per partition)
  RecalibrateBaseQualities.apply_table         :66-76   (apply, one C call per partition)
  RecalTable (++, finalize_table, deltas)      core/rdd/recalibration/RecalTable.scala
  SnpTable                                     core/models/SnpTable.scala
  adam_bqsr(partitions, dbsnp)                 core/rdd/AdamRDDFunctions.scala:104-107

An "RDD" here is a list of ``RecordBatch`` partitions.  Partition tables are
merged in partition order (the reference merges in Spark task-completion
order).  Every exception the reference would throw surfaces
as ``BQSRError`` with the matching status (``.name``: NULL_RG, MD_PARSE, ...).
All compute runs in libadam_bqsr.so on a HIP device; nothing here computes
covariates on the CPU.
"""
from __future__ import annotations

import contextlib
import ctypes
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

from . import _capi
from ._capi import BQSRError, Dims, check, lib
from .records import (F_DUPLICATE, F_HAS_MD, F_MAPPED, F_PRIMARY, ADAMRecord, RecordBatch)

MAX_REASONABLE_QSCORE = 60  # RecalUtil.Constants, recalibration/RecalUtil.scala:26


class Context:
    """One library context per HIP device (bqsr_context)."""

    _by_device: Dict[int, "Context"] = {}

    def __init__(self, device: int = 0):
        h = ctypes.c_void_p()
        check(lib().bqsr_context_create(device, ctypes.byref(h)))
        self.handle = h
        self.device = device

    @classmethod
    def get(cls, device: int = 0) -> "Context":
        if device not in cls._by_device:
            cls._by_device[device] = Context(device)
        return cls._by_device[device]

    # bqsr_context_tune knobs (include/adam_bqsr.h): layout choices of the
    # batches created afterwards, for tests and A/B runs; None = leave as is
    _KNOBS = {"order": 1, "fronts": 2, "key_major": 3, "bgzf": 5}
    _DEFAULTS = {"order": -1, "fronts": -1, "key_major": 0, "bgzf": 1}

    def tune(self, **knobs) -> Dict[str, int]:
        """Set layout knobs (order: -1 auto / 0 read / 1 read-group buckets;
        fronts: -1 auto / 0 none / f; key_major: 1 / 0; bgzf: 1 device / 0 host
        inflate of BAM input); returns the settings they replace."""
        cur = getattr(self, "_tuned", dict(self._DEFAULTS))
        prev = {}
        for k, v in knobs.items():
            if v is None:
                continue
            if isinstance(v, str):
                v = {"auto": -1, "read": 0, "group": 1}[v]
            check(lib().bqsr_context_tune(self.handle, self._KNOBS[k], int(v)))
            prev[k] = cur[k]
            cur[k] = int(v)
        self._tuned = cur
        return prev

    @contextlib.contextmanager
    def tuned(self, **knobs):
        """tune() for a block, the previous settings restored after it"""
        prev = self.tune(**knobs)
        try:
            yield self
        finally:
            self.tune(**prev)


class SnpTable:
    """Known-site mask (models/SnpTable.scala:12-47): contig -> set of raw VCF POS values."""

    def __init__(self, table: Optional[Dict[str, Iterable[int]]] = None):
        self.table = {k: np.unique(np.asarray(list(v), dtype=np.int64)) for k, v in (table or {}).items()}
        self._handles: Dict[int, ctypes.c_void_p] = {}

    @property
    def contigs(self) -> List[str]:
        return list(self.table.keys())

    @staticmethod
    def from_vcf(path: str) -> "SnpTable":
        """SnpTable.apply(File) (SnpTable.scala:32-47): lines not starting with '#',
        split on tab, (split(0), split(1).toLong).  POS is kept 1-based (quirk Q7)."""
        t: Dict[str, List[int]] = {}
        with open(path, "r", encoding="latin-1") as fh:
            for line in fh:
                line = line.rstrip("\n")
                if line.startswith("#"):
                    continue
                f = line.split("\t")
                t.setdefault(f[0], []).append(int(f[1]))
        return SnpTable(t)

    def handle(self, ctx: Context):
        if ctx.device not in self._handles:
            names = [c.encode() for c in self.contigs]
            arrs = [np.ascontiguousarray(self.table[c]) for c in self.contigs]
            n = len(arrs)
            cnames = (ctypes.c_char_p * max(1, n))(*names)
            cpos = (ctypes.c_void_p * max(1, n))(*[a.ctypes.data for a in arrs])
            cn = np.asarray([len(a) for a in arrs] or [0], dtype=np.uint64)
            h = ctypes.c_void_p()
            check(lib().bqsr_sites_create(ctx.handle, ctypes.cast(cnames, ctypes.c_void_p),
                                          ctypes.cast(cpos, ctypes.c_void_p), cn.ctypes.data, n, ctypes.byref(h)))
            self._handles[ctx.device] = h
        return self._handles[ctx.device]

    def __del__(self):
        L = _capi._lib
        if L is not None:
            for h in getattr(self, "_handles", {}).values():
                L.bqsr_sites_destroy(h)


def dims_of(batches: Sequence[RecordBatch]) -> Dims:
    n_rg = max([b.n_rg() for b in batches] or [1])
    max_len = max([b.max_len() for b in batches] or [1])
    return Dims(n_rg, max_len)


class ErrorCount:
    """ErrorCount (RecalTable.scala:194-215): bases observed / mismatches."""

    def __init__(self, bases_observed: int = 0, mismatches: int = 0):
        self.bases_observed = int(bases_observed)
        self.mismatches = int(mismatches)

    def __add__(self, other: "ErrorCount") -> "ErrorCount":  # ErrorCount.++
        return ErrorCount(self.bases_observed + other.bases_observed, self.mismatches + other.mismatches)

    def get_error_prob(self) -> Optional[float]:
        if self.bases_observed == 0:
            return None
        return max(10.0 ** (-60 / 10.0), self.mismatches / self.bases_observed)

    def __repr__(self):
        return "ErrorCount(%d, %d)" % (self.bases_observed, self.mismatches)


class RecalTable:
    """Dense device-resident RecalTable ([touched K][obs K*(C+X)][mm K*(C+X)] int64)."""

    def __init__(self, dims: Dims, ctx: Optional[Context] = None, expected_mismatch: float = 0.0):
        self.ctx = ctx or Context.get()
        self.dims = Dims(dims.n_rg, dims.max_len)
        h = ctypes.c_void_p()
        check(lib().bqsr_table_create(self.ctx.handle, self.dims, None, ctypes.byref(h)))
        self.handle = h
        self.expected_mismatch = float(expected_mismatch)

    def __del__(self):
        L = _capi._lib
        if L is not None and getattr(self, "handle", None):
            L.bqsr_table_destroy(self.handle)
            self.handle = None

    # geometry
    @property
    def K(self) -> int:
        return 60 * (self.dims.n_rg - 1) + 128

    @property
    def C(self) -> int:
        return 2 * self.dims.max_len + 1

    @property
    def cells(self) -> int:
        return self.C + 21

    def words(self) -> np.ndarray:
        w = np.zeros(lib().bqsr_table_words(self.dims), dtype=np.int64)
        check(lib().bqsr_table_download(self.handle, w.ctypes.data))
        return w

    def set_words(self, w: np.ndarray):
        w = np.ascontiguousarray(w, dtype=np.int64)
        check(lib().bqsr_table_upload(self.handle, w.ctypes.data))

    def counts(self) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """(touched[K], obs[K, cells], mm[K, cells]); cells = cycle slots (c + max_len) then contexts (x + 4)."""
        w = self.words()
        K, cells = self.K, self.cells
        return w[:K], w[K:K + K * cells].reshape(K, cells), w[K + K * cells:].reshape(K, cells)

    def merge(self, other: "RecalTable") -> "RecalTable":
        """``this ++ other`` (RecalTable.scala:90-108): int64 sums, expectedMismatch = this + other."""
        out = RecalTable(self.dims, self.ctx)
        out.set_words(self.words())
        em = ctypes.c_double(self.expected_mismatch)
        check(lib().bqsr_table_merge(out.handle, other.handle, ctypes.byref(em), other.expected_mismatch))
        out.expected_mismatch = em.value
        return out

    def merge_into(self, other: "RecalTable"):
        em = ctypes.c_double(self.expected_mismatch)
        check(lib().bqsr_table_merge(self.handle, other.handle, ctypes.byref(em), other.expected_mismatch))
        self.expected_mismatch = em.value

    def finalize_table(self) -> "FinalizedTable":
        return FinalizedTable(self)


class FinalizedTable:
    """RecalTable after finalizeTable (RecalTable.scala:117-152) plus the device apply tables."""

    def __init__(self, table: RecalTable):
        self.table = table
        h = ctypes.c_void_p()
        check(lib().bqsr_finalize(table.ctx.handle, table.handle, table.expected_mismatch, ctypes.byref(h)))
        self.handle = h
        st = _capi.FinalStats()
        check(lib().bqsr_lut_stats(h, ctypes.byref(st)))
        self.average_reported_error = st.average_reported_error
        self.global_error = st.global_error
        self.global_counts = ErrorCount(st.global_obs, st.global_mm)

    def __del__(self):
        L = _capi._lib
        if L is not None and getattr(self, "handle", None):
            L.bqsr_lut_destroy(self.handle)
            self.handle = None

    def read_group_counts(self, r: int) -> Optional[ErrorCount]:
        o, m = ctypes.c_int64(), ctypes.c_int64()
        k = lib().bqsr_lut_group(self.handle, r, ctypes.byref(o), ctypes.byref(m))
        if k < 0:
            check(_capi.DEVICE)
        return ErrorCount(o.value, m.value) if k == 1 else None

    def get_error_rate_shifts(self, qual_by_rg: int, qual: int, cycle: int, context: int):
        """getErrorRateShifts (RecalTable.scala:147-152) -> ([rg, qual, cycle, context] deltas, new phred)."""
        sh = np.zeros(4, dtype=np.float64)
        q = ctypes.c_int32()
        check(lib().bqsr_lut_shifts(self.handle, qual_by_rg, qual, cycle, context, sh.ctypes.data, ctypes.byref(q)))
        return sh, q.value

    def get_read_group_delta(self, qual_by_rg: int) -> float:
        """getReadGroupDelta (RecalTable.scala:128-131)."""
        # (qualByRG - 1) / 60 in Java truncates toward zero: key 0 -> group 0,
        # keys <= -59 -> group -1 or below, which never exist (MISSING_KEY)
        num = qual_by_rg - 1
        r = num // MAX_REASONABLE_QSCORE if num >= 0 else -((-num) // MAX_REASONABLE_QSCORE)
        ec = self.read_group_counts(r)
        if ec is None:
            raise BQSRError(_capi.MISSING_KEY, "read group %d" % r)
        p = ec.get_error_prob()
        avg = self.average_reported_error
        return (p if p is not None else avg) - avg


class Partition:
    """One partition's recalibrated qualities: Java chars in the input's
    qual_offset layout; read r's new qual string is chars[qo[r] : qo[r] + out_len[r]]."""

    def __init__(self, batch: RecordBatch, chars: np.ndarray, out_len: np.ndarray):
        self.batch = batch
        self.chars = chars
        self.out_len = out_len

    def qual(self, r: int) -> str:
        o = int(self.batch.qual_offset[r])
        return "".join(map(chr, self.chars[o:o + int(self.out_len[r])]))

    def records(self) -> List[ADAMRecord]:
        recs = self.batch.to_records()
        for r, rec in enumerate(recs):
            if rec.qual is not None or self.out_len[r]:
                rec.qual = self.qual(r)
        return recs


class RecalibrateBaseQualities:
    """RecalibrateBaseQualities (core/rdd/RecalibrateBaseQualities.scala:27-77)."""

    def __init__(self, ctx: Optional[Context] = None, dims: Optional[Dims] = None):
        self.ctx = ctx or Context.get()
        self.dims = dims

    @staticmethod
    def usable_read(rec: ADAMRecord) -> bool:
        """readMapped && primaryAlignment && !duplicateRead && mismatchingPositions != null (:29-32)."""
        return rec.read_mapped and rec.primary_alignment and not rec.duplicate_read and \
            rec.mismatching_positions is not None

    @classmethod
    def apply(cls, partitions: Sequence[RecordBatch], dbsnp: Optional[SnpTable] = None,
              ctx: Optional[Context] = None) -> List[Partition]:
        """RecalibrateBaseQualities.apply (:34-46): compute the table over usable reads, then apply it."""
        parts = list(partitions)
        rbq = cls(ctx, dims_of(parts))
        table = rbq.compute_table(parts, dbsnp or SnpTable())
        return rbq.apply_table(table, parts)

    def _records(self, batch: RecordBatch, dbsnp: Optional[SnpTable]):
        return batch.c_struct(batch.contig_ids_for(dbsnp.contigs if dbsnp else None))

    def compute_table(self, partitions: Sequence[RecordBatch], dbsnp: SnpTable) -> RecalTable:
        """computeTable (:52-64): one observe call per partition, each folding
        from a zero table; partition tables merged in order by ``++``."""
        dims = self.dims or dims_of(partitions)
        acc = RecalTable(dims, self.ctx)
        sites = dbsnp.handle(self.ctx) if dbsnp is not None else None
        for batch in partitions:
            s, keep = self._records(batch, dbsnp)
            h = ctypes.c_void_p()
            em = ctypes.c_double(0.0)
            check(lib().bqsr_observe_records(self.ctx.handle, ctypes.byref(s), sites, dims, ctypes.byref(h),
                                             ctypes.byref(em)))
            part = RecalTable.__new__(RecalTable)
            part.ctx, part.dims, part.handle, part.expected_mismatch = self.ctx, dims, h, em.value
            acc.merge_into(part)
        return acc

    def apply_table(self, table: RecalTable, partitions: Sequence[RecordBatch]) -> List[Partition]:
        """applyTable (:66-76): finalize, then recalibrate every eligible read."""
        fin = table.finalize_table()
        out = []
        for batch in partitions:
            s, keep = self._records(batch, None)
            chars = np.zeros(max(1, int(batch.qual_offset[-1])), dtype=np.uint16)
            out_len = np.zeros(max(1, batch.n_reads), dtype=np.uint32)
            check(lib().bqsr_apply_records(self.ctx.handle, ctypes.byref(s), fin.handle, chars.ctypes.data,
                                           out_len.ctypes.data))
            out.append(Partition(batch, chars, out_len))
        return out


def adam_bqsr(partitions: Sequence[RecordBatch], dbsnp: Optional[SnpTable] = None,
              ctx: Optional[Context] = None) -> List[Partition]:
    """AdamRecordRDDFunctions.adamBQSR (core/rdd/AdamRDDFunctions.scala:104-107)."""
    return RecalibrateBaseQualities.apply(partitions, dbsnp, ctx)
