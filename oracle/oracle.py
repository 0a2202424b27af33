"""ctypes front-end of the CPU oracle (liboracle.so).  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  See bqsr_oracle.cpp for the reference file:line each function
restates.  Run ``make -C oracle`` (or __graft_entry__.build()) first.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


class Dims(ctypes.Structure):
    _fields_ = [("n_rg", ctypes.c_int32), ("max_len", ctypes.c_int32)]


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError("oracle not built: run `make -C oracle`")
        L = ctypes.CDLL(path)
        vp, i64, i32, dbl = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_double
        L.oracle_pow10cache.restype = dbl
        L.oracle_pow10cache.argtypes = [ctypes.c_int]
        L.oracle_log10.restype = dbl
        L.oracle_log10.argtypes = [dbl]
        L.oracle_error_prob_to_phred.restype = i32
        L.oracle_error_prob_to_phred.argtypes = [dbl]
        L.oracle_table_words.restype = i64
        L.oracle_table_words.argtypes = [Dims]
        L.oracle_sites_create.restype = vp
        L.oracle_sites_create.argtypes = [vp, vp, i32]
        L.oracle_sites_destroy.argtypes = [vp]
        L.oracle_observe.restype = ctypes.c_int
        L.oracle_observe.argtypes = [vp, i64, i64, vp, Dims, vp, vp, vp]
        L.oracle_finalize.restype = vp
        L.oracle_finalize.argtypes = [Dims, vp, dbl, vp]
        L.oracle_final_destroy.argtypes = [vp]
        L.oracle_final_avg.restype = dbl
        L.oracle_final_avg.argtypes = [vp]
        L.oracle_final_global.argtypes = [vp, vp, vp]
        L.oracle_final_group.restype = ctypes.c_int
        L.oracle_final_group.argtypes = [vp, i32, vp, vp]
        L.oracle_shifts.restype = ctypes.c_int
        L.oracle_shifts.argtypes = [vp, i32, i32, i32, i32, vp, vp]
        L.oracle_apply.restype = ctypes.c_int
        L.oracle_apply.argtypes = [vp, i64, i64, vp, vp, vp, vp]
        L.oracle_bqsr.restype = ctypes.c_int
        L.oracle_bqsr.argtypes = [vp, i32, vp, Dims, i32, vp, vp, vp, vp, vp]
        L.oracle_bqsr_fold1.restype = ctypes.c_int
        L.oracle_bqsr_fold1.argtypes = [vp, i32, vp, Dims, i32, vp, vp, vp, vp, vp]
        L.oracle_observe_mt.restype = ctypes.c_int
        L.oracle_observe_mt.argtypes = [vp, i32, vp, Dims, i32, i32, vp, vp, vp]
        L.oracle_apply_mt.restype = ctypes.c_int
        L.oracle_apply_mt.argtypes = [vp, i32, Dims, i32, vp, dbl, vp, vp, vp]
        L.oracle_em_fold.restype = None
        L.oracle_em_fold.argtypes = [vp, i64, i64, vp]
        L.oracle_compare_device_output.restype = i64
        L.oracle_compare_device_output.argtypes = [vp, vp, vp, vp, vp, vp, vp, i64, i32, i32, vp]
        L.oracle_compare_compact_output.restype = i64
        L.oracle_compare_compact_output.argtypes = [vp, vp, vp, vp, vp, vp, i64, i32, vp]
        L.oracle_reference_positions.restype = i64
        L.oracle_reference_positions.argtypes = [vp, ctypes.c_uint64, i64, vp, i64]
        L.oracle_reference_end.restype = i64
        L.oracle_reference_end.argtypes = [vp, ctypes.c_uint64, i64]
        L.oracle_md_runs.restype = i64
        L.oracle_md_runs.argtypes = [vp, ctypes.c_uint64, i64, vp, i64]
        L.oracle_read_covariates.restype = i64
        L.oracle_read_covariates.argtypes = [vp, i64, vp, vp, i64]
        _LIB = L
    return _LIB


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


class OracleError(RuntimeError):
    def __init__(self, code: int, read: int = -1):
        super().__init__("oracle status %d at read %d" % (code, read))
        self.code = code
        self.read = read


class Sites:
    """Known-site table (SnpTable.scala:32-47): contig name -> positions."""

    def __init__(self, table: dict):
        self.contigs = list(table.keys())
        self._arrs = [np.ascontiguousarray(np.asarray(table[c], dtype=np.int64)) for c in self.contigs]
        ptrs = (ctypes.c_void_p * max(1, len(self._arrs)))(*[a.ctypes.data for a in self._arrs])
        ns = np.asarray([len(a) for a in self._arrs] or [0], dtype=np.uint64)
        self._h = lib().oracle_sites_create(ctypes.cast(ptrs, ctypes.c_void_p), _p(ns), len(self._arrs))

    @property
    def handle(self):
        return self._h

    def __del__(self):
        if getattr(self, "_h", None) and _LIB is not None:
            _LIB.oracle_sites_destroy(self._h)
            self._h = None


def dims_for(batch, n_rg: Optional[int] = None, max_len: Optional[int] = None) -> Dims:
    return Dims(n_rg if n_rg is not None else batch.n_rg(), max_len if max_len is not None else batch.max_len())


def table_words(d: Dims) -> int:
    return lib().oracle_table_words(d)


def split_table(d: Dims, words: np.ndarray):
    K = 60 * (d.n_rg - 1) + 128
    cells = 2 * d.max_len + 1 + 21
    touched = words[:K]
    obs = words[K:K + K * cells].reshape(K, cells)
    mm = words[K + K * cells:].reshape(K, cells)
    return touched, obs, mm


def observe(batch, sites: Optional[Sites], d: Dims, r0: int = 0, r1: Optional[int] = None,
            words: Optional[np.ndarray] = None, em: float = 0.0) -> Tuple[np.ndarray, float]:
    """One partition of computeTable: fold reads [r0, r1) from a zero table / 0.0."""
    r1 = batch.n_reads if r1 is None else r1
    cid = batch.contig_ids_for(sites.contigs if sites else None)
    s, keep = batch.c_struct(cid)
    if words is None:
        words = np.zeros(table_words(d), dtype=np.int64)
    emv = ctypes.c_double(em)
    err = ctypes.c_int64(-1)
    st = lib().oracle_observe(ctypes.byref(s), r0, r1, sites.handle if sites else None, d, _p(words),
                              ctypes.byref(emv), ctypes.byref(err))
    if st != 0:
        raise OracleError(st, err.value)
    return words, emv.value


class Final:
    """RecalTable after finalizeTable (RecalTable.scala:117-126)."""

    def __init__(self, d: Dims, words: np.ndarray, em: float):
        self.d = d
        self.words = np.ascontiguousarray(words, dtype=np.int64)
        status = ctypes.c_int(0)
        self._h = lib().oracle_finalize(d, _p(self.words), em, ctypes.byref(status))
        if not self._h:
            raise OracleError(status.value)

    def __del__(self):
        if getattr(self, "_h", None) and _LIB is not None:
            _LIB.oracle_final_destroy(self._h)
            self._h = None

    @property
    def average_reported_error(self) -> float:
        return lib().oracle_final_avg(self._h)

    def global_counts(self) -> Tuple[int, int]:
        o, m = ctypes.c_int64(), ctypes.c_int64()
        lib().oracle_final_global(self._h, ctypes.byref(o), ctypes.byref(m))
        return o.value, m.value

    def group_counts(self, r: int):
        o, m = ctypes.c_int64(), ctypes.c_int64()
        if not lib().oracle_final_group(self._h, r, ctypes.byref(o), ctypes.byref(m)):
            return None
        return o.value, m.value

    def shifts(self, key: int, qual: int, cyc: int, ctx: int):
        sh = np.zeros(4, dtype=np.float64)
        q = ctypes.c_int32()
        st = lib().oracle_shifts(self._h, key, qual, cyc, ctx, _p(sh), ctypes.byref(q))
        if st != 0:
            raise OracleError(st)
        return sh, q.value


def apply(batch, fin: Final, r0: int = 0, r1: Optional[int] = None, out: Optional[np.ndarray] = None,
          out_len: Optional[np.ndarray] = None):
    """applyTable over reads [r0, r1): returns (uint16 chars in qual_offset layout, out_len)."""
    r1 = batch.n_reads if r1 is None else r1
    s, keep = batch.c_struct()
    if out is None:
        out = np.zeros(max(1, int(batch.qual_offset[-1])), dtype=np.uint16)
    if out_len is None:
        out_len = np.zeros(max(1, batch.n_reads), dtype=np.uint32)
    err = ctypes.c_int64(-1)
    st = lib().oracle_apply(ctypes.byref(s), r0, r1, fin._h, _p(out), _p(out_len), ctypes.byref(err))
    if st != 0:
        raise OracleError(st, err.value)
    return out, out_len


def bqsr(batch, sites: Optional[Sites], d: Dims, n_parts: int = 1, nthreads: int = 1, fold1: bool = False):
    """Whole BQSR (observe per partition -> merge in partition order -> finalize
    -> apply) on nthreads std::threads.  Returns (words, em, out, out_len).
    fold1: expectedMismatch as if the batch were ONE partition (the table is
    partition-order free; em is folded sequentially over all reads by one more
    thread) -- the job one GPU runs over its shard."""
    cid = batch.contig_ids_for(sites.contigs if sites else None)
    s, keep = batch.c_struct(cid)
    out = np.zeros(max(1, int(batch.qual_offset[-1])), dtype=np.uint16)
    out_len = np.zeros(max(1, batch.n_reads), dtype=np.uint32)
    words = np.zeros(table_words(d), dtype=np.int64)
    em = ctypes.c_double(0.0)
    err = ctypes.c_int64(-1)
    fn = lib().oracle_bqsr_fold1 if fold1 else lib().oracle_bqsr
    st = fn(ctypes.byref(s), n_parts, sites.handle if sites else None, d, nthreads, _p(out),
                           _p(out_len), _p(words), ctypes.byref(em), ctypes.byref(err))
    if st != 0:
        raise OracleError(st, err.value)
    return words, em.value, out, out_len


def observe_mt(batch, sites: Optional[Sites], d: Dims, n_parts: int = 1, nthreads: int = 1,
               fold1: bool = False) -> Tuple[np.ndarray, float]:
    """computeTable over the batch as n_parts partitions on nthreads threads
    (merged in partition order); fold1: expectedMismatch as ONE partition."""
    cid = batch.contig_ids_for(sites.contigs if sites else None)
    s, keep = batch.c_struct(cid)
    words = np.zeros(table_words(d), dtype=np.int64)
    em = ctypes.c_double(0.0)
    err = ctypes.c_int64(-1)
    st = lib().oracle_observe_mt(ctypes.byref(s), n_parts, sites.handle if sites else None, d, nthreads, int(fold1),
                                 _p(words), ctypes.byref(em), ctypes.byref(err))
    if st != 0:
        raise OracleError(st, err.value)
    return words, em.value


def apply_mt(batch, d: Dims, words: np.ndarray, em: float, n_parts: int = 1, nthreads: int = 1):
    """finalizeTable(words, em) then applyTable over the batch on nthreads
    threads: (uint16 chars in qual_offset layout, out_len)."""
    s, keep = batch.c_struct()
    words = np.ascontiguousarray(words, dtype=np.int64)
    out = np.zeros(max(1, int(batch.qual_offset[-1])), dtype=np.uint16)
    out_len = np.zeros(max(1, batch.n_reads), dtype=np.uint32)
    err = ctypes.c_int64(-1)
    st = lib().oracle_apply_mt(ctypes.byref(s), n_parts, d, nthreads, _p(words), em, _p(out), _p(out_len),
                               ctypes.byref(err))
    if st != 0:
        raise OracleError(st, err.value)
    return out, out_len


def em_fold(batch, r0: int = 0, r1: Optional[int] = None, em: float = 0.0) -> float:
    """expectedMismatch of reads [r0, r1) folded as one partition (error-free input)."""
    r1 = batch.n_reads if r1 is None else r1
    s, keep = batch.c_struct()
    v = ctypes.c_double(em)
    lib().oracle_em_fold(ctypes.byref(s), r0, r1, ctypes.byref(v))
    return v.value


def compare_device_output(batch, ref_out: np.ndarray, ref_len: np.ndarray, got_qual: np.ndarray,
                          got_start: np.ndarray, got_len: np.ndarray, exceptions: Optional[np.ndarray] = None,
                          aligned: bool = True, nthreads: int = 8) -> Tuple[int, int]:
    """(number of reads whose recalibrated chars differ, first such read or -1)
    between the oracle's output and the HIP apply output in the packed device
    layout (u8 per slot, per-read start/length, exception list for chars > 0xFF)."""
    s, keep = batch.c_struct()
    ref_out = np.ascontiguousarray(ref_out, dtype=np.uint16)
    ref_len = np.ascontiguousarray(ref_len, dtype=np.uint32)
    got_qual = np.ascontiguousarray(got_qual, dtype=np.uint8)
    got_start = np.ascontiguousarray(got_start).view(np.uint32)
    got_len = np.ascontiguousarray(got_len).view(np.uint32)
    exc = np.ascontiguousarray(exceptions if exceptions is not None else np.zeros(1, np.int64)).view(np.uint64)
    n_exc = 0 if exceptions is None else len(exceptions)
    first = ctypes.c_int64(-1)
    bad = lib().oracle_compare_device_output(ctypes.byref(s), _p(ref_out), _p(ref_len), _p(got_qual), _p(got_start),
                                             _p(got_len), _p(exc), n_exc, int(aligned), nthreads,
                                             ctypes.byref(first))
    return int(bad), int(first.value)


def compare_compact_output(batch, ref_out: np.ndarray, ref_len: np.ndarray, got_chars: np.ndarray,
                           got_off: np.ndarray, exceptions: Optional[np.ndarray] = None,
                           nthreads: int = 8) -> Tuple[int, int]:
    """compare_device_output for the compacted streamed outputs (chars at
    u32 offsets per read, exceptions keyed by position in the chars)."""
    s, keep = batch.c_struct()
    ref_out = np.ascontiguousarray(ref_out, dtype=np.uint16)
    ref_len = np.ascontiguousarray(ref_len, dtype=np.uint32)
    got_chars = np.ascontiguousarray(got_chars, dtype=np.uint8)
    if got_chars.size == 0:
        got_chars = np.zeros(1, np.uint8)
    got_off = np.ascontiguousarray(got_off).view(np.uint32)
    exc = np.ascontiguousarray(exceptions if exceptions is not None else np.zeros(1, np.int64)).view(np.uint64)
    n_exc = 0 if exceptions is None else len(exceptions)
    first = ctypes.c_int64(-1)
    bad = lib().oracle_compare_compact_output(ctypes.byref(s), _p(ref_out), _p(ref_len), _p(got_chars), _p(got_off),
                                              _p(exc), n_exc, nthreads, ctypes.byref(first))
    return int(bad), int(first.value)


def reference_positions(cigar: Sequence[int], start: int):
    c = np.ascontiguousarray(np.asarray(cigar, dtype=np.uint32))
    if c.size == 0:
        c = np.zeros(1, dtype=np.uint32)
        n = 0
    else:
        n = len(cigar)
    out = np.zeros(100000, dtype=np.int64)
    k = lib().oracle_reference_positions(_p(c), n, start, _p(out), len(out))
    if k < 0:
        raise OracleError(int(-k))
    return [None if v == np.iinfo(np.int64).min else int(v) for v in out[:k]]


def reference_end(cigar: Sequence[int], start: int) -> int:
    c = np.ascontiguousarray(np.asarray(list(cigar) or [0], dtype=np.uint32))
    return lib().oracle_reference_end(_p(c), len(cigar), start)


def md_runs(md: str, start: int):
    b = np.frombuffer(md.encode("latin-1") or b"\0", dtype=np.uint8).copy()
    out = np.zeros(20000, dtype=np.int64)
    k = lib().oracle_md_runs(_p(b), len(md), start, _p(out), len(out))
    if k < 0:
        raise OracleError(int(-k))
    return [(int(out[2 * i]), int(out[2 * i + 1])) for i in range(k)]


def read_covariates(batch, r: int, sites: Optional[Sites] = None):
    """Per-base BaseCovariates of read r: list of (qualByRG, cycle, context, qual, isMismatch, isMasked)."""
    cid = batch.contig_ids_for(sites.contigs if sites else None)
    s, keep = batch.c_struct(cid)
    out = np.zeros(6 * 70000, dtype=np.int32)
    k = lib().oracle_read_covariates(ctypes.byref(s), r, sites.handle if sites else None, _p(out), 70000)
    if k < 0:
        raise OracleError(int(-k), r)
    o = out[:6 * k].reshape(k, 6)
    return [(int(a), int(b), int(c), int(d), bool(e), bool(f)) for a, b, c, d, e, f in o]


def pow10cache(q: int) -> float:
    return lib().oracle_pow10cache(q)


def error_prob_to_phred(p: float) -> int:
    return lib().oracle_error_prob_to_phred(p)
