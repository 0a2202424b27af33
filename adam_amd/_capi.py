"""ctypes binding of libadam_bqsr.so (include/adam_bqsr.h).

The HIP library is the only compute path: importing a function that needs it
raises ``NativeLibraryMissing`` when the in-tree build is absent -- there is no
CPU fallback.  Build with ``python -c "import __graft_entry__ as g; g.build()"``.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# ADAM_BQSR_LIB: an instrumented build of the same sources (tools/*.sh profiling)
LIB_PATH = os.environ.get("ADAM_BQSR_LIB") or os.path.join(_HERE, "libadam_bqsr.so")

BQSR_OK = 0
STAGE_RESET, STAGE_KERNEL, STAGE_FOLD, STAGE_PREP, STAGE_LUT, STAGE_NO_LUT = 1, 2, 4, 8, 16, 32
STATUS_NAMES = ["OK", "NULL_RG", "MD_PARSE", "CIGAR_SHORT", "BAD_REVCOMP_BASE", "EMPTY_TABLE", "MISSING_KEY",
                "QUAL_RANGE", "NULL_FIELD", "SEQ_SHORT", "CIGAR_INVALID", "INVALID_ARG", "DEVICE", "UNSUPPORTED",
                "SAM_PARSE"]
(NULL_RG, MD_PARSE, CIGAR_SHORT, BAD_REVCOMP_BASE, EMPTY_TABLE, MISSING_KEY, QUAL_RANGE, NULL_FIELD, SEQ_SHORT,
 CIGAR_INVALID, INVALID_ARG, DEVICE, UNSUPPORTED, SAM_PARSE) = range(1, 15)

# every symbol include/adam_bqsr.h declares
EXPORTS = [
    "bqsr_abi_version", "bqsr_last_error", "bqsr_last_error_read", "bqsr_status_name", "bqsr_context_create",
    "bqsr_context_destroy", "bqsr_context_tune", "bqsr_sites_create", "bqsr_sites_destroy", "bqsr_batch_create", "bqsr_batch_destroy",
    "bqsr_batch_reads", "bqsr_batch_bases", "bqsr_batch_dims", "bqsr_batch_relayout", "bqsr_batch_layout_times", "bqsr_batch_wrap_device", "bqsr_table_words",
    "bqsr_table_create", "bqsr_table_destroy", "bqsr_table_dims", "bqsr_table_device_ptr", "bqsr_table_download",
    "bqsr_table_upload", "bqsr_observe", "bqsr_observe_records", "bqsr_table_merge", "bqsr_finalize",
    "bqsr_lut_destroy", "bqsr_lut_stats", "bqsr_lut_shifts", "bqsr_apply", "bqsr_apply_records",
    "bqsr_stage_records", "bqsr_staged_destroy", "bqsr_staged_bytes", "bqsr_staged_reads", "bqsr_staged_bases",
    "bqsr_batch_create_staged", "bqsr_batch_upload_async", "bqsr_em_fold_async", "bqsr_batch_em_copy_async",
    "bqsr_finalize_device", "bqsr_observe_stage", "bqsr_apply_stage", "bqsr_job_reset_async", "bqsr_job_result", "bqsr_copy_async",
    "bqsr_job_errors_export_async", "bqsr_job_errors_import_async", "bqsr_job_status_async", "bqsr_job_status_get",
    "bqsr_copy_dyn_async", "bqsr_compact_outputs_async", "bqsr_batch_exception_count_ptr",
]


class NativeLibraryMissing(RuntimeError):
    pass


class BQSRError(RuntimeError):
    """A status the C ABI returned; ``.status`` mirrors the JVM exception class."""

    def __init__(self, status: int, message: str = "", read: int = -1):
        name = STATUS_NAMES[status] if 0 <= status < len(STATUS_NAMES) else str(status)
        super().__init__("%s: %s" % (name, message))
        self.status = status
        self.name = name
        self.read = read


class Dims(ctypes.Structure):
    _fields_ = [("n_rg", ctypes.c_int32), ("max_len", ctypes.c_int32)]


class FinalStats(ctypes.Structure):
    _fields_ = [("average_reported_error", ctypes.c_double), ("global_error", ctypes.c_double),
                ("global_obs", ctypes.c_int64), ("global_mm", ctypes.c_int64), ("n_groups", ctypes.c_int32)]


class DeviceReads(ctypes.Structure):
    _fields_ = [("n_reads", ctypes.c_int64), ("n_slots", ctypes.c_int64), ("meta", ctypes.c_void_p),
                ("align", ctypes.c_void_p), ("qual", ctypes.c_void_p), ("bases", ctypes.c_void_p),
                ("cigar", ctypes.c_void_p), ("md", ctypes.c_void_p), ("dims", Dims),
                ("slots_aligned", ctypes.c_int32)]


_lib = None
_lock = threading.Lock()


def lib():
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise NativeLibraryMissing("%s is not built; run __graft_entry__.build()" % LIB_PATH)
        # one HIP runtime per process: let torch load and initialise its
        # libamdhip64 first, so the library binds to the same one (loading ours
        # first left whichever initialised second without a device on the box)
        try:
            import torch
            if torch.cuda.is_available():
                torch.cuda.init()
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        vp, i32, i64, dbl = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_double
        pp = ctypes.POINTER(ctypes.c_void_p)
        sig = {
            "bqsr_abi_version": (ctypes.c_int, []),
            "bqsr_last_error": (ctypes.c_char_p, []),
            "bqsr_last_error_read": (i64, []),
            "bqsr_status_name": (ctypes.c_char_p, [ctypes.c_int]),
            "bqsr_context_create": (ctypes.c_int, [ctypes.c_int, pp]),
            "bqsr_context_destroy": (None, [vp]),
            "bqsr_context_tune": (ctypes.c_int, [vp, ctypes.c_int, i64]),
            "bqsr_batch_relayout": (ctypes.c_int, [vp, vp, ctypes.POINTER(dbl)]),
            "bqsr_batch_layout_times": (ctypes.c_int, [vp, ctypes.POINTER(dbl), ctypes.POINTER(dbl)]),
            "bqsr_sites_create": (ctypes.c_int, [vp, vp, vp, vp, i32, pp]),
            "bqsr_sites_destroy": (None, [vp]),
            "bqsr_batch_create": (ctypes.c_int, [vp, vp, vp, pp]),
            "bqsr_batch_destroy": (None, [vp]),
            "bqsr_batch_reads": (i64, [vp]),
            "bqsr_batch_bases": (i64, [vp]),
            "bqsr_batch_slots": (i64, [vp]),
            "bqsr_batch_dims": (Dims, [vp]),
            "bqsr_batch_wrap_device": (ctypes.c_int, [vp, ctypes.POINTER(DeviceReads), pp]),
            "bqsr_stage_records": (ctypes.c_int, [vp, vp, pp]),
            "bqsr_staged_destroy": (None, [vp]),
            "bqsr_staged_bytes": (i64, [vp]),
            "bqsr_staged_reads": (i64, [vp]),
            "bqsr_staged_bases": (i64, [vp]),
            "bqsr_batch_create_staged": (ctypes.c_int, [vp, vp, pp]),
            "bqsr_batch_upload_async": (ctypes.c_int, [vp, vp, vp]),
            "bqsr_batch_set_window": (ctypes.c_int, [vp, i32, i32]),
            "bqsr_batch_reads_per_tile": (i32, [vp]),
            "bqsr_table_words": (i64, [Dims]),
            "bqsr_table_create": (ctypes.c_int, [vp, Dims, vp, pp]),
            "bqsr_table_destroy": (None, [vp]),
            "bqsr_table_dims": (Dims, [vp]),
            "bqsr_table_device_ptr": (vp, [vp]),
            "bqsr_table_download": (ctypes.c_int, [vp, vp]),
            "bqsr_table_upload": (ctypes.c_int, [vp, vp]),
            "bqsr_observe": (ctypes.c_int, [vp, vp, vp, vp, ctypes.POINTER(dbl), vp]),
            "bqsr_observe_async": (ctypes.c_int, [vp, vp, vp, vp, vp]),
            "bqsr_observe_result": (ctypes.c_int, [vp, ctypes.POINTER(dbl), vp]),
            "bqsr_observe_stage": (ctypes.c_int, [vp, vp, vp, vp, i32, vp]),
            "bqsr_table_zero_async": (ctypes.c_int, [vp, vp]),
            "bqsr_batch_em_device_ptr": (vp, [vp]),
            "bqsr_apply_stage": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, i64, i32, vp]),
            "bqsr_observe_records": (ctypes.c_int, [vp, vp, vp, Dims, pp, ctypes.POINTER(dbl)]),
            "bqsr_table_merge": (ctypes.c_int, [vp, vp, ctypes.POINTER(dbl), dbl]),
            "bqsr_finalize": (ctypes.c_int, [vp, vp, dbl, pp]),
            "bqsr_finalize_async": (ctypes.c_int, [vp, vp, dbl, pp, vp]),
            "bqsr_finalize_result": (ctypes.c_int, [vp, vp]),
            "bqsr_finalize_device": (ctypes.c_int, [vp, vp, vp, pp, vp]),
            "bqsr_batch_em_copy_async": (ctypes.c_int, [vp, vp, vp]),
            "bqsr_em_fold_async": (ctypes.c_int, [vp, vp, i64, vp, vp]),
            "bqsr_lut_destroy": (None, [vp]),
            "bqsr_lut_stats": (ctypes.c_int, [vp, ctypes.POINTER(FinalStats)]),
            "bqsr_lut_group": (ctypes.c_int, [vp, i32, ctypes.POINTER(i64), ctypes.POINTER(i64)]),
            "bqsr_lut_shifts": (ctypes.c_int, [vp, i32, i32, i32, i32, vp, ctypes.POINTER(i32)]),
            "bqsr_phred_threshold_table": (i32, [vp, i32, ctypes.POINTER(i32)]),
            "bqsr_apply": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, i64, ctypes.POINTER(i64), vp]),
            "bqsr_apply_async": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, i64, vp]),
            "bqsr_apply_result": (ctypes.c_int, [vp, ctypes.POINTER(i64), vp]),
            "bqsr_apply_records": (ctypes.c_int, [vp, vp, vp, vp, vp]),
            "bqsr_job_reset_async": (ctypes.c_int, [vp, vp, vp]),
            "bqsr_job_result": (ctypes.c_int, [vp, vp, ctypes.POINTER(dbl), ctypes.POINTER(i64), vp]),
            "bqsr_copy_async": (ctypes.c_int, [vp, vp, vp, i64, vp]),
            "bqsr_copy_dyn_async": (ctypes.c_int, [vp, vp, vp, vp, i32, i64, i64, vp]),
            "bqsr_compact_outputs_async": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, i64, vp, vp, vp, vp]),
            "bqsr_batch_exception_count_ptr": (vp, [vp]),
            "bqsr_job_errors_export_async": (ctypes.c_int, [vp, i64, vp, vp]),
            "bqsr_job_errors_import_async": (ctypes.c_int, [vp, vp, vp]),
            "bqsr_job_status_async": (ctypes.c_int, [vp, vp, i32, vp]),
            "bqsr_job_status_get": (ctypes.c_int, [vp, i32, i32, ctypes.POINTER(dbl), ctypes.POINTER(i64)]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(status: int):
    if status != BQSR_OK:
        L = lib()
        raise BQSRError(status, L.bqsr_last_error().decode(), L.bqsr_last_error_read())
