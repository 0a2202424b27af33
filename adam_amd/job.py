"""One rank's whole BQSR job over a device-resident read shard.

This is the step ``bench.py`` times and the multi-rank GPU test runs (two
ranks sharing one GPU over gloo): the rank's shard is one partition of the
job (RecalibrateBaseQualities.scala:52-76 over an RDD whose partitions are the
ranks' shards, in rank order).  One ``step``:

1. zero the count table (``new RecalTable``) and the job's error words (one kernel);
2. observe: prep (trimming, CIGAR / MD / known-site masks), the observe kernel
   (+ window reduce), the exact expectedMismatch fold -- all on one HIP stream;
3. N > 1: the int64 table all-reduce and the expectedMismatch of every
   rank's partition folded in rank order on the device (adam_amd/distributed.py);
4. finalize on the device (expectedMismatch read from HBM: no host round trip);
5. apply into device outputs (u8 chars per packed slot, per-read start and
   length, exception list for chars above 0xFF);
6. N > 1: the ranks' error keys (global read order) MIN-reduced, so every
   rank raises the job's first error, as the reference's one Spark job fails
   on its first failing partition;
7. the job's errors, in the order the reference raises them (one transfer, one sync).

Only the HIP library computes; this module orders launches.
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional

import numpy as np

from . import _capi, bqsr
from . import distributed as D
from ._capi import check
from .records import RecordBatch


class ResidentJob:
    STAGES = ("prep", "observe", "fold", "apply")

    def __init__(self, batch: Optional[RecordBatch], dims, snp: Optional["bqsr.SnpTable"] = None, device: int = 0,
                 max_exc: int = 1 << 16, read_base: Optional[int] = None, sam=None, handle=None):
        """read_base: global index of the shard's first read (reads of the
        ranks before this one): errors are reported in global read order.
        Required when several ranks run the job.  sam: a parse (sam.SamText)
        whose records become the batch on the device (bqsr_sam_batch_create)
        in place of a host RecordBatch; handle: a bqsr_batch* built on the
        device (parquet.ArrowReads.device_batch), owned by the job from here;
        dims None = the batch's own."""
        import torch
        self.torch = torch
        self.L = L = _capi.lib()
        self.dev = torch.device("cuda", device)
        self.ctx = bqsr.Context.get(device)
        self.stream = torch.cuda.current_stream(self.dev)
        self.sp = ctypes.c_void_p(self.stream.cuda_stream)
        self.batch = batch
        self.dims = dims
        self.snp = snp
        self.bh = ctypes.c_void_p()
        if sam is not None or handle is not None:
            self.bh = handle if handle is not None else sam.device_batch(snp.contigs if snp else None, self.sp)
            self.n_reads = int(L.bqsr_batch_reads(self.bh))
            self.n_bases = int(L.bqsr_batch_bases(self.bh))
            if dims is None:
                dims = L.bqsr_batch_dims(self.bh)
                self.dims = dims
        else:
            s, keep = batch.c_struct(batch.contig_ids_for(snp.contigs if snp else None))
            check(L.bqsr_batch_create(self.ctx.handle, ctypes.byref(s), self.sp, ctypes.byref(self.bh)))
            del keep
            self.n_reads = batch.n_reads
            self.n_bases = batch.n_bases
        self.n_slots = int(L.bqsr_batch_slots(self.bh))
        words = int(L.bqsr_table_words(dims))
        self.table = torch.zeros(words, dtype=torch.int64, device=self.dev)
        self.th = ctypes.c_void_p()
        check(L.bqsr_table_create(self.ctx.handle, dims, ctypes.c_void_p(self.table.data_ptr()), ctypes.byref(self.th)))
        self.sites_h = snp.handle(self.ctx) if snp else None
        self.out_qual = torch.empty(self.n_slots + 64, dtype=torch.uint8, device=self.dev)
        self.out_start = torch.empty(max(1, self.n_reads), dtype=torch.int32, device=self.dev)
        self.out_len = torch.empty(max(1, self.n_reads), dtype=torch.int32, device=self.dev)
        self.max_exc = max_exc
        self.exc = torch.empty(max_exc, dtype=torch.int64, device=self.dev)
        self.em_part = torch.zeros(1, dtype=torch.float64, device=self.dev)
        self.lut = ctypes.c_void_p()
        self.world = D.dist.get_world_size() if D._multi() else 1
        if read_base is None and self.world > 1:
            raise ValueError("several ranks: read_base (reads of the ranks before this one) is required")
        self.read_base = int(read_base or 0)
        self.err_keys = torch.empty(2, dtype=torch.int64, device=self.dev)
        self.ev = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
        self.kt: Dict[str, List[float]] = {k: [] for k in self.STAGES}
        self.n_exc = 0
        self.em = None  # the job's expectedMismatch (device, 1 double) of the last step
        torch.cuda.synchronize(self.dev)

    def _ptr(self, t):
        return ctypes.c_void_p(t.data_ptr())

    def layout_ms(self, reps: int = 3):
        """Wall time (ms, mean of reps) of the layout a bucketed batch builds
        once at creation -- piece-key sort, key-major copy -- redone on this
        batch (bqsr_batch_relayout); None for a batch without one."""
        ms = []
        for _ in range(reps):
            v = ctypes.c_double()
            check(self.L.bqsr_batch_relayout(self.bh, self.sp, ctypes.byref(v)))
            if v.value < 0:
                return None
            ms.append(v.value)
        return sum(ms) / len(ms)

    def layout_times(self):
        """(alloc_ms, build_ms) of the layout when the batch was created
        (bqsr_batch_layout_times); None for a batch without one."""
        a, b = ctypes.c_double(), ctypes.c_double()
        check(self.L.bqsr_batch_layout_times(self.bh, ctypes.byref(a), ctypes.byref(b)))
        return None if b.value < 0 else (a.value, b.value)

    def step(self, record: bool = False):
        """One job.  record: bracket the stages with timing events (each event
        record costs the stream ~30 us on this runtime, so callers sample)."""
        L, ctx, bh, th, sp, ev, stream = self.L, self.ctx.handle, self.bh, self.th, self.sp, self.ev, self.stream
        check(L.bqsr_job_reset_async(bh, th, sp))  # new RecalTable; the job's error words reset
        mark = (lambda i: ev[i].record(stream)) if record else (lambda i: None)
        mark(5)
        check(L.bqsr_observe_stage(ctx, bh, self.sites_h, th, _capi.STAGE_PREP, sp))
        mark(0)
        check(L.bqsr_observe_stage(ctx, bh, self.sites_h, th, _capi.STAGE_KERNEL, sp))
        mark(1)
        check(L.bqsr_observe_stage(ctx, bh, self.sites_h, th, _capi.STAGE_FOLD, sp))
        mark(2)
        if self.world > 1:
            # RecalTable.++ across ranks: exact int64 all-reduce (RCCL over
            # xGMI), expectedMismatch of every rank's partition folded in rank
            # order on the device
            check(L.bqsr_batch_em_copy_async(bh, self._ptr(self.em_part), sp))
            D.allreduce_table(self.table)
            self.em = D.fold_partition_ems_device(self.em_part, [1] * self.world, self.ctx, stream)
            em_ptr = self._ptr(self.em)
        else:
            self.em = None
            em_ptr = ctypes.c_void_p(L.bqsr_batch_em_device_ptr(bh))
        check(L.bqsr_finalize_device(ctx, th, em_ptr, ctypes.byref(self.lut), sp))
        args = (ctx, bh, self.lut, self._ptr(self.out_qual), self._ptr(self.out_start), self._ptr(self.out_len),
                self._ptr(self.exc), self.max_exc)
        if record:  # the char tables first, so the bracket holds the apply kernel alone
            check(L.bqsr_apply_stage(*args, _capi.STAGE_LUT, sp))
            mark(3)
            check(L.bqsr_apply_stage(*args, _capi.STAGE_KERNEL | _capi.STAGE_NO_LUT, sp))
            mark(4)
        else:
            check(L.bqsr_apply_stage(*args, _capi.STAGE_KERNEL, sp))
        if self.world > 1:
            check(L.bqsr_job_errors_export_async(bh, self.read_base, self._ptr(self.err_keys), sp))
            D.allreduce_error_keys(self.err_keys)
            check(L.bqsr_job_errors_import_async(bh, self._ptr(self.err_keys), sp))
        # the job's results and errors, in the order the reference raises them
        # (one transfer and one sync)
        em = ctypes.c_double()
        nexc = ctypes.c_int64()
        check(L.bqsr_job_result(bh, self.lut, ctypes.byref(em), ctypes.byref(nexc), sp))
        self.n_exc = int(nexc.value)
        if self.n_exc > self.max_exc:
            raise _capi.BQSRError(_capi.UNSUPPORTED, "%d chars above 0xFF exceed the exception list" % self.n_exc)
        if record:
            self.kt["prep"].append(ev[5].elapsed_time(ev[0]))
            self.kt["observe"].append(ev[0].elapsed_time(ev[1]))
            self.kt["fold"].append(ev[1].elapsed_time(ev[2]))
            self.kt["apply"].append(ev[3].elapsed_time(ev[4]))

    def kernel_ms(self) -> Dict[str, float]:
        return {k: float(np.mean(v)) if v else float("nan") for k, v in self.kt.items()}

    def expected_mismatch(self) -> float:
        """The job's expectedMismatch (after step)."""
        if self.em is not None:
            return float(self.em.cpu()[0])
        v = ctypes.c_double()
        check(self.L.bqsr_observe_result(self.bh, ctypes.byref(v), self.sp))
        return v.value

    def results(self):
        """(table words, job expectedMismatch, out_qual u8 per slot, out_start,
        out_len, exception list) of the last step, on the host."""
        self.torch.cuda.synchronize(self.dev)
        return (self.table.cpu().numpy(), self.expected_mismatch(), self.out_qual.cpu().numpy()[:self.n_slots],
                self.out_start.cpu().numpy()[:self.n_reads], self.out_len.cpu().numpy()[:self.n_reads],
                self.exc.cpu().numpy()[:self.n_exc])

    def close(self):
        L = self.L
        if self.lut:
            L.bqsr_lut_destroy(self.lut)
            self.lut = ctypes.c_void_p()
        if self.th:
            L.bqsr_table_destroy(self.th)
            self.th = ctypes.c_void_p()
        if self.bh:
            L.bqsr_batch_destroy(self.bh)
            self.bh = ctypes.c_void_p()
