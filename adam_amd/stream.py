"""Streamed BQSR over host-resident partitions (BASELINE cfg5).

A shard of reads lives on the host as partitions already flattened into the
device layout in pinned memory (``bqsr_stage_records`` -- what the JNI side
hands over per Spark partition).  One job (``StreamedShard.run``):

1. observe, partition by partition: the partition's H2D copy on the copy
   stream, then prep + observe + the exact expectedMismatch fold on the
   compute stream, which waits on the copy's event -- so partition i+1 moves
   over PCIe while partition i is on the CUs.  Every partition counts into the
   one device table (``RecalTable.++`` is an integer sum); its
   expectedMismatch stays on the device.
2. on several ranks the int64 all-reduce of the table; then
   ``((0.0 + e_0) + e_1) + ...`` over every partition of the job in global
   partition order (this rank's partitions after those of lower ranks: Spark's
   per-partition ``aggregate`` merged in partition order), on
   the device (adam_amd/distributed.py, ``bqsr_em_fold_async``).
3. finalize on the device, then apply partition by partition from the
   partitions still resident in HBM, each partition's recalibrated qualities
   (and per-read start / length) copied back to pinned host memory on the
   download stream while the next partition is applied (double-buffered
   device output).
4. the job's status words snapshot into pinned memory (``bqsr_job_status_async``).

Jobs pipeline over both link directions: uploads run on a stream of their
own, and job k+1's upload of partition i starts as soon as job k's apply is
done with it, while job k's results still move back on the download stream.
``finish`` checks a job's snapshot (errors in the reference's order) after
the next job has been enqueued.

Reference: RecalibrateBaseQualities.scala:34-76 (computeTable / applyTable over
an RDD's partitions).  Only the HIP library computes; this module orders
copies and launches.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence

from . import _capi
from . import distributed as D
from ._capi import check


class StreamedShard:
    """Partitions of one rank's shard: pinned host copies + device batches."""

    def __init__(self, ctx, parts: Sequence, dims, sites_handle=None, device: int = 0, max_exc: int = 1 << 16,
                 site_contigs: Optional[Sequence[str]] = None, read_base: Optional[int] = None,
                 zero_copy: bool = False,
                 d2h: str = "kernel", compact: Optional[bool] = None):
        """read_base: global index of the shard's first read (reads of the
        ranks before this one): multi-rank errors are raised in global order;
        required when several ranks run the job."""
        import torch
        self.torch = torch
        self.L = L = _capi.lib()
        self.ctx = ctx
        self.dims = dims
        self.sites = sites_handle
        self.dev = torch.device("cuda", device)
        self.staged: List[ctypes.c_void_p] = []
        self.batches: List[ctypes.c_void_p] = []
        self.n_reads: List[int] = []
        self.n_slots: List[int] = []
        self.n_bases = 0
        self.staged_bytes = 0
        self.site_contigs = site_contigs
        if read_base is None and D._multi():
            raise ValueError("several ranks: read_base (reads of the ranks before this one) is required")
        self.read_base = int(read_base or 0)
        # zero_copy: apply writes its outputs straight into the pinned host
        # buffers (device stores over PCIe, no download copies)
        self.zero_copy = bool(zero_copy)
        # d2h: "kernel" -- results copied back by a kernel (bqsr_copy_async),
        # which runs beside the next job's DMA uploads (the two directions at
        # once: 85 GB/s in all, against 57 for two DMA copies, tools/link_probe.hip);
        # "dma" -- hipMemcpyAsync copies
        if d2h not in ("kernel", "dma"):
            raise ValueError("d2h must be 'kernel' or 'dma'")
        self.d2h = d2h
        # compact: each partition's recalibrated chars go back compacted (chars
        # at u32 offsets per read, bqsr_compact_outputs_async) instead of the
        # padded slot array; needs the kernel copies (sizes known on the device only)
        self.compact = (not self.zero_copy and d2h == "kernel") if compact is None else bool(compact)
        if self.compact and (self.zero_copy or d2h != "kernel"):
            raise ValueError("compact outputs need d2h='kernel' and no zero_copy")
        for p in parts:
            self.add_partition(p)
        if parts:
            self.alloc_outputs(max_exc)

    def add_partition(self, part):
        """Flatten one partition into pinned host memory (device layout) and
        allocate its device batch; ``part`` may be dropped afterwards."""
        L = self.L
        s, keep = part.c_struct(part.contig_ids_for(self.site_contigs))
        sh = ctypes.c_void_p()
        check(L.bqsr_stage_records(self.ctx.handle, ctypes.byref(s), ctypes.byref(sh)))
        del keep
        bh = ctypes.c_void_p()
        st = L.bqsr_batch_create_staged(self.ctx.handle, sh, ctypes.byref(bh))
        if st != _capi.BQSR_OK:
            L.bqsr_staged_destroy(sh)
            check(st)
        self.staged.append(sh)
        self.batches.append(bh)
        self.n_reads.append(int(L.bqsr_batch_reads(bh)))
        self.n_slots.append(int(L.bqsr_batch_slots(bh)))
        self.n_bases += int(L.bqsr_batch_bases(bh))
        self.staged_bytes += int(L.bqsr_staged_bytes(sh))

    def alloc_outputs(self, max_exc: int = 1 << 16):
        torch = self.torch
        dev = self.dev
        ms = max(self.n_slots or [1]) + 64
        mr = max(self.n_reads or [1])
        self.out_qual = [torch.empty(ms, dtype=torch.uint8, device=dev) for _ in range(2)]
        self.out_start = [torch.empty(max(1, mr), dtype=torch.int32, device=dev) for _ in range(2)]
        self.out_len = [torch.empty(max(1, mr), dtype=torch.int32, device=dev) for _ in range(2)]
        if self.compact:
            # device: the compacted chars, offsets and u16 lengths (double-buffered);
            # host, pinned: per partition the chars and the lengths (the link
            # carries 2 B a read; read r = chars[off[r] : off[r + 1]], off their
            # prefix sum, built on the host when a result is read)
            self.cchars = [torch.empty(ms, dtype=torch.uint8, device=dev) for _ in range(2)]
            self.coff = [torch.empty(mr + 1, dtype=torch.int32, device=dev) for _ in range(2)]
            self.clen = [torch.empty(max(1, mr), dtype=torch.int16, device=dev) for _ in range(2)]
            self.host_chars = [torch.empty(n + 64, dtype=torch.uint8, pin_memory=True) for n in self.n_slots]
            self.host_len16 = [torch.empty(max(1, n), dtype=torch.int16, pin_memory=True) for n in self.n_reads]
            self._offs = {}
            self.host_qual = self.host_start = self.host_len = None
        else:
            # host results, pinned: qualities by packed slot, per-read start / length
            self.host_qual = [torch.empty(n + 64, dtype=torch.uint8, pin_memory=True) for n in self.n_slots]
            self.host_start = [torch.empty(max(1, n), dtype=torch.int32, pin_memory=True) for n in self.n_reads]
            self.host_len = [torch.empty(max(1, n), dtype=torch.int32, pin_memory=True) for n in self.n_reads]
        # exception lists (chars above 0xFF, Q14): one slice of max_exc entries
        # per partition, copied back with the partition's qualities
        n = len(self.batches)
        self.exc = torch.empty(max(1, n) * max_exc, dtype=torch.int64, device=dev)
        self.host_exc = torch.empty(max(1, n) * max_exc, dtype=torch.int64, pin_memory=True)
        self.n_exc = [0] * n
        self.max_exc = max_exc
        self.counts = None  # every rank's partition count (exchanged on the first multi-rank job)
        self.em = torch.zeros(max(1, len(self.batches)), dtype=torch.float64, device=dev)
        # H2D and D2H on copy streams of their own: a job's uploads overlap
        # the previous job's downloads (both link directions)
        self.up_stream = torch.cuda.Stream(dev)
        self.dn_stream = torch.cuda.Stream(dev)
        self.copy_stream = self.dn_stream
        self.ev_up = [torch.cuda.Event() for _ in range(n)]
        self.ev_ap = [torch.cuda.Event() for _ in range(n)]
        self.ev_dl = [torch.cuda.Event() for _ in range(2)]
        self.ev_exc = [torch.cuda.Event() for _ in range(n)]  # partition i's exception list copied back
        self.dl_used = [False, False]
        self.ev_status = [torch.cuda.Event() for _ in range(2)]
        self.ev_done = [torch.cuda.Event() for _ in range(2)]
        self.ev_apply_t = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                           for _ in range(n)]
        self.lut = ctypes.c_void_p()
        self.jobs = 0
        self.pending: List[int] = []  # status slots of jobs run but not finished, oldest first

    def run(self, table_handle, table_words=None, record_apply: bool = False):
        """Enqueue one whole job over the shard (no host sync); returns the
        job's expectedMismatch tensor (device).  Jobs pipeline: this job's
        uploads start as soon as the previous job's apply is done with each
        partition, while its results still move back on the other copy
        stream.  At most two jobs may be pending; ``finish`` raises a job's
        errors.  The host results (host_qual / host_start / host_len /
        host_exc) are shared by the jobs: they hold the last job's results
        once no job is pending (``exceptions`` / ``qual_chars`` refuse to read
        them before), since a pending job's apply and copies overwrite them."""
        torch, L = self.torch, self.L
        if self.compact:
            self._offs = {}  # the offsets of the last job's lengths
        if len(self.pending) >= 2:
            raise RuntimeError("two jobs pending: finish() one first")
        comp = torch.cuda.current_stream(self.dev)
        up, dn = self.up_stream, self.dn_stream
        sp = ctypes.c_void_p(comp.cuda_stream)
        upp = ctypes.c_void_p(up.cuda_stream)
        ctx = self.ctx.handle
        slot = self.jobs & 1
        check(L.bqsr_table_zero_async(table_handle, sp))
        # (1) stream the partitions in, observing each as it lands
        for i, bh in enumerate(self.batches):
            if self.jobs:
                up.wait_event(self.ev_ap[i])  # the previous job's apply is done with partition i's columns
            check(L.bqsr_batch_upload_async(bh, self.staged[i], upp))
            self.ev_up[i].record(up)
            comp.wait_event(self.ev_up[i])
            check(L.bqsr_observe_async(ctx, bh, self.sites, table_handle, sp))
            check(L.bqsr_batch_em_copy_async(bh, ctypes.c_void_p(self.em.data_ptr() + 8 * i), sp))
        # (2) the table all-reduce across ranks, then the expectedMismatch of
        # every partition of the job folded in global partition order:
        # ((0.0 + e_0) + e_1) + ...
        n = len(self.batches)
        if table_words is not None:
            D.allreduce_table(table_words)
        if self.counts is None:
            self.counts = D.partition_counts(n, self.dev)
        acc = D.fold_partition_ems_device(self.em[:n], self.counts, self.ctx, comp)
        self._em_keep = acc
        check(L.bqsr_finalize_device(ctx, table_handle, ctypes.c_void_p(acc.data_ptr()), ctypes.byref(self.lut), sp))
        # (3) apply from the resident partitions, results streamed back
        for i, bh in enumerate(self.batches):
            k = i & 1
            if self.zero_copy:
                if self.jobs:
                    comp.wait_event(self.ev_done[slot])  # the job two back is done with these host buffers
                oq, os_, ol = self.host_qual[i], self.host_start[i], self.host_len[i]
            else:
                if self.dl_used[k]:
                    comp.wait_event(self.ev_dl[k])  # output buffer k drained to the host
                oq, os_, ol = self.out_qual[k], self.out_start[k], self.out_len[k]
            if self.jobs:
                comp.wait_event(self.ev_exc[i])  # the previous job's exception list of partition i is on the host
            if record_apply:
                self.ev_apply_t[i][0].record(comp)
            exc_i = ctypes.c_void_p(self.exc.data_ptr() + 8 * i * self.max_exc)
            check(L.bqsr_apply_stage(ctx, bh, self.lut, ctypes.c_void_p(oq.data_ptr()),
                                     ctypes.c_void_p(os_.data_ptr()), ctypes.c_void_p(ol.data_ptr()), exc_i,
                                     self.max_exc, _capi.STAGE_RESET | _capi.STAGE_KERNEL, sp))
            if record_apply:
                self.ev_apply_t[i][1].record(comp)
            if self.compact:
                check(L.bqsr_compact_outputs_async(ctx, bh, ctypes.c_void_p(oq.data_ptr()),
                                                   ctypes.c_void_p(os_.data_ptr()), ctypes.c_void_p(ol.data_ptr()),
                                                   exc_i, self.max_exc, ctypes.c_void_p(self.cchars[k].data_ptr()),
                                                   ctypes.c_void_p(self.coff[k].data_ptr()),
                                                   ctypes.c_void_p(self.clen[k].data_ptr()), sp))
            self.ev_ap[i].record(comp)
            dn.wait_event(self.ev_ap[i])
            ns, nr = self.n_slots[i], max(1, self.n_reads[i])
            e0 = i * self.max_exc
            if self.compact:
                # sizes on the device: the chars (offset n), the exception count
                dnp = ctypes.c_void_p(dn.cuda_stream)
                n_i = self.n_reads[i]
                cp = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
                check(L.bqsr_copy_dyn_async(ctx, cp(self.host_chars[i]), cp(self.cchars[k]),
                                            ctypes.c_void_p(self.coff[k].data_ptr() + 4 * n_i), 4, 1, ns, dnp))
                if n_i:
                    check(L.bqsr_copy_async(ctx, cp(self.host_len16[i]), cp(self.clen[k]), 2 * n_i, dnp))
                check(L.bqsr_copy_dyn_async(ctx, ctypes.c_void_p(self.host_exc.data_ptr() + 8 * e0),
                                            ctypes.c_void_p(self.exc.data_ptr() + 8 * e0),
                                            ctypes.c_void_p(L.bqsr_batch_exception_count_ptr(bh)), 8, 8,
                                            8 * self.max_exc, dnp))
                self.ev_dl[k].record(dn)
                self.ev_exc[i].record(dn)
                self.dl_used[k] = True
                continue
            pairs = [] if self.zero_copy else [(self.host_qual[i][:ns], self.out_qual[k][:ns]),
                                               (self.host_start[i][:nr], self.out_start[k][:nr]),
                                               (self.host_len[i][:nr], self.out_len[k][:nr])]
            pairs.append((self.host_exc[e0:e0 + self.max_exc], self.exc[e0:e0 + self.max_exc]))
            if self.d2h == "kernel":
                dnp = ctypes.c_void_p(dn.cuda_stream)
                for h, d in pairs:
                    check(L.bqsr_copy_async(ctx, ctypes.c_void_p(h.data_ptr()), ctypes.c_void_p(d.data_ptr()),
                                            h.numel() * h.element_size(), dnp))
            else:
                with torch.cuda.stream(dn):
                    for h, d in pairs:
                        h.copy_(d, non_blocking=True)
            self.ev_dl[k].record(dn)
            self.ev_exc[i].record(dn)
            self.dl_used[k] = True
        # (4) several ranks: the job's first error in global read order on every rank
        if D._multi():
            self._exchange_errors(sp)
        # (5) the job's status, snapshot for `finish` (the next job resets the live words)
        for bh in self.batches:
            check(L.bqsr_job_status_async(bh, self.lut, slot, sp))
        self.ev_status[slot].record(comp)
        self.ev_done[slot].record(dn)
        self.pending.append(slot)
        self.jobs += 1
        return acc

    def finish(self):
        """Wait for the oldest pending job, then raise its first error in the
        reference's order (observe errors partition by partition, finalize,
        apply).  Returns the number of recalibrated chars above 0xFF (Q14);
        their codes are in ``exceptions(i)`` and ``qual_chars`` applies them."""
        L = self.L
        if not self.pending:
            raise RuntimeError("no job pending")
        slot = self.pending.pop(0)
        self.ev_status[slot].synchronize()
        self.ev_done[slot].synchronize()
        em = ctypes.c_double()
        nexc = ctypes.c_int64()
        for bh in self.batches:
            check(L.bqsr_job_status_get(bh, slot, 0, ctypes.byref(em), ctypes.byref(nexc)))
        if self.batches:
            check(L.bqsr_job_status_get(self.batches[0], slot, 1, ctypes.byref(em), ctypes.byref(nexc)))
        total = 0
        for i, bh in enumerate(self.batches):
            check(L.bqsr_job_status_get(bh, slot, 2, ctypes.byref(em), ctypes.byref(nexc)))
            self.n_exc[i] = int(nexc.value)
            if self.n_exc[i] > self.max_exc:
                raise _capi.BQSRError(_capi.UNSUPPORTED, "partition %d: %d chars above 0xFF exceed the exception "
                                      "list (%d)" % (i, self.n_exc[i], self.max_exc))
            total += self.n_exc[i]
        return total

    def _exchange_errors(self, sp):
        """Several ranks: the first observe error and the first apply error of
        the whole job (global read order) on every rank -- the partitions'
        error keys rebased to global reads, MIN over partitions and ranks, and
        written back into every partition (the first partition carries them,
        the others none), so every rank raises the same error in `finish`."""
        torch, L = self.torch, self.L
        n = len(self.batches)
        keys = torch.empty(max(1, n), 2, dtype=torch.int64, device=self.dev)
        base = self.read_base
        for i, bh in enumerate(self.batches):
            check(L.bqsr_job_errors_export_async(bh, base, ctypes.c_void_p(keys[i].data_ptr()), sp))
            base += self.n_reads[i]
        red = keys[:max(1, n)].min(dim=0).values.contiguous() if n else torch.full((2,), 2 ** 63 - 1,
                                                                                     dtype=torch.int64,
                                                                                     device=self.dev)
        D.allreduce_error_keys(red)
        none = torch.full((2,), 2 ** 63 - 1, dtype=torch.int64, device=self.dev)
        for i, bh in enumerate(self.batches):
            check(L.bqsr_job_errors_import_async(bh, ctypes.c_void_p((red if i == 0 else none).data_ptr()), sp))
        self._err_keep = (keys, red, none)

    def _results_ready(self):
        if self.pending:
            raise RuntimeError("a job is pending: its apply and copies overwrite the host results; finish() it first")

    def exceptions(self, i: int):
        """Partition i's chars above 0xFF of the last job: (position, Java char)
        pairs -- the slot in the padded layout, the index into host_chars[i]
        when compact."""
        self._results_ready()
        a = self.host_exc[i * self.max_exc: i * self.max_exc + self.n_exc[i]].numpy()
        return [(int(v) >> 16, int(v) & 0xFFFF) for v in a]

    def qual_chars(self, i: int, slot: int, r: int):
        """Read r's recalibrated quality string of partition i as Java chars
        (uint16): the u8 output with the partition's exceptions applied (slot:
        the read's packed slot, used by the padded layout only)."""
        import numpy as np
        self._results_ready()
        if self.compact:
            off = self._offsets(i)
            a, b = int(off[r]), int(off[r + 1])
        else:
            st, ln = int(self.host_start[i][r]), int(self.host_len[i][r])
            a, b = slot + st, slot + st + ln
        out = (self.host_chars[i] if self.compact else self.host_qual[i])[a:b].numpy().astype(np.uint16)
        for s, code in self.exceptions(i):
            if a <= s < b:
                out[s - a] = code
        return out

    def outputs(self, i: int):
        """Partition i's results of the last job for a checker: ("compact",
        chars, offsets u32, exceptions) or ("slots", qual by slot, start, len,
        exceptions); exceptions as the raw (position << 16 | char) words."""
        self._results_ready()
        exc = self.host_exc[i * self.max_exc: i * self.max_exc + self.n_exc[i]].numpy()
        nr = self.n_reads[i]
        if self.compact:
            off = self._offsets(i)
            return "compact", self.host_chars[i].numpy()[:int(off[nr]) if nr else 0], off, exc
        return ("slots", self.host_qual[i].numpy()[:self.n_slots[i]], self.host_start[i].numpy()[:nr],
                self.host_len[i].numpy()[:nr], exc)

    def d2h_bytes(self) -> int:
        """Bytes the last finished job copied back to the host."""
        if not self.compact:
            return sum(self.n_slots) + 8 * sum(self.n_reads) + 8 * self.max_exc * len(self.batches)
        return sum(int(self._offsets(i)[self.n_reads[i]]) + 2 * self.n_reads[i] + 8 * self.n_exc[i]
                   for i in range(len(self.batches)))

    def _offsets(self, i: int):
        """u32 offsets [n + 1] of partition i's compacted chars: the prefix
        sum of the shipped u16 lengths (cached until the next job)"""
        import numpy as np
        if i not in self._offs:
            n = self.n_reads[i]
            off = np.zeros(n + 1, np.uint32)
            if n:
                np.cumsum(self.host_len16[i].numpy()[:n].view(np.uint16), out=off[1:], dtype=np.uint32)
            self._offs[i] = off
        return self._offs[i]

    def n_bases_of(self, i: int) -> int:
        """bases of partition i"""
        return int(self.L.bqsr_batch_bases(self.batches[i]))

    def apply_probe_ms(self, i: int = 0, reps: int = 3) -> Optional[float]:
        """The apply kernel alone on partition i, no copies in flight (no job
        pending): its char tables first, then the kernel bracketed by HIP
        events on the compute stream, `reps` times; the mean in ms.  Writes
        the device output buffers only (the host results stay)."""
        torch, L = self.torch, self.L
        if self.pending or not self.lut or not self.batches:
            return None
        torch.cuda.synchronize(self.dev)
        comp = torch.cuda.current_stream(self.dev)
        sp = ctypes.c_void_p(comp.cuda_stream)
        bh = self.batches[i]
        oq = self.host_qual[i] if self.zero_copy else self.out_qual[0]
        os_ = self.host_start[i] if self.zero_copy else self.out_start[0]
        ol = self.host_len[i] if self.zero_copy else self.out_len[0]
        p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        exc_i = ctypes.c_void_p(self.exc.data_ptr() + 8 * i * self.max_exc)
        args = (self.ctx.handle, bh, self.lut, p(oq), p(os_), p(ol), exc_i, self.max_exc)
        check(L.bqsr_apply_stage(*args, _capi.STAGE_LUT, sp))
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        t = []
        for _ in range(reps):
            ev[0].record(comp)
            check(L.bqsr_apply_stage(*args, _capi.STAGE_RESET | _capi.STAGE_KERNEL | _capi.STAGE_NO_LUT, sp))
            ev[1].record(comp)
            ev[1].synchronize()
            t.append(ev[0].elapsed_time(ev[1]))
        return sum(t) / len(t)

    def apply_ms(self) -> Optional[float]:
        """Mean apply-kernel time per partition of the last recorded job."""
        try:
            t = [a.elapsed_time(b) for a, b in self.ev_apply_t]
        except RuntimeError:
            return None
        return sum(t) / max(1, len(t))

    def close(self):
        L = self.L
        if self.lut:
            L.bqsr_lut_destroy(self.lut)
            self.lut = ctypes.c_void_p()
        for bh in self.batches:
            L.bqsr_batch_destroy(bh)
        for sh in self.staged:
            L.bqsr_staged_destroy(sh)
        self.batches, self.staged = [], []
