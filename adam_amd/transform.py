"""`adam transform`: the CLI harness around the device path
(adam-cli/.../cli/Transform.scala:38-110).

    python -m adam_amd.transform INPUT.sam OUTPUT.sam [-mark_duplicate_reads]
        [-recalibrate_base_qualities] [-dbsnp_sites SITES.vcf]
    python -m adam_amd.transform INPUT.{adam,parquet,sam} OUTPUT.{adam,parquet} [...]

SAM or BAM in goes through the device path described below, out as SAM text
or as ADAMRecord Parquet part files (adamSave, adam_save.py).  ADAMRecord
Parquet in goes through ``transform_parquet``: Arrow decodes the Parquet
pages on host threads, the column buffers go to the device as they are
(parquet.ArrowReads), MarkDuplicates, the BQSR batch and the recalibrated
qual column are built there, and the records are written back as Parquet
with the qual (and duplicateRead) columns replaced.

Steps in Transform.run's order (:66-90): load (the SAM text parsed on the
device, SAMRecordConverter semantics), MarkDuplicates (`adamMarkDuplicates`),
BQSR (`adamBQSR(loadSnpTable)`: an empty SnpTable without -dbsnp_sites,
:96-105), save.  The output is ADAMRecord Parquet part files, as the
reference's adamSave writes them (core/rdd/AdamRDDFunctions.scala:37-56;
OUTPUT.adam / .parquet / a directory), or SAM text -- the input records with
their QUAL fields replaced by the recalibrated strings (and FLAG 0x400 by
MarkDuplicates' result).  -sort_reads, -coalesce and
-realignIndels are outside this build and are refused.

Partitions: an input whose records exceed ``partition_bytes`` is cut at line
boundaries into partitions (the Hadoop splits the reference's RDD is read
as, each parsed with the header as a SAM file of its own) that stream through
the device: every partition is parsed and packed into a resident batch and
observed into the one count table (computeTable's per-partition aggregate
merged by ``RecalTable.++``, RecalibrateBaseQualities.scala:52-64), the
per-partition expectedMismatch values folded in partition order, then per
partition: apply, its text re-read (the reference re-reads its input per
stage, cli/Transform.scala:62-97), QUAL rewritten on the device and the
records appended to the output.  Errors are raised in the reference's order:
observe errors partition by partition, finalize, then apply errors partition
by partition; the output file appears only when the job succeeds.
MarkDuplicates groups reads across the whole input (its groupBy): with
-mark_duplicate_reads every partition is parsed once more up front and its
reads' compact MarkDuplicates records (sam.DupSet, bqsr_dup_set_*) collected
on the device; the duplicate bits, found over all partitions, are set on each
partition's parse before BQSR observes it and before it is written.
"""
from __future__ import annotations

import argparse
import ctypes
import mmap
import os
import shutil
import sys
import time
from typing import Dict, List, Optional, Tuple

import numpy as np

from . import _capi, bqsr
from . import distributed as D
from ._capi import check
from .sam import SamText

DEFAULT_PARTITION_BYTES = 8 << 30  # SAM text per partition: ~3x that in HBM while parsed (288 GB per GPU)


def sam_partitions(data, partition_bytes: int) -> Tuple[bytes, List[Tuple[int, int]]]:
    """(header, ranges): the SAM header lines and the byte ranges [a, b) of
    the records, each range cut after the first newline at or beyond
    partition_bytes from its start (so every record lies in one range)."""
    n = len(data)
    pos = 0
    while pos < n and data[pos:pos + 1] == b"@":
        nl = data.find(b"\n", pos)
        pos = n if nl < 0 else nl + 1
    ranges = []
    a = pos
    step = max(1, int(partition_bytes))
    while a < n:
        b = min(n, a + step)
        if b < n:
            nl = data.find(b"\n", b - 1)
            b = n if nl < 0 else nl + 1
        ranges.append((a, b))
        a = b
    return bytes(data[:pos]), ranges


def _bqsr_partitions(data, header: bytes, ranges: List[Tuple[int, int]], snp, ctx, device: int, emit,
                     max_exc: int = 1 << 16, dups=None) -> Dict[str, float]:
    """BQSR over several partitions of one SAM input (see the module doc);
    emit(i, sam) gets every partition's parse with its QUAL fields rewritten,
    in partition order (emit(i, sam, quals): quals = the apply's outputs for
    the parse, handed to the sink).  dups: a finished sam.DupSet over the same
    partitions (MarkDuplicates' bits set on every parse before its batch is
    built and before it is rewritten)."""
    import torch
    L = _capi.lib()
    dev = torch.device("cuda", device)
    stream = torch.cuda.current_stream(dev)
    sp = ctypes.c_void_p(stream.cuda_stream)
    h = ctx.handle
    contigs = snp.contigs if snp else None
    sites_h = snp.handle(ctx) if snp else None
    batches: List[ctypes.c_void_p] = []
    th, lut = ctypes.c_void_p(), ctypes.c_void_p()
    n_reads = 0
    try:
        # (1) every partition parsed on the device and packed into a resident batch
        n_rg = max_len = 1
        slots, reads = [], []
        for a, b in ranges:
            sam = SamText(header + bytes(data[a:b]), ctx)
            try:
                if dups is not None:
                    dups.apply(len(batches), sam)
                bh = sam.device_batch(contigs, sp)  # packed on the device
            finally:
                sam.close()
            batches.append(bh)
            d = L.bqsr_batch_dims(bh)
            n_rg, max_len = max(n_rg, d.n_rg), max(max_len, d.max_len)
            slots.append(int(L.bqsr_batch_slots(bh)))
            reads.append(int(L.bqsr_batch_reads(bh)))
        n_reads = sum(reads)
        # (2) computeTable: every partition observed into the one table, its
        # errors raised partition by partition, expectedMismatch folded in
        # partition order
        dims = _capi.Dims(n_rg, max_len)
        table = torch.zeros(int(L.bqsr_table_words(dims)), dtype=torch.int64, device=dev)
        check(L.bqsr_table_create(h, dims, ctypes.c_void_p(table.data_ptr()), ctypes.byref(th)))
        em = torch.zeros(max(1, len(batches)), dtype=torch.float64, device=dev)
        for i, bh in enumerate(batches):
            check(L.bqsr_observe_async(h, bh, sites_h, th, sp))
            check(L.bqsr_batch_em_copy_async(bh, ctypes.c_void_p(em.data_ptr() + 8 * i), sp))
        for bh in batches:
            v = ctypes.c_double()
            check(L.bqsr_observe_result(bh, ctypes.byref(v), sp))
        acc = D.fold_partition_ems_device(em[:len(batches)], [len(batches)], ctx, stream)
        check(L.bqsr_finalize_device(h, th, ctypes.c_void_p(acc.data_ptr()), ctypes.byref(lut), sp))
        # (3) applyTable partition by partition, each partition's records
        # re-read, rewritten on the device and appended
        out_qual = torch.empty(max(slots or [0]) + 64, dtype=torch.uint8, device=dev)
        out_start = torch.empty(max(1, max(reads or [1])), dtype=torch.int32, device=dev)
        out_len = torch.empty_like(out_start)
        exc = torch.empty(max_exc, dtype=torch.int64, device=dev)
        ptr = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        for i, (a, b) in enumerate(ranges):
            bh = batches[i]
            check(L.bqsr_apply_stage(h, bh, lut, ptr(out_qual), ptr(out_start), ptr(out_len), ptr(exc), max_exc,
                                     _capi.STAGE_RESET | _capi.STAGE_KERNEL, sp))
            v, nexc = ctypes.c_double(), ctypes.c_int64()
            check(L.bqsr_job_result(bh, lut, ctypes.byref(v), ctypes.byref(nexc), sp))
            if nexc.value > max_exc:
                raise _capi.BQSRError(_capi.UNSUPPORTED, "partition %d: %d chars above 0xFF exceed the exception "
                                      "list" % (i, nexc.value))
            sam = SamText(header + bytes(data[a:b]), ctx)
            try:
                if dups is not None:
                    dups.apply(i, sam)
                emit(i, sam, (bh, ptr(out_qual), ptr(out_start), ptr(out_len), ptr(exc), nexc.value, sp))
            finally:
                sam.close()
            L.bqsr_batch_destroy(bh)
            batches[i] = None
    finally:
        if lut:
            L.bqsr_lut_destroy(lut)
        if th:
            L.bqsr_table_destroy(th)
        for bh in batches:
            if bh:
                L.bqsr_batch_destroy(bh)
    return {"reads": n_reads, "partitions": len(ranges)}


def _partitions(data, header: bytes, ranges, mark_duplicates: bool, recalibrate: bool, dbsnp, ctx, device: int,
                emit) -> Dict[str, float]:
    """A SAM input of several partitions: MarkDuplicates over all of them
    (a DupSet: every partition parsed once for its compact records), then
    BQSR over the partitions streamed through the device, or (without BQSR)
    every partition re-parsed, its FLAG fields rewritten and emitted."""
    from .sam import DupSet
    dups = None
    stats: Dict[str, float] = {}
    try:
        if mark_duplicates:
            dups = DupSet(ctx)
            for a, b in ranges:
                sam = SamText(header + bytes(data[a:b]), ctx)
                try:
                    dups.add(sam)
                finally:
                    sam.close()
            n_dup = dups.finish()
        if recalibrate:
            snp = bqsr.SnpTable.from_vcf(dbsnp) if dbsnp else bqsr.SnpTable()
            stats = _bqsr_partitions(data, header, ranges, snp if snp.table else None, ctx, device, emit,
                                     dups=dups)
        else:
            n_reads = 0
            for i, (a, b) in enumerate(ranges):
                sam = SamText(header + bytes(data[a:b]), ctx)
                try:
                    n_reads += sam.counts().n_reads
                    dups.apply(i, sam)
                    emit(i, sam, None)
                finally:
                    sam.close()
            stats = {"reads": n_reads, "partitions": len(ranges)}
        if dups is not None:
            stats["duplicates"] = n_dup
    finally:
        if dups is not None:
            dups.close()
    return stats


def is_parquet(path: str) -> bool:
    """ADAM's own format: a Parquet file (magic PAR1) or a directory of part
    files (what adamSave writes), or a .adam / .parquet name."""
    if path.endswith((".adam", ".parquet")) or os.path.isdir(path):
        return True
    try:
        with open(path, "rb") as fh:
            return fh.read(4) == b"PAR1"
    except OSError:
        return False


def _check_out(path: str, overwrite: bool, adam: bool) -> None:
    """The output path must not exist (adamSave's FileOutputFormat refuses an
    existing one); with overwrite, only a regular file, or (ADAM output) a
    directory of nothing but part files, may be replaced."""
    from .adam_save import is_adam_output
    for p in (path, path + ".partial"):
        if not os.path.lexists(p):
            continue
        if not overwrite:
            raise FileExistsError("output path %s already exists" % p)
        if os.path.isdir(p) and not (adam and is_adam_output(p)):
            raise FileExistsError("refusing to replace directory %s" % p)


def transform_parquet(inp: str, out: str, mark_duplicates: bool = False, recalibrate: bool = False,
                      dbsnp: Optional[str] = None, device: int = 0, overwrite: bool = False) -> Dict[str, float]:
    """`transform` with ADAMRecord Parquet output (adamSave,
    core/rdd/AdamRDDFunctions.scala:37-56): the input -- Parquet (adamLoad,
    AdamContext.scala:318-331, every column kept and written back) or SAM
    (parsed on the host); for Parquet input the Arrow columns go to the device
    (parquet.ArrowReads): MarkDuplicates, the BQSR batch and the rebuilt qual
    column all built there; the qual (and duplicateRead) columns replaced."""
    from . import parquet as P
    from .records import RecordBatch, read_sam_records
    _check_out(out, overwrite, True)
    t0 = time.perf_counter()
    batch = None
    A = None
    if is_parquet(inp):
        table = P.read_table(inp)
    else:
        if mark_duplicates:  # (the host SAM parse carries no library / mateMapped: use SAM output or ADAM input)
            raise ValueError("-mark_duplicate_reads with SAM input and ADAM output is not supported")
        recs = read_sam_records(inp)
        batch = RecordBatch.from_records(recs)
        table = P.batch_to_table(batch, [r.read_name for r in recs])
    n = table.num_rows
    stats: Dict[str, float] = {"reads": n}
    if is_parquet(inp) and (mark_duplicates or recalibrate):
        # the Arrow columns on the device: MarkDuplicates there, the batch
        # packed there, the qual column rebuilt there after apply
        cols = [c for c in table.column_names if c in P.BQSR_PROJECTION or c in P.MARKDUP_PROJECTION]
        A = P.ArrowReads(table.select(cols), bqsr.Context.get(device), markdup=mark_duplicates)
    try:
        return _transform_table(A, table, batch, inp, out, mark_duplicates, recalibrate, dbsnp, device, stats, t0)
    finally:
        if A is not None:
            A.close()


def _transform_table(A, table, batch, inp, out, mark_duplicates, recalibrate, dbsnp, device, stats, t0):
    import pyarrow.parquet as pq

    from . import parquet as P
    from .records import F_DUPLICATE
    n = table.num_rows
    if mark_duplicates:
        stats["duplicates"] = A.mark_duplicates()
        dcol = A.flag_column(F_DUPLICATE)
        table = (table.set_column(table.column_names.index("duplicateRead"), "duplicateRead", dcol)
                 if "duplicateRead" in table.column_names else table.append_column("duplicateRead", dcol))
    if recalibrate:
        snp = bqsr.SnpTable.from_vcf(dbsnp) if dbsnp else bqsr.SnpTable()
        if A is not None:
            from .job import ResidentJob
            job = ResidentJob(None, None, snp if snp.table else None, device,
                              handle=A.device_batch(snp.contigs if snp.table else None))
            try:
                job.step()
                qcol = A.qual_column(job)
            finally:
                job.close()
        else:
            parts = bqsr.adam_bqsr([batch], snp if snp.table else None, bqsr.Context.get(device))
            qcol = P.recalibrated_qual_column(parts, n)
        table = (table.set_column(table.column_names.index("qual"), "qual", qcol)
                 if "qual" in table.column_names else table.append_column("qual", qcol))
    # the new file first, then the old output goes (a failed write leaves the
    # previous output in place); a leftover part-file directory at the
    # .partial path (_check_out allowed it under overwrite) is removed first
    tmp = out + ".partial"
    if os.path.isdir(tmp):
        shutil.rmtree(tmp)
    pq.write_table(table, tmp)
    if os.path.isdir(out):  # (transform_parquet checked it: overwrite of a part-file directory)
        shutil.rmtree(out)
    os.replace(tmp, out)
    stats["seconds"] = time.perf_counter() - t0
    return stats


class _SamOut:
    """SAM text output (records appended partition by partition; the file
    appears when the job succeeds)."""

    def __init__(self, path: str, overwrite: bool = False):
        _check_out(path, overwrite, False)
        self.path = path
        self.tmp = path + ".partial"
        self.fh = open(self.tmp, "wb")
        self.first = True

    def emit(self, i, sam, quals=None):
        """quals: (batch, out_qual, out_start, out_len, exceptions, n, stream)
        of an apply over the parse (None: QUAL kept; FLAG after MarkDuplicates)"""
        if quals is None:
            sam.rewrite(None)
        else:
            check(_capi.lib().bqsr_sam_rewrite_quals(sam.ctx.handle, sam.h, *quals))
        text = sam.text()
        self.fh.write(text if self.first else text[self._header_len(sam):])
        self.first = False

    @staticmethod
    def _header_len(sam) -> int:
        from .adam_save import _lib
        n = ctypes.c_int64()
        check(_lib().bqsr_sam_header_text(sam.h, None, 0, ctypes.byref(n)))
        return int(n.value)

    def close(self, ok: bool = True):
        self.fh.close()
        if ok:
            os.replace(self.tmp, self.path)
        elif os.path.exists(self.tmp):
            os.remove(self.tmp)


class _AdamOut:
    """ADAM output (adamSave): part files of `part_reads` records each."""

    def __init__(self, path: str, compression: str, part_reads: int, overwrite: bool = False):
        from .adam_save import AdamWriter
        self.w = AdamWriter(path, compression, overwrite=overwrite)
        self.part_reads = part_reads

    def emit(self, i, sam, quals=None):
        """the ADAM columns with the apply's quals (no text rewrite)"""
        from .adam_save import set_quals
        if quals is not None:
            set_quals(sam, *quals)
        self.w.emit(sam, self.part_reads)

    def close(self, ok: bool = True):
        self.w.close(ok)


class _Phases:
    """wall time per named phase (the stats' phase split)"""

    def __init__(self):
        self.t: Dict[str, float] = {}

    def __call__(self, name: str):
        import contextlib

        @contextlib.contextmanager
        def cm():
            t0 = time.perf_counter()
            try:
                yield
            finally:
                self.t[name] = self.t.get(name, 0.0) + time.perf_counter() - t0
        return cm()


def _host_bytes(data):
    """the input as a bytes-like object ctypes can pass without a copy: a
    read-only mmap is passed as a numpy view's address"""
    if isinstance(data, mmap.mmap):
        return np.frombuffer(data, np.uint8)
    return data


def is_bam(data) -> bool:
    return bytes(data[:4]) == b"\x1f\x8b\x08\x04"


def transform(inp: str, out: str, mark_duplicates: bool = False, recalibrate: bool = False,
              dbsnp: Optional[str] = None, device: int = 0, partition_bytes: int = DEFAULT_PARTITION_BYTES,
              compression: str = "gzip", part_reads: int = 1 << 19, overwrite: bool = False) -> Dict[str, float]:
    """Transform.run (cli/Transform.scala:62-97) over SAM or BAM input: the
    records parsed on the device (a BAM's records become SAM lines there),
    MarkDuplicates, BQSR, then adamSave (OUT.adam / .parquet / a directory:
    ADAMRecord Parquet part files, adam_save.py) or SAM text.  ADAM Parquet
    input goes through transform_parquet (Arrow reads it on the host)."""
    if is_parquet(inp):
        return transform_parquet(inp, out, mark_duplicates, recalibrate, dbsnp, device, overwrite)
    t0 = time.perf_counter()
    # ADAM output by name, or over an earlier adamSave directory (never just
    # because `out` is some existing directory: the sinks refuse that)
    from .adam_save import is_adam_output
    adam_out = out.endswith((".adam", ".parquet")) or is_adam_output(out)
    sink = _AdamOut(out, compression, part_reads, overwrite) if adam_out else _SamOut(out, overwrite)
    try:
        ctx = bqsr.Context.get(device)
    except BaseException:
        sink.close(False)
        raise
    ok = False
    stats: Dict[str, float] = {}
    try:
        with open(inp, "rb") as fh:
            data = mmap.mmap(fh.fileno(), 0, access=mmap.ACCESS_READ) if os.path.getsize(inp) else b""
            try:
                bam = is_bam(data)
                ranges = None
                if (recalibrate or mark_duplicates) and not bam and len(data):
                    header, ranges = sam_partitions(data, partition_bytes)
                if ranges is not None and len(ranges) > 1:
                    stats = _partitions(data, header, ranges, mark_duplicates, recalibrate, dbsnp, ctx, device,
                                        sink.emit)
                else:
                    ph = _Phases()
                    with ph("parse"):
                        sam = SamText(_host_bytes(data), ctx, bam=bam)
                    try:
                        stats["reads"] = sam.counts().n_reads
                        if mark_duplicates:
                            with ph("markdup"):
                                stats["duplicates"] = sam.mark_duplicates()
                        if recalibrate:
                            from .job import ResidentJob
                            snp = bqsr.SnpTable.from_vcf(dbsnp) if dbsnp else bqsr.SnpTable()
                            with ph("batch"):
                                job = ResidentJob(None, None, snp if snp.table else None, device, sam=sam)
                            try:
                                with ph("bqsr"):
                                    job.step()
                                p = job._ptr
                                with ph("emit"):
                                    sink.emit(0, sam, (job.bh, p(job.out_qual), p(job.out_start), p(job.out_len),
                                                       p(job.exc), job.n_exc, job.sp))
                            finally:
                                job.close()
                        else:
                            with ph("emit"):
                                sink.emit(0, sam, None)
                    finally:
                        sam.close()
                    stats["phases"] = ph.t
            finally:
                if isinstance(data, mmap.mmap):
                    data.close()
        ok = True
    finally:
        t1 = time.perf_counter()
        sink.close(ok)
        stats.setdefault("phases", {})["close"] = time.perf_counter() - t1
    if adam_out:
        stats["parts"] = sink.w.parts
    stats["seconds"] = time.perf_counter() - t0
    return stats


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="adam_amd.transform", description=__doc__.split("\n\n")[0])
    ap.add_argument("input")
    ap.add_argument("output")
    ap.add_argument("-mark_duplicate_reads", action="store_true")
    ap.add_argument("-recalibrate_base_qualities", action="store_true")
    ap.add_argument("-dbsnp_sites", default=None)
    for flag in ("-sort_reads", "-realignIndels"):
        ap.add_argument(flag, action="store_true")
    ap.add_argument("-coalesce", type=int, default=-1)
    ap.add_argument("-partition_bytes", type=int, default=DEFAULT_PARTITION_BYTES,
                    help="records per streamed partition, in bytes of SAM text")
    ap.add_argument("-parquet_compression", default="gzip", choices=("gzip", "snappy", "zstd", "none"),
                    help="ADAM output: the part files' codec (adamSave's default: GZIP)")
    ap.add_argument("-part_reads", type=int, default=1 << 19, help="ADAM output: records per part file")
    ap.add_argument("-overwrite", action="store_true",
                    help="replace an existing output (a file, or a directory of ADAM part files only)")
    a = ap.parse_args(argv)
    if a.sort_reads or a.realignIndels or a.coalesce != -1:
        ap.error("-sort_reads / -coalesce / -realignIndels are outside this build")
    st = transform(a.input, a.output, a.mark_duplicate_reads, a.recalibrate_base_qualities, a.dbsnp_sites,
                   partition_bytes=a.partition_bytes, compression=a.parquet_compression, part_reads=a.part_reads,
                   overwrite=a.overwrite)
    print(" ".join("%s=%s" % kv for kv in st.items()), file=sys.stderr)
    return 0


if __name__ == "__main__":
    sys.exit(main())
