"""End-to-end `transform IN.sam OUT.adam [-mark_duplicate_reads]
-recalibrate_base_qualities` throughput (§8 f2): synthetic cfg2-like reads as
SAM text (or BAM) in a file, the whole transform timed -- device parse,
MarkDuplicates, BQSR, ADAM columns on the device, Parquet part files written
by host threads -- and one JSON line printed with the phase split.

    python tools/bench_adam.py --reads 10000000 [--bam] [--no-markdup]
        [--compression none|snappy|gzip] [--part-reads N] [--partition-bytes B]
"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


CHUNK = 500_000


def log(msg):
    print("[bench_adam] " + msg, file=sys.stderr, flush=True)


def _chunk(args):
    from adam_amd import synth
    from adam_amd.samgen import sam_text
    r0, n, read_len, total = args
    b = synth.generate(n, (read_len,), 2, 20261015 + 2, first_read=r0)
    text = sam_text(b, n_rg=2, qname="c%d_" % (r0 // CHUNK))
    if r0:  # the header once
        text = b"".join(l + b"\n" for l in text.split(b"\n") if l and not l.startswith(b"@"))
    return text


def synthetic_sam(n_reads: int, read_len: int) -> bytes:
    """cfg2-like reads as SAM text, generated in slices by a process pool
    (before the GPU is touched); QNAMEs unique per read"""
    from multiprocessing import get_context
    jobs = [(r0, min(CHUNK, n_reads - r0), read_len, n_reads) for r0 in range(0, n_reads, CHUNK)]
    # close() + join(), not the context manager: its terminate() SIGTERMs
    # workers still unwinding (under rocprofv3 the signal handler prints an
    # abort trace)
    pool = get_context("fork").Pool(min(16, max(1, len(jobs)), os.cpu_count() or 1))
    try:
        parts = []
        for i, t in enumerate(pool.imap(_chunk, jobs)):
            parts.append(t)
            log("slice %d / %d" % (i + 1, len(jobs)))
        pool.close()
    except BaseException:
        pool.terminate()
        raise
    finally:
        pool.join()
    return b"".join(parts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=2_000_000)
    ap.add_argument("--len", type=int, default=100)
    ap.add_argument("--bam", action="store_true")
    ap.add_argument("--bgzf", type=int, default=1, help="BAM: 1 inflate on the device (default), 0 on host threads")
    ap.add_argument("--no-markdup", action="store_true")
    ap.add_argument("--compression", default="snappy")
    ap.add_argument("--part-reads", type=int, default=1 << 19)
    ap.add_argument("--partition-bytes", type=int, default=8 << 30)
    ap.add_argument("--reps", type=int, default=1)
    ap.add_argument("--dir", default=None, help="scratch directory (default: a temporary one)")
    a = ap.parse_args()
    t0 = time.perf_counter()
    data = synthetic_sam(a.reads, a.len)
    if a.bam:
        from adam_amd.bam_writer import sam_to_bam_parallel
        data = sam_to_bam_parallel(data, min(16, os.cpu_count() or 1),
                                   progress=lambda i, n: log("bam slice %d / %d" % (i, n)) if i % 8 == 0 else None)
    t_gen = time.perf_counter() - t0
    log("generated %d bytes in %.1f s" % (len(data), t_gen))
    import torch
    from adam_amd import bqsr
    from adam_amd import transform as T
    torch.zeros(1, device="cuda")
    bqsr.Context.get(0).tune(bgzf=a.bgzf)
    work = a.dir or tempfile.mkdtemp(prefix="bench_adam_")
    os.makedirs(work, exist_ok=True)
    src = os.path.join(work, "in.bam" if a.bam else "in.sam")
    with open(src, "wb") as fh:
        fh.write(data)
    n_bytes = len(data)
    del data
    out = os.path.join(work, "out.adam")
    try:
        # warm: the first call builds the context and loads pyarrow
        log("warm-up transform")
        T.transform(src, out, mark_duplicates=not a.no_markdup, recalibrate=True,
                    partition_bytes=a.partition_bytes, compression=a.compression, part_reads=a.part_reads,
                    overwrite=True)
        best = None
        for _ in range(a.reps):
            log("timed transform")
            t0 = time.perf_counter()
            st = T.transform(src, out, mark_duplicates=not a.no_markdup, recalibrate=True,
                             partition_bytes=a.partition_bytes, compression=a.compression, part_reads=a.part_reads,
                             overwrite=True)
            dt = time.perf_counter() - t0
            if best is None or dt < best[0]:
                best = (dt, st)
        dt, st = best
        out_bytes = sum(os.path.getsize(os.path.join(out, f)) for f in os.listdir(out))
        if st["reads"] != a.reads:
            raise SystemExit("transformed %d reads, expected %d" % (st["reads"], a.reads))
        print(json.dumps({
            "metric": "transform %s -> ADAM Parquet reads/s (device parse, %sBQSR, ADAM columns on the device, "
                      "part files by host threads)" % ("BAM" if a.bam else "SAM",
                                                       "" if a.no_markdup else "MarkDuplicates, "),
            "reads": a.reads, "read_len": a.len, "input_bytes": n_bytes, "output_bytes": out_bytes,
            "seconds": dt, "reads_per_s": a.reads / dt, "compression": a.compression,
            "bgzf": (("device" if a.bgzf else "host threads") if a.bam else None),
            "part_reads": a.part_reads, "partition_bytes": a.partition_bytes, "gen_seconds": t_gen,
            "stats": {k: v for k, v in st.items()}}))
    finally:
        if not a.dir:
            shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()
