"""SAM / BAM ingest throughput (§8 f1): synthetic SAM text (cfg2-like reads)
parsed by bqsr_sam_parse, or the same records as BAM (adam_amd/bam_writer.py)
through bqsr_bam_parse (BGZF inflated on the device or, --bgzf 0, on host
threads; records decoded on the device); prints one JSON line.  Run under rocprofv3 --kernel-trace --stats to
split the device kernels from the H2D copy."""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=2_000_000)
    ap.add_argument("--len", type=int, default=100)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--bam", action="store_true", help="BAM input (BGZF) instead of SAM text")
    ap.add_argument("--bgzf", type=int, default=1, help="BAM: 1 inflate on the device (default), 0 on host threads")
    a = ap.parse_args()
    import numpy as np
    import torch
    from adam_amd import bqsr, synth
    from adam_amd._capi import check
    from adam_amd.sam import _lib
    from adam_amd.samgen import sam_text
    torch.zeros(1, device="cuda")
    t0 = time.perf_counter()
    b = synth.generate(a.reads, (a.len,), 1, 20261015 + 2)
    data = sam_text(b)
    if a.bam:
        from adam_amd.bam_writer import sam_to_bam
        data = sam_to_bam(data)
    t_gen = time.perf_counter() - t0
    ctx = bqsr.Context.get(0)
    ctx.tune(bgzf=a.bgzf)
    # pinned host copy: the H2D runs at the link's rate
    pinned = torch.empty(len(data), dtype=torch.uint8, pin_memory=True)
    pinned.numpy()[:] = np.frombuffer(data, np.uint8)
    L = _lib()
    parse = L.bqsr_bam_parse if a.bam else L.bqsr_sam_parse
    times = []
    n_reads = 0
    for _ in range(a.reps):
        h = ctypes.c_void_p()
        t0 = time.perf_counter()
        check(parse(ctx.handle, ctypes.c_char_p(pinned.data_ptr()), len(data), None, ctypes.byref(h)))
        times.append(time.perf_counter() - t0)
        from adam_amd.sam import SamCounts
        c = SamCounts()
        check(L.bqsr_sam_get_counts(h, ctypes.byref(c)))
        n_reads = c.n_reads
        L.bqsr_sam_destroy(h)
    if n_reads != a.reads:
        raise SystemExit("parsed %d records, expected %d" % (n_reads, a.reads))
    t = min(times)
    fmt = ("BAM (BGZF in pinned host memory -> inflate on %s -> device columns)" %
           ("the device" if a.bgzf else "host threads")) if a.bam else "SAM text in pinned host memory -> device columns"
    print(json.dumps({"metric": "%s ingest reads/s (%s)" % ("BAM" if a.bam else "SAM", fmt),
                      "reads": a.reads, "read_len": a.len, "input_bytes": len(data), "seconds": t,
                      "reads_per_s": a.reads / t, "GB_per_s": len(data) / t / 1e9, "gen_seconds": t_gen,
                      "inflate": ("device" if a.bgzf else "host %d threads" % min(16, os.cpu_count() or 1)) if a.bam else None}))


if __name__ == "__main__":
    main()
