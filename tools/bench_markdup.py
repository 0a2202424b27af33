"""MarkDuplicates throughput (§8 f3): synthetic SAM text (pairs and
fragments, 2 read groups / libraries) parsed on the device, then
bqsr_sam_mark_duplicates timed; prints one JSON line."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=10_000_000)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import ctypes
    import numpy as np
    import torch
    from adam_amd import bqsr, synth
    from adam_amd._capi import check
    from adam_amd.sam import _lib
    torch.zeros(1, device="cuda")
    t0 = time.perf_counter()
    # cfg2-like reads on a 30x-deep 3.3 Mbp stretch: many same-position buckets
    b = synth.generate(a.reads, (100,), 2, 20261015 + 6, contig_len=a.reads * 100 // 30, p_duplicate=0.0)
    from adam_amd.samgen import sam_text
    text = sam_text(b, n_rg=2, qname="q")
    t_gen = time.perf_counter() - t0
    ctx = bqsr.Context.get(0)
    pinned = torch.empty(len(text), dtype=torch.uint8, pin_memory=True)
    pinned.numpy()[:] = np.frombuffer(text, np.uint8)
    L = _lib()
    times, nd = [], 0
    for _ in range(a.reps):
        h = ctypes.c_void_p()
        check(L.bqsr_sam_parse(ctx.handle, ctypes.c_char_p(pinned.data_ptr()), len(text), None, ctypes.byref(h)))
        n = ctypes.c_int64()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        check(L.bqsr_sam_mark_duplicates(h, ctypes.byref(n)))
        times.append(time.perf_counter() - t0)
        nd = int(n.value)
        L.bqsr_sam_destroy(h)
    t = min(times)
    print(json.dumps({"metric": "MarkDuplicates reads/s (device columns of a parsed SAM, flags rewritten in place)",
                      "reads": a.reads, "duplicates": nd, "seconds": t, "reads_per_s": a.reads / t,
                      "path": os.environ.get("ADAM_BQSR_MARKDUP", "device"), "gen_seconds": t_gen}))


if __name__ == "__main__":
    main()
