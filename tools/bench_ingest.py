"""SAM ingest throughput (§8 f1): synthetic SAM text (cfg2-like reads)
parsed by bqsr_sam_parse; prints one JSON line.  Run under rocprofv3
--kernel-trace --stats to split the device kernels from the H2D copy."""
import argparse
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
    a = ap.parse_args()
    import numpy as np
    import torch
    from adam_amd import bqsr, synth
    from adam_amd.records import read_sam  # noqa: F401  (the restatement the columns match)
    from adam_amd.sam import SamText
    from adam_amd.samgen import sam_text
    torch.zeros(1, device="cuda")
    t0 = time.perf_counter()
    b = synth.generate(a.reads, (a.len,), 1, 20261015 + 2)
    text = sam_text(b)
    t_gen = time.perf_counter() - t0
    ctx = bqsr.Context.get(0)
    # pinned host copy: the H2D runs at the link's rate
    pinned = torch.empty(len(text), dtype=torch.uint8, pin_memory=True)
    pinned.numpy()[:] = np.frombuffer(text, np.uint8)
    import ctypes
    from adam_amd.sam import _lib
    L = _lib()
    times = []
    for _ in range(a.reps):
        h = ctypes.c_void_p()
        t0 = time.perf_counter()
        from adam_amd._capi import check
        check(L.bqsr_sam_parse(ctx.handle, ctypes.c_char_p(pinned.data_ptr()), len(text), None, ctypes.byref(h)))
        times.append(time.perf_counter() - t0)
        L.bqsr_sam_destroy(h)
    t = min(times)
    print(json.dumps({"metric": "SAM ingest reads/s (text in pinned host memory -> device columns)",
                      "reads": a.reads, "read_len": a.len, "text_bytes": len(text), "seconds": t,
                      "reads_per_s": a.reads / t, "GB_per_s": len(text) / t / 1e9, "gen_seconds": t_gen}))


if __name__ == "__main__":
    main()
