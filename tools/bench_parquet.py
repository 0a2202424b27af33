"""ADAMRecord Parquet read throughput (§8 f1, adamLoad with the BQSR
projection): a synthetic cfg2-like file written once, then timed: Arrow
decodes the projected columns on host threads, the buffers go to the device
as they are (parquet.ArrowReads) and are packed into a BQSR batch there.
Prints one JSON line with the split (Arrow decode / device load / batch)."""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=2_000_000)
    ap.add_argument("--len", type=int, default=100)
    ap.add_argument("--compression", default="snappy")
    ap.add_argument("--row-group", type=int, default=0,
                    help="rows per row group (0: 128 MB of column data, parquet-mr's block size in adamSave)")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import pyarrow.parquet as pq
    from adam_amd import parquet as P, synth
    t0 = time.perf_counter()
    b = synth.generate(a.reads, (a.len,), 2, 20261015 + 2)
    table = P.batch_to_table(b)
    del b
    work = tempfile.mkdtemp(prefix="bench_parquet_")
    path = os.path.join(work, "reads.parquet")
    rg = a.row_group or max(1, (128 << 20) * table.num_rows // max(1, table.nbytes))
    pq.write_table(table, path, compression=a.compression, row_group_size=rg)
    del table
    t_gen = time.perf_counter() - t0
    print("[bench_parquet] wrote %d bytes in %.1f s" % (os.path.getsize(path), t_gen), file=sys.stderr, flush=True)
    import torch
    from adam_amd import bqsr
    from adam_amd._capi import lib
    torch.zeros(1, device="cuda")
    ctx = bqsr.Context.get(0)
    L = lib()
    best = None
    try:
        for _ in range(a.reps + 1):  # the first is a warm-up
            t0 = time.perf_counter()
            t = P.read_table(path, P.BQSR_PROJECTION)
            t1 = time.perf_counter()
            A = P.ArrowReads(t, ctx)
            t2 = time.perf_counter()
            bh = A.device_batch()
            t3 = time.perf_counter()
            n = int(L.bqsr_batch_reads(bh))
            L.bqsr_batch_destroy(bh)
            A.close()
            del t
            if n != a.reads:
                raise SystemExit("read %d records, expected %d" % (n, a.reads))
            split = (t3 - t0, t1 - t0, t2 - t1, t3 - t2)
            if best is None or split[0] < best[0]:
                best = split
    finally:
        shutil.rmtree(work, ignore_errors=True)
    tot, dec, load, pack = best
    print(json.dumps({"metric": "ADAM Parquet read reads/s (Arrow decode on host threads -> buffers to the device -> "
                                "parse layout and BQSR batch on the device)",
                      "reads": a.reads, "read_len": a.len, "compression": a.compression, "row_group_rows": rg,
                      "seconds": tot, "reads_per_s": a.reads / tot,
                      "split_s": {"arrow_decode": dec, "device_load": load, "batch_pack": pack},
                      "gen_seconds": t_gen}))


if __name__ == "__main__":
    main()
