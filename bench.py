#!/usr/bin/env python3
"""BQSR (observe + apply) throughput on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg2]

One step = one whole BQSR job over the GPU's read shard, inputs resident in
HBM: zero the covariate table, observe (+ the exact expectedMismatch fold),
[N > 1: RCCL int64 all-reduce of the table, all-gather of the per-shard
expectedMismatch folded in rank order], finalize, apply.  `bases` = sum of the
sequence lengths of ALL reads (filtered ones included).  The ranks' shards
are consecutive read ranges of one synthetic dataset (cfg2 / cfg4: the
config's reads per GPU, weak scaling; cfg3: the 60M-read set split over the
ranks), the job's partitions in rank order.  After the timed jobs every rank
checks the last job's table, expectedMismatch and recalibrated chars against
the oracle (oracle/, outside the timed region); rank 0 prints one JSON line.
See DESIGN.md "Measurement".
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "BQSR bases/sec (observe+apply) at 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s HBM3E peak (spec)

WORKLOADS = {
    "cfg2": "cfg2: synthetic 10M x 100 bp reads, 1 read group, no known sites (per GPU)",
    "cfg3": "cfg3: synthetic 60M x 101 bp reads on a 64.4 Mbp contig, ~1.3M known sites (sharded)",
    "cfg4": "cfg4: synthetic 20M reads 150/250 bp, 96 read groups (per GPU)",
    "cfg5": "cfg5: whole-genome 30x slice, 150 bp reads streamed from pinned host memory in 4M-read partitions, "
            "H2D/D2H overlapped with compute (600M reads / 8 GPUs = 75M reads per GPU)",
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU).  Without WORLD_SIZE in the environment and N > 1 this process "
                         "launches the N ranks itself; under torch.distributed.run it must equal WORLD_SIZE")
    ap.add_argument("--backend", default="nccl", choices=("nccl", "gloo"),
                    help="torch.distributed backend (nccl = RCCL over xGMI; gloo: host collectives, ranks may "
                         "share a GPU -- tests)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="cfg2", choices=sorted(WORKLOADS))
    ap.add_argument("--reads", type=int, default=None, help="reads per GPU (default: the config's)")
    ap.add_argument("--sorted", action="store_true",
                    help="coordinate-sorted reads (as after transform -sort_reads; the known-site A/B of cfg3)")
    ap.add_argument("--cpu-reads", type=int, default=10_000_000, help="oracle baseline sample (reads)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true", help="skip the oracle check of the timed job's results")
    ap.add_argument("--event-steps", type=int, default=3,
                    help="untimed jobs after the timed region whose stages are timed with HIP events")
    ap.add_argument("--tune", action="append", default=[], metavar="KNOB=V",
                    help="bqsr_context_tune layout knob for an A/B run (order, fronts, key_major)")
    ap.add_argument("--traffic", default=None,
                    help="PMC traffic json (default profiles/pmc_traffic_<config>.json)")
    ap.add_argument("--part-reads", type=int, default=4_000_000, help="cfg5: reads per streamed partition")
    ap.add_argument("--stream-mode", default="pipe", choices=("pipe", "serial", "zerocopy"),
                    help="cfg5: jobs pipelined over both link directions, one at a time, or pipelined with "
                         "apply writing into pinned host memory")
    ap.add_argument("--d2h", default="kernel", choices=("kernel", "dma"),
                    help="cfg5: results copied back by a kernel (beside the DMA uploads) or by DMA copies")
    return ap.parse_args(argv)


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch(n: int, child_argv, poll_s: float = 0.2, out=None) -> int:
    """Start `n` ranks of `child_argv` (a command list) as fresh child
    processes -- RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT
    set, the way torch.distributed.run would -- wait for all of them, relay
    rank 0's stdout (the JSON line) and return 0, or the first failing rank's
    exit status (the other ranks are then terminated: a rank left waiting in
    a collective would never return).  The launcher itself never touches the
    GPU (it does not import torch)."""
    import subprocess
    import tempfile
    out = out or sys.stdout
    port = _free_port()
    procs = []
    line0 = tempfile.TemporaryFile()
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(child_argv, env=env, stdout=line0 if r == 0 else 2))
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                break
            if all(c == 0 for c in codes):
                break
            time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    line0.seek(0)
    text = line0.read().decode()
    line0.close()
    if rc == 0:
        out.write(text)
        out.flush()
    else:
        sys.stderr.write(text)
        print("bench: a rank failed (exit status %d); no result line" % rc, file=sys.stderr, flush=True)
    return rc


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and (args.gpus or 1) > 1:
        # bench.py --gpus N without a launcher: start the N ranks here
        sys.exit(launch(args.gpus, [sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:]))
    import numpy as np
    import torch
    import torch.distributed as dist

    from adam_amd import _capi, bqsr, synth
    from adam_amd import distributed as D
    from adam_amd._capi import Dims, check

    world = int(env_world or "1")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus is not None and args.gpus != world:
        raise SystemExit("bench: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    # a rank per GPU; with gloo (tests) ranks beyond the device count share GPUs.
    # device_count() does not initialise the GPU on this runtime.
    n_dev = torch.cuda.device_count()
    if n_dev < 1:
        raise SystemExit("bench: no HIP device")
    if world > n_dev and args.backend == "nccl":
        raise SystemExit("bench: %d ranks over RCCL need %d GPUs (%d visible); use --backend gloo to share" %
                         (world, world, n_dev))
    dev_index = local % n_dev
    dev = torch.device("cuda", dev_index)
    torch.cuda.set_device(dev)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            torch.zeros(1, device=dev)  # torch's HIP runtime up before the library's
            dist.init_process_group("gloo")
        if dist.get_world_size() != world:
            raise SystemExit("bench: process group has %d ranks, expected %d" % (dist.get_world_size(), world))
    L = _capi.lib()
    ctx = bqsr.Context.get(dev_index)
    if args.tune:
        ctx.tune(**{k: (v if v in ("auto", "read", "group") else int(v)) for k, v in (t.split("=", 1) for t in args.tune)})

    cfg = dict(synth.CONFIGS[args.config])
    if args.config == "cfg5":
        return main_stream(args, cfg, world, rank, dev, ctx)
    # one dataset per job (seed, config): cfg3 is the 60M-read set sharded by
    # read index over the ranks; cfg2 / cfg4 give every rank the config's read
    # count (weak scaling) as reads [rank*n, (rank+1)*n) of one bigger set --
    # the ranks' shards are the job's partitions in rank order either way
    if args.config == "cfg3":
        total = args.reads or cfg["n_reads"]
        r0, r1 = D.shard_bounds(total, rank, world)
    else:
        n = args.reads or cfg["n_reads"]
        r0, r1 = rank * n, (rank + 1) * n
    n_reads = r1 - r0
    t_gen = time.time()
    total = (args.reads or cfg["n_reads"]) * (1 if args.config == "cfg3" else world)
    batch = synth.generate(n_reads, cfg["lens"], cfg["n_rg"], cfg["seed"], first_read=r0,
                           sorted_total=total if args.sorted else 0)
    sites = synth.known_sites(cfg["sites"]) if cfg["sites"] else None
    snp = bqsr.SnpTable(sites) if sites else None
    t_gen = time.time() - t_gen
    n_bases = batch.n_bases

    from adam_amd.job import ResidentJob
    job = ResidentJob(batch, Dims(cfg["n_rg"], max(cfg["lens"])), snp, dev_index, read_base=r0)

    for _ in range(args.warmup):
        job.step(False)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        job.step(False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # per-stage times: HIP events on the launch stream over extra jobs after
    # the timed region (an event record costs the stream ~30 us, so the timed
    # jobs carry none; the stage times include their launch gaps)
    for _ in range(max(0, args.event_steps)):
        job.step(True)
    torch.cuda.synchronize()
    # what a bucketed batch pays once at creation, outside the repeated job:
    # the piece-key sort and the key-major copy (bqsr_batch_relayout)
    layout_ms = job.layout_ms()
    layout_created = job.layout_times()
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        D.allreduce(t, dist.ReduceOp.MAX)
        elapsed = float(t.item())
        nb = torch.tensor([n_bases], dtype=torch.int64, device=dev)
        D.allreduce(nb)
        total_bases = int(nb.item())
    else:
        total_bases = n_bases
    kt = job.kt

    # parity of the last job's results against the oracle (every rank checks
    # its own shard; N > 1 with the all-reduced oracle table), outside the
    # timed region; the CPU baseline on rank 0 at N = 1
    cpu_line, parity = None, None
    if world == 1:
        ref = None
        if not args.no_cpu_baseline:
            cpu_line, ref = cpu_baseline(args, cfg, batch, sites, whole=not args.no_parity)
        if not args.no_parity:
            if ref is None:
                ref = oracle_shard(cfg, batch, sites)
            parity = parity_check(job, batch, ref)
            del ref
    elif not args.no_parity:
        parity = parity_multi(job, cfg, batch, sites, world, rank, dev)

    if rank == 0:
        ms = {k: float(np.mean(v)) for k, v in kt.items() if v}
        R = batch.n_reads
        # algorithmic bytes: observe 1.75 B/base + 16 B/read, apply 2.5 B/base + 16 B/read
        alg = {"observe": 1.75 * n_bases + 16 * R, "apply": 2.5 * n_bases + 16 * R}
        tpath = args.traffic or os.path.join(ROOT, "profiles", "pmc_traffic_%s.json" % args.config)
        tr = _profile_json(tpath, args.config, R)  # PMC bytes per launch (tools/make_traffic.py)
        kpath = os.path.join(ROOT, "profiles", "kernel_stats_%s.json" % args.config)
        ks = _profile_json(kpath, args.config, R)  # rocprofv3 kernel averages (tools/make_kstats.py)
        # the dominant kernel: the longer one by rocprof's kernel-only averages of
        # this tree's committed profile; by the live HIP events without one
        rp = {k: ks["kernels"][k]["avg_ms"] for k in alg if ks and k in ks["kernels"]}
        src = rp if len(rp) == 2 else ms
        dom = "observe" if src.get("observe", 0) >= src.get("apply", 0) else "apply"
        kernels = {}
        for k in alg:
            e = {"alg_bytes_per_launch": alg[k], "events_ms": ms.get(k),
                 "events_frac": alg[k] / (ms[k] * 1e-3) / 1e9 / HBM_PEAK_GBS if ms.get(k) else None}
            if k in rp:
                e.update(kernel=ks["kernels"][k]["kernel"], rocprof_ms=rp[k],
                         rocprof_frac=alg[k] / (rp[k] * 1e-3) / 1e9 / HBM_PEAK_GBS)
            if tr and k in tr["kernels"]:
                e.update(traffic=tr["kernels"][k]["hbm_bytes_per_launch"],
                         traffic_x_alg=tr["kernels"][k]["hbm_bytes_per_launch"] / alg[k])
            kernels[k] = e
        kernels["dominant"] = dom
        achieved = alg[dom] / (ms[dom] * 1e-3) / 1e9 if dom in ms else None
        traffic = kernels[dom].get("traffic")
        kname = kernels[dom].get("kernel", "bqsr_%s" % dom)
        value = args.steps * total_bases / elapsed
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "bases/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak" if args.config != "cfg3" else "strong",
            "vs_baseline": None,
            "dtype": "u8 in, int64 counts, f64 recalibration",
            "data": "synthetic (deterministic generator, SURVEY.md 8d spec), resident in HBM",
            "config": {
                "workload": WORKLOADS[args.config] + (" (coordinate-sorted)" if args.sorted else ""),
                "reads_per_gpu": R,
                "bases_per_gpu": n_bases,
                "reads_total": R * world if args.config != "cfg3" else (args.reads or cfg["n_reads"]),
                "read_len": list(cfg["lens"]),
                "read_groups": cfg["n_rg"],
                "known_sites": int(sum(len(v) for v in sites.values())) if sites else 0,
                "parallelism": "dp%d: read shards per GPU, RCCL int64 table all-reduce" % world,
            },
            "roofline": {
                "bound": "hbm",
                "kernel": kname,
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS if achieved else None,
                "traffic": traffic,
                "traffic_source": tpath if traffic is not None else None,
                "alg_bytes_per_launch": alg[dom],
                "kernel_ms": ms,
                "kernel_ms_method": "HIP events on the launch stream around each stage over %d untimed jobs after "
                                    "the timed region (apply: the kernel alone, its char tables before the "
                                    "bracket)" % args.event_steps,
                "kernels": kernels,
                "kernels_source": {"rocprof": kpath if rp else None, "commit": ks.get("commit") if ks else None},
            },
            "hbm_roofline_frac_step": (total_bases / world) * (4.25 + 32.0 / max(cfg["lens"])) /
                                      (elapsed / args.steps) / (HBM_PEAK_GBS * 1e9),
            "layout_ms": layout_ms,
            "layout_alloc_ms": layout_created[0] if layout_created else None,
            "layout_build_ms": layout_created[1] if layout_created else None,
            "job_with_layout_ms": ((elapsed / args.steps * 1e3 + layout_created[0] + layout_created[1])
                                   if layout_created else None),
            "layout_note": ("bucketed batch: the piece-key sort (and, with key_major=1, the key-major copy of "
                            "quals / codes) runs once when the batch is created (outside the timed jobs); "
                            "layout_alloc_ms / layout_build_ms are its allocation and kernel wall times at creation, "
                            "layout_ms the kernels redone on the batch, job_with_layout_ms a single job that pays "
                            "both -- the single-pass cost of a partition")
                           if layout_created else None,
            "gen_s": t_gen,
        }
        if cpu_line is not None:
            line["cpu_baseline"] = cpu_line
        if parity is not None:
            line["parity"] = parity
        print(json.dumps(line), flush=True)
    job.close()
    if world > 1:
        dist.destroy_process_group()


def _profile_json(path, config, reads):
    """A committed profile summary (profiles/*.json) when it was taken on
    this config and shard size, else None."""
    try:
        with open(path) as fh:
            d = json.load(fh)
    except (OSError, ValueError):
        return None
    if d.get("config") != config or d.get("reads_per_gpu") != reads or "kernels" not in d:
        return None
    return d


def oracle_shard(cfg, batch, sites):
    """The oracle over the whole shard as ONE partition (table by partitions in
    parallel, expectedMismatch folded sequentially), for the parity check."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    cores, _ = host_cores()
    osites = O.Sites(sites) if sites else None
    d = O.Dims(cfg["n_rg"], max(cfg["lens"]))
    words, em = O.observe_mt(batch, osites, d, n_parts=cores, nthreads=cores, fold1=True)
    out, out_len = O.apply_mt(batch, d, words, em, n_parts=cores, nthreads=cores)
    return words, em, out, out_len


def parity_check(job, batch, ref):
    """The timed job's own results (last step) against the oracle run over the
    same shard as ONE partition: table words and expectedMismatch bit for bit,
    every read's recalibrated chars (outside the timed region)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle as O
    t = time.perf_counter()
    words, em, q, st, ln, exc = job.results()
    rw, rem, rout, rlen = ref
    table_ok = bool(np.array_equal(words, rw))
    em_ok = em == rem
    bad, first = O.compare_device_output(batch, rout, rlen, q, st, ln, exc if len(exc) else None,
                                         nthreads=max(1, len(os.sched_getaffinity(0))))
    return {"checked": True, "ok": bool(table_ok and em_ok and bad == 0), "table_words_equal": table_ok,
            "expected_mismatch_equal": bool(em_ok), "expected_mismatch": float(em).hex(),
            "reads_checked": batch.n_reads, "reads_differing": bad, "first_differing_read": first,
            "chars_above_0xff": int(len(exc)),
            "against": "oracle/ (C++ restatement of ADAM BQSR) on the same shard as one partition, "
                       "table built by partitions in parallel, expectedMismatch folded sequentially",
            "check_s": time.perf_counter() - t}


def parity_multi(job, cfg, batch, sites, world, rank, dev):
    """N > 1 (called on every rank): each rank runs the oracle's observe over
    its own shard as one partition; the oracle tables are all-reduced and the
    shards' expectedMismatch values folded in rank order (the job's partitions
    merged in partition order, RecalibrateBaseQualities.scala:63); each rank
    then checks the GPU's all-reduced table, the job's expectedMismatch and
    its own recalibrated chars against the oracle's apply with that table.
    Mismatch counts and equalities are reduced to every rank."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import torch
    import torch.distributed as dist
    import oracle as O
    from adam_amd import distributed as D
    t = time.perf_counter()
    cores, _ = host_cores()
    osites = O.Sites(sites) if sites else None
    d = O.Dims(cfg["n_rg"], max(cfg["lens"]))
    words, em_shard = O.observe_mt(batch, osites, d, n_parts=cores, nthreads=cores, fold1=True)
    wt = torch.from_numpy(words).to(dev)
    D.allreduce_table(wt)
    rwords = wt.cpu().numpy()
    rem = D.fold_expected_mismatch(em_shard, dev)
    rout, rlen = O.apply_mt(batch, d, rwords, rem, n_parts=cores, nthreads=cores)
    gw, gem, q, st, ln, exc = job.results()
    table_ok = bool(np.array_equal(gw, rwords))
    em_ok = gem == rem
    bad, first = O.compare_device_output(batch, rout, rlen, q, st, ln, exc if len(exc) else None,
                                         nthreads=max(1, cores))
    first_g = (job.read_base + first) if bad else np.iinfo(np.int64).max
    red = torch.tensor([bad, int(not table_ok), int(not em_ok), len(exc), batch.n_reads], dtype=torch.int64,
                       device=dev)
    D.allreduce(red)
    fr = torch.tensor([first_g], dtype=torch.int64, device=dev)
    D.allreduce(fr, dist.ReduceOp.MIN)
    red = red.cpu().tolist()
    fr = int(fr.item())
    return {"checked": True, "ok": red[0] == 0 and red[1] == 0 and red[2] == 0,
            "table_words_equal": red[1] == 0, "expected_mismatch_equal": red[2] == 0,
            "expected_mismatch": float(gem).hex(), "reads_checked": red[4], "reads_differing": red[0],
            "first_differing_read": fr if red[0] else -1, "chars_above_0xff": red[3], "ranks": world,
            "against": "oracle/ (C++ restatement of ADAM BQSR): every rank's shard as one partition, oracle tables "
                       "all-reduced, shard expectedMismatch folded in rank order; every rank checks its own chars",
            "check_s": time.perf_counter() - t}


def main_stream(args, cfg, world, rank, dev, ctx):
    """cfg5: the rank's 1/8 of a 600M x 150 bp whole genome (75M reads), held
    on the host as pinned 4M-read partitions in the device layout; one step =
    upload + observe every partition (copy stream overlapped with compute),
    partition-order expectedMismatch fold, [N > 1: all-reduce + rank fold],
    finalize, apply every partition with its results copied back to pinned
    host memory.  PCIe-inclusive, end to end."""
    import numpy as np
    import torch
    import torch.distributed as dist

    from adam_amd import _capi, synth
    from adam_amd import distributed as D
    from adam_amd._capi import Dims, check
    from adam_amd.stream import StreamedShard

    L = _capi.lib()
    n_reads = args.reads or cfg["n_reads"] // 8
    pr = max(1, args.part_reads)
    dims = Dims(cfg["n_rg"], max(cfg["lens"]))
    t_gen = time.time()
    # rank r holds reads [r*n, (r+1)*n) of the one 600M-read dataset (the
    # generator is indexed by global read), as partitions of `pr` reads
    base = rank * n_reads
    sh = StreamedShard(ctx, [], dims, None, dev.index, zero_copy=args.stream_mode == "zerocopy", d2h=args.d2h,
                       read_base=base)
    first = None
    for i, r0 in enumerate(range(0, n_reads, pr)):
        part = synth.generate(min(pr, n_reads - r0), cfg["lens"], cfg["n_rg"], cfg["seed"], first_read=base + r0)
        sh.add_partition(part)
        if first is None:
            first = part
        del part
        if rank == 0 and i % 4 == 0:
            print("cfg5: staged %d / %d reads" % (min(n_reads, r0 + pr), n_reads), file=sys.stderr, flush=True)
    sh.alloc_outputs()
    t_gen = time.time() - t_gen
    words = int(L.bqsr_table_words(dims))
    table_t = torch.zeros(words, dtype=torch.int64, device=dev)
    th = ctypes.c_void_p()
    check(L.bqsr_table_create(ctx.handle, dims, ctypes.c_void_p(table_t.data_ptr()), ctypes.byref(th)))
    torch.cuda.synchronize()

    def step(record):
        # jobs pipeline (stream.py): this job's uploads overlap the previous
        # job's downloads; its status is checked one job later
        sh.run(th, table_t if world > 1 else None, record_apply=record)
        if len(sh.pending) > (0 if args.stream_mode == "serial" else 1):
            sh.finish()

    for _ in range(args.warmup):
        step(False)
    while sh.pending:
        sh.finish()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i == args.steps - 1)
    while sh.pending:  # every job's results on the host, every status checked
        sh.finish()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    apply_ms = [sh.apply_ms()]
    probe_ms = sh.apply_probe_ms(0)  # the kernel alone (no copies in flight), for the roofline
    n_bases = sh.n_bases
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        D.allreduce(t, dist.ReduceOp.MAX)
        elapsed = float(t.item())
        nb = torch.tensor([n_bases], dtype=torch.int64, device=dev)
        D.allreduce(nb)
        total_bases = int(nb.item())
    else:
        total_bases = n_bases
    parity = None
    if not args.no_parity:  # every rank (collectives inside)
        parity = parity_stream(cfg, sh, table_t, n_reads, pr, rank, world, dims, dev)
    if rank == 0:
        ms_step = elapsed / args.steps * 1e3
        parts_n = len(sh.batches)
        am = float(np.mean([a for a in apply_ms if a is not None])) if apply_ms else None
        R_part = n_reads / parts_n
        R0 = sh.n_reads[0]
        B0 = sh.n_bases_of(0)
        alg_part = 2.5 * B0 + 16 * R0  # partition 0's algorithmic bytes
        achieved = alg_part / (probe_ms * 1e-3) / 1e9 if probe_ms else None
        h2d = sh.staged_bytes
        d2h = sh.d2h_bytes()
        line = {
            "metric": METRIC,
            "value": args.steps * total_bases / elapsed,
            "unit": "bases/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8 in, int64 counts, f64 recalibration",
            "data": "synthetic (deterministic generator, SURVEY.md 8d spec), streamed from pinned host memory "
                    "(PCIe-inclusive: H2D of every partition and D2H of every result inside the timed region)",
            "config": {
                "workload": WORKLOADS["cfg5"],
                "reads_per_gpu": n_reads,
                "bases_per_gpu": n_bases,
                "read_len": list(cfg["lens"]),
                "read_groups": cfg["n_rg"],
                "known_sites": 0,
                "partitions_per_gpu": parts_n,
                "stream_mode": args.stream_mode,
                "d2h": args.d2h,
                "outputs": "compacted chars + u16 lengths" if sh.compact else "padded slots + start/len",
                "parallelism": "dp%d: read shards per GPU, RCCL int64 table all-reduce" % world,
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "bqsr_apply_kernel (partition 0: %d reads)" % int(R0),
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS if achieved else None,
                "traffic": None,
                "alg_bytes_per_launch": alg_part,
                "kernel_ms": {"apply_alone": probe_ms, "apply_in_pipeline_per_partition": am},
                "kernel_ms_method": "apply_alone: HIP events around the apply kernel on partition 0 after the timed "
                                    "jobs, no copies in flight (mean of 3); in_pipeline: the recorded timed job's "
                                    "brackets, sharing the GPU with the copies of the other partitions",
                "bound_note": "cfg5 is PCIe-bound: see `pcie` (the link, not HBM, sets the job time)",
            },
            "pcie": {"h2d_bytes_per_step": h2d, "d2h_bytes_per_step": d2h,
                     "achieved_GBps": (h2d + d2h) / (ms_step * 1e-3) / 1e9},
            "gen_s": t_gen,
        }
        if world == 1 and not args.no_cpu_baseline:
            args.cpu_reads = min(args.cpu_reads, 2_000_000)
            line["cpu_baseline"] = cpu_baseline(args, cfg, first, None)[0]
        if parity is not None:
            line["parity"] = parity
        print(json.dumps(line), flush=True)
    sh.close()
    if world > 1:
        dist.destroy_process_group()


def parity_stream(cfg, sh, table_t, n_reads, pr, rank, world, dims, dev):
    """cfg5 (called on every rank): the last job's table words and
    expectedMismatch against the oracle over every partition of every rank
    (each observed as one partition; the tables summed across ranks, the
    expectedMismatch values folded in global partition order -- rank 0's
    partitions first), and the recalibrated chars of each rank's first and
    last partitions (outside the timed region; partitions regenerated from
    the dataset's global read indices).  Counts and equalities are reduced
    to every rank."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import torch
    import torch.distributed as dist
    import oracle as O
    from adam_amd import distributed as D
    from adam_amd import synth
    t = time.perf_counter()
    cores, _ = host_cores()
    d = O.Dims(dims.n_rg, dims.max_len)
    words = np.zeros(O.table_words(d), dtype=np.int64)
    base = rank * n_reads
    starts = list(range(0, n_reads, pr))
    sampled = {0, len(starts) - 1}
    keep = {}
    ems = []
    for i, r0 in enumerate(starts):
        part = synth.generate(min(pr, n_reads - r0), cfg["lens"], cfg["n_rg"], cfg["seed"], first_read=base + r0)
        w, e = O.observe_mt(part, None, d, n_parts=cores, nthreads=cores, fold1=True)
        words += w
        ems.append(e)
        if i in sampled:
            keep[i] = part
        del part
    if world > 1:
        wt = torch.from_numpy(words).to(dev)
        D.allreduce_table(wt)
        words = wt.cpu().numpy()
        all_ems = D.gather_partition_ems(torch.tensor(ems, dtype=torch.float64, device=dev)).cpu().tolist()
    else:
        all_ems = ems
    em = 0.0
    for e in all_ems:  # ((0.0 + e_0) + e_1) + ... in global partition order
        em = em + e
    gw = table_t.cpu().numpy()
    gem = float(sh._em_keep.cpu()[0])
    table_ok = bool(np.array_equal(gw, words))
    em_ok = gem == em
    bad_total, checked, first_bad = 0, 0, np.iinfo(np.int64).max
    for i, part in sorted(keep.items()):
        out, out_len = O.apply_mt(part, d, words, em, n_parts=cores, nthreads=cores)
        bad, first = compare_stream_outputs(O, sh, i, part, out, out_len, cores)
        bad_total += bad
        checked += part.n_reads
        if bad:
            first_bad = min(first_bad, base + sum(sh.n_reads[:i]) + first)
    red = torch.tensor([bad_total, int(not table_ok), int(not em_ok), checked], dtype=torch.int64, device=dev)
    D.allreduce(red)
    fr = torch.tensor([first_bad], dtype=torch.int64, device=dev)
    D.allreduce(fr, dist.ReduceOp.MIN)
    red = red.cpu().tolist()
    fr = int(fr.item())
    return {"checked": True, "ok": red[0] == 0 and red[1] == 0 and red[2] == 0, "table_words_equal": red[1] == 0,
            "expected_mismatch_equal": red[2] == 0, "expected_mismatch": float(gem).hex(),
            "reads_checked": red[3], "partitions_checked_per_rank": sorted(keep), "reads_differing": red[0],
            "first_differing_read": fr if red[0] else -1, "ranks": world,
            "against": "oracle/ (C++ restatement of ADAM BQSR): table and expectedMismatch over every partition of "
                       "every rank (tables summed, expectedMismatch folded in global partition order), chars of "
                       "each rank's first and last partitions",
            "check_s": time.perf_counter() - t}


def compare_stream_outputs(O, sh, i, part, out, out_len, cores):
    """(reads differing, first) between the oracle's chars and a streamed
    partition's results (compacted or by slot)."""
    res = sh.outputs(i)
    if res[0] == "compact":
        _, chars, off, exc = res
        return O.compare_compact_output(part, out, out_len, chars, off, exc if len(exc) else None, nthreads=cores)
    _, q, st, ln, exc = res
    return O.compare_device_output(part, out, out_len, q, st, ln, exc if len(exc) else None, nthreads=cores)


def host_cores():
    """(threads to use, description): the CPUs this process can actually
    keep busy -- its affinity mask, capped by the cgroup CPU quota (the GPU
    box shows the machine's 256 CPUs but allows 16) -- with the machine's
    count and the quota stated."""
    import math
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
            if q != "max":
                quota = float(q) / float(per)
    except (OSError, ValueError):
        quota = None
    n = aff if quota is None else max(1, min(aff, int(math.ceil(quota))))
    return n, {"affinity": aff, "nproc": os.cpu_count(), "cgroup_cpu_quota": quota, "threads_used": n}


def cpu_baseline(args, cfg, batch, sites, whole=False):
    """The oracle (oracle/: the C++ restatement of ADAM BQSR; Spark cannot run
    here) timed on this host's cores over a bounded sample of the same
    workload: the first --cpu-reads reads of the GPU's own shard, observe per
    partition -> merge in order -> finalize -> apply, one std::thread per
    partition; plus one thread on an eighth of the sample.  With `whole` and a
    sample that is the whole shard, the run is the single-partition form
    (oracle_bqsr_fold1: expectedMismatch folded over the shard in order by one
    more thread) and its outputs are returned for the parity check."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    cores, cinfo = host_cores()
    n = min(args.cpu_reads, batch.n_reads)
    sample = batch.slice(0, n) if n < batch.n_reads else batch
    fold1 = whole and n == batch.n_reads
    osites = O.Sites(sites) if sites else None
    d = O.Dims(cfg["n_rg"], max(cfg["lens"]))
    t = time.perf_counter()
    res = O.bqsr(sample, osites, d, n_parts=cores, nthreads=cores, fold1=fold1)
    dt = time.perf_counter() - t
    one = sample.slice(0, max(1, n // 8))
    t1 = time.perf_counter()
    O.bqsr(one, osites, d, n_parts=1, nthreads=1)
    dt1 = time.perf_counter() - t1
    line = {"value": sample.n_bases / dt, "unit": "bases/s", "cores": cores, "kind": "port",
            "label": "C++ restatement of ADAM BQSR (oracle/), not Spark: no JVM on the box",
            "host": cinfo,
            "sample": "first %d reads (%d bases) of the %s shard, observe+merge+finalize+apply, %d partitions "
                      "on %d threads (%.1f s)%s; value_1thread on the first %d reads (%.1f s)" %
                      (n, sample.n_bases, args.config, cores, cores, dt,
                       " + one thread folding expectedMismatch over the shard as one partition" if fold1 else "",
                       one.n_reads, dt1),
            "value_1thread": one.n_bases / dt1}
    return line, (res if fold1 else None)

if __name__ == "__main__":
    main()
