"""The multi-rank HIP sequence, two ranks sharing one GPU over gloo.

Each rank is a separate process on cuda:0 running exactly what a rank of
``bench.py --gpus N`` runs (adam_amd/job.py ResidentJob.step: staged observe ->
int64 table all-reduce -> expectedMismatch of every rank's partition folded in
rank order on the device -> finalize from HBM -> apply), and what a rank of the
streamed path runs (adam_amd/stream.py StreamedShard.run over several
partitions per rank, the table all-reduced, expectedMismatch folded over every
partition of the job in global partition order).  The results must equal the
CPU oracle folding the same partitions in that order as one job
(RecalibrateBaseQualities.scala:63: aggregate over partitions, merged in
partition order), bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from _parity import run_oracle

pytestmark = pytest.mark.gpu

WORLD = 2
N_READS = 24000
PARTS_PER_RANK = 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _data():
    from adam_amd import synth
    batch = synth.generate(N_READS, (100, 150), 2, 977)
    sites = synth.known_sites(300_000, seed=5)
    return batch, sites


def _rank_parts(batch, rank):
    from adam_amd.distributed import shard_bounds
    r0, r1 = shard_bounds(batch.n_reads, rank, WORLD)
    shard = batch.slice(r0, r1)
    cuts = [shard.n_reads * i // PARTS_PER_RANK for i in range(PARTS_PER_RANK + 1)]
    return shard, [shard.slice(cuts[i], cuts[i + 1]) for i in range(PARTS_PER_RANK)]


def _rank_main(rank, port, out_dir):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import ctypes

    import torch
    import torch.distributed as dist

    from adam_amd import _capi, bqsr
    from adam_amd.job import ResidentJob
    from adam_amd.stream import StreamedShard

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.zeros(1, device=dev)  # torch's HIP runtime first, as bench.py does
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        batch, sites = _data()
        snp = bqsr.SnpTable(sites)
        dims = bqsr.dims_of([batch])
        shard, parts = _rank_parts(batch, rank)
        # ---- bench.py's step: the shard as one partition ----
        r0 = sum(_rank_parts(batch, r)[0].n_reads for r in range(rank))
        job = ResidentJob(shard, dims, snp, 0, read_base=r0)
        for _ in range(2):  # steady state: the second job reuses every buffer
            job.step(False)
        words, em, q, st, ln, exc = job.results()
        job.close()
        # ---- the streamed path: PARTS_PER_RANK partitions on this rank ----
        L = _capi.lib()
        ctx = bqsr.Context.get(0)
        words_t = torch.zeros(int(L.bqsr_table_words(dims)), dtype=torch.int64, device=dev)
        th = ctypes.c_void_p()
        _capi.check(L.bqsr_table_create(ctx.handle, dims, ctypes.c_void_p(words_t.data_ptr()), ctypes.byref(th)))
        sh = StreamedShard(ctx, parts, dims, snp.handle(ctx), 0, site_contigs=snp.contigs, read_base=r0)
        try:
            for _ in range(2):
                em_s = sh.run(th, words_t)
                n_exc = sh.finish()
            s_words = words_t.cpu().numpy()
            s_em = float(em_s.cpu()[0])
            outs = [sh.outputs(i) for i in range(len(parts))]  # compacted: chars, offsets
            s_q = [o[1].copy() for o in outs]
            s_st = [o[2].copy() for o in outs]
            s_ln = [np.zeros(1, np.int32) for _ in outs]
        finally:
            sh.close()
            L.bqsr_table_destroy(th)
        np.savez(os.path.join(out_dir, "rank%d.npz" % rank), words=words, em=np.array([em]), q=q, st=st, ln=ln,
                 exc=exc, s_words=s_words, s_em=np.array([s_em]), s_exc=np.array([n_exc]),
                 **{"s_q%d" % i: s_q[i] for i in range(len(parts))},
                 **{"s_st%d" % i: s_st[i] for i in range(len(parts))},
                 **{"s_ln%d" % i: s_ln[i] for i in range(len(parts))})
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(400)
def test_two_ranks_one_gpu(tmp_path):
    import oracle as O
    ctx = mp.start_processes(_rank_main, args=(_free_port(), str(tmp_path)), nprocs=WORLD, join=False,
                             start_method="spawn")
    for _ in range(600):  # at most ~10 minutes, normally well under one
        if ctx.join(timeout=1):
            break
    else:
        for p in ctx.processes:
            p.kill()
        pytest.fail("ranks did not finish")
    batch, sites = _data()
    shards = [_rank_parts(batch, r) for r in range(WORLD)]
    # bench.py's job: partitions = the ranks' shards, in rank order
    o = run_oracle([s for s, _ in shards], sites)
    assert o.error is None
    # streamed: partitions = every rank's partitions, rank 0's first
    all_parts = [p for _, ps in shards for p in ps]
    os_ = run_oracle(all_parts, sites)
    assert os_.error is None
    for rank in range(WORLD):
        z = np.load(tmp_path / ("rank%d.npz" % rank))
        shard, parts = shards[rank]
        assert np.array_equal(z["words"], o.words)
        assert z["em"][0] == o.em, (z["em"][0], o.em)
        ref_out, ref_len = o.outs[rank]
        bad, first = O.compare_device_output(shard, ref_out, ref_len, z["q"], z["st"], z["ln"],
                                             z["exc"] if len(z["exc"]) else None)
        assert bad == 0, first
        # streamed
        assert np.array_equal(z["s_words"], os_.words)
        assert z["s_em"][0] == os_.em, (z["s_em"][0], os_.em)
        assert int(z["s_exc"][0]) == 0
        for i, p in enumerate(parts):
            ref_out, ref_len = os_.outs[rank * PARTS_PER_RANK + i]
            bad, first = O.compare_compact_output(p, ref_out, ref_len, z["s_q%d" % i], z["s_st%d" % i])
            assert bad == 0, (rank, i, first)


def _bad_md(shard, k):
    """Read k's MD tag made unparseable (MdTag.scala:52: must start with a digit)."""
    a = int(shard.md_offset[k])
    f = int(shard.flags[k])
    usable = (f & 2) and (f & 16) and not (f & 32)  # mapped, primary, not a duplicate (include/adam_bqsr.h)
    if usable and int(shard.md_offset[k + 1]) > a:
        shard.md[a] = ord("Z")
        return True
    return False


def _rank_err_main(rank, port, out_dir, bad_rank):
    """bench.py's multi-rank step with one bad MD tag on `bad_rank` (and, on
    the other rank, a later bad one), then bench.parity_multi on clean data."""
    import json
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import torch
    import torch.distributed as dist

    import bench
    from adam_amd import _capi, bqsr, synth
    from adam_amd.distributed import shard_bounds
    from adam_amd.job import ResidentJob
    from adam_amd.stream import StreamedShard

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.zeros(1, device=dev)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    out = {}
    try:
        cfg = dict(lens=(100,), n_rg=1)
        n = 6000
        r0, r1 = shard_bounds(n, rank, WORLD)
        dims = _capi.Dims(1, 100)
        # clean: the parity leg of bench.py on the real job
        shard = synth.generate(r1 - r0, cfg["lens"], 1, 31337, first_read=r0)
        job = ResidentJob(shard, dims, None, 0, read_base=r0)
        job.step(False)
        out["parity"] = bench.parity_multi(job, cfg, shard, None, WORLD, rank, dev)
        job.close()
        # errors: the first bad read of the job in global read order
        shard = synth.generate(r1 - r0, cfg["lens"], 1, 31337, first_read=r0)
        # bad_rank 0: both ranks hold a bad read, rank 0's comes first in
        # global order; bad_rank 1: only rank 1 holds one (its global index
        # = read_base + local index).  Both past the stream's first partition
        # (1000 reads).
        out["bad_local"] = None
        if rank == bad_rank or bad_rank == 0:
            k = 2100 if rank == bad_rank else 2900
            while not _bad_md(shard, k):
                k += 1
            out["bad_local"] = k
        job = ResidentJob(shard, dims, None, 0, read_base=r0)
        try:
            job.step(False)
            out["raised"] = None
        except _capi.BQSRError as e:
            out["raised"] = [e.name, e.read]
        job.close()
        # the streamed path: the same shard as two partitions, the bad read in
        # the second one -- the error key is rebased by read_base + the reads
        # of the partitions before (stream.py _exchange_errors)
        import ctypes
        L = _capi.lib()
        ctx = bqsr.Context.get(0)
        half = shard.n_reads // 3
        parts = [shard.slice(0, half), shard.slice(half, shard.n_reads)]
        words_t = torch.zeros(int(L.bqsr_table_words(dims)), dtype=torch.int64, device=dev)
        th = ctypes.c_void_p()
        _capi.check(L.bqsr_table_create(ctx.handle, dims, ctypes.c_void_p(words_t.data_ptr()), ctypes.byref(th)))
        sh = StreamedShard(ctx, parts, dims, None, 0, read_base=r0)
        try:
            sh.run(th, words_t)
            sh.finish()
            out["raised_stream"] = None
        except _capi.BQSRError as e:
            out["raised_stream"] = [e.name, e.read]
        finally:
            while sh.pending:
                try:
                    sh.finish()
                except _capi.BQSRError:
                    pass
            sh.close()
            L.bqsr_table_destroy(th)
        with open(os.path.join(out_dir, "err%d.json" % rank), "w") as fh:
            json.dump(out, fh)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(400)
@pytest.mark.parametrize("bad_rank", [0, 1])
def test_two_ranks_raise_the_jobs_first_error_and_parity_leg(tmp_path, bad_rank):
    import json
    ctx = mp.start_processes(_rank_err_main, args=(_free_port(), str(tmp_path), bad_rank), nprocs=WORLD,
                             join=False, start_method="spawn")
    for _ in range(600):
        if ctx.join(timeout=1):
            break
    else:
        for p in ctx.processes:
            p.kill()
        pytest.fail("ranks did not finish")
    res = [json.load(open(tmp_path / ("err%d.json" % r))) for r in range(WORLD)]
    from adam_amd.distributed import shard_bounds
    first = min(shard_bounds(6000, r, WORLD)[0] + res[r]["bad_local"] for r in range(WORLD)
                if res[r]["bad_local"] is not None)
    assert first >= 3000 if bad_rank == 1 else first < 3000
    for z in res:
        p = z["parity"]
        assert p["ok"] and p["reads_checked"] == 6000, json.dumps(p)
        assert z["raised"] == ["MD_PARSE", first], (z["raised"], first)
        assert z["raised_stream"] == ["MD_PARSE", first], (z["raised_stream"], first)
