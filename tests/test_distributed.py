"""The multi-rank path (adam_amd/distributed.py) with world_size 2 on gloo:
each rank observes its contiguous shard, the int64 tables are all-reduced, the
expectedMismatch doubles are all-gathered and folded in rank order, and every
rank finalizes the same table.  The per-rank observe here is the CPU oracle
(the same call sequence the GPU ranks make through the C ABI in bench.py);
the result must equal a single process folding the same shards as
consecutive partitions."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

WORLD = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_main(rank, port, out_dir):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "oracle"))
    import torch
    import torch.distributed as dist

    import oracle as O
    from adam_amd import distributed as D
    from adam_amd import synth

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        batch = synth.generate(3000, (100,), 2, 77)
        d = O.Dims(2, 100)
        r0, r1 = D.shard_bounds(batch.n_reads, rank, WORLD)
        words, em = O.observe(batch, None, d, r0, r1)
        t = torch.from_numpy(words.copy())
        D.allreduce_table(t)
        total = D.fold_expected_mismatch(em)
        # the device form the benchmark uses (gloo: CPU tensors) folds identically
        dev_total = float(D.fold_expected_mismatch_device(torch.tensor([em], dtype=torch.float64))[0])
        assert dev_total == total
        fin = O.Final(d, t.numpy(), total)
        out, out_len = O.apply(batch, fin, r0, r1)
        np.savez(os.path.join(out_dir, "rank%d.npz" % rank), words=t.numpy(), em=np.array([total]),
                 out=out, out_len=out_len, r0=r0, r1=r1)
    finally:
        dist.destroy_process_group()


def test_two_rank_table_allreduce_and_rank_order_fold(tmp_path):
    import oracle as O
    from adam_amd import synth
    from adam_amd.distributed import shard_bounds

    mp.start_processes(_rank_main, args=(_free_port(), str(tmp_path)), nprocs=WORLD, join=True,
                       start_method="spawn")
    batch = synth.generate(3000, (100,), 2, 77)
    d = O.Dims(2, 100)
    # single process, the two shards as consecutive partitions merged in order
    words = np.zeros(O.table_words(d), dtype=np.int64)
    em = 0.0
    for rank in range(WORLD):
        r0, r1 = shard_bounds(batch.n_reads, rank, WORLD)
        w, e = O.observe(batch, None, d, r0, r1)
        words += w
        em = em + e
    fin = O.Final(d, words, em)
    ref_out, ref_len = O.apply(batch, fin)
    for rank in range(WORLD):
        z = np.load(tmp_path / ("rank%d.npz" % rank))
        assert np.array_equal(z["words"], words)
        assert z["em"][0] == em  # bit-exact: rank-order fold == partition-order merge
        r0, r1 = int(z["r0"]), int(z["r1"])
        a, b = int(batch.qual_offset[r0]), int(batch.qual_offset[r1])
        assert np.array_equal(z["out"][a:b], ref_out[a:b])
        assert np.array_equal(z["out_len"][r0:r1], ref_len[r0:r1])


def _rank_parts_main(rank, port, out_dir):
    """Several partitions per rank (2 on rank 0, 3 on rank 1): each partition
    observed from zero, the tables all-reduced, and every partition's
    expectedMismatch gathered and folded in global partition order."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "oracle"))
    import torch
    import torch.distributed as dist

    import oracle as O
    from adam_amd import distributed as D
    from adam_amd import synth

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        batch = synth.generate(5000, (100,), 1, 78)
        d = O.Dims(1, 100)
        cuts = _PART_CUTS[rank]
        words = np.zeros(O.table_words(d), dtype=np.int64)
        ems = []
        for a, b in zip(cuts[:-1], cuts[1:]):
            w, e = O.observe(batch, None, d, a, b)
            words += w
            ems.append(e)
        t = torch.from_numpy(words)
        D.allreduce_table(t)
        counts = D.partition_counts(len(ems))
        em = float(D.fold_partition_ems_device(torch.tensor(ems, dtype=torch.float64), counts)[0])
        np.savez(os.path.join(out_dir, "p%d.npz" % rank), words=t.numpy(), em=np.array([em]),
                 counts=np.array(counts))
    finally:
        dist.destroy_process_group()


_PART_CUTS = {0: [0, 1000, 2600], 1: [2600, 3000, 4100, 5000]}


def test_two_ranks_several_partitions_each_fold_in_partition_order(tmp_path):
    import oracle as O
    from adam_amd import synth
    mp.start_processes(_rank_parts_main, args=(_free_port(), str(tmp_path)), nprocs=WORLD, join=True,
                       start_method="spawn")
    batch = synth.generate(5000, (100,), 1, 78)
    d = O.Dims(1, 100)
    words = np.zeros(O.table_words(d), dtype=np.int64)
    em = 0.0
    bounds = _PART_CUTS[0] + _PART_CUTS[1][1:]
    for a, b in zip(bounds[:-1], bounds[1:]):  # partitions 0..4 in order, one driver merge each
        w, e = O.observe(batch, None, d, a, b)
        words += w
        em = em + e
    for rank in range(WORLD):
        z = np.load(tmp_path / ("p%d.npz" % rank))
        assert z["counts"].tolist() == [2, 3]
        assert np.array_equal(z["words"], words)
        assert z["em"][0] == em


@pytest.mark.parametrize("n,world", [(0, 1), (1, 2), (10, 3), (1001, 8)])
def test_shard_bounds_cover_in_order(n, world):
    from adam_amd.distributed import shard_bounds
    bounds = [shard_bounds(n, r, world) for r in range(world)]
    assert bounds[0][0] == 0 and bounds[-1][1] == n
    assert all(bounds[i][1] == bounds[i + 1][0] for i in range(world - 1))
    sizes = [b - a for a, b in bounds]
    assert max(sizes) - min(sizes) <= 1


class _StubJob:
    """Stands in for adam_amd.job.ResidentJob on a CPU rank: `results()` in the
    device layout (u8 chars per 16-aligned packed slot, per-read start and
    length, exception list) built from a single-process oracle run over every
    rank's shard -- what a correct multi-rank GPU job returns."""

    def __init__(self, shard, words, em, out, out_len, read_base, corrupt=None):
        lq = np.diff(shard.qual_offset.astype(np.int64))
        ls = np.diff(shard.seq_offset.astype(np.int64))
        span = (np.maximum(lq, ls) + 15) // 16 * 16
        slot = np.concatenate([[0], np.cumsum(span)])
        q = np.zeros(int(slot[-1]) + 16, dtype=np.uint8)
        for r in range(shard.n_reads):
            a = int(shard.qual_offset[r])
            q[slot[r]:slot[r] + out_len[r]] = out[a:a + out_len[r]]
        if corrupt is not None:
            q[slot[corrupt]] ^= 1
        self._res = (words, em, q, np.zeros(shard.n_reads, np.int32), out_len[:shard.n_reads].astype(np.int32),
                     np.zeros(0, np.int64))
        self.read_base = read_base

    def results(self):
        return self._res


def _parity_rank_main(rank, port, out_dir, corrupt):
    """bench.py's N > 1 parity leg (bench.parity_multi), on gloo CPU ranks."""
    import json
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "oracle"))
    import torch.distributed as dist

    import bench
    import oracle as O
    from adam_amd import distributed as D
    from adam_amd import synth

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        cfg = dict(lens=(100, 150), n_rg=2)
        n = 2000
        r0, r1 = D.shard_bounds(n, rank, WORLD)
        shard = synth.generate(r1 - r0, cfg["lens"], cfg["n_rg"], 4242, first_read=r0)
        sites = synth.known_sites(20_000, contig_len=2_000_000)
        # the job's expected results: the ranks' shards as partitions in order
        d = O.Dims(2, 150)
        osites = O.Sites(sites)
        words = np.zeros(O.table_words(d), dtype=np.int64)
        em = 0.0
        for rr in range(WORLD):
            a, b = D.shard_bounds(n, rr, WORLD)
            part = synth.generate(b - a, cfg["lens"], cfg["n_rg"], 4242, first_read=a)
            w, e = O.observe(part, osites, d)
            words += w
            em = em + e
        out, out_len = O.apply(shard, O.Final(d, words, em))
        job = _StubJob(shard, words, em, out, out_len, r0, corrupt if rank == 1 else None)
        res = bench.parity_multi(job, cfg, shard, sites, WORLD, rank, "cpu")
        with open(os.path.join(out_dir, "parity%d.json" % rank), "w") as fh:
            json.dump({"res": res, "r0": r0}, fh)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("corrupt", [None, 7])
def test_bench_multi_rank_parity_leg(tmp_path, corrupt):
    """Every rank checks its own shard against the oracle with the all-reduced
    table and rank-order expectedMismatch; counts reach every rank."""
    import json
    mp.start_processes(_parity_rank_main, args=(_free_port(), str(tmp_path), corrupt), nprocs=WORLD, join=True,
                       start_method="spawn")
    res = [json.load(open(tmp_path / ("parity%d.json" % r))) for r in range(WORLD)]
    for z in res:
        p = z["res"]
        assert p["checked"] and p["table_words_equal"] and p["expected_mismatch_equal"]
        assert p["reads_checked"] == 2000 and p["ranks"] == WORLD
        if corrupt is None:
            assert p["ok"] and p["reads_differing"] == 0 and p["first_differing_read"] == -1
        else:
            assert not p["ok"] and p["reads_differing"] == 1
            assert p["first_differing_read"] == res[1]["r0"] + corrupt
