"""Multi-GPU BQSR: one process per GPU, reads sharded by contiguous ranges.

The reference aggregates per-partition RecalTables with Spark's
`RDD.aggregate` (RecalibrateBaseQualities.scala:52-64): every partition folds
its reads from an empty table, the driver merges the partial tables with
`RecalTable.++` (RecalTable.scala:90-108).  Here every rank holds a run of
consecutive partitions of the job (rank 0 the first ones):

* the int64 count tables are summed exactly with one all-reduce (RCCL over
  xGMI on the GPU box; any torch.distributed backend works -- the CPU tests use
  gloo), since integer addition is order-free;
* the per-partition expectedMismatch doubles are NOT summed by the collective:
  floating-point addition is order-dependent, so every rank's
  per-partition values are all-gathered and folded
  ``((0.0 + e_0) + e_1) + ...`` in global partition order (rank 0's partitions,
  then rank 1's, ...), the merge order of partitions 0, 1, ... on the driver --
  on the device, by the library (``bqsr_em_fold_async``);
* every rank then finalizes the identical table and recalibrates its own shard
  (no second exchange).

With gloo (the CPU tests, or two ranks sharing one GPU in the GPU tests) the
collectives run on host copies of device tensors; with RCCL on the tensors
themselves.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist


def shard_bounds(n_reads: int, rank: int, world: int) -> Tuple[int, int]:
    """Reads [r0, r1) of `rank`: contiguous, in rank order, sizes differing by at most one."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank / world size")
    return n_reads * rank // world, n_reads * (rank + 1) // world


def _multi() -> bool:
    return dist.is_initialized() and dist.get_world_size() > 1


def _host_coll(t: torch.Tensor) -> bool:
    """gloo runs these collectives on host tensors only."""
    return t.device.type != "cpu" and dist.get_backend() == "gloo"


def allreduce(t: torch.Tensor, op=None) -> torch.Tensor:
    """In-place all-reduce of `t` (SUM by default) on any backend: RCCL on
    device tensors, gloo on a host copy.  For the bench's timing and parity
    reductions (not on the data path)."""
    op = dist.ReduceOp.SUM if op is None else op
    if _multi():
        if _host_coll(t):
            h = t.cpu()
            dist.all_reduce(h, op=op)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=op)
    return t


def allreduce_table(words: torch.Tensor) -> torch.Tensor:
    """Exact int64 sum of the ranks' count tables, in place (RecalTable.++ on counts)."""
    if words.dtype != torch.int64:
        raise TypeError("covariate tables are int64")
    if _multi():
        if _host_coll(words):
            h = words.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.SUM)
            words.copy_(h)
        else:
            dist.all_reduce(words, op=dist.ReduceOp.SUM)
    return words


def allreduce_error_keys(keys: torch.Tensor) -> torch.Tensor:
    """MIN over the ranks of the int64 error keys (global read order; no error
    = INT64_MAX), in place: the job's first error, which every rank raises."""
    if keys.dtype != torch.int64:
        raise TypeError("error keys are int64")
    if _multi():
        if _host_coll(keys):
            h = keys.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.MIN)
            keys.copy_(h)
        else:
            dist.all_reduce(keys, op=dist.ReduceOp.MIN)
    return keys


def _all_gather(t: torch.Tensor) -> torch.Tensor:
    """[world * n] = every rank's 1-D `t` (same n on every rank), rank-major."""
    world = dist.get_world_size()
    if _host_coll(t):
        h = t.cpu()
        out = torch.empty(world * h.numel(), dtype=h.dtype)
        dist.all_gather(list(out.chunk(world)), h)
        return out.to(t.device)
    out = torch.empty(world * t.numel(), dtype=t.dtype, device=t.device)
    if t.device.type == "cpu":
        dist.all_gather(list(out.chunk(world)), t)
    else:
        dist.all_gather_into_tensor(out, t)
    return out


def partition_counts(n_local: int, device: torch.device | str = "cpu") -> List[int]:
    """Every rank's number of partitions, in rank order (one host round trip;
    a shard's partition count is fixed, so callers exchange it once)."""
    if not _multi():
        return [int(n_local)]
    t = torch.tensor([int(n_local)], dtype=torch.int64, device=device)
    return [int(v) for v in _all_gather(t).tolist()]


def gather_partition_ems(ems: torch.Tensor, counts: Optional[Sequence[int]] = None) -> torch.Tensor:
    """All ranks' per-partition expectedMismatch values in global partition
    order (rank 0's partitions first), as one float64 tensor on ems.device.
    `counts` = partition_counts(...) when known (saves the exchange)."""
    if ems.dtype != torch.float64 or ems.dim() != 1:
        raise TypeError("per-partition expectedMismatch is a 1-D float64 tensor")
    if not _multi():
        return ems
    if counts is None:
        counts = partition_counts(ems.numel(), ems.device)
    if ems.numel() != counts[dist.get_rank()]:
        raise ValueError("partition count differs from the exchanged one")
    m = max(1, max(counts))
    pad = torch.zeros(m, dtype=torch.float64, device=ems.device)
    pad[:ems.numel()] = ems
    allv = _all_gather(pad).view(len(counts), m)
    return torch.cat([allv[r, :c] for r, c in enumerate(counts)])


def fold_ems_device(ems: torch.Tensor, ctx=None, stream: Optional[torch.cuda.Stream] = None) -> torch.Tensor:
    """((0.0 + ems[0]) + ems[1]) + ... as a 1-element float64 tensor.  Device
    tensors are folded by the HIP library (bqsr_em_fold_async) on `stream`
    without a host round trip; host tensors (gloo CPU tests) one IEEE addition
    at a time."""
    out = torch.zeros(1, dtype=torch.float64, device=ems.device)
    if ems.device.type == "cpu":
        s = 0.0
        for v in ems.tolist():
            s = s + v
        out[0] = s
        return out
    from . import _capi, bqsr
    ctx = ctx or bqsr.Context.get(ems.device.index or 0)
    st = stream or torch.cuda.current_stream(ems.device)
    e = ems.contiguous()
    _capi.check(_capi.lib().bqsr_em_fold_async(ctx.handle, ctypes.c_void_p(e.data_ptr()), e.numel(),
                                               ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(st.cuda_stream)))
    out._keep = e  # the fold reads `e` asynchronously
    return out


def fold_partition_ems_device(ems: torch.Tensor, counts: Optional[Sequence[int]] = None, ctx=None,
                              stream: Optional[torch.cuda.Stream] = None) -> torch.Tensor:
    """The job's expectedMismatch: this rank's per-partition values gathered
    with every other rank's and folded in global partition order."""
    return fold_ems_device(gather_partition_ems(ems, counts), ctx, stream)


def fold_expected_mismatch(em: float, device: torch.device | str = "cpu") -> float:
    """Host form for one partition per rank: all-gather every rank's
    expectedMismatch and fold them in rank order."""
    if not _multi():
        return 0.0 + em
    mine = torch.tensor([em], dtype=torch.float64, device=device)
    total = 0.0
    for v in _all_gather(mine).tolist():
        total = total + v
    return total


def fold_expected_mismatch_device(mine: torch.Tensor, ctx=None) -> torch.Tensor:
    """One partition per rank, on the device: `mine` is this rank's
    expectedMismatch (1 float64); returns the rank-order fold as a 1-element
    tensor."""
    if mine.dtype != torch.float64 or mine.numel() != 1:
        raise TypeError("expectedMismatch is one float64")
    return fold_partition_ems_device(mine.reshape(1), [1] * (dist.get_world_size() if _multi() else 1), ctx)
