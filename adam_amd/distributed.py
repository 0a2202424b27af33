"""Multi-GPU BQSR: one process per GPU, reads sharded by contiguous ranges.

The reference aggregates per-partition RecalTables with Spark's
`RDD.aggregate` (RecalibrateBaseQualities.scala:52-64): every partition folds
its reads from an empty table, the driver merges the partial tables with
`RecalTable.++` (RecalTable.scala:90-108).  Here every rank is one partition
(or a run of consecutive partitions) of the job:

* the int64 count tables are summed exactly with one all-reduce (RCCL over
  xGMI on the GPU box; any torch.distributed backend works -- the CPU tests use
  gloo), since integer addition is order-free;
* the per-rank expectedMismatch doubles are NOT summed by the collective:
  floating-point addition is order-dependent, so they are
  all-gathered and folded ``((0.0 + e_0) + e_1) + ...`` in rank order, the
  merge order of partitions 0, 1, ... on the driver;
* every rank then finalizes the identical table and recalibrates its own shard
  (no second exchange).
"""
from __future__ import annotations

from typing import Tuple

import torch
import torch.distributed as dist


def shard_bounds(n_reads: int, rank: int, world: int) -> Tuple[int, int]:
    """Reads [r0, r1) of `rank`: contiguous, in rank order, sizes differing by at most one."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank / world size")
    return n_reads * rank // world, n_reads * (rank + 1) // world


def allreduce_table(words: torch.Tensor) -> torch.Tensor:
    """Exact int64 sum of the ranks' count tables, in place (RecalTable.++ on counts)."""
    if words.dtype != torch.int64:
        raise TypeError("covariate tables are int64")
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(words, op=dist.ReduceOp.SUM)
    return words


def fold_expected_mismatch(em: float, device: torch.device | str = "cpu") -> float:
    """All-gather every rank's expectedMismatch and fold them in rank order
    (RecalTable.++: this.expectedMismatch + other.expectedMismatch)."""
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return 0.0 + em
    world = dist.get_world_size()
    mine = torch.tensor([em], dtype=torch.float64, device=device)
    ems = torch.zeros(world, dtype=torch.float64, device=device)
    dist.all_gather_into_tensor(ems, mine)
    total = 0.0
    for v in ems.tolist():
        total = total + v
    return total


def fold_expected_mismatch_device(mine: torch.Tensor) -> torch.Tensor:
    """fold_expected_mismatch without leaving the device: `mine` is this
    rank's expectedMismatch as a 1-element float64 tensor; returns the
    rank-order fold ((0.0 + e_0) + e_1) + ... as a 1-element tensor (each `+`
    one IEEE double addition, as on the host)."""
    if mine.dtype != torch.float64 or mine.numel() != 1:
        raise TypeError("expectedMismatch is one float64")
    total = torch.zeros(1, dtype=torch.float64, device=mine.device)
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return total + mine.reshape(1)
    world = dist.get_world_size()
    ems = torch.empty(world, dtype=torch.float64, device=mine.device)
    dist.all_gather_into_tensor(ems, mine.reshape(1))
    for i in range(world):
        total = total + ems[i:i + 1]
    return total
