"""Sharding of independent alignment pairs over ranks (one process per GPU).

The hot path has no cross-pair dependency: a batch of pairs (C4: 1024 pairs of
4,000 x 4,000) is split into contiguous blocks, one per rank, and every rank
fills its block with its own stripe kernel launch.  The only collective is the
tiny score all-gather at the end (RCCL over xGMI on MI355X, gloo in the CPU
tests) -- there is no data-path exchange, so scaling is weak.

This mirrors how the reference parallelises *across* subproblems
(main_alignment.cpp:389-401: independent Subproblem objects handed to threads)
one level up: pairs -> ranks instead of subproblems -> threads.
"""
from __future__ import annotations

from typing import Callable, List, Sequence, Tuple


def shard_range(n_units: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous block [lo, hi) of ``n_units`` owned by ``rank`` (ceil split; late ranks may be short/empty)."""
    if world <= 0 or not 0 <= rank < world or n_units < 0:
        raise ValueError("bad shard arguments")
    per = (n_units + world - 1) // world
    lo = min(n_units, rank * per)
    return lo, min(n_units, lo + per)


def gather_scores(local, n_units: int, rank: int, world: int, group=None):
    """All-gather every rank's int64 score block into the full ``n_units`` vector (same device as ``local``)."""
    import torch
    import torch.distributed as dist

    per = (n_units + world - 1) // world
    lo, hi = shard_range(n_units, rank, world)
    if local.numel() != hi - lo:
        raise ValueError(f"rank {rank} holds {local.numel()} scores, expected {hi - lo}")
    pad = torch.zeros(per, dtype=torch.int64, device=local.device)
    pad[: hi - lo] = local.to(torch.int64)
    if world == 1:
        return pad[:n_units].clone()
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad, group=group)
    return torch.cat(parts)[:n_units]


def sharded_scores(pairs: Sequence, scorer: Callable[[Sequence], List[int]], rank: int, world: int, device="cpu",
                   group=None):
    """Score ``pairs`` across ranks: rank r runs ``scorer`` on its block, then all ranks get every score.

    ``scorer`` is the per-rank compute (on a GPU box: a ``Plan`` over the block's
    pairs, see bench.py workload c4)."""
    import torch

    lo, hi = shard_range(len(pairs), rank, world)
    mine = torch.tensor(list(scorer(pairs[lo:hi])) if hi > lo else [], dtype=torch.int64, device=device)
    return gather_scores(mine, len(pairs), rank, world, group=group)
