"""Sharding of independent alignment pairs over ranks (one process per GPU).

The hot path has no cross-pair dependency: a batch of pairs (C4: 1024 pairs of
4,000 x 4,000) is split into contiguous blocks, one per rank, and every rank
fills its block with its own kernel launch.  The only collectives are the
broadcast of the shared reference sequence (once) and the score all-gather at
the end of every step (RCCL over xGMI on MI355X, gloo in the CPU tests) --
there is no data-path exchange.  The batch is fixed and split over the ranks,
so adding ranks shrinks each rank's share (strong scaling of the batch); below
two workgroups' worth of pairs per CU a rank's plan splits every pair over
several CUs (split mode).

This mirrors how the reference parallelises *across* pairs
(testing.cpp:112-158: one std::thread per pair, each calling
main_alignment_function) one level up: pairs -> ranks instead of pairs ->
threads.  ``bench.py`` (workload c4) and ``tests/test_dist_gloo.py`` drive the
same ``ShardedBatch``; only the per-rank scorer differs (a device Plan vs the
CPU oracle).
"""
from __future__ import annotations

from typing import Callable, Tuple


def shard_range(n_units: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous block [lo, hi) of ``n_units`` owned by ``rank`` (ceil split; late ranks may be short/empty)."""
    if world <= 0 or not 0 <= rank < world or n_units < 0:
        raise ValueError("bad shard arguments")
    per = (n_units + world - 1) // world
    lo = min(n_units, rank * per)
    return lo, min(n_units, lo + per)


def broadcast_reference(ref, src: int = 0, group=None):
    """Every rank gets rank ``src``'s reference-sequence codes (in place; no-op at world size 1)."""
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.broadcast(ref, src=src, group=group)
    return ref


def gather_scores(local, n_units: int, rank: int, world: int, group=None):
    """All-gather every rank's score block into the full ``n_units`` int64 vector (on ``local``'s device)."""
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


class ShardedBatch:
    """``n_units`` independent pairs split over ``world`` ranks.

    ``score_block(lo, hi)`` computes the scores of pairs [lo, hi) on this rank
    and returns them as an integer tensor (device-resident on a GPU box: a Plan
    built once for the block, run, then ``Plan.scores_into``).  ``step()`` runs
    it and all-gathers every rank's scores."""

    def __init__(self, n_units: int, rank: int, world: int, score_block: Callable, group=None):
        self.n_units, self.rank, self.world, self.group = n_units, rank, world, group
        self.lo, self.hi = shard_range(n_units, rank, world)
        self.score_block = score_block

    def step(self):
        local = self.score_block(self.lo, self.hi)
        return gather_scores(local, self.n_units, self.rank, self.world, group=self.group)
