"""One pair over several GPUs: the reference's own single-pair split.

The reference can align one pair as independent sub-alignments: the partial
scorer finds a balanced partition of the DP matrix into (i, j, node type)
points (partial.cpp:149-163, ``findPartialBalancedPartitionParallel``) and
``optimal_alignment`` (main_alignment.cpp:202-351) aligns the pieces between
consecutive points as ``Subproblem``s with fixed start / end node types, then
stitches their node lists (:344-348).  The pieces do not depend on each other,
so they shard over ranks with no data-path exchange:

* rank 0 finds the partition on its GPU (``msa_partial_partition``) and
  broadcasts the points;
* every rank solves its share of the subproblems the reference solves (its
  three-round selection, main_alignment.cpp:232-341, mirrored by
  ``solve_order``), each one fill + ``find_alignment`` walk on its own GPU
  (``msa_subproblem``), shares assigned largest-first to the least-loaded rank;
* one all-gather of the node lists lets every rank stitch the path and print
  the text ``msa_optimal_alignment`` prints on one GPU (bp lines per solved
  subproblem, then ``print_seq``, main_alignment.cpp:32-55).

``partition_fn`` / ``solve_fn`` default to the GPU C-ABI; tests substitute the
CPU oracle to check the orchestration with gloo on CPU.
"""
from __future__ import annotations

import ctypes as C
from concurrent.futures import ThreadPoolExecutor
from typing import Callable, Dict, List, Optional, Sequence, Tuple

from . import _lib as LB

Node = Tuple[int, int, int]
_HDR = "bp1\nbp1.2\nbp2\nbp3\nbp4\n"


def solve_order(num: int, fix_all: bool) -> List[int]:
    """The subproblems ``optimal_alignment`` solves, in its order (main_alignment.cpp:232-341: three
    rounds over k = r, r+3, ... with the last three handled by the rounds' tails; with <= 3
    subproblems only the first round runs)."""
    if fix_all:
        return list(range(num))
    order: List[int] = []
    many = num > 3
    for r in range(3):
        if r > 0 and not many:
            break
        i = r
        while many and i < num - 3:
            order.append(i)
            i += 3
        if i < num:
            order.append(i)
    return order


def check_partition(bp: Sequence[Node], m: int, n: int) -> None:
    """The checks msa_optimal_alignment makes (a decreasing coordinate would wrap size_t in the
    reference; an empty subproblem crashes it, :258)."""
    if len(bp) < 2:
        raise ValueError("a partition needs at least two points")
    for (i0, j0, _), (i1, j1, _) in zip(bp, bp[1:]):
        if i1 < i0 or j1 < j0 or i1 > m or j1 > n or (i1 == i0 and j1 == j0):
            raise ValueError(f"bad partition step ({i0},{j0}) -> ({i1},{j1})")


def assign(order: Sequence[int], bp: Sequence[Node], world: int) -> List[List[int]]:
    """Subproblems per rank: largest area first onto the least-loaded rank (deterministic on every rank)."""
    area = {k: (bp[k + 1][0] - bp[k][0] + 1) * (bp[k + 1][1] - bp[k][1] + 1) for k in order}
    load = [0] * world
    share: List[List[int]] = [[] for _ in range(world)]
    for k in sorted(order, key=lambda k: (-area[k], k)):
        r = min(range(world), key=lambda x: (load[x], x))
        share[r].append(k)
        load[r] += area[k]
    return share


def stitch(nodes: Dict[int, List[Node]], num: int, fix_all: bool) -> List[Node]:
    """main_alignment.cpp:344-348: end of subproblem k-1 -> begin of k for k = 1 .. num-2; the link into
    the last subproblem is never made (fix_all: made); an unsolved or empty subproblem ends the walk."""
    out: List[Node] = []
    last_link = num - 1 if fix_all else (num - 2 if num >= 2 else 0)
    for k in range(num):
        part = nodes.get(k)
        if not part:
            break
        out.extend(part)
        if k + 1 > last_link or k + 1 >= num:
            break
    return out


def text_of(A1: bytes, B1: bytes, m: int, n: int, n_solved: int, path: Sequence[Node]) -> str:
    """The stdout of optimal_alignment: the five bp lines per solved subproblem, then print_seq
    (main_alignment.cpp:32-55) of the stitched path; indices past the buffers print '?'."""
    l1 = "".join((chr(A1[i]) if i <= m else "?") if t in (1, 3) else "-" for (i, _, t) in path)
    l2 = "".join((chr(B1[j]) if j <= n else "?") if t in (1, 2) else "-" for (_, j, t) in path)
    return _HDR * n_solved + l1 + "\n" + l2 + "\n"


def gpu_partition(A1: bytes, B1: bytes, m: int, n: int, p: int, g: float, h: float) -> List[Node]:
    """findPartialBalancedPartitionParallel(A, B, m, n, p, g, h, -1, -1) on this rank's GPU (partial.cpp
    reads A[i-1]: the 0-based view of the 1-based buffers)."""
    from .api import findPartialBalancedPartitionParallel

    return [a.as_tuple() for a in findPartialBalancedPartitionParallel(A1[1:], B1[1:], m, n, p, g, h, -1, -1)]


def gpu_subproblem(A1: bytes, B1: bytes, bp: Sequence[Node], k: int, g: float, h: float) -> List[Node]:
    """Subproblem k (OptimalAlignmentMapThread, main_alignment.cpp:11-22): fill + find_alignment on this
    rank's GPU (msa_subproblem), its node list."""
    (i0, j0, t0), (i1, j1, t1) = bp[k], bp[k + 1]
    lenA, lenB = i1 - i0, j1 - j0
    cap = lenA + lenB + 2
    nodes = (LB.Node * cap)()
    cnt = C.c_size_t()
    endn = LB.Node()
    inv = C.c_int()
    LB.check(LB.lib().msa_subproblem(A1, B1, lenA, lenB, i0, j0, t0, -t1, g, h, None, None, None, nodes, cap,
                                     C.byref(cnt), C.byref(endn), C.byref(inv)), "msa_subproblem")
    return [(int(nodes[x].i), int(nodes[x].j), int(nodes[x].t)) for x in range(cnt.value)]


def optimal_alignment_distributed(A1: bytes, B1: bytes, m: int, n: int, p: int, g: float, h: float,
                                  fix_all: bool = False, bp: Optional[Sequence[Node]] = None,
                                  partition_fn: Optional[Callable] = None, solve_fn: Optional[Callable] = None,
                                  group=None):
    """main_alignment_function with the partition split, over every rank of the default (or ``group``)
    process group (world size 1 without torch.distributed): returns (stdout text, stitched path), the
    same on every rank.  ``bp`` skips the partition (optimal_alignment over a given partition).  Each
    rank computes on its current device (``torch.cuda.set_device(local_rank)`` first)."""
    import torch.distributed as dist

    A1, B1 = bytes(A1), bytes(B1)
    on = dist.is_available() and dist.is_initialized()
    rank = dist.get_rank(group) if on else 0
    world = dist.get_world_size(group) if on else 1
    part = partition_fn or gpu_partition
    solve = solve_fn or gpu_subproblem
    box = [list(bp) if bp is not None else None]
    if bp is None and rank == 0:
        try:
            box[0] = part(A1, B1, m, n, p, g, h)
        except Exception as e:  # the other ranks must not wait on the broadcast forever
            box[0] = RuntimeError(f"rank 0: partition failed: {e}")
    if world > 1 and bp is None:
        # src is a GLOBAL rank: the group's rank 0 (which computed the partition above)
        src = dist.get_global_rank(group, 0) if group is not None else 0
        dist.broadcast_object_list(box, src=src, group=group)
    if isinstance(box[0], Exception):
        raise box[0]
    points = [tuple(int(v) for v in x) for x in box[0]]
    check_partition(points, m, n)
    order = solve_order(len(points) - 1, fix_all)
    mine = assign(order, points, world)[rank]
    # this rank's subproblems run concurrently (msa_subproblem is reentrant: each call takes its own
    # pooled stream; ctypes drops the GIL), as msa_optimal_alignment runs them on one GPU.  libmsa
    # works on the calling thread's current device: the workers take this rank's.
    import torch

    dev = torch.cuda.current_device() if torch.cuda.is_available() else None

    def run(k):
        if dev is not None:
            torch.cuda.set_device(dev)
        return solve(A1, B1, points, k, g, h)

    # a failing subproblem must not leave this rank out of the all-gather (the others would wait in it
    # until the backend's timeout): the error travels in the gathered dict and every rank raises it
    try:
        with ThreadPoolExecutor(max_workers=max(1, min(8, len(mine)))) as pool:
            local = dict(zip(mine, pool.map(run, mine)))
    except Exception as e:
        if world == 1:
            raise
        local = {"__err__": f"rank {rank}: subproblem failed: {e!r}"}
    if world > 1:
        every: List[Optional[Dict[int, List[Node]]]] = [None] * world
        dist.all_gather_object(every, local, group=group)
        errs = [d["__err__"] for d in every if "__err__" in d]
        if errs:
            raise RuntimeError("; ".join(errs))
        solved: Dict[int, List[Node]] = {}
        for d in every:
            solved.update(d)
    else:
        solved = local
    path = stitch(solved, len(points) - 1, fix_all)
    return text_of(A1, B1, m, n, len(order), path), path
