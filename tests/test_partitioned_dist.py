"""One pair over several ranks (partitioned.py) on CPU with gloo, world size 2 and 3.

The partition is found on rank 0 and broadcast, the subproblems
``optimal_alignment`` solves (main_alignment.cpp:232-341) are split over the
ranks, their node lists all-gathered and stitched (:344-348).  Here the oracle
stands in for the GPU partition and subproblem solver, so the split, the
broadcast, the gather and the stitch are checked without a GPU against
tests/golden/optimal.json (text and path produced by the reference itself, 77
partitions, reference behaviour and fix_all) and against the oracle's
single-process chain over the partitions partial.cpp finds."""
import json
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import GOLDEN

OPT = json.loads((GOLDEN / "optimal.json").read_text())
# (m, n, p, seed): partition found by the (oracle) partial scorer on rank 0
# (the first two give partitions msa_optimal_alignment refuses: a coordinate goes backwards)
PARTS = [(60, 75, 6, 1), (90, 40, 8, 2), (60, 75, 6, 4), (33, 33, 3, 3), (100, 100, 4, 1), (80, 80, 2, 2),
         (300, 280, 8, 3), (64, 64, 4, 4)]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _pair(m, n, seed):
    rng = np.random.default_rng(seed)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    A = rng.choice(acgt, m).tobytes()
    B = bytearray(A[:n] if n <= m else A + rng.choice(acgt, n - m).tobytes())
    for k in rng.integers(0, n, size=max(1, n // 8)):
        B[k] = b"ACGT"[int(rng.integers(0, 4))]
    return A, bytes(B)


def _oracle_fns():
    from oracle import oracle as O

    def part(A1, B1, m, n, p, g, h):
        return O.partial_partition(A1[1:m + 1], B1[1:n + 1], p, g, h, -1, -1)

    def solve(A1, B1, bp, k, g, h):
        (i0, j0, t0), (i1, j1, t1) = bp[k], bp[k + 1]
        return O.subproblem_align(A1[1:-1], B1[1:-1], t0, -t1, g, h, idA=i0, idB=j0, m=i1 - i0, n=j1 - j0)["nodes"]

    return part, solve


def _run_all(rank, world):
    """Every case through optimal_alignment_distributed: (text, path, subproblems this rank solved)
    or the ValueError text for a partition msa_optimal_alignment refuses."""
    from cse305_parallel_sequence_alignment_amd.partitioned import optimal_alignment_distributed

    part, solve = _oracle_fns()
    calls = []

    def counted(A1, B1, bp, k, g, h):
        calls.append(k)
        return solve(A1, B1, bp, k, g, h)

    def refuse(*a):
        raise AssertionError("only rank 0 finds the partition")

    res = []
    for c in OPT:
        A, B = c["A"].encode(), c["B"].encode()
        for fix in (False, True):
            calls.clear()
            text, path = optimal_alignment_distributed(b"\0" + A + b"\0", b"\0" + B + b"\0", len(A), len(B), 4,
                                                       c["g"], c["h"], fix_all=fix, bp=c["bp"], solve_fn=counted)
            res.append((text, [list(x) for x in path], sorted(calls)))
    for (m, n, p, seed) in PARTS:
        A, B = _pair(m, n, seed)
        for fix in (False, True):
            calls.clear()
            try:
                text, path = optimal_alignment_distributed(b"\0" + A + b"\0", b"\0" + B + b"\0", m, n, p, 1.0, 2.0,
                                                           fix_all=fix, partition_fn=part if rank == 0 else refuse,
                                                           solve_fn=counted)
                res.append((text, [list(x) for x in path], sorted(calls)))
            except ValueError as e:
                res.append(("refused", str(e), []))
    return res


def _want():
    from oracle import oracle as O

    want = []
    for c in OPT:
        for key in ("ref", "fix_all"):
            want.append((c[key]["text"], c[key]["path"], c["bp"], key == "fix_all"))
    for (m, n, p, seed) in PARTS:
        A, B = _pair(m, n, seed)
        bp = O.partial_partition(A, B, p, 1.0, 2.0, -1, -1)
        mono = all(bp[k + 1][0] >= bp[k][0] and bp[k + 1][1] >= bp[k][1] and bp[k + 1][:2] != bp[k][:2]
                   and bp[k + 1][0] <= m and bp[k + 1][1] <= n for k in range(len(bp) - 1))
        for fix in (False, True):
            if not mono:
                want.append(("refused", None, bp, fix))
                continue
            text, path = O.optimal_alignment(A, B, bp, 1.0, 2.0, fix)
            want.append((text, [list(x) for x in path], bp, fix))
    return want


def _worker(rank, world, port, q):
    import sys
    import traceback

    from conftest import ROOT

    sys.path.insert(0, str(ROOT))
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        try:
            q.put((rank, _run_all(rank, world)))
        finally:
            dist.destroy_process_group()
    except Exception:
        q.put((rank, traceback.format_exc()))


def _check(results_per_rank, world):
    from cse305_parallel_sequence_alignment_amd.partitioned import solve_order

    want = _want()
    n_mono = 0
    for c, (text, path, bp, fix) in enumerate(want):
        solved = []
        for r in range(world):
            got_text, got_path, calls = results_per_rank[r][c]
            assert got_text == text, (r, c, bp, fix)
            if text != "refused":
                assert got_path == path, (r, c, bp, fix)
            solved.extend(calls)
        if text != "refused":
            n_mono += 1
            # every subproblem the reference solves is solved exactly once, on some rank
            assert sorted(solved) == sorted(solve_order(len(bp) - 1, fix)), (c, bp, fix)
    assert n_mono == 2 * len(OPT) + 2 * (len(PARTS) - 2)


@pytest.mark.parametrize("world", [2, 3])
def test_partitioned_world(world):
    from oracle import oracle as O

    O.build()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    try:
        out = dict(q.get(timeout=120) for _ in ps)
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for r in range(world):
        assert not isinstance(out[r], str), out[r]
    for p in ps:
        assert p.exitcode == 0
    _check(out, world)


def _worker_edge(rank, world, port, q):
    """A subgroup whose rank 0 is not global rank 0 (ranks [1, 2] of world 3), and a subproblem that fails
    on one rank (world-wide: every rank raises instead of waiting in the all-gather)."""
    import sys
    import traceback

    from conftest import ROOT

    sys.path.insert(0, str(ROOT))
    import torch.distributed as dist

    from cse305_parallel_sequence_alignment_amd.partitioned import optimal_alignment_distributed

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        try:
            part, solve = _oracle_fns()
            A, B = _pair(300, 280, 3)
            sub = dist.new_group([1, 2])
            out = {}
            if rank in (1, 2):
                def part1(*a):
                    assert rank == 1, "only the group's rank 0 (global rank 1) finds the partition"
                    return part(*a)

                out["sub"] = optimal_alignment_distributed(b"\0" + A + b"\0", b"\0" + B + b"\0", 300, 280, 8, 1.0,
                                                           2.0, fix_all=True, partition_fn=part1, solve_fn=solve,
                                                           group=sub)[0]

            def bad(A1, B1, bp, k, g, h):
                if rank == world - 1:
                    raise RuntimeError("injected solve failure")
                return solve(A1, B1, bp, k, g, h)

            try:
                optimal_alignment_distributed(b"\0" + A + b"\0", b"\0" + B + b"\0", 300, 280, 8, 1.0, 2.0,
                                              fix_all=True, partition_fn=part, solve_fn=bad)
                out["fail"] = "no error"
            except RuntimeError as e:
                out["fail"] = str(e)
            q.put((rank, out))
        finally:
            dist.destroy_process_group()
    except Exception:
        q.put((rank, traceback.format_exc()))


def test_partitioned_subgroup_and_solve_failure():
    from oracle import oracle as O

    O.build()
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker_edge, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    try:
        out = dict(q.get(timeout=120) for _ in ps)
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for r in range(world):
        assert not isinstance(out[r], str), out[r]
    A, B = _pair(300, 280, 3)
    bp = O.partial_partition(A, B, 8, 1.0, 2.0, -1, -1)
    want, _ = O.optimal_alignment(A, B, bp, 1.0, 2.0, True)
    assert out[1]["sub"] == out[2]["sub"] == want
    for r in range(world):
        assert "injected solve failure" in out[r]["fail"] and f"rank {world - 1}" in out[r]["fail"], out[r]


def test_partitioned_world1_matches_oracle():
    """No process group: the same code on one rank (the GPU box's world-1 run)."""
    from oracle import oracle as O

    O.build()
    _check({0: _run_all(0, 1)}, 1)


def test_solve_order_assign_stitch():
    from cse305_parallel_sequence_alignment_amd.partitioned import assign, check_partition, solve_order, stitch

    assert solve_order(2, False) == [0]
    assert solve_order(3, False) == [0]
    assert solve_order(4, False) == [0, 3, 1, 2]
    assert solve_order(7, False) == [0, 3, 6, 1, 4, 2, 5]
    assert solve_order(5, True) == [0, 1, 2, 3, 4]
    bp = [(0, 0, -1), (10, 12, 1), (11, 30, 2), (40, 41, 1), (41, 50, 3)]
    order = solve_order(4, True)
    for w in (1, 2, 3, 5):
        share = assign(order, bp, w)
        assert sorted(k for s in share for k in s) == order
    # the largest subproblem (k=2: 30 x 12) goes first, to rank 0
    assert assign(order, bp, 2)[0][0] == 2
    nodes = {0: [(1, 1, 1)], 1: [(2, 2, 1)], 2: [(3, 3, 1)], 3: [(4, 4, 1)]}
    assert stitch(nodes, 4, True) == [(1, 1, 1), (2, 2, 1), (3, 3, 1), (4, 4, 1)]
    assert stitch(nodes, 4, False) == [(1, 1, 1), (2, 2, 1), (3, 3, 1)]   # the link into the last is never made
    assert stitch({0: [(1, 1, 1)], 2: [(3, 3, 1)]}, 4, True) == [(1, 1, 1)]   # an unsolved one ends the walk
    with pytest.raises(ValueError):
        check_partition([(0, 0, -1), (5, 5, 1), (5, 5, 1)], 10, 10)
    with pytest.raises(ValueError):
        check_partition([(0, 0, -1), (5, 5, 1), (4, 9, 1)], 10, 10)
