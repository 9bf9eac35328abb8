"""GPU parity of the one-pair-over-several-ranks path (partitioned.py): partition on rank 0's
GPU, subproblems on each rank's GPU through msa_subproblem, node lists all-gathered and
stitched.  Checked exactly against the reference-produced fixtures (tests/golden/optimal.json)
and against the one-process C-ABI chain (msa_main_alignment_partitioned).  The world-2 case
runs both ranks on the one GPU of the box (gloo carries the partition and the node lists)."""
import json
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

OPT = json.loads((GOLDEN / "optimal.json").read_text())


def _pairs():
    """(A, B, p): synthetic related pairs, partitions with and without backward steps."""
    rng = np.random.default_rng(7)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    out = []
    for (m, n, p) in ((300, 280, 8), (1000, 993, 8), (2000, 1990, 5), (640, 700, 16), (100, 100, 4)):
        A = rng.choice(acgt, m).tobytes()
        B = bytearray((A + rng.choice(acgt, max(0, n - m)).tobytes())[:n])
        for k in rng.integers(0, n, size=n // 10):
            B[k] = b"ACGT"[int(rng.integers(0, 4))]
        out.append((A, bytes(B), p))
    return out


def _run(rank):
    from cse305_parallel_sequence_alignment_amd.partitioned import optimal_alignment_distributed

    res = []
    for c in OPT:
        A, B = c["A"].encode(), c["B"].encode()
        for fix in (False, True):
            text, path = optimal_alignment_distributed(b"\0" + A, b"\0" + B, len(A), len(B), 4, c["g"], c["h"],
                                                       fix_all=fix, bp=c["bp"])
            res.append((text, [list(x) for x in path]))
    for (A, B, p) in _pairs():
        for fix in (False, True):
            try:
                text, _ = optimal_alignment_distributed(b"\0" + A, b"\0" + B, len(A), len(B), p, 1.0, 2.0,
                                                        fix_all=fix)
            except ValueError:
                text = "refused"
            res.append((text, None))
    return res


def _want():
    from cse305_parallel_sequence_alignment_amd import _lib as LB
    from cse305_parallel_sequence_alignment_amd import api

    want = [(c[key]["text"], c[key]["path"]) for c in OPT for key in ("ref", "fix_all")]
    for (A, B, p) in _pairs():
        for fix in (False, True):
            try:
                text = api.main_alignment_partitioned_text(b"\0" + A, b"\0" + B, len(A), len(B), p, 1, 2, fix)
            except LB.MsaError:
                text = "refused"
            want.append((text, None))
    return want


def _check(got, want):
    assert len(got) == len(want)
    assert sum(t != "refused" for t, _ in want) > 2 * len(OPT)
    for c, ((gt, gp), (wt, wp)) in enumerate(zip(got, want)):
        assert gt == wt, c
        if wp is not None:
            assert gp == wp, c


def test_partitioned_world1(dev):
    _check(_run(0), _want())


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


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
            q.put((rank, _run(rank)))
        finally:
            dist.destroy_process_group()
    except Exception:
        q.put((rank, traceback.format_exc()))


def test_partitioned_world2_one_gpu(dev):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    try:
        out = dict(q.get(timeout=100) for _ in ps)
    finally:
        for p in ps:
            p.join(timeout=20)
            if p.is_alive():
                p.kill()
    want = _want()
    for r in range(world):
        assert not isinstance(out[r], str), out[r]
        _check(out[r], want)
