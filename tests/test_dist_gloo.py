"""World-size-2 sharding path on CPU (gloo): pairs split over ranks, scores all-gathered.

The per-rank compute on a GPU box is the stripe kernel; here each rank scores
its block with the oracle so the sharding/gather logic (shard.py, used by
bench.py's multi-GPU c4 workload) is checked without a GPU."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n_pairs, q):
    import sys

    from conftest import ROOT

    sys.path.insert(0, str(ROOT))
    import torch.distributed as dist

    from cse305_parallel_sequence_alignment_amd.shard import shard_range, sharded_scores
    from oracle import oracle as O

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(42)
        pairs = [(rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), 50 + 7 * k).tobytes(),
                  rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), 60).tobytes()) for k in range(n_pairs)]
        seen = []

        def scorer(block):
            seen.extend(block)
            return [O.sw(a, b, 2, -1, 1, 1)["score"] for a, b in block]

        got = sharded_scores(pairs, scorer, rank, world)
        lo, hi = shard_range(n_pairs, rank, world)
        q.put((rank, got.tolist(), len(seen), hi - lo))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_pairs", [7, 8, 1])
def test_sharded_scores_world2(n_pairs):
    from oracle import oracle as O

    O.build()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, n_pairs, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    rng = np.random.default_rng(42)
    pairs = [(rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), 50 + 7 * k).tobytes(),
              rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), 60).tobytes()) for k in range(n_pairs)]
    want = [O.sw(a, b, 2, -1, 1, 1)["score"] for a, b in pairs]
    for rank, got, nseen, nblock in out:
        assert got == want
        assert nseen == nblock
    assert sum(o[2] for o in out) == n_pairs


def test_shard_range_partitions():
    from cse305_parallel_sequence_alignment_amd.shard import shard_range

    for n in (0, 1, 5, 1024, 1023):
        for w in (1, 2, 3, 8):
            blocks = [shard_range(n, r, w) for r in range(w)]
            covered = [i for lo, hi in blocks for i in range(lo, hi)]
            assert covered == list(range(n))
