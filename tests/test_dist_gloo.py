"""World-size-2 sharding path on CPU (gloo): pairs split over ranks, scores all-gathered.

bench.py's multi-GPU c4 workload runs ``shard.ShardedBatch`` with a device Plan
as the per-rank scorer; here the same class runs with the oracle as the
scorer, so the split, the reference broadcast and the gather are checked
without a GPU."""
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

    import torch

    from cse305_parallel_sequence_alignment_amd.shard import ShardedBatch, broadcast_reference, shard_range
    from oracle import oracle as O

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(42)
        queries = [rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), 50 + 7 * k).tobytes() for k in range(n_pairs)]
        # only rank 0 holds the reference sequence; the broadcast gives it to every rank
        ref = torch.from_numpy(np.frombuffer(b"ACGT" * 15, dtype=np.uint8).copy()) if rank == 0 else \
            torch.zeros(60, dtype=torch.uint8)
        ref = bytes(broadcast_reference(ref).numpy())
        seen = []

        def score_block(lo, hi):
            seen.extend(range(lo, hi))
            return torch.tensor([O.sw(queries[k], ref, 2, -1, 1, 1)["score"] for k in range(lo, hi)],
                                dtype=torch.int32)

        got = ShardedBatch(n_pairs, rank, world, score_block).step()
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
    queries = [rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), 50 + 7 * k).tobytes() for k in range(n_pairs)]
    want = [O.sw(a, b"ACGT" * 15, 2, -1, 1, 1)["score"] for a in queries]
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
