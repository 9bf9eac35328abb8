"""Minimal driver for rocprofv3 runs: a few launches of one bench workload (same plans as bench.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from cse305_parallel_sequence_alignment_amd import _lib as LB
from cse305_parallel_sequence_alignment_amd.plan import Plan
from oracle.oracle import load_dataset

wl = sys.argv[1] if len(sys.argv) > 1 else "c2"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
seqs = load_dataset()[1]
enc = lambda s: torch.from_numpy(np.frombuffer(s.translate(bytes.maketrans(b"ACGT", b"\x00\x01\x02\x03")),
                                               dtype=np.uint8).copy()).cuda()
out = None
if wl in ("c2", "c2n"):
    A, B = seqs[1][:10000], seqs[0][:10000]
    cells = LB.CELLS_H if wl == "c2" else LB.CELLS_NONE
    pl = Plan(LB.SW_LINEAR, cells, [10000], [10000], [0], [0], match=1, mismatch=0, gap_open=1, gap_extend=1)
elif wl in ("c5", "c5h"):
    from cse305_parallel_sequence_alignment_amd import data

    A, B = data.c5_pair(0, False)  # the bench's C5 pair (c5h: its first 10k x 10k, a plane under the L3's size)
    if wl == "c5h":
        A, B = A[:10000], B[:10000]
    pl = Plan(LB.SW_AFFINE, LB.CELLS_DIR, [len(A)], [len(B)], [0], [0], match=1, mismatch=0, gap_open=3,
              gap_extend=1, track_end=True)
elif wl in ("ref", "ref20", "refwhole"):
    L = {"ref": 10000, "ref20": 20000, "refwhole": None}[wl]
    # the bench's ref pairs (main_alignment_function's path); refwhole = bench --ref-pair 3,4 --ref-len 0
    A, B = (seqs[0][:L], seqs[1][:L]) if L else (seqs[3], seqs[4])
    L = len(A)
    pl = Plan(LB.REF_GOTOH, LB.CELLS_DIR, [len(A)], [len(B)], [0], [0], match=1, mismatch=0, gap_open=3,
              gap_extend=1, start_type=-1)
elif wl == "c3":
    from cse305_parallel_sequence_alignment_amd import data

    A, B = data.c3_pair(False)
    pl = Plan(LB.NW_BANDED, LB.CELLS_H, [len(A)], [len(B)], [0], [0], match=1, mismatch=0, gap_open=3,
              gap_extend=1, band=512)
else:  # c4 (1024 pairs) / c4_128 (the first 128: one rank's share at 8 GPUs, split mode)
    L, K = 4000, (128 if wl == "c4_128" else 1024)
    rng = np.random.default_rng(0x5EED0004)
    offs = rng.integers(0, 13309 - L, size=1024)  # the same windows as data.c4_offsets()
    A = b"".join(seqs[k % 20][offs[k]:offs[k] + L] for k in range(K))
    B = seqs[0][:L]
    pl = Plan(LB.SW_LINEAR, LB.CELLS_NONE, [L] * K, [L] * K, [k * L for k in range(K)], [0] * K, match=1,
              mismatch=0, gap_open=1, gap_extend=1)
if pl.cells != LB.CELLS_NONE:
    out = torch.empty(pl.cells_elems, dtype=torch.uint8 if pl.cells == LB.CELLS_DIR else torch.int32, device="cuda")
dA, dB = enc(A), enc(B)
tb = None
if wl in ("c5", "c5h", "ref", "ref20", "refwhole"):  # the bench's step: fill, then the traceback walk on the device
    tb = (torch.empty(len(A) + len(B) + 2, dtype=torch.uint8, device="cuda"),
          torch.zeros(8, dtype=torch.int64, device="cuda"))
for _ in range(reps):
    pl.run(dA, dB, out)
    if tb is not None:
        if wl in ("c5", "c5h"):
            pl.traceback_async(out, *tb)
        else:
            pl.traceback_gotoh_async(out, *tb, -1)
torch.cuda.synchronize()
print("score", pl.results()[0]["score"], "kernel_ms", pl.kernel_ms())
