"""Minimal driver for rocprofv3 runs: a few launches of one workload."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from cse305_parallel_sequence_alignment_amd import _lib as LB
from cse305_parallel_sequence_alignment_amd.plan import Plan
from oracle.oracle import load_dataset

wl = sys.argv[1] if len(sys.argv) > 1 else "c2"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
seqs = load_dataset()[1]
enc = lambda s: torch.from_numpy(np.frombuffer(s.translate(bytes.maketrans(b"ACGT", b"\x00\x01\x02\x03")), dtype=np.uint8).copy()).cuda()
if wl == "c2n":
    A, B = seqs[1][:10000], seqs[0][:10000]
    pl = Plan(LB.SW_LINEAR, LB.CELLS_NONE, [10000], [10000], [0], [0], match=1, mismatch=0, gap_open=1, gap_extend=1)
    out = None
elif wl == "c2":
    A, B = seqs[1][:10000], seqs[0][:10000]
    pl = Plan(LB.SW_LINEAR, LB.CELLS_H, [10000], [10000], [0], [0], match=1, mismatch=0, gap_open=1, gap_extend=1)
    out = torch.empty(pl.cells_elems, dtype=torch.int32, device="cuda")
else:
    L, K = 4000, 1024
    rng = np.random.default_rng(0x5EED0004)
    offs = rng.integers(0, 13309 - L, size=K)
    A = b"".join(seqs[k % 20][offs[k]:offs[k] + L] for k in range(K)); B = seqs[0][:L]
    pl = Plan(LB.SW_LINEAR, LB.CELLS_NONE, [L] * K, [L] * K, [k * L for k in range(K)], [0] * K, match=1, mismatch=0, gap_open=1, gap_extend=1)
    out = None
dA, dB = enc(A), enc(B)
for _ in range(reps):
    pl.run(dA, dB, out)
torch.cuda.synchronize()
print("score", pl.results()[0]["score"], "kernel_ms", pl.kernel_ms())
