"""Diagnostic: wall time per plan.run step of C2 (like bench.py's timed loop)."""
import sys, os, time
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from cse305_parallel_sequence_alignment_amd import _lib as LB
from cse305_parallel_sequence_alignment_amd.plan import Plan
from oracle.oracle import load_dataset
seqs = load_dataset()[1]
enc = lambda s: torch.from_numpy(np.frombuffer(s.translate(bytes.maketrans(b"ACGT", b"\x00\x01\x02\x03")), dtype=np.uint8).copy()).cuda()
A, B = seqs[1][:10000], seqs[0][:10000]
pl = Plan(LB.SW_LINEAR, LB.CELLS_H, [10000], [10000], [0], [0], match=1, mismatch=0, gap_open=1, gap_extend=1)
out = torch.empty(pl.cells_elems, dtype=torch.int32, device="cuda")
dA, dB = enc(A), enc(B)
for rep in range(3):
    for _ in range(3):
        pl.run(dA, dB, out)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        pl.run(dA, dB, out)
    torch.cuda.synchronize()
    print("ms/step", round((time.perf_counter() - t0) / 20 * 1e3, 4), "score", pl.results()[0]["score"], flush=True)
