"""Diagnostic: single-pair SW-linear kernel time vs m at fixed n (slope = per-stripe lag)."""
import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from cse305_parallel_sequence_alignment_amd import _lib as LB
from cse305_parallel_sequence_alignment_amd.plan import Plan
from oracle.oracle import load_dataset
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
ms = [int(x) for x in (sys.argv[2].split(",") if len(sys.argv) > 2 else "64,256,1024,2560,5120,10000".split(","))]
seqs = load_dataset()[1]
enc = lambda s: torch.from_numpy(np.frombuffer(s.translate(bytes.maketrans(b"ACGT", b"\x00\x01\x02\x03")), dtype=np.uint8).copy()).cuda()
for mode in ("h", "n"):
    for m in ms:
        A, B = (seqs[1] * 8)[:m], (seqs[0] * 8)[:n]
        pl = Plan(LB.SW_LINEAR, LB.CELLS_H if mode == "h" else LB.CELLS_NONE, [m], [n], [0], [0],
                  match=1, mismatch=0, gap_open=1, gap_extend=1)
        out = torch.empty(max(1, pl.cells_elems), dtype=torch.int32, device="cuda") if mode == "h" else None
        dA, dB = enc(A), enc(B)
        ts = []
        for it in range(6):
            pl.run(dA, dB, out)
            torch.cuda.synchronize()
            ts.append(pl.kernel_ms())
        print(mode, "m", m, "n", n, "ms", round(min(ts[1:]), 4), "score", pl.results()[0]["score"], flush=True)
