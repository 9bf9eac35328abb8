#!/usr/bin/env python3
"""Diagnostic: per-stripe best cells of a packed C4-shape batch (cflow kernels) against the oracle's H matrix,
to find the first stripe a kernel variant gets wrong.  MSA_C4_KERNEL selects the kernel.

    MSA_C4_KERNEL=cflow4 python3 scripts/dbg_cflow.py --pairs 2 --len 1000
"""
import argparse
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np
import torch

from cse305_parallel_sequence_alignment_amd import _lib as LB
from cse305_parallel_sequence_alignment_amd.plan import Plan
from oracle import oracle as O

ap = argparse.ArgumentParser()
ap.add_argument("--pairs", type=int, default=2)
ap.add_argument("--len", type=int, default=1000)
args = ap.parse_args()
rng = np.random.default_rng(7)
L, K = args.len, args.pairs
acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
As = [rng.choice(acgt, L).tobytes() for _ in range(K)]
B = rng.choice(acgt, L).tobytes()
tr = bytes.maketrans(b"ACGT", b"\x00\x01\x02\x03")
enc = lambda s: torch.from_numpy(np.frombuffer(s.translate(tr), dtype=np.uint8).copy()).cuda()
pl = Plan(LB.SW_LINEAR, LB.CELLS_NONE, [L] * K, [L] * K, [k * L for k in range(K)], [0] * K, match=1, mismatch=0,
          gap_open=1, gap_extend=1, single=False)
info = pl.launch_info()
pl.run(enc(b"".join(As)), enc(B))
res = pl.results()
meta = pl.stripe_meta()
out = dict(launch=info, pairs=[])
for k in range(min(K, 4)):
    o = O.sw(As[k], B, 1, 0, 1, 1, want_h=True)
    H = o["H"]
    S = (L + 63) // 64
    g0 = pl.geom[k].stripe0
    bad = []
    for s in range(S):
        want = int(H[64 * s + 1:min(L, 64 * s + 64) + 1, :].max())
        got = int(meta[g0 + s, 2])
        if got != want:
            bad.append((s, got, want))
    out["pairs"].append(dict(pair=k, score=res[k]["score"], want=o["score"], first_bad=bad[:6], n_bad=len(bad)))
print(json.dumps(out))
