#!/usr/bin/env python3
"""Diagnostic: per-stripe best cells of a packed C4-shape batch (cflow_kernel) against the oracle's H
matrix, over several launches of one plan, to find the stripes a kernel build gets wrong and whether
the error repeats (a deterministic defect) or moves (a race).  MSA_C4_KERNEL selects the kernel,
MSA_LIB_PATH the library build.

A stripe's best is over every cell its lanes compute, the virtual columns right of n included: lane r
runs columns up to cs + 16 P - 1 - r, and a virtual column scores as a mismatch (code 7: H(i, n + d) can
equal H(i - d, n), a real cell of a row above -- possibly of the stripe above).  The expectation here
is the oracle's H over B extended by never-matching columns, so a stripe may legitimately report a
real cell of an earlier stripe (the pair's score, the maximum over stripes, is unaffected; round 5
read those stripes as wrong cells).

    MSA_LIB_PATH=vlib/libmsa_wpe5.so python3 scripts/dbg_cflow.py --pairs 4 --len 4000 --reps 5

Prints one JSON line: the launch shape and, per launch, every (pair, stripe, got, want) that differs.
"""
import argparse
import json
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
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--seed", type=int, default=7)
args = ap.parse_args()
rng = np.random.default_rng(args.seed)
L, K = args.len, args.pairs
acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
As = [rng.choice(acgt, L).tobytes() for _ in range(K)]
B = rng.choice(acgt, L).tobytes()
tr = bytes.maketrans(b"ACGT", b"\x00\x01\x02\x03")


def enc(s):
    return torch.from_numpy(np.frombuffer(s.translate(tr), dtype=np.uint8).copy()).cuda()


pl = Plan(LB.SW_LINEAR, LB.CELLS_NONE, [L] * K, [L] * K, [k * L for k in range(K)], [0] * K, match=1, mismatch=0,
          gap_open=1, gap_extend=1, single=False)
S = (L + 63) // 64
dA, dB = enc(b"".join(As)), enc(B)
pl.run(dA, dB)
meta0 = pl.stripe_meta()
EXT = 64 + 16 * int(meta0[:, 1].max())  # virtual columns any lane can reach
want = []
for k in range(K):
    H = O.sw(As[k], B + b"N" * EXT, 1, 0, 1, 1, want_h=True)["H"]
    g0 = pl.geom[k].stripe0
    row = []
    for s in range(S):
        cs, P = int(meta0[g0 + s, 0]), int(meta0[g0 + s, 1])
        row.append(max(int(H[64 * s + 1 + r, 1:min(cs + 16 * P - 1 - r, L + EXT) + 1].max())
                       for r in range(min(64, L - 64 * s))))
    want.append(row)
out = dict(launch=pl.launch_info(), pairs=K, len=L, runs=[])
for rep in range(args.reps):
    pl.run(dA, dB)
    meta = pl.stripe_meta()
    bad = []
    for k in range(K):
        g0 = pl.geom[k].stripe0
        for s in range(S):
            got = int(meta[g0 + s, 2])
            if got != want[k][s]:
                bad.append((k, s, got, want[k][s]))
    out["runs"].append(dict(n_bad=len(bad), bad=bad[:12], err=pl.error()))
print(json.dumps(out))
