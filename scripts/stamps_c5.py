#!/usr/bin/env python3
"""Diagnostic (needs a -DMSA_STAMPS build of libmsa.so): per-stripe start / end times and slow-path
phase counts of the C5 affine flow kernel's pass 1, items < 64 (stripes < 256).

    python3 scripts/stamps_c5.py [--len 20000]
"""
import argparse
import ctypes as C
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np
import torch

from cse305_parallel_sequence_alignment_amd import _lib as LB, data
from cse305_parallel_sequence_alignment_amd.plan import Plan

ap = argparse.ArgumentParser()
ap.add_argument("--len", type=int, default=20000)
args = ap.parse_args()
A, B = data.c5_pair(0)
A, B = A[: args.len], B[: args.len]
pl = Plan(LB.SW_AFFINE, LB.CELLS_DIR, [len(A)], [len(B)], [0], [0], match=1, mismatch=0, gap_open=3, gap_extend=1,
          track_end=True)
dA = torch.from_numpy(data.encode(A)).cuda()
dB = torch.from_numpy(data.encode(B)).cuda()
D = torch.empty(pl.cells_elems, dtype=torch.uint8, device="cuda")
st = torch.zeros(64 * 16 * 4096 * 4, dtype=torch.int64, device="cuda")
lib = LB.lib()
lib.msa_debug_stamps.argtypes = [C.c_void_p, C.c_void_p]
for rep in range(3):
    st.zero_()
    lib.msa_debug_stamps(pl._h, C.c_void_p(st.data_ptr()))
    pl.run(dA, dB, D)
    torch.cuda.synchronize()
    print("kernel ms", pl.kernel_ms())
s = st.cpu().numpy().reshape(64, 16, 4096, 4)[:, :4, 0, :]  # item, wave, slot
t0 = s[0, 0, 0]
rows = []
for it in range(64):
    for w in range(4):
        a, b, ns = s[it, w, 0], s[it, w, 1], s[it, w, 2]
        if a == 0:
            continue
        rows.append((4 * it + w, (a - t0) / 100.0, (b - t0) / 100.0, (b - a) / 100.0, ns))
for k, a, b, d, ns in rows[:12] + rows[-6:]:
    print(f"stripe {k:4d} start {a:8.2f} us end {b:8.2f} us dur {d:8.2f} us slow {ns}")
ks = np.array([r[0] for r in rows]); starts = np.array([r[1] for r in rows]); durs = np.array([r[3] for r in rows])
lag = np.diff(starts)
print("mean start lag us", lag.mean(), "intra-WG", lag[(ks[1:] % 4) != 0].mean(), "inter-WG", lag[(ks[1:] % 4) == 0].mean())
print("mean duration us", durs.mean(), "slow phases mean", np.mean([r[4] for r in rows]))
