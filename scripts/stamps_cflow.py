#!/usr/bin/env python3
"""Diagnostic (needs a -DMSA_STAMPS build of libmsa.so): the chains of cflow_kernel (C4 packed couples,
msa_cflow.hip) for couples 0..3 -- per stripe its start / end (s_memrealtime, 100 MHz, chip-wide), the
phases that waited on their producer and the s_memtime ticks spent waiting on producer / consumer.
Prints one JSON line: mean phase time, mean start lag between consecutive stripes inside an item and
across items, chain length, wait shares.

    python3 scripts/stamps_cflow.py --lib variants/libmsa_stamps.so --pairs 128
"""
import argparse
import ctypes as C
import json
import os
import sys
from pathlib import Path

ap = argparse.ArgumentParser()
ap.add_argument("--lib", required=True)
ap.add_argument("--pairs", type=int, default=128)
ap.add_argument("--tag", default="")
args = ap.parse_args()
os.environ["MSA_LIB_PATH"] = str(Path(args.lib).resolve())
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np
import torch

from cse305_parallel_sequence_alignment_amd import _lib as LB, data
from cse305_parallel_sequence_alignment_amd.plan import Plan

L = data.C4_LEN
qs = data.c4_queries(0, args.pairs)
B = data.c4_reference()
pl = Plan(LB.SW_LINEAR, LB.CELLS_NONE, [L] * len(qs), [L] * len(qs), [k * L for k in range(len(qs))],
          [0] * len(qs), match=1, mismatch=0, gap_open=1, gap_extend=1)
info = pl.launch_info()
dA = torch.from_numpy(data.encode(b"".join(qs))).cuda()
dB = torch.from_numpy(data.encode(B)).cuda()
st = torch.zeros(64 * 16 * 4096 * 4, dtype=torch.int64, device="cuda")
lib = LB.lib()
lib.msa_debug_stamps.argtypes = [C.c_void_p, C.c_void_p]
kms = []
for rep in range(3):
    st.zero_()
    lib.msa_debug_stamps(pl._h, C.c_void_p(st.data_ptr()))
    pl.run(dA, dB)
    torch.cuda.synchronize()
    kms.append(pl.kernel_ms())
lib.msa_debug_stamps(pl._h, C.c_void_p(0))
S = st.cpu().numpy().reshape(64, 16, 4096, 4)
W = 4
ncpl = (len(qs) + 1) // 2
nstr = (L + 63) // 64
P = (L + 15 + 63) // 16 + 1  # fl_P of a full stripe (cs in [-15, 0])
res = dict(tag=args.tag, pairs=args.pairs, launch=info, kernel_ms=[round(k, 4) for k in kms])
chains = []
for cpl in range(min(4, ncpl)):
    rows = []
    for k in range(nstr):
        grp, w = divmod(k, W)
        s = S[cpl * 16 + grp, w]
        t0, t1 = s[0, 0], s[0, 1]
        if t0 == 0 or t1 == 0:
            continue
        rows.append(dict(k=k, start=t0 / 100.0, end=t1 / 100.0, nslow=int(s[0, 2]), tw_in=int(s[0, 3]),
                         tw_cons=int(s[1, 0]), claim=S[cpl * 16 + grp, W, 1, 1] / 100.0))
    if len(rows) < 2:
        continue
    base = rows[0]["start"]
    starts = np.array([r["start"] - base for r in rows])
    ends = np.array([r["end"] - base for r in rows])
    ks = np.array([r["k"] for r in rows])
    durs = ends - starts
    lag = np.diff(starts)
    inner = [lag[i] for i in range(len(lag)) if ks[i + 1] % W != 0]
    cross = [lag[i] for i in range(len(lag)) if ks[i + 1] % W == 0]
    ph = float(np.mean(durs)) / P
    claims = [r["claim"] - base for r in rows if r["k"] % W == 0 and r["claim"] > 0]
    chains.append(dict(
        couple=cpl, stripes=len(rows), chain_us=round(float(ends.max()), 2), phase_us=round(ph, 4),
        lag_inner_us=round(float(np.mean(inner)), 3) if inner else None,
        lag_cross_us=round(float(np.mean(cross)), 3) if cross else None,
        lag_inner_phases=round(float(np.mean(inner)) / ph, 2) if inner else None,
        lag_cross_phases=round(float(np.mean(cross)) / ph, 2) if cross else None,
        nslow_mean=round(float(np.mean([r["nslow"] for r in rows])), 1),
        wait_in_share=round(float(np.mean([r["tw_in"] / 2400.0 / max(1e-9, d) for r, d in zip(rows, durs)])), 3),
        wait_cons_share=round(float(np.mean([r["tw_cons"] / 2400.0 / max(1e-9, d) for r, d in zip(rows, durs)])), 3),
        claim_minus_start_us=[round(c - s, 1) for c, s in zip(claims, starts[ks % W == 0])][:16],
        # per item boundary (item g-1 -> g): the start lag of its first stripe, in phases
        cross_lags_phases=[round(float(lag[i]) / ph, 1) for i in range(len(lag)) if ks[i + 1] % W == 0],
        item_starts_us=[round(float(t), 1) for t, k in zip(starts, ks) if k % W == 0]))
res["chains"] = chains
print(json.dumps(res))
