#!/usr/bin/env python3
"""Diagnostic (needs a -DMSA_STAMPS build of libmsa.so; -DMSA_STAMPS_RT for chip-wide 100 MHz clocks):
where the C4 split-mode batch (stripe_kernel, kp.single == 3: every packed couple split into items of
8 stripes chained through granules) spends its phases.  Items < 64 are recorded (couples 0..7, all their
groups).  Per phase and item: every wave's arrival at the phase barrier (slot 0), release (slot 1) and,
for compute waves, the end of its compute (slot 2).  Prints one JSON line:

* phase_us by group: mean barrier-to-barrier time of an item's phases (group 0 has no loader work);
* loader_last: fraction of phases whose last arrival at the barrier is the loader wave (w = 8), and
  its mean lateness over the last compute wave;
* item_start_us: release of each item's first phase relative to item 0 of the same couple (RT clocks only).

    python3 scripts/stamps_split.py --lib variants/libmsa_stamps.so [--pairs 128] [--rt]
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
ap.add_argument("--rt", action="store_true", help="the build records s_memrealtime (100 MHz)")
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
dA = torch.from_numpy(data.encode(b"".join(qs))).cuda()
dB = torch.from_numpy(data.encode(B)).cuda()
NPH = 4096
st = torch.zeros(64 * 16 * NPH * 4, dtype=torch.int64, device="cuda")
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
S = np.asarray(st.cpu().numpy().reshape(64, 16, NPH, 4), dtype=np.float64)
tick_us = 0.01 if args.rt else 1.0 / 2400.0  # memrealtime 100 MHz; memtime ~ shader clock
W = 8
groups = (L + 63) // 64 // W + (1 if ((L + 63) // 64) % W else 0)
res = dict(tag=args.tag, pairs=args.pairs, kernel_ms=[round(k, 4) for k in kms], groups=groups, rt=args.rt)
ph_by_group = {}
last_loader = []
late = []
starts = {}
for it in range(64):
    rel = S[it, 0, :, 1]
    nph = int(np.count_nonzero(rel))
    if nph < 2:
        continue
    g = it % groups
    rel = rel[:nph]
    ph_by_group.setdefault(g, []).append(float(np.mean(np.diff(rel))) * tick_us)
    arr = S[it, :W + 1, :nph, 0]  # arrivals, waves 0..8
    lastw = np.argmax(arr, axis=0)
    last_loader.append(float(np.mean(lastw == W)))
    late.append(float(np.mean(np.clip(arr[W] - np.max(arr[:W], axis=0), 0, None))) * tick_us)
    starts[it] = float(rel[0])
res["phase_us_by_group"] = {str(g): round(float(np.mean(v)), 4) for g, v in sorted(ph_by_group.items())}
# compute waves' phase split (MSA_MARK slots: 3 = LDS inputs + codes in registers, 2 = the phase's steps
# done, 0 = at the barrier, 1 = released): start = slot3 - previous release, steps = slot2 - slot3,
# tail = slot0 - slot2 (hand-off, outputs), barrier = slot1 - slot0; phases where the wave computed
split = {"start": [], "steps": [], "tail": [], "barrier": []}
for it in range(64):
    for w in range(W):
        rel = S[it, w, :, 1]
        n_ = int(np.count_nonzero(rel))
        if n_ < 3:
            continue
        s3, s2, s0, s1 = S[it, w, 1:n_, 3], S[it, w, 1:n_, 2], S[it, w, 1:n_, 0], S[it, w, 1:n_, 1]
        prev = S[it, w, 0:n_ - 1, 1]
        ok = (s3 > 0) & (s2 > 0)
        if not np.any(ok):
            continue
        split["start"].append(np.mean((s3 - prev)[ok]))
        split["steps"].append(np.mean((s2 - s3)[ok]))
        split["tail"].append(np.mean((s0 - s2)[ok]))
        split["barrier"].append(np.mean((s1 - s0)[ok]))
res["compute_phase_split_us"] = {k: round(float(np.mean(v)) * tick_us, 4) for k, v in split.items() if v}
res["phases_recorded_item0"] = int(np.count_nonzero(S[0, 0, :, 1]))
res["loader_last_frac_by_item"] = [round(x, 3) for x in last_loader]
res["loader_lateness_us_mean"] = round(float(np.mean(late)), 4) if late else None
if args.rt:
    res["item_start_us"] = {str(it): round((t - starts[(it // groups) * groups]) * tick_us, 2)
                            for it, t in starts.items() if (it // groups) * groups in starts}
    ends = {it: float(S[it, 0, int(np.count_nonzero(S[it, 0, :, 1])) - 1, 1]) for it in starts}
    t00 = min(starts.values())
    res["couple_start_us"] = [round((starts[c] - t00) * tick_us, 2) for c in range(0, 64, groups) if c in starts]
    res["item_end_us"] = {str(it): round((t - starts[(it // groups) * groups]) * tick_us, 2)
                          for it, t in ends.items() if (it // groups) * groups in starts}
print(json.dumps(res))
