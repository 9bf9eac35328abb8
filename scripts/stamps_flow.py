#!/usr/bin/env python3
"""Diagnostic (needs a -DMSA_STAMPS build of libmsa.so, optionally with -DMSA_ABL ablations):
per-stripe start / end times and slow-path phase counts of a flow kernel's pass 1 (items < 64),
for the C2 (SW linear, H, two rows per lane), C5 (SW affine, direction bytes) or ref
(Gotoh, tag bytes) single pair.  Prints one JSON summary line.

    python3 scripts/stamps_flow.py --workload c2 [--tag name]
"""
import argparse
import ctypes as C
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np
import torch

from cse305_parallel_sequence_alignment_amd import _lib as LB, data
from cse305_parallel_sequence_alignment_amd.plan import Plan

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="c2", choices=["c2", "c5", "ref"])
ap.add_argument("--tag", default="")
ap.add_argument("--ref-len", type=int, default=10000, help="ref: prefix length (0 = whole sequences)")
ap.add_argument("--ref-pair", default="0,1")
args = ap.parse_args()
wl = args.workload
if wl == "c2":
    A, B = data.c2_pair(0)
    pl = Plan(LB.SW_LINEAR, LB.CELLS_H, [len(A)], [len(B)], [0], [0], match=1, mismatch=0, gap_open=1, gap_extend=1)
    out = torch.empty(pl.cells_elems, dtype=torch.int32, device="cuda")
    rows = 128
elif wl == "c5":
    A, B = data.c5_pair(0)
    pl = Plan(LB.SW_AFFINE, LB.CELLS_DIR, [len(A)], [len(B)], [0], [0], match=1, mismatch=0, gap_open=3,
              gap_extend=1, track_end=True)
    out = torch.empty(pl.cells_elems, dtype=torch.uint8, device="cuda")
    rows = 64
else:
    ia, ib = (int(x) for x in args.ref_pair.split(","))
    A, B = data.bundled()[ia], data.bundled()[ib]
    if args.ref_len:
        A, B = A[:args.ref_len], B[:args.ref_len]
    pl = Plan(LB.REF_GOTOH, LB.CELLS_DIR, [len(A)], [len(B)], [0], [0], match=1, mismatch=0, gap_open=3,
              gap_extend=1, start_type=-1)
    out = torch.empty(pl.cells_elems, dtype=torch.uint8, device="cuda")
    rows = 64
dA = torch.from_numpy(data.encode(A)).cuda()
dB = torch.from_numpy(data.encode(B)).cuda()
st = torch.zeros(64 * 16 * 4096 * 4, dtype=torch.int64, device="cuda")
lib = LB.lib()
lib.msa_debug_stamps.argtypes = [C.c_void_p, C.c_void_p]
kms = []
for rep in range(4):
    st.zero_()
    lib.msa_debug_stamps(pl._h, C.c_void_p(st.data_ptr()))
    pl.run(dA, dB, out)
    torch.cuda.synchronize()
    kms.append(pl.kernel_ms())
full = st.cpu().numpy().reshape(64, 16, 4096, 4)
s = full[:, :4, 0, :]  # item, wave, slot
wq = full[:, :4, 1, :]  # SW-linear waves: ticks waiting on the producer, on consumers, consumer waits
t0 = s[0, 0, 0]
recs = []
for it in range(64):
    for w in range(4):
        a, b, ns = s[it, w, 0], s[it, w, 1], s[it, w, 2]
        if a == 0:
            continue
        recs.append((4 * it + w, (a - t0) / 100.0, (b - t0) / 100.0, (b - a) / 100.0, int(ns)))
ks = np.array([r[0] for r in recs])
starts = np.array([r[1] for r in recs])
durs = np.array([r[3] for r in recs])
lag = np.diff(starts)
P0 = (len(B) + 63) // 16 + 1
out = dict(tag=args.tag, workload=wl, kernel_ms=[round(x, 4) for x in kms], stripes=len(recs),
           dur0_us=round(float(durs[0]), 2), phase0_us=round(float(durs[0]) / P0, 4),
           cycles_per_step0=round(float(durs[0]) / P0 / 16 * 2400, 1),
           dur_by_wave_us=[round(float(durs[ks % 4 == w].mean()), 2) for w in range(4)],
           dur_mean_us=round(float(durs.mean()), 2), dur_max_us=round(float(durs.max()), 2),
           lag_intra_us=round(float(lag[(ks[1:] % 4) != 0].mean()), 3) if len(lag) else None,
           lag_inter_us=round(float(lag[(ks[1:] % 4) == 0].mean()), 3) if len(lag) else None,
           last_end_us=round(float(max(r[2] for r in recs)), 2),
           slow_by_wave=[round(float(np.mean([r[4] for r in recs if r[0] % 4 == w])), 1) for w in range(4)],
           rows_per_stripe=rows,
           wait_in_ticks_s0=int(wq[0, 0, 0]), wait_cons_ticks_s0=int(wq[0, 0, 1]), ncons_s0=int(wq[0, 0, 2]),
           wait_in_ticks_mean=float(np.mean([wq[r[0] // 4, r[0] % 4, 0] for r in recs])),
           wait_cons_ticks_mean=float(np.mean([wq[r[0] // 4, r[0] % 4, 1] for r in recs])),
           ncons_mean=float(np.mean([wq[r[0] // 4, r[0] % 4, 2] for r in recs])))
wg = full[63, 15, :2048, :]
started = wg[:, 0] > 0
if started.any():
    ws, we, role = wg[started, 0], wg[started, 1], wg[started, 2]
    out.update(wg_count=int(started.sum()), wg_first_start_us=round(float((ws.min() - t0) / 100.0), 2),
               wg_last_end_us=round(float((we.max() - t0) / 100.0), 2),
               pass1_last_end_us=round(float((we[role == 1].max() - t0) / 100.0), 2) if (role == 1).any() else None,
               pass2_last_end_us=round(float((we[role == 2].max() - t0) / 100.0), 2) if (role == 2).any() else None,
               wg_last_start_us=round(float((ws.max() - t0) / 100.0), 2),
               wg_started_after_100us=int(((ws - t0) / 100.0 > 100).sum()),
               wg_pass1=int((role == 1).sum()), wg_pass2=int((role == 2).sum()),
               pass2_started_after_100us=int((((ws - t0) / 100.0) > 100)[role == 2].sum()))
cl = full[63, 15, 2048:, :]
claimed = cl[:, 2] > 0
if claimed.any():
    it0 = np.where(cl[:, 2] == 1)[0]
    if len(it0):
        b0 = it0[0]
        out.update(item0_wg_start_us=round(float((wg[b0, 0] - t0) / 100.0), 2),
                   item0_role_us=round(float((cl[b0, 0] - t0) / 100.0), 2),
                   item0_claim_us=round(float((cl[b0, 1] - t0) / 100.0), 2),
                   claim_us_max=round(float((cl[claimed, 1].max() - t0) / 100.0), 2))
    io0 = full[0, 4, 0, 0]
    if io0:
        out.update(item0_codes_loaded_us=round(float((io0 - t0) / 100.0), 2))
p2 = full[62, 15, 0, :]  # pass-2 block totals (Gotoh fill blocks): wait, load, compute ticks, blocks
if p2[3]:
    out.update(p2_blocks=int(p2[3]), p2_wait_ticks_per_block=round(float(p2[0]) / p2[3], 1),
               p2_load_ticks_per_block=round(float(p2[1]) / p2[3], 1),
               p2_compute_ticks_per_block=round(float(p2[2]) / p2[3], 1))
print(json.dumps(out), flush=True)
