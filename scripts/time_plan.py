#!/usr/bin/env python3
"""Diagnostic: DP-kernel time (HIP events on the launch stream) of one single-pair plan, no checks --
for ablation builds (-DMSA_ABL, loaded through MSA_LIB_PATH) whose results are wrong by design.

    MSA_LIB_PATH=variants/libmsa_abl1.so python3 scripts/time_plan.py --workload ref --ref-pair 3,4 --ref-len 0
"""
import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch

from cse305_parallel_sequence_alignment_amd import _lib as LB, data
from cse305_parallel_sequence_alignment_amd.plan import Plan

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="ref", choices=["c2", "c5", "ref", "c3", "c3d", "c3syn"])
ap.add_argument("--ref-len", type=int, default=10000)
ap.add_argument("--ref-pair", default="0,1")
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--check", action="store_true", help="c2: compare the H checksum with the oracle's")
args = ap.parse_args()
if args.workload == "c2":
    A, B = data.c2_pair(0)
    pl = Plan(LB.SW_LINEAR, LB.CELLS_H, [len(A)], [len(B)], [0], [0], match=1, mismatch=0, gap_open=1, gap_extend=1)
    out = torch.empty(pl.cells_elems, dtype=torch.int32, device="cuda")
elif args.workload.startswith("c3"):
    if args.workload == "c3d":  # a dissimilar real pair (rank convergence fails: the exact launch runs)
        A, B = data.bundled()[0][:81835], data.bundled()[15][:81835]
    else:
        A, B = data.c3_pair(synthetic=args.workload == "c3syn")
    pl = Plan(LB.NW_BANDED, LB.CELLS_H, [len(A)], [len(B)], [0], [0], match=1, mismatch=0, gap_open=3,
              gap_extend=1, band=512)
    out = torch.empty(pl.cells_elems, dtype=torch.int32, device="cuda")
elif args.workload == "c5":
    A, B = data.c5_pair(0)
    pl = Plan(LB.SW_AFFINE, LB.CELLS_DIR, [len(A)], [len(B)], [0], [0], match=1, mismatch=0, gap_open=3,
              gap_extend=1, track_end=True)
    out = torch.empty(pl.cells_elems, dtype=torch.uint8, device="cuda")
else:
    ia, ib = (int(x) for x in args.ref_pair.split(","))
    A, B = data.bundled()[ia], data.bundled()[ib]
    if args.ref_len:
        A, B = A[:args.ref_len], B[:args.ref_len]
    pl = Plan(LB.REF_GOTOH, LB.CELLS_DIR, [len(A)], [len(B)], [0], [0], match=1, mismatch=0, gap_open=3,
              gap_extend=1, start_type=-1)
    out = torch.empty(pl.cells_elems, dtype=torch.uint8, device="cuda")
dA = torch.from_numpy(data.encode(A)).cuda()
dB = torch.from_numpy(data.encode(B)).cuda()
kms = []
for _ in range(args.reps):
    pl.run(dA, dB, out)
    kms.append(pl.kernel_ms())
res = dict(workload=args.workload, m=len(A), n=len(B), lib=str(LB.LIB_PATH.name), kernel_ms=kms, error=pl.error(),
           median_ms=sorted(kms)[len(kms) // 2])
if args.workload.startswith("c3"):
    res["run_info"] = pl.run_info()
if args.check and args.workload.startswith("c3"):
    from oracle import oracle as O

    score, digest = O.banded_ref(A, B, 512, 1.0, 2.0, want_digest=True)
    res["h_ok"] = bool(pl.checksum(out) == digest and pl.results()[0]["score"] == int(score))
if args.check and args.workload == "c2":
    from oracle import oracle as O

    o = O.sw(A, B, 1, 0, 1, 1, want_h=True)
    res["h_ok"] = bool(pl.checksum(out) == O.checksum_h(o["H"]) and pl.results()[0]["score"] == o["score"])
print(json.dumps(res), flush=True)
