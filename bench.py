#!/usr/bin/env python3
"""Benchmark of the hot path (BASELINE.json metric: GCUPS, 10k x 10k Smith-Waterman).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c2|c4|c3|c5]

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI when
launched by torch.distributed.run).  A "step" is one pass of the DP fill over
one batch of input already resident in HBM:

* c2 (default, the BASELINE metric's config): every rank aligns its own
  10,000 x 10,000 pair (rank r: query seq(r+1)[:10000] vs the reference
  seq0[:10000] that rank 0 broadcasts once with RCCL), Smith-Waterman, linear
  gap, int32 scores, the full int32 H matrix written to HBM; the step ends
  with an RCCL all-gather of the per-rank scores.  Weak scaling.
* c4: 1024 pairs of 4,000 x 4,000 SW (score only), sharded over ranks.
* c3: one 100k x 100k banded (|i-j| <= 512) reference-Gotoh fill, H written.
* c5: one 20k x 20k affine SW fill writing 1 B/cell traceback bits.

Prints ONE JSON line (rank 0) with value = whole-job GCUPS, the roofline of
the stripe kernel (HIP events around that kernel on its own stream) and the
reference CPU path timed on this host (bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E peak 8.0 TB/s (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c2", choices=["c2", "c4", "c3", "c5"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--synthetic", action="store_true", help="i.i.d. ACGT (splitmix seed) instead of the dataset")
    return ap.parse_args()


def dataset():
    from oracle.oracle import load_dataset  # plain FASTA reader of the committed data file

    return load_dataset()[1]


def encode(s: bytes) -> np.ndarray:
    return np.frombuffer(s.translate(bytes.maketrans(b"ACGT", b"\x00\x01\x02\x03")), dtype=np.uint8).copy()


def synth(n: int, seed: int) -> bytes:
    rng = np.random.default_rng(seed)
    return rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), n).tobytes()


def cpu_baseline(workload: str, A: bytes, B: bytes):
    """The reference's own CPU fill (oracle/_ref, compiled from its sources) on a
    bounded sample of the workload; the C restatement if _ref is absent."""
    from oracle import oracle as O

    if O.ref_available():
        L = min(len(A), len(B), 10000)
        r = O.ref_subproblem(A[:L], B[:L], -1, -1, 1.0, 2.0, p=1, tables=False, traceback=False)
        secs = r["fill_seconds"]
        return dict(value=round(L * L / secs / 1e9, 4), unit="GCUPS", cores=1, kind="reference",
                    sample=f"Subproblem::compute_tables (subproblem_alignment.cpp:329) p'=1 on {L}x{L} "
                           f"of the same pair, reference sources built -O2 by oracle/Makefile; "
                           f"{secs:.2f} s fill (table allocation excluded)")
    L = min(len(A), len(B), 6000)
    t0 = time.perf_counter()
    O.sw(A[:L], B[:L], 1, 0, 1, 1)
    secs = time.perf_counter() - t0
    return dict(value=round(L * L / secs / 1e9, 4), unit="GCUPS", cores=1, kind="port",
                sample=f"oracle orc_sw (C restatement) {L}x{L}, {secs:.2f} s")


def load_traffic(workload: str):
    """Per-launch HBM bytes of the stripe kernel from the committed PMC profile
    (profiles/<round>_<workload>_pmc.json written by scripts/pmc_summary.py:
    2 x FETCH_SIZE + WRITE_SIZE, per the MI355X guide's gfx950 correction), or None."""
    for p in sorted((REPO / "profiles").glob("*_pmc.json"), reverse=True):
        try:
            d = json.loads(p.read_text())
        except Exception:
            continue
        if d.get("workload") == workload and d.get("hbm_bytes_per_launch"):
            return float(d["hbm_bytes_per_launch"]["total"])
    return None


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    from cse305_parallel_sequence_alignment_amd import _lib as LB
    from cse305_parallel_sequence_alignment_amd.plan import Plan

    seqs = None if args.synthetic else dataset()

    def seq(k, L, salt):
        if seqs is None:
            return synth(L, 0x5EED0000 + salt * 1000 + k)
        s = seqs[k % len(seqs)]
        return s[:L]

    wl = args.workload
    if wl == "c2":
        m = n = 10000
        B = seq(0, n, 1)  # the reference sequence (rank 0 owns it, bcast)
        A = seq(1 + rank, m, 1)
        pairs_m, pairs_n, a_off, b_off = [m], [n], [0], [0]
        plan_kw = dict(alg=LB.SW_LINEAR, cells=LB.CELLS_H, match=1, mismatch=0, gap_open=1, gap_extend=1)
        cells_per_step = m * n
        algo_bytes_per_cell = 4.0  # int32 H written once
        desc = "sw-linear 10000x10000, match 1 mismatch 0 gap 1, int32 H written"
        dtype = "int32"
    elif wl == "c3":
        m = n = 100000
        B = seq(0, n, 3) if seqs is None else (seqs[3][:97403] + seqs[4][:2597])[:n]
        A = seq(1 + rank, m, 3) if seqs is None else (seqs[4][:97403] + seqs[3][:2597])[:m]
        m, n = len(A), len(B)
        pairs_m, pairs_n, a_off, b_off = [m], [n], [0], [0]
        band = 512
        plan_kw = dict(alg=LB.NW_BANDED, cells=LB.CELLS_H, match=1, mismatch=0, gap_open=3, gap_extend=1, band=band)
        cells_per_step = sum(min(n, i + band) - max(1, i - band) + 1 for i in range(1, m + 1))
        algo_bytes_per_cell = 4.0
        desc = f"banded reference Gotoh {m}x{n}, band 512, g=1 h=2, int32 H written"
        dtype = "int32"
    elif wl == "c5":
        m = n = 20000
        B = seq(0, n, 5)
        A = seq(1 + rank, m, 5)
        pairs_m, pairs_n, a_off, b_off = [m], [n], [0], [0]
        plan_kw = dict(alg=LB.SW_AFFINE, cells=LB.CELLS_DIR, match=1, mismatch=0, gap_open=3, gap_extend=1,
                       track_end=True)
        cells_per_step = m * n
        algo_bytes_per_cell = 1.0
        desc = "sw-affine 20000x20000, open 3 extend 1, 1 B/cell traceback bits written"
        dtype = "int32"
    else:  # c4
        L = 4000
        total_pairs = 1024
        per = (total_pairs + world - 1) // world
        lo, hi = rank * per, min(total_pairs, (rank + 1) * per)
        B = seq(0, L, 4)
        rng = np.random.default_rng(0x5EED0004)
        offs = rng.integers(0, 13309 - L, size=total_pairs)
        qs = [(seqs[k % 20][offs[k]:offs[k] + L] if seqs is not None else synth(L, 0x5EED0004 + k)) for k in
              range(lo, hi)]
        A = b"".join(qs)
        pairs_m = [L] * len(qs)
        pairs_n = [L] * len(qs)
        a_off = [k * L for k in range(len(qs))]
        b_off = [0] * len(qs)
        plan_kw = dict(alg=LB.SW_LINEAR, cells=LB.CELLS_NONE, match=1, mismatch=0, gap_open=1, gap_extend=1)
        cells_per_step = L * L * len(qs)
        algo_bytes_per_cell = 0.0
        desc = f"{total_pairs} x (4000x4000) sw-linear score-only, shard {len(qs)} pairs/rank"
        dtype = "int32"

    dA = torch.from_numpy(encode(A)).to(dev)
    dB = torch.from_numpy(encode(B)).to(dev)
    if world > 1:
        dist.broadcast(dB, src=0)  # RCCL: the shared reference sequence
    plan = Plan(cells=plan_kw.pop("cells"), ms=pairs_m, ns=pairs_n, a_offs=a_off, b_offs=b_off, **plan_kw)
    out = torch.empty(max(plan.cells_elems, 1), dtype=torch.uint8 if plan.cells == LB.CELLS_DIR else torch.int32,
                      device=dev) if plan.cells != LB.CELLS_NONE else None
    score_buf = torch.zeros(1, dtype=torch.int64, device=dev)
    gathered = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]

    def step():
        plan.run(dA, dB, out)
        if world > 1:
            # scores of every rank -> every rank (tiny RCCL all-gather over xGMI)
            dist.all_gather(gathered, score_buf)

    plan.set_timing(False)  # no event records inside the timed steps (kernel_ms pass below re-enables)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    res = plan.results()
    # stripe-kernel duration from HIP events on the launch stream (separate pass)
    kms = []
    plan.set_timing(True)
    for _ in range(max(3, min(args.steps, 10))):
        plan.run(dA, dB, out)
        kms.append(plan.kernel_ms())
    kern_ms = float(np.mean(kms))

    total_cells = cells_per_step * args.steps * world
    gcups = total_cells / elapsed / 1e9
    if rank == 0:
        achieved = algo_bytes_per_cell * cells_per_step / (kern_ms * 1e-3) / 1e9
        traffic = load_traffic(wl)
        roof = dict(bound="hbm", achieved=round(achieved, 2), peak=HBM_PEAK_GBS, unit="GB/s",
                    frac=round(achieved / HBM_PEAK_GBS, 4), traffic=traffic,
                    note="algorithmic bytes = %.0f B/cell x cells / DP-kernel time (flow_kernel for C2); bound by the "
                         "per-wave DP dependency chain of the anti-diagonal wavefront, not by HBM (DESIGN.md)"
                         % algo_bytes_per_cell)
        cpu = None
        if not args.no_cpu_baseline:
            try:
                cpu = cpu_baseline(wl, A[:m] if wl != "c4" else A[:4000], B)
            except Exception as e:  # pragma: no cover
                cpu = dict(value=None, unit="GCUPS", cores=1, kind="reference", sample=f"failed: {e}")
        score_ok = None
        if wl == "c2":
            from oracle import oracle as O  # CPU checker for the max score
            score_ok = bool(O.sw(A, B, 1, 0, 1, 1)["score"] == res[0]["score"])
        line = {
            "metric": "GCUPS (DP cell updates/s) + max-score match vs CPU, 10k×10k SW",
            "value": round(gcups, 3),
            "unit": "GCUPS",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": dtype,
            "data": "synthetic i.i.d. ACGT" if seqs is None else "gene_sequences_test (reference's bundled FASTA)",
            "config": {"workload": wl + ": " + desc, "cells_per_step_per_gpu": int(cells_per_step),
                       "parallelism": f"dp{world} (one pair per GPU; RCCL bcast of the reference + all-gather)"
                       if wl != "c4" else f"dp{world} (pairs sharded over GPUs)",
                       "score_rank0": int(res[0]["score"]), "score_matches_cpu": score_ok,
                       "stripe_kernel_ms": round(kern_ms, 4)},
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
