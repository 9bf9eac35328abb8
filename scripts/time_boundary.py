#!/usr/bin/env python3
"""Diagnostic: where a main_alignment_function boundary call's time goes at 10k (steady state):
the whole call (msa_main_alignment), a plan create + destroy, and the device work (fill + walk)
of a resident plan.  Prints one JSON line."""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch

from cse305_parallel_sequence_alignment_amd import _lib as LB, api, data
from cse305_parallel_sequence_alignment_amd.plan import Plan

L = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
A, B = data.bundled()[0][:L], data.bundled()[1][:L]
m, n = len(A), len(B)


def best(fn, reps=10):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(min(ts) * 1e3, 4), round(sorted(ts)[len(ts) // 2] * 1e3, 4)


out = {}
out["boundary_call_ms"] = best(lambda: api.main_alignment_text(b"\0" + A, b"\0" + B, m, n, 32, 1.0, 2.0))


def mk():
    p = Plan(LB.REF_GOTOH, LB.CELLS_DIR, [m], [n], [0], [0], match=1, mismatch=0, gap_open=3, gap_extend=1,
             start_type=-1)
    p.close() if hasattr(p, "close") else None
    del p


out["plan_create_destroy_ms"] = best(mk)
pl = Plan(LB.REF_GOTOH, LB.CELLS_DIR, [m], [n], [0], [0], match=1, mismatch=0, gap_open=3, gap_extend=1,
          start_type=-1)
dA = torch.from_numpy(data.encode(A)).cuda()
dB = torch.from_numpy(data.encode(B)).cuda()
D = torch.empty(pl.cells_elems, dtype=torch.uint8, device="cuda")
ops = torch.empty(m + n + 2, dtype=torch.uint8, device="cuda")
info = torch.zeros(8, dtype=torch.int64, device="cuda")


def dev():
    pl.run(dA, dB, D)
    pl.traceback_gotoh_async(D, ops, info, -1)
    torch.cuda.synchronize()


out["device_fill_walk_ms"] = best(dev)


def dev_res():
    pl.run(dA, dB, D)
    pl.traceback_gotoh_async(D, ops, info, -1)
    pl.results()
    k = int(info[0].item())
    ops[:k].cpu()


out["device_fill_walk_results_ops_ms"] = best(dev_res)
print(json.dumps(out), flush=True)
