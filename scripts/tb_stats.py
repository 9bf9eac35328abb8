#!/usr/bin/env python3
"""Diagnostic (needs a -DMSA_TB_STATS build of libmsa.so): where the device walk's time goes, for
the C5 (SW affine) and ref (Gotoh, 10k) walks.  In that build the walk's info words are
{ops, -, ticks prefetching, diagonal runs, ticks waiting for group loads, windows, ticks total,
ticks inside groups}.

    python3 scripts/tb_stats.py --workload c5
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
ap.add_argument("--workload", default="c5", choices=["c5", "ref"])
args = ap.parse_args()
if args.workload == "c5":
    A, B = data.c5_pair(0)
    pl = Plan(LB.SW_AFFINE, LB.CELLS_DIR, [len(A)], [len(B)], [0], [0], match=1, mismatch=0, gap_open=3,
              gap_extend=1, track_end=True)
else:
    A, B = data.bundled()[0][:10000], data.bundled()[1][:10000]
    pl = Plan(LB.REF_GOTOH, LB.CELLS_DIR, [len(A)], [len(B)], [0], [0], match=1, mismatch=0, gap_open=3,
              gap_extend=1, start_type=-1)
dA = torch.from_numpy(data.encode(A)).cuda()
dB = torch.from_numpy(data.encode(B)).cuda()
out = torch.empty(pl.cells_elems, dtype=torch.uint8, device="cuda")
ops = torch.empty(len(A) + len(B) + 16, dtype=torch.uint8, device="cuda")
info = torch.zeros(8, dtype=torch.int64, device="cuda")
pl.run(dA, dB, out)
rows = []
for rep in range(4):
    if args.workload == "c5":
        pl.traceback_async(out, ops, info)
    else:
        pl.traceback_gotoh_async(out, ops, info, -1)
    torch.cuda.synchronize()
    rows.append(info.cpu().tolist())
k = rows[-1]
print(json.dumps(dict(workload=args.workload, ops=k[0], t_prefetch=k[2], n_run=k[3], t_wait=k[4], n_win=k[5],
                      t_total=k[6], t_in_groups=k[7], t_other=k[6] - k[7] - k[2] - k[4],
                      totals=[r[6] for r in rows])), flush=True)
