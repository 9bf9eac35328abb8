#!/usr/bin/env python3
"""Diagnostic (needs a -DMSA_TB_STATS build of libmsa.so): where the device walk's time goes, for
the C5 (SW affine) and ref (Gotoh, 10k) walks.  In that build the walk's info words are
{ops, begin i, begin j, status, ticks waiting for the loader, diagonal runs, windows, ticks inside groups, walk
total, groups staged on demand, ticks in diagonal runs, decoder busy ticks, stripes entered, loader requests, loader
ticks issuing, loader ticks waiting, sum of issue-to-publish ticks, groups staged};
the walk's total comes from HIP events around it.

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
ap.add_argument("--workload", default="c5", choices=["c5", "ref", "refwhole"])
ap.add_argument("--trace", default="", help="save the event traces (.npz)")
args = ap.parse_args()
if args.workload == "c5":
    A, B = data.c5_pair(0)
    pl = Plan(LB.SW_AFFINE, LB.CELLS_DIR, [len(A)], [len(B)], [0], [0], match=1, mismatch=0, gap_open=3,
              gap_extend=1, track_end=True)
else:
    A, B = data.bundled()[0], data.bundled()[1]
    if args.workload == "ref":
        A, B = A[:10000], B[:10000]
    pl = Plan(LB.REF_GOTOH, LB.CELLS_DIR, [len(A)], [len(B)], [0], [0], match=1, mismatch=0, gap_open=3,
              gap_extend=1, start_type=-1)
dA = torch.from_numpy(data.encode(A)).cuda()
dB = torch.from_numpy(data.encode(B)).cuda()
out = torch.empty(pl.cells_elems, dtype=torch.uint8, device="cuda")
ops = torch.empty(len(A) + len(B) + 16, dtype=torch.uint8, device="cuda")
info = torch.zeros(32 + 2 * 16384, dtype=torch.int64, device="cuda")
pl.run(dA, dB, out)
rows, ms = [], []
for rep in range(4):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    if args.workload == "c5":
        pl.traceback_async(out, ops, info)
    else:
        pl.traceback_gotoh_async(out, ops, info, -1)
    e1.record()
    torch.cuda.synchronize()
    rows.append(info.cpu().tolist() if rep == 3 else info[:32].cpu().tolist())
    ms.append(e0.elapsed_time(e1))
k = rows[-1]
if args.trace:
    # event traces of the last walk: walker group lookups {t << 32 | s, asked, ready word seen, got},
    # loader groups {b0 << 32 | s, issue start, issue end, published}
    import numpy as np
    tr = np.array(k[32:32 + 16384], dtype=np.int64).reshape(-1, 4)
    lg = np.array(k[32 + 16384:], dtype=np.int64).reshape(-1, 4)
    np.savez(args.trace, walker=tr[:min(k[12] + k[13] + 64, 4096)], loader=lg[:min(k[17], 4096)])
assert k[3] == 0, f"walk status {k[3]}"
print(json.dumps(dict(workload=args.workload, ops=k[0], t_total=k[8], t_wait=k[4], t_in_groups=k[7],
                      t_runs=k[10], t_decoder=k[11], n_run=k[5], n_win=k[6], n_switch=k[12], n_demand=k[9],
                      n_req=k[13], ld_issue=k[14], ld_wait=k[15], ld_issue_to_publish=k[16], ld_groups=k[17], ld_paths=k[18:22], ld_path_ticks=k[22:26], ld_sel_ticks=k[26], ld_sels=k[27],
                      walk_ms=[round(x, 4) for x in ms])), flush=True)
