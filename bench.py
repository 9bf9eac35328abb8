#!/usr/bin/env python3
"""Benchmark of the hot path (BASELINE.json metric: GCUPS, 10k x 10k Smith-Waterman).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c2|c4|c3|c5|ref] [--ref-len L]
                    [--ref-pair a,b]

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI when
launched by torch.distributed.run).  A "step" is one pass of the DP fill over
one batch of input already resident in HBM:

* c2 (default, the BASELINE metric's config): every rank aligns its own
  10,000 x 10,000 pair (rank r: query seq(r+1)[:10000] against the reference
  seq0[:10000], which rank 0 broadcasts once with RCCL), Smith-Waterman, linear
  gap, int32 scores, the full int32 H matrix written to HBM.  Independent
  pairs, no collective inside the step: weak scaling.
* c4: 1024 pairs of 4,000 x 4,000 SW (score only), sharded over ranks
  (shard.ShardedBatch); every step ends with an RCCL all-gather of the scores.
* c3: one 97,403 x 97,403 banded (|i-j| <= 512) reference-Gotoh fill, H written.
* c5: one 20k x 20k affine SW fill writing 1 B/cell traceback bits, then the
  traceback on the device (one wave walks the bits from the end cell): a step
  is fill + traceback.
* ref: the reference's own boundary, main_alignment_function (global Gotoh,
  g=1 h=2, start/end type -1) on seq a x seq b (--ref-pair, default 0,1) at --ref-len (10k default;
  0 = the whole sequences, as the reference's own callers pass them, testing.cpp:261,345):
  a step is the fill writing 1 B/cell direction bytes + find_alignment's walk
  on the device, inputs resident in HBM.  The whole C-ABI call (host buffers
  in, printed text out: PCIe, plan set-up, node list and print_seq included)
  is timed separately and reported as boundary_call_ms, never as the value.

After the timed steps (outside the timed region) the run is checked: the
plan's sticky error word must be 0 (every timed step completed its waits), the
score must equal the CPU oracle's, for c2 the checksum of the whole H matrix
the timed steps wrote must equal the oracle's, for c4 the gathered scores must
equal the committed fixture.  Prints ONE JSON line (rank 0) with value =
whole-job GCUPS, the roofline of the DP kernel (HIP events around that kernel
on its stream, separate pass) and the reference's CPU method timed on this
host (oracle/cpu_rowsweep.cpp, p' = 1 and p' = host cores, bounded sample).
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
# MI355X_MICROARCH.md: 256 CUs x 4 SIMD-32 x 2.4 GHz, a wave64 VALU op issues in 2 cycles per SIMD
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12  # = 78.64 T int32 lane-ops/s
# algorithmic bytes / ops per cell, fixed up front
BYTES_PER_CELL = {"c2": 4.0, "c3": 4.0}
OPS_PER_CELL = {"c4": 8.0, "c5": 12.0, "ref": 13.0}  # ref: T1 add + 2 max, T2 / T3 3 sub + 2 max each


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks); default 1, or WORLD_SIZE when a launcher (torchrun) started this process")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c2", choices=["c2", "c4", "c3", "c5", "ref"])
    ap.add_argument("--ref-len", type=int, default=10000,
                    help="ref workload: prefix length of both sequences (0 = whole sequences)")
    ap.add_argument("--ref-pair", default="0,1", help="ref workload: dataset indices a,b of the pair")
    ap.add_argument("--pairs", type=int, default=0,
                    help="c4: run only the first PAIRS of the 1024 pairs (e.g. 128 = one rank's share at N=8)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-c4-strong", action="store_true",
                    help="c2: skip the same-run C4 strong-scaling sub-record (config.c4_strong)")
    ap.add_argument("--synthetic", action="store_true", help="i.i.d. ACGT (splitmix seed) instead of the dataset")
    return ap.parse_args()


def cpu_baseline(wl: str, A: bytes, B: bytes, cores: int, pairs=None):
    """The reference's CPU method (row sweep, fresh std::threads per row phase, prefix-max
    horizontal gap: oracle/cpu_rowsweep.cpp) on this host, p' = 1 and p' = cores, bounded samples.
    c3: the reference's full tables cannot hold a 97k x 97k pair, so its baseline is
    the banded CPU oracle (oracle/msa_oracle.c orc_banded_ref2, one thread) over the whole band."""
    from oracle import oracle as O

    if wl == "c3":
        t0 = time.perf_counter()
        O.banded_ref(A, B, 512, 1.0, 2.0)
        secs = time.perf_counter() - t0
        cells = sum(min(len(B), i + 512) - max(1, i - 512) + 1 for i in range(1, len(A) + 1))
        return dict(value=round(cells / secs / 1e9, 4), unit="GCUPS", cores=1, kind="port",
                    sample=f"the banded CPU oracle (oracle/msa_oracle.c orc_banded_ref2: the reference's Gotoh "
                           f"recurrence, subproblem_alignment.cpp:396-398, restricted to |i-j| <= 512; -O2, one "
                           f"thread) over the whole {len(A)} x {len(B)} band, {secs:.2f} s; host nproc "
                           f"{os.cpu_count()}",
                    points=[dict(threads=1, rows=len(A), cols=len(B), seconds=round(secs, 3))])

    if wl == "c4" and pairs:
        # the reference's pair-level fan-out (testing.cpp:269-280: one std::thread per pair, each calling
        # main_alignment_function): whole 4,000 x 4,000 pairs, p' = 1 each, `cores` at a time
        from concurrent.futures import ThreadPoolExecutor

        sample = pairs[:8 * cores]
        O.rowsweep(sample[0][:200], B[:200], p=1, mode=1)  # load the library outside the timed region
        t0 = time.perf_counter()
        with ThreadPoolExecutor(max_workers=cores) as ex:  # (ctypes releases the GIL during each call)
            list(ex.map(lambda q: O.rowsweep(q, B, p=1, mode=1, g=1.0, match=1, mismatch=0), sample))
        secs = time.perf_counter() - t0
        cells = sum(len(q) * len(B) for q in sample)
        return dict(value=round(cells / secs / 1e9, 4), unit="GCUPS", cores=cores, kind="port",
                    sample=f"the reference's pair-level fan-out (testing.cpp:269-280, one thread per pair) over "
                           f"the first {len(sample)} of this rank's C4 pairs, whole {len(sample[0])} x {len(B)} "
                           f"pairs, each the reference's row-sweep method at p'=1 (oracle/cpu_rowsweep.cpp, "
                           f"SW-linear int32), {cores} pairs at a time on {cores} threads, {secs:.2f} s; host "
                           f"nproc {os.cpu_count()}, this job's CPU share {cores}",
                    points=[dict(threads=cores, pairs=len(sample), seconds=round(secs, 3))])

    # c3 / c5 / ref (affine gaps): the reference's own Gotoh recurrence; c2 / c4: SW linear int32
    mode = 0 if wl in ("c3", "c5", "ref") else 1
    L = min(len(A), len(B), 10000)
    A, B = A[:L], B[:L]
    pts = []
    # ref: p' = 11 is what the reference's harness runs (main_alignment_function(..., p=32): p' = (p+2)/3)
    for p, rows in ((1, L), ((11 if wl == "ref" else cores), min(L, 1500))):
        _, secs = O.rowsweep(A, B, p=p, mode=mode, g=1.0, h=2.0, match=1, mismatch=0, rows=rows)
        pts.append(dict(threads=p, rows=rows, cols=L, seconds=round(secs, 3), gcups=round(rows * L / secs / 1e9, 4)))
    best = max(pts, key=lambda x: x["gcups"])
    return dict(value=best["gcups"], unit="GCUPS", cores=best["threads"], kind="port",
                sample=f"the reference's CPU method (subproblem_alignment.cpp:251-332 row sweep, prefix-max "
                       f"T2 :13-103, fresh std::threads per phase) restated in oracle/cpu_rowsweep.cpp, "
                       f"{'Gotoh' if mode == 0 else 'SW-linear int32'} recurrence (two-row buffers, -O2: faster "
                       f"than the reference's full double tables at -O0) on the first rows of the same pair; p'=1 and "
                       f"p'={11 if wl == 'ref' else cores} (host nproc {os.cpu_count()}, this job's share "
                       f"{cores}); best shown",
                points=pts)


def _pmc_profile(wl: str, shape: str):
    """The newest committed PMC profile (profiles/<round>_<name>_pmc.json, scripts/pmc_summary.py) of THIS
    workload and shape ("m,n", or "pairs=P" for a c4 rank's share): a profile of another size or another
    rank share is never used for this run's line."""
    for p in sorted((REPO / "profiles").glob("*_pmc.json"), reverse=True):
        try:
            d = json.loads(p.read_text())
        except Exception:
            continue
        if d.get("workload", "").startswith(wl) and d.get("shape") == shape:
            return p.name, d
    return None, None


def load_wave_time(wl: str, shape: str):
    """Where the DP kernel's waves spend their time (parked on s_waitcnt / barriers, issue-stalled,
    issuing VALU / LDS / SALU; fractions of SQ_WAVE_CYCLES), or None."""
    name, d = _pmc_profile(wl, shape)
    return dict(d["wave_time"], source=name) if d and d.get("wave_time") else None


def load_traffic(wl: str, shape: str):
    """Per-launch HBM bytes of the DP kernel (2 x FETCH_SIZE + WRITE_SIZE per the MI355X guide's gfx950
    correction) and the profile it comes from, or (None, None)."""
    name, d = _pmc_profile(wl, shape)
    if d and d.get("hbm_bytes_per_launch"):
        return float(d["hbm_bytes_per_launch"]["total"]), name
    return None, None


def c4_strong(rank: int, world: int, dev, steps: int, warmup: int, syn: bool):
    """The north_star's batch-scaling measurement, taken in the same run as the line's value: C4's fixed
    1,024 pairs of 4k x 4k (score only) split over the job's ranks (the reference's pair-level fan-out,
    testing.cpp:112-158 / :269-280), RCCL all-gather of the scores every step, timed between barriers, max
    over ranks.  Returns the sub-record (rank 0) with GCUPS, ms per step, the all-gather's share and the
    world size RCCL reports; the scores are checked against the committed fixture."""
    import torch
    import torch.distributed as dist

    from cse305_parallel_sequence_alignment_amd import _lib as LB
    from cse305_parallel_sequence_alignment_amd import data
    from cse305_parallel_sequence_alignment_amd.plan import Plan
    from cse305_parallel_sequence_alignment_amd.shard import ShardedBatch, broadcast_reference, gather_scores, \
        shard_range

    total, L = data.C4_PAIRS, data.C4_LEN
    lo, hi = shard_range(total, rank, world)
    qs = data.c4_queries(lo, hi, syn)
    dA = torch.from_numpy(data.encode(b"".join(qs))).to(dev)
    dB = broadcast_reference(torch.from_numpy(data.encode(data.c4_reference(syn))).to(dev))
    plan = Plan(LB.SW_LINEAR, LB.CELLS_NONE, [L] * len(qs), [L] * len(qs), [k * L for k in range(len(qs))],
                [0] * len(qs), match=1, mismatch=0, gap_open=1, gap_extend=1)
    plan.set_timing(False)
    local = torch.empty(len(qs), dtype=torch.int32, device=dev)

    def block(lo_, hi_):
        plan.run(dA, dB)
        plan.scores_into(local)
        return local

    batch = ShardedBatch(total, rank, world, block)
    for _ in range(warmup):
        batch.step()

    def timed(fn, k):
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = None
        for _ in range(k):
            out = fn()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el, out

    el, got = timed(batch.step, steps)
    gel, _ = timed(lambda: gather_scores(local, total, rank, world), steps)
    if plan.error():
        raise SystemExit(f"rank {rank}: c4_strong: a kernel wait hit its spin limit")
    ok = True
    fx = REPO / "tests" / "golden" / "c4_scores.json"
    if not syn and fx.exists():
        ok = [int(x) for x in got.cpu().tolist()] == json.loads(fx.read_text())["scores"][:total]
    okt = torch.tensor([int(ok)], dtype=torch.int32, device=dev)
    if world > 1:
        dist.all_reduce(okt, op=dist.ReduceOp.MIN)
    ms = el / steps * 1e3
    return dict(pairs_total=total, pairs_per_rank=hi - lo, world_size=dist.get_world_size() if world > 1 else 1,
                value=round(total * L * L / (el / steps) / 1e9, 3), unit="GCUPS", ms_per_step=round(ms, 4),
                steps=steps, score_allgather_ms=round(gel / steps * 1e3, 4),
                score_allgather_share=round(gel / el, 4), launch=plan.launch_info()["mode"],
                scores_match_fixture=bool(okt.item()), scaling="strong",
                note="C4's 1,024 pairs split over the ranks, measured in this run after the C2 steps; "
                     "one RCCL all-gather of the scores per step")


def launch_ranks(gpus: int) -> int:
    """``bench.py --gpus N`` started without a launcher: run the same command under torch.distributed.run
    (N ranks, one per GPU) as a CHILD process -- nothing in this process has touched the GPU, and it never
    replaces itself (no exec) -- and return the child's exit code.  Rank 0's JSON line reaches stdout through
    the inherited descriptor."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", str(Path(__file__).resolve())] + sys.argv[1:]
    return subprocess.call(cmd, env=env)


def main():
    args = parse()
    if args.gpus is None:  # `torchrun --nproc-per-node N bench.py` without --gpus: the launcher's world
        args.gpus = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py --gpus {args.gpus} but the launcher started {world} rank(s) (WORLD_SIZE)")
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"RCCL sees {dist.get_world_size()} ranks, --gpus {args.gpus}")
    dev = torch.device("cuda", local)
    from cse305_parallel_sequence_alignment_amd import _lib as LB
    from cse305_parallel_sequence_alignment_amd import data
    from cse305_parallel_sequence_alignment_amd.plan import Plan
    from cse305_parallel_sequence_alignment_amd.shard import ShardedBatch, broadcast_reference

    syn = args.synthetic
    wl = args.workload
    batch = None
    if wl == "c2":
        A, B = data.c2_pair(rank, syn)
        m, n = len(A), len(B)
        pairs_m, pairs_n, a_off, b_off = [m], [n], [0], [0]
        plan_kw = dict(alg=LB.SW_LINEAR, cells=LB.CELLS_H, match=1, mismatch=0, gap_open=1, gap_extend=1)
        cells_per_step = m * n
        desc = "sw-linear 10000x10000, match 1 mismatch 0 gap 1, int32 H written"
    elif wl == "c3":
        A, B = data.c3_pair(syn)
        m, n = len(A), len(B)
        band = 512
        pairs_m, pairs_n, a_off, b_off = [m], [n], [0], [0]
        plan_kw = dict(alg=LB.NW_BANDED, cells=LB.CELLS_H, match=1, mismatch=0, gap_open=3, gap_extend=1, band=band)
        cells_per_step = sum(min(n, i + band) - max(1, i - band) + 1 for i in range(1, m + 1))
        desc = f"banded reference Gotoh {m}x{n}, band 512, g=1 h=2, int32 H written"
    elif wl == "c5":
        A, B = data.c5_pair(rank, syn)
        m, n = len(A), len(B)
        pairs_m, pairs_n, a_off, b_off = [m], [n], [0], [0]
        plan_kw = dict(alg=LB.SW_AFFINE, cells=LB.CELLS_DIR, match=1, mismatch=0, gap_open=3, gap_extend=1,
                       track_end=True)
        cells_per_step = m * n
        desc = ("sw-affine 20000x20000, open 3 extend 1, 1 B/cell traceback bits written + traceback on the "
                "device (ops + begin cell)")
    elif wl == "ref":
        L = args.ref_len
        ia, ib = (int(x) for x in args.ref_pair.split(","))
        A, B = data.bundled()[ia], data.bundled()[ib]
        if L > 0:
            A, B = A[:L], B[:L]
        m, n = len(A), len(B)
        pairs_m, pairs_n, a_off, b_off = [m], [n], [0], [0]
        plan_kw = dict(alg=LB.REF_GOTOH, cells=LB.CELLS_DIR, match=1, mismatch=0, gap_open=3, gap_extend=1,
                       start_type=-1)
        cells_per_step = m * n
        desc = (f"main_alignment_function's path: reference Gotoh {m}x{n} (seq{ia} x seq{ib}{'' if L > 0 else ', whole'}, g=1 h=2, start/end type -1), "
                f"1 B/cell direction bytes + find_alignment's walk on the device")
    else:  # c4
        total = args.pairs if args.pairs > 0 else data.C4_PAIRS
        L = data.C4_LEN
        B = data.c4_reference(syn)
        from cse305_parallel_sequence_alignment_amd.shard import shard_range

        lo, hi = shard_range(total, rank, world)
        qs = data.c4_queries(lo, hi, syn)
        A = b"".join(qs)
        pairs_m = [L] * len(qs)
        pairs_n = [L] * len(qs)
        a_off = [k * L for k in range(len(qs))]
        b_off = [0] * len(qs)
        plan_kw = dict(alg=LB.SW_LINEAR, cells=LB.CELLS_NONE, match=1, mismatch=0, gap_open=1, gap_extend=1)
        cells_per_step = L * L * len(qs)
        desc = f"{total} x (4000x4000) sw-linear score-only, {len(qs)} pairs on this rank"

    dA = torch.from_numpy(data.encode(A)).to(dev)
    dB = torch.from_numpy(data.encode(B)).to(dev)
    broadcast_reference(dB)  # RCCL over xGMI: rank 0's reference sequence to every rank (once)
    plan = Plan(cells=plan_kw.pop("cells"), ms=pairs_m, ns=pairs_n, a_offs=a_off, b_offs=b_off, **plan_kw)
    out = torch.empty(max(plan.cells_elems, 1), dtype=torch.uint8 if plan.cells == LB.CELLS_DIR else torch.int32,
                      device=dev) if plan.cells != LB.CELLS_NONE else None

    if wl == "c4":
        local_scores = torch.empty(len(pairs_m), dtype=torch.int32, device=dev)

        def score_block(lo_, hi_):
            assert (lo_, hi_) == (lo, hi)
            plan.run(dA, dB, out)
            plan.scores_into(local_scores)
            return local_scores

        batch = ShardedBatch(total, rank, world, score_block)

        def step():
            return batch.step()  # fill this rank's pairs, then RCCL all-gather of every rank's scores
    elif wl == "c5":
        tb_ops = torch.empty(m + n + 2, dtype=torch.uint8, device=dev)
        tb_info = torch.zeros(8, dtype=torch.int64, device=dev)

        def step():
            plan.run(dA, dB, out)
            plan.traceback_async(out, tb_ops, tb_info)  # same stream: walks the bits this run wrote
    elif wl == "ref":
        tb_ops = torch.empty(m + n + 2, dtype=torch.uint8, device=dev)
        tb_info = torch.zeros(8, dtype=torch.int64, device=dev)

        def step():
            plan.run(dA, dB, out)
            plan.traceback_gotoh_async(out, tb_ops, tb_info, -1)  # find_alignment's walk, same stream
    else:
        def step():
            plan.run(dA, dB, out)

    plan.set_timing(False)  # no event records inside the timed steps (the kernel_ms pass below re-enables)
    for _ in range(args.warmup):
        step()
    if out is not None:
        # poison the cell output the warm-up wrote (outside the timed region): the checks after the
        # timed steps then prove that those steps rewrote every cell
        out.fill_(0x5A if out.dtype == torch.uint8 else -0x5A5A5A5A)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        gathered = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # ---- checks of what the timed steps produced (outside the timed region) ----
    err = plan.error()
    if err:
        raise SystemExit(f"rank {rank}: a kernel wait hit its spin limit (site {err}) during the timed steps")
    res = plan.results()
    from oracle import oracle as O  # CPU checker

    checks = {}
    dp_launch = None
    gather_ms = None
    if wl == "c2":
        o = O.sw(A, B, 1, 0, 1, 1, want_h=(rank == 0))
        checks["score_matches_cpu"] = bool(o["score"] == res[0]["score"])
        if rank == 0:
            checks["h_matches_cpu"] = bool(plan.checksum(out) == O.checksum_h(o["H"]))
            del o
    elif wl == "c5":
        from cse305_parallel_sequence_alignment_amd.plan import cigar_of

        o = O.sw(A, B, 1, 0, 3, 1, want_tb=(rank == 0))
        checks["score_matches_cpu"] = bool(o["score"] == res[0]["score"] and tuple(o["end"]) == tuple(res[0]["end"]))
        if rank == 0:
            inf = tb_info.cpu().tolist()
            cig = cigar_of(bytes(tb_ops[:inf[0]].cpu().numpy().tobytes()))
            checks["traceback_matches_cpu"] = bool(inf[3] == 0 and cig == o["cigar"] and
                                                   (inf[1], inf[2]) == tuple(o["beg"]))
    elif wl == "c3":
        score, digest = O.banded_ref(A, B, 512, 1.0, 2.0, want_digest=True)
        checks["score_matches_cpu"] = bool(int(score) == res[0]["score"])
        checks["h_matches_cpu"] = bool(plan.checksum(out) == digest)  # every in-band cell the timed steps wrote
        dp_launch = plan.run_info()  # chunked: converged = 1 means the chunk launch produced the cells
    elif wl == "ref":
        import hashlib

        from cse305_parallel_sequence_alignment_amd import api

        inf = tb_info.cpu().tolist()
        # the reference's own outputs at this size (make_golden.py at_size), else the 1 B/cell oracle's
        # whole-sequence fixtures (make_whole.py), else the 1 B/cell oracle itself (bounded)
        fx = [c for c in json.loads((REPO / "tests" / "golden" / "at_size.json").read_text())
              if (c["a"], c["b"], c["L"], c["g"], c["h"]) == (ia, ib, m, 1.0, 2.0) and m == n]
        fxw = [c for c in json.loads((REPO / "tests" / "golden" / "whole.json").read_text())
               if (c["a"], c["b"], c["m"], c["n"]) == (ia, ib, m, n)]
        # the boundary call itself (host buffers in, text out), timed outside the device-resident steps,
        # after one untimed call (its first call in this process fills the device-block pool)
        api.main_alignment_text(b"\0" + A, b"\0" + B, m, n, 32, 1.0, 2.0)
        tb0 = time.perf_counter()
        for _ in range(3):
            text, sc = api.main_alignment_text(b"\0" + A, b"\0" + B, m, n, 32, 1.0, 2.0)
        boundary_ms = (time.perf_counter() - tb0) / 3 * 1e3
        lines = text.split("\n")[5:7]
        checks["walk_status_ok"] = bool(inf[3] == 0 and min(inf[1], inf[2]) == 1)
        if fx:  # the reference's own outputs at this size (make_golden.py at_size)
            checks["score_matches_reference"] = bool(sc == fx[0]["score"] == max(res[0]["fin"]))
            checks["text_matches_reference"] = bool(
                hashlib.md5((lines[0] + "\n" + lines[1] + "\n").encode()).hexdigest() == fx[0]["lines_md5"] and
                len(lines[0]) == fx[0]["n_nodes"] == inf[0])
        elif fxw:
            checks["score_matches_cpu"] = bool(sc == fxw[0]["score"] == max(res[0]["fin"]))
            checks["text_matches_cpu"] = bool(
                hashlib.md5(text.encode("latin-1")).hexdigest() == fxw[0]["text_md5"] and
                len(lines[0]) == fxw[0]["n_nodes"] == inf[0])
        elif m * n <= 2.5e9:
            o = O.main_alignment_text_dir(A, B, 1, 2)
            checks["text_matches_cpu"] = bool(text == o[0])
    else:
        # the score all-gather's share of a step (outside the timed region): the collective alone, on
        # this rank's last scores
        from cse305_parallel_sequence_alignment_amd.shard import gather_scores

        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        g0 = time.perf_counter()
        for _ in range(20):
            gather_scores(local_scores, total, rank, world)
        torch.cuda.synchronize()
        gather_ms = (time.perf_counter() - g0) / 20 * 1e3
        got = [int(x) for x in gathered.cpu().tolist()]
        fx = REPO / "tests" / "golden" / "c4_scores.json"
        if not syn and fx.exists():
            checks["scores_match_fixture"] = got == json.loads(fx.read_text())["scores"][:total]
        checks["score_rank_block_matches_cpu_sample"] = all(
            got[lo + k] == O.sw(qs[k], B, 1, 0, 1, 1)["score"] for k in (0, len(qs) // 2, len(qs) - 1) if qs)
    ok = torch.tensor([int(all(checks.values()))], dtype=torch.int32, device=dev)
    if world > 1:
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)

    # DP-kernel duration from HIP events on the launch stream (separate pass; same plan and buffers)
    kms = []
    plan.set_timing(True)
    for _ in range(max(3, min(args.steps, 10))):
        plan.run(dA, dB, out)
        kms.append(plan.kernel_ms())
    kern_ms = float(np.mean(kms))
    tb_ms = None
    if wl in ("c5", "ref"):  # the device traceback alone (torch events: it runs on torch's current stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            if wl == "c5":
                plan.traceback_async(out, tb_ops, tb_info)
            else:
                plan.traceback_gotoh_async(out, tb_ops, tb_info, -1)
        e1.record()
        torch.cuda.synchronize()
        tb_ms = e0.elapsed_time(e1) / 5
        inf = tb_info.cpu().tolist()
        tb_walk = dict(ops=inf[0], group_switches=inf[4], fetched_on_demand=inf[5], memtime_ticks=inf[6],
                       loader_requests=inf[7])
    if plan.error():
        raise SystemExit(f"rank {rank}: a kernel wait hit its spin limit in the timing pass")

    # the north_star's batch scaling, measured in the same run (C2's value is unchanged by it)
    strong = c4_strong(rank, world, dev, args.steps, args.warmup, syn) if (wl == "c2" and not args.no_c4_strong) \
        else None
    if strong is not None and not strong["scores_match_fixture"]:  # (all-reduced: every rank agrees)
        raise SystemExit(f"rank {rank}: c4_strong: gathered scores differ from tests/golden/c4_scores.json")

    total_cells = cells_per_step * args.steps * world
    gcups = total_cells / elapsed / 1e9
    if rank == 0:
        kern_gcups = cells_per_step / (kern_ms * 1e-3) / 1e9
        shape = f"pairs={len(qs)}" if wl == "c4" else f"{m},{n}"
        traffic, traffic_src = load_traffic(wl, shape)
        if wl in BYTES_PER_CELL:
            achieved = BYTES_PER_CELL[wl] * kern_gcups
            roof = dict(bound="hbm", achieved=round(achieved, 2), peak=HBM_PEAK_GBS, unit="GB/s",
                        frac=round(achieved / HBM_PEAK_GBS, 4), traffic=traffic, traffic_source=traffic_src,
                        note=f"algorithmic bytes = {BYTES_PER_CELL[wl]:.0f} B/cell x {cells_per_step} cells per "
                             f"launch / DP-kernel mean time {kern_ms:.4f} ms (HIP events on the launch stream); "
                             f"traffic = committed PMC HBM bytes per launch. The kernel is bound by the "
                             f"wavefront's dependency chain, not by HBM (DESIGN.md)")
        else:
            achieved = OPS_PER_CELL[wl] * kern_gcups / 1000.0
            roof = dict(bound="valu", achieved=round(achieved, 3), peak=round(VALU_PEAK_TOPS, 2),
                        unit="T int32 lane-ops/s", frac=round(achieved / VALU_PEAK_TOPS, 4),
                        traffic=traffic, traffic_source=traffic_src,
                        note=f"algorithmic ops = {OPS_PER_CELL[wl]:.0f} int32 ops/cell (SURVEY §8(d)) x cells / "
                             f"DP-kernel mean time {kern_ms:.4f} ms; peak = 256 CU x 4 SIMD x 32 lanes x 2.4 GHz")
        roof["pmc_wave_time"] = load_wave_time(wl, shape)
        cpu = None
        if not args.no_cpu_baseline:
            try:
                # the job's CPU share: 16 host threads per GPU on this pool (the box's nproc counts the whole
                # machine); the line states both
                cpu = cpu_baseline(wl, A[:data.C4_LEN] if wl == "c4" else A, B, min(16, os.cpu_count() or 1),
                                   pairs=qs if wl == "c4" else None)
            except Exception as e:  # pragma: no cover
                cpu = dict(value=None, unit="GCUPS", cores=1, kind="port", sample=f"failed: {e}")
        line = {
            "metric": "GCUPS (DP cell updates/s) + max-score match vs CPU, 10k×10k SW",
            "value": round(gcups, 3),
            "unit": "GCUPS",
            "n_gpus": dist.get_world_size() if world > 1 else 1,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if wl == "c4" else "weak",  # c4: a fixed 1024-pair batch split over ranks
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic i.i.d. ACGT" if syn else "gene_sequences_test (reference's bundled FASTA)",
            "config": dict(workload=wl + ": " + desc, cells_per_step_per_gpu=int(cells_per_step),
                           parallelism=(f"dp{world} (pairs sharded over GPUs; RCCL bcast of the reference, "
                                        f"all-gather of scores every step)" if wl == "c4" else
                                        f"dp{world} (one independent pair per GPU; RCCL bcast of the reference "
                                        f"once; no collective in the step)"),
                           score_rank0=int(res[0]["score"]), checks_all_ranks=bool(ok.item()), **checks,
                           kernel_errors=0, dp_kernel_ms=round(kern_ms, 4),
                           **({"traceback_ms": round(tb_ms, 4), "traceback_walk": tb_walk} if tb_ms is not None
                              else {}),
                           **({"dp_launch": dp_launch} if dp_launch is not None else {}),
                           **({"c4_strong": strong} if strong is not None else {}),
                           **({"score_allgather_ms": round(gather_ms, 4),
                               "score_allgather_share": round(gather_ms / (elapsed / args.steps * 1e3), 4)}
                              if gather_ms is not None else {}),
                           **({"boundary_call_ms": round(boundary_ms, 3),
                               "boundary_note": "msa_main_alignment with host buffers (plan set-up, H2D codes, fill, "
                                                "device walk, D2H ops, node list, print_seq text): PCIe-inclusive, "
                                                "not the value"} if wl == "ref" else {})),
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if not bool(ok.item()):
        raise SystemExit(f"rank {rank}: result check failed: {checks}")


if __name__ == "__main__":
    main()
