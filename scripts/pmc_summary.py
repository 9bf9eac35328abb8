"""Summarise a scripts/prof.sh output directory into profiles/ (committed evidence).

    python scripts/pmc_summary.py gpurun_out/prof_c2 c2 r01 [shape]

Writes profiles/<round>_<wl>_kernel_stats.csv (rocprofv3 --stats summary),
profiles/<round>_<wl>_pmc.json: per-launch averages of the SQ counters of the
stripe kernel and its HBM traffic: FETCH_SIZE (doubled: on gfx950 it reports
half the bytes of wide coalesced reads, MI355X_MICROARCH.md "HBM") + WRITE_SIZE,
both in KB as rocprofv3 reports them, converted to bytes per launch.
"""
import csv
import json
import shutil
import sys
from collections import defaultdict
from pathlib import Path

src, wl, rnd = Path(sys.argv[1]), sys.argv[2], sys.argv[3]
# the DP kernel of the workload: flow_kernel (single-pair SW linear, pass 1 + pass-2
# blocks in one launch) or stripe_kernel (everything else)
KERNELS = ("flow_kernel", "stripe_kernel", "band_kernel", "cflow_kernel")
dst = Path(__file__).resolve().parent.parent / "profiles"
dst.mkdir(exist_ok=True)


# the DP kernel = the matching kernel with the largest total time in the trace (a chunked
# banded run also launches the exact fallback, which exits at once)
MAIN = None
_stats = src / "trace" / "run_kernel_stats.csv"
if _stats.exists():
    best = -1.0
    for r in csv.DictReader(open(_stats)):
        if any(k in r["Name"] for k in KERNELS) and float(r["TotalDurationNs"]) > best:
            best, MAIN = float(r["TotalDurationNs"]), r["Name"]


def _is_main(name):
    return name == MAIN if MAIN else any(k in name for k in KERNELS)


# Dispatches of the DP kernel are selected by DURATION, not by name alone: a chunked banded run also
# launches the exact fallback instance of the same kernel, which exits at once (C3: min 4 us, max
# 400 us).  Kept: dispatches lasting at least half the longest one of the same run.
KEEP_FRAC = 0.5
selection = {}


def _keep(durs):
    top = max(durs.values()) if durs else 0
    return {d for d, t in durs.items() if t >= KEEP_FRAC * top}


def per_dispatch(sub, match=None):
    f = src / sub / "run_counter_collection.csv"
    if not f.exists():
        return {}
    match = match or _is_main
    acc = defaultdict(lambda: defaultdict(float))
    durs = {}
    for r in csv.DictReader(open(f)):
        if not match(r["Kernel_Name"]):
            continue
        acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
        if "Start_Timestamp" in r and r["Start_Timestamp"]:
            durs[r["Dispatch_Id"]] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    keep = _keep(durs) if durs else None
    if match is _is_main:
        selection[sub] = dict(dispatches=len(durs) or None, kept=len(keep) if keep is not None else None)
    out = {}
    for k, v in acc.items():
        vals = [x for d, x in v.items() if keep is None or d in keep]
        out[k] = sum(vals) / len(vals) if vals else 0.0
    return out


out = {"workload": wl, "round": rnd, "kernel": MAIN or "/".join(KERNELS), "per_launch": {}}


def shape_of(name):
    """The shape bench.py keys PMC profiles on ("m,n", or "pairs=P" for a c4 rank share), for the
    scripts/prof_run.py workloads."""
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
    from cse305_parallel_sequence_alignment_amd import data

    s = data.bundled()
    if name.startswith("c4"):
        return "pairs=128" if name == "c4_128" else "pairs=1024"
    pair = {"c2": lambda: data.c2_pair(0), "c3": lambda: data.c3_pair(False), "c5": lambda: data.c5_pair(0, False),
            "ref": lambda: (s[0][:10000], s[1][:10000]), "ref20": lambda: (s[0][:20000], s[1][:20000]),
            "refwhole": lambda: (s[3], s[4])}.get(name)
    if pair is None:
        return None
    A, B = pair()
    return f"{len(A)},{len(B)}"


# the workload's shape (bench.load_traffic matches on it)
out["shape"] = sys.argv[4] if len(sys.argv) > 4 else shape_of(wl)
for sub in ("pmc1", "pmc2", "pmc_fetch", "pmc_write"):
    out["per_launch"].update(per_dispatch(sub))
out["dispatch_selection"] = dict(rule=f"dispatches of the DP kernel lasting >= {KEEP_FRAC} x the longest", **selection)
pl = out["per_launch"]
if "FETCH_SIZE" in pl or "WRITE_SIZE" in pl:
    fetch = 2.0 * pl.get("FETCH_SIZE", 0.0) * 1024.0
    write = pl.get("WRITE_SIZE", 0.0) * 1024.0
    out["hbm_bytes_per_launch"] = {"fetch_corrected": fetch, "write": write, "total": fetch + write}
    # a long pair's pass 2 is a launch of its own (flow_fill_kernel) inside the same timed DP region:
    # its bytes belong to the same per-run traffic
    fill = {}
    for sub in ("pmc_fetch", "pmc_write"):
        fill.update(per_dispatch(sub, lambda name: "flow_fill_kernel" in name))
    if fill:
        ff, fw = 2.0 * fill.get("FETCH_SIZE", 0.0) * 1024.0, fill.get("WRITE_SIZE", 0.0) * 1024.0
        h = out["hbm_bytes_per_launch"]
        h.update(fill_fetch_corrected=ff, fill_write=fw, dp_kernel_only_total=h["total"], total=h["total"] + ff + fw)
# where the DP kernel's waves spend their time (SQ counters summed over waves; WAIT_ANY +
# WAIT_INST_ANY + ACTIVE_INST_ANY ~= WAVE_CYCLES, MI355X_MICROARCH.md "rocprofv3 PMC slots"):
# parked on s_waitcnt / s_barrier, stalled at issue, issuing VALU, issuing LDS
wc = pl.get("SQ_WAVE_CYCLES", 0.0)
if wc > 0:
    out["wave_time"] = {
        "parked_waitcnt_or_barrier": round(pl.get("SQ_WAIT_ANY", 0.0) / wc, 4),
        "issue_stall": round(pl.get("SQ_WAIT_INST_ANY", 0.0) / wc, 4),
        "valu_active": round(pl.get("SQ_ACTIVE_INST_VALU", 0.0) / wc, 4),
        "lds_active": round(pl.get("SQ_ACTIVE_INST_LDS", 0.0) / wc, 4),
        "salu_active": round(pl.get("SQ_ACTIVE_INST_SCA", 0.0) / wc, 4),
    }
stats = src / "trace" / "run_kernel_stats.csv"
if stats.exists():
    shutil.copy(stats, dst / f"{rnd}_{wl}_kernel_stats.csv")
    for r in csv.DictReader(open(stats)):
        if _is_main(r["Name"]):
            out["trace_avg_ns_all_calls"] = float(r["AverageNs"])
            out["trace_calls"] = int(r["Calls"])
trace = src / "trace" / "run_kernel_trace.csv"
if trace.exists():
    durs = {r["Dispatch_Id"]: float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
            for r in csv.DictReader(open(trace)) if _is_main(r["Kernel_Name"])}
    keep = _keep(durs)
    if keep:
        out["trace_avg_ns"] = sum(durs[d] for d in keep) / len(keep)
        out["trace_kept_calls"] = len(keep)
(dst / f"{rnd}_{wl}_pmc.json").write_text(json.dumps(out, indent=1))
print(json.dumps(out, indent=1))
