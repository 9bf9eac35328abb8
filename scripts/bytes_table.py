#!/usr/bin/env python3
"""Per-buffer HBM-side byte attribution of a flow-kernel workload (ref 10k, C5 20k) from
scripts/prof_bytes.sh runs on the production library and on MSA_ABL ablation builds (msa_flow.hip:
1 = no pass-2 work, 2 = no SNAP stores, 4 = no bottom-row (BR) stores), against the buffer sizes the
plan allocates.  Prints one JSON object (and writes profiles/<round>_<wl>_bytes.json):

    python scripts/bytes_table.py gpurun_out/pb2 r05 ref c5     (runs gpurun_out/pb2_<wl>_<variant>)
"""
import csv
import json
import sys
from pathlib import Path

prefix, rnd = sys.argv[1], sys.argv[2]
wls = sys.argv[3:] or ["ref", "c5"]
ROOT = Path(__file__).resolve().parent.parent


def flow_bytes(d: Path):
    """Mean FETCH_SIZE (doubled: gfx950 reports half of wide coalesced reads) and WRITE_SIZE (KB -> bytes)
    per dispatch of the longest flow kernel in the run, and its mean duration."""
    out = {}
    trace = d / "trace" / "run_kernel_trace.csv"
    dur = {}
    if trace.exists():
        for r in csv.DictReader(open(trace)):
            if "flow_kernel" in r["Kernel_Name"] or "flow_fill" in r["Kernel_Name"]:
                dur.setdefault(r["Kernel_Name"], []).append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
    for sub, name, scale in (("pmc_fetch", "FETCH_SIZE", 2.0), ("pmc_write", "WRITE_SIZE", 1.0),
                             ("pmc_sq", "SQ_INSTS_VALU", 1.0 / 1024.0), ("pmc_sq", "SQ_INSTS_SALU", 1.0 / 1024.0),
                             ("pmc_sq", "SQ_INSTS_LDS", 1.0 / 1024.0), ("pmc_sq", "SQ_WAVES", 1.0 / 1024.0)):
        f = d / sub / "run_counter_collection.csv"
        if not f.exists():
            continue
        acc = {}
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != name or "flow" not in r["Kernel_Name"]:
                continue
            acc.setdefault(r["Kernel_Name"], {}).setdefault(r["Dispatch_Id"], 0.0)
            acc[r["Kernel_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
        out[name] = {k: scale * 1024.0 * sum(v.values()) / len(v) for k, v in acc.items()}
    out["dur_us"] = {k: sum(v) / len(v) / 1e3 for k, v in dur.items()}
    return out


def sizes(wl: str):
    """Bytes of the buffers a flow plan (R = 2, two values per link column) writes per run."""
    m = n = 10000 if wl == "ref" else 20000
    R = 2
    S = (m + 64 * R - 1) // (64 * R)
    P = (n + 15 + 63) // 16 + 1  # fl_P of a full stripe, 16-step phases
    plane = S * P * 16 * 64 * R  # 1 B per cell of the R = 2 layout
    brw = 16 * P + 16
    br = 2 * S * brw * 8
    nseg = (P + 7) // 8
    snap = S * nseg * 128 * (R + 1) * 8
    items = (S + 3) // 4
    gran = (items - 1) * 2 * (n + 2 * 128 + 16) * 8
    return dict(plane=plane, br=br, snap=snap, granules=gran, cells=m * n)


res = {}
for wl in wls:
    runs = {v: flow_bytes(Path(f"{prefix}_{wl}_{v}")) for v in ("prod", "abl1", "abl2", "abl4", "abl8")
            if Path(f"{prefix}_{wl}_{v}", "pmc_write").exists()}
    sz = sizes(wl)

    def tot(v, key):
        return sum(runs[v].get(key, {}).values())

    w = {v: tot(v, "WRITE_SIZE") for v in runs}
    f = {v: tot(v, "FETCH_SIZE") for v in runs}
    res[wl] = dict(
        buffers_bytes=sz,
        writes_counted=w, fetches_counted=f,
        # prod - abl1 = pass 2's bytes; prod - abl8 = pass 2's cell stores alone; abl1 = pass 1's (BR, SNAP, granules)
        write_attributed={k: w["prod"] - w[v] for k, v in (("pass2", "abl1"), ("snap", "abl2"), ("br", "abl4"),
                                                           ("pass2_cells", "abl8")) if v in w},
        fetch_attributed={k: f["prod"] - f[v] for k, v in (("pass2", "abl1"), ("snap", "abl2"), ("br", "abl4"),
                                                           ("pass2_cells", "abl8")) if v in f},
        pass1_writes_vs_buffers=(w["abl1"] / (sz["br"] + sz["snap"] + sz["granules"])) if "abl1" in w else None,
        pass2_writes_vs_plane=((w["prod"] - w["abl1"]) / sz["plane"]) if "abl1" in w else None,
        traffic_vs_plane=(w["prod"] + f["prod"]) / sz["plane"],
        dur_us={v: runs[v].get("dur_us") for v in runs},
        # wave instructions per launch; x 64 lanes / cells = lane-ops per cell (pass 2 = prod - abl1)
        valu_lane_ops_per_cell={v: 64.0 * tot(v, "SQ_INSTS_VALU") / sz["cells"] for v in runs},
        salu_wave_instrs_per_64_cells={v: 64.0 * tot(v, "SQ_INSTS_SALU") / sz["cells"] for v in runs},
        lds_wave_instrs_per_64_cells={v: 64.0 * tot(v, "SQ_INSTS_LDS") / sz["cells"] for v in runs})
(ROOT / "profiles").mkdir(exist_ok=True)
for wl, r in res.items():
    (ROOT / "profiles" / f"{rnd}_{wl}_bytes.json").write_text(json.dumps(r, indent=1))
print(json.dumps(res, indent=1))
