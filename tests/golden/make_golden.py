"""Generate the golden fixtures from the REFERENCE'S OWN CODE.

Runs only in the build container, where oracle/_ref/ holds the reference's
unmodified subproblem_alignment.cpp / partial.cpp compiled by oracle/Makefile.
The fixtures written here are data (inputs + expected outputs) and are
committed; the GPU box never needs /root/reference.

    python tests/golden/make_golden.py            # small fixtures
    python tests/golden/make_golden.py at_size    # 10k / 20k fixtures (at_size.json)

Outputs (tests/golden/):
  kat.json             known-answer tests + harness-pair outputs
  subproblem_tables.npz  full T1/T2/T3 for small random pairs, every start/end type
  subproblem_paths.json  find_alignment node lists for the same + dataset prefixes
  partial.json         findPartialBalancedPartitionParallel partitions (wrap semantics)
  at_size.json         scores / node lists / H digests at 10k and 20k (reference p'=1)
"""
from __future__ import annotations

import hashlib
import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent.parent))
from oracle import oracle as O  # noqa: E402

GH = [(1.0, 2.0), (1.0, 0.0), (2.0, 1.0), (3.0, 5.0)]
TYPES = [-1, -2, -3, 1, 2, 3]


def rseq(rng, n):
    return rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), n).tobytes()


def to_i32(T):
    """Reference tables hold integral doubles or -inf; stored as int32 with
    INT32_MIN standing for -inf (all fixtures use integral g, h)."""
    assert np.all(~np.isfinite(T) | (T == np.round(T)))
    return np.where(np.isfinite(T), T, np.iinfo(np.int32).min).astype(np.int32)


def print_seq_lines(A: bytes, B: bytes, nodes):
    """print_seq (main_alignment.cpp:32-55) on 1-based A,B (given 0-based here)."""
    a = b"\0" + A
    b = b"\0" + B
    l1 = "".join(chr(a[i]) if t in (1, 3) else "-" for i, j, t in nodes)
    l2 = "".join(chr(b[j]) if t in (1, 2) else "-" for i, j, t in nodes)
    return l1, l2


def at_size():
    """Reference-produced fixtures at C2/C5 sizes: the reference's own
    Subproblem (p'=1) on seq0 x seq1 at 10k and 20k, seq0 x seq5 at 20k and h = 0 at 10k: score,
    final cell, node count, md5 of print_seq's two lines, and the H digest (checksum_h of
    max(T1,T2,T3)) where the fixture says so.  Writes tests/golden/at_size.json."""
    if not O.ref_available():
        O.build()
    assert O.ref_available(), "oracle/_ref not built (needs /root/reference)"
    _, seqs = O.load_dataset()
    out = []
    for (ia, ib, L, g, h, dig) in [(0, 1, 10000, 1.0, 2.0, True), (0, 1, 10000, 1.0, 0.0, False),
                                   (0, 1, 20000, 1.0, 2.0, True), (0, 5, 20000, 1.0, 2.0, False)]:
        A, B = seqs[ia][:L], seqs[ib][:L]
        r = O.ref_subproblem(A, B, -1, -1, g, h, p=1, tables=False, digest=dig)
        l1, l2 = print_seq_lines(A, B, r["nodes"])
        d = dict(a=ia, b=ib, L=L, g=g, h=h, score=float(max(r["fin"])), fin=list(r["fin"]),
                 n_nodes=len(r["nodes"]), lines_md5=hashlib.md5((l1 + "\n" + l2 + "\n").encode()).hexdigest())
        if dig:
            d["h_checksum"] = str(r["h_digest"])
        out.append(d)
        print("at_size", ia, ib, L, h, d["score"], flush=True)
    (HERE / "at_size.json").write_text(json.dumps(out, indent=1))


def main():
    if not O.ref_available():
        O.build()
    assert O.ref_available(), "oracle/_ref not built (needs /root/reference)"
    rng = np.random.default_rng(0x5EED0005)
    names, seqs = O.load_dataset()

    # ---- KATs ---------------------------------------------------------------
    kat = {}
    r = O.ref_subproblem(b"AGGA", b"ATGTC", -1, -1, 2.0, 1.0, p=3)
    kat["AGGA_ATGTC_g2_h1"] = dict(A="AGGA", B="ATGTC", g=2.0, h=1.0, nodes=r["nodes"],
                                   score=float(max(r["T1"][-1, -1], r["T2"][-1, -1], r["T3"][-1, -1])))
    r = O.ref_subproblem(b"AGGA", b"AGTGC", -1, -1, 1.0, 2.0, p=3)
    l1, l2 = print_seq_lines(b"AGGA", b"AGTGC", r["nodes"])
    kat["AGGA_AGTGC_g1_h2"] = dict(A="AGGA", B="AGTGC", g=1.0, h=2.0, nodes=r["nodes"], lines=[l1, l2],
                                   score=float(max(r["T1"][-1, -1], r["T2"][-1, -1], r["T3"][-1, -1])))
    # harness pairs: test_input_size (testing.cpp:26-80) picks seq3 x seq3 and
    # seq10 x seq11 at 1000 with glibc's unseeded rand(); main.cpp's default
    # test_input_size_thread picks seq2 x seq15 at 50.
    harness = []
    for (ia, ib, L) in [(3, 3, 1000), (10, 11, 1000), (2, 15, 50)]:
        A, B = seqs[ia][:L], seqs[ib][:L]
        r = O.ref_subproblem(A, B, -1, -1, 1.0, 2.0, p=11)
        l1, l2 = print_seq_lines(A, B, r["nodes"])
        score = float(max(r["T1"][-1, -1], r["T2"][-1, -1], r["T3"][-1, -1]))
        stdout = "bp1\nbp1.2\nbp2\nbp3\nbp4\n" + l1 + "\n" + l2 + "\n"
        harness.append(dict(a=ia, b=ib, L=L, score=score, n_nodes=len(r["nodes"]),
                            stdout=stdout if L <= 1000 else None,
                            stdout_md5=hashlib.md5(stdout.encode()).hexdigest()))
    kat["harness"] = harness
    lines4 = []
    for hp in harness[:2]:
        lines4 += hp["stdout"].split("\n")[5:7]
    kat["harness_1k_lines_md5"] = hashlib.md5(("\n".join(lines4) + "\n").encode()).hexdigest()
    # dataset prefixes seq0 x seq1 (scores quoted in BASELINE.md), plus H digest
    prefixes = []
    for L in (1000, 2000, 4000):
        A, B = seqs[0][:L], seqs[1][:L]
        r = O.ref_subproblem(A, B, -1, -1, 1.0, 2.0, p=1)
        Hm = np.maximum(np.maximum(r["T1"], r["T2"]), r["T3"])
        Hi = np.where(np.isfinite(Hm), Hm, 0).astype(np.int32)
        l1, l2 = print_seq_lines(A, B, r["nodes"])
        prefixes.append(dict(L=L, score=float(Hm[-1, -1]), n_nodes=len(r["nodes"]),
                             lines_md5=hashlib.md5((l1 + "\n" + l2 + "\n").encode()).hexdigest(),
                             h_checksum=str(O.checksum_h(Hi))))
        print("prefix", L, prefixes[-1]["score"], flush=True)
    kat["seq0_seq1_prefixes"] = prefixes
    (HERE / "kat.json").write_text(json.dumps(kat, indent=1))

    # ---- full tables for small pairs, all start/end types -------------------
    tabs = {}
    paths = []
    case = 0
    for st in TYPES:
        for et in TYPES:
            g, h = GH[case % len(GH)]
            m, n = int(rng.integers(1, 33)), int(rng.integers(1, 33))
            A, B = rseq(rng, m), rseq(rng, n)
            r = O.ref_subproblem(A, B, st, et, g, h, p=int(rng.integers(1, 4)))
            key = f"c{case:03d}"
            tabs[key + "_T"] = to_i32(np.stack([r["T1"], r["T2"], r["T3"]]))
            paths.append(dict(key=key, A=A.decode(), B=B.decode(), start=st, end=et, g=g, h=h,
                              invert=r["invert"], nodes=r["nodes"], end_node=r["end"]))
            case += 1
    # a few larger square/rectangular ones (start -1 only: the live path)
    for (m, n) in [(64, 64), (60, 64), (64, 37), (127, 129), (200, 130)]:
        g, h = GH[case % len(GH)]
        A, B = rseq(rng, m), rseq(rng, n)
        r = O.ref_subproblem(A, B, -1, -1, g, h, p=2)
        key = f"c{case:03d}"
        tabs[key + "_T"] = to_i32(np.stack([r["T1"], r["T2"], r["T3"]]))
        paths.append(dict(key=key, A=A.decode(), B=B.decode(), start=-1, end=-1, g=g, h=h,
                          invert=r["invert"], nodes=r["nodes"], end_node=r["end"]))
        case += 1
    np.savez_compressed(HERE / "subproblem_tables.npz", **tabs)
    (HERE / "subproblem_paths.json").write_text(json.dumps(paths))

    # ---- partial (wrap) -----------------------------------------------------
    parts = []
    for (m, n, p) in [(40, 40, 4), (40, 50, 4), (200, 200, 8), (17, 33, 5), (64, 64, 3)]:
        for st in (-1, 1, 2, 3):
            for et in (-1, 1, 2, 3):
                g, h = GH[len(parts) % len(GH)]
                if (m, n, p) == (40, 40, 4) and st == 1 and et == 1:
                    A, B = seqs[0][:40], seqs[1][:40]
                else:
                    A, B = rseq(rng, m), rseq(rng, n)
                out = O.ref_partial(A, B, p, g, h, st, et)
                parts.append(dict(A=A.decode(), B=B.decode(), p=p, g=g, h=h, start=st, end=et, partition=out))
    (HERE / "partial.json").write_text(json.dumps(parts))
    print("wrote fixtures to", HERE)


def partial_ties():
    """partial_ties.json: partitions with p >= 16 whose points tie on (i, j) (bands with no cell above
    INT_MIN give (0,0,0) when p > m or p > n; equal winners of different bands), so the reference's
    std::sort (partial.cpp:141-143, introsort: not stable past 16 elements) fixes their order."""
    rng = np.random.default_rng(0x5EED0016)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    out = []
    for (m, n) in [(5, 5), (10, 30), (30, 10), (15, 15), (20, 20), (12, 40), (40, 12), (64, 64), (3, 200),
                   (100, 100)]:
        for p in (16, 17, 20, 24, 32, 40, 64):
            for st, et in ((-1, -1), (1, 1), (2, 3), (3, -1)):
                A, B = rng.choice(acgt, m).tobytes(), rng.choice(acgt, n).tobytes()
                g, h = GH[len(out) % len(GH)]
                part = O.ref_partial(A, B, p, g, h, st, et)
                keys = [(i, j) for (i, j, _) in part]
                if len(set(keys)) == len(keys):
                    continue  # no tie: nothing the sort order decides
                # a stable sort keeps the input order among ties: (0,0,-1) pushed first stays first among
                # the (0,0,*) points and (m,n,1) pushed last stays last among the (m,n,*) ones
                z = [t for (i, j, t) in part if (i, j) == (0, 0)]
                e = [t for (i, j, t) in part if (i, j) == (m, n)]
                out.append(dict(A=A.decode(), B=B.decode(), p=p, g=g, h=h, start=st, end=et, partition=part,
                                differs_from_stable=bool(z[0] != -1 or e[-1] != 1)))
    (HERE / "partial_ties.json").write_text(json.dumps(out))
    print("partial_ties:", len(out), "cases,", sum(c["differs_from_stable"] for c in out), "differ from a stable sort")


if __name__ == "__main__":
    if sys.argv[1:] == ["at_size"]:
        at_size()
    elif sys.argv[1:] == ["partial_ties"]:
        partial_ties()
    else:
        main()
