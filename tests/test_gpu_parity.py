"""Bit-exact parity of the HIP stripe kernels (through libmsa.so's C-ABI) with the oracle and golden fixtures.

Integer DP: every comparison is exact (scores, end cells, full H matrices,
direction-derived tracebacks, node lists, stdout text)."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)


def enc(s: bytes) -> np.ndarray:
    return np.frombuffer(s.translate(bytes.maketrans(b"ACGT", b"\x00\x01\x02\x03")), dtype=np.uint8).copy()


def rs(rng, n):
    return rng.choice(ACGT, n).tobytes()


def _dev(x, dev):
    import torch

    return torch.from_numpy(enc(x)).to(dev)


@pytest.fixture(scope="module")
def LB():
    from cse305_parallel_sequence_alignment_amd import _lib

    return _lib


# (match, mismatch, gap): a negative mismatch runs the floored kernel; all
# scores >= 0 run the floor-free one (MSA_ALG_SWL0, zero-score virtual cells)
SW_SCORINGS = [(2, -1, 1), (1, 0, 1), (3, 1, 2), (1, 0, 3)]


# track_end=False is what bench.py's C2 line times (flow_kernel<..., TRACKPOS=false, 2>); True adds the end cell
@pytest.mark.parametrize("track_end", [False, True])
@pytest.mark.parametrize("scoring", SW_SCORINGS)
@pytest.mark.parametrize("single", [True, False])
def test_sw_linear_H_small(oracle, dev, LB, single, scoring, track_end):
    import torch
    from cse305_parallel_sequence_alignment_amd.plan import Plan

    ma, mi, g = scoring
    rng = np.random.default_rng(7)
    for (m, n) in [(1, 1), (5, 7), (64, 64), (65, 100), (130, 70), (200, 513), (511, 300), (700, 650), (520, 40)]:
        A, B = rs(rng, m), rs(rng, n)
        pl = Plan(LB.SW_LINEAR, LB.CELLS_H, [m], [n], [0], [0], match=ma, mismatch=mi, gap_open=g, gap_extend=g,
                  track_end=track_end, single=single)
        H = torch.empty(pl.cells_elems, dtype=torch.int32, device=dev)
        pl.run(_dev(A, dev), _dev(B, dev), H)
        res = pl.results()[0]
        Hd = pl.deskew(H.cpu().numpy(), 0, pl.stripe_meta())
        o = oracle.sw(A, B, ma, mi, g, g, want_h=True)
        assert res["score"] == o["score"], (m, n)
        if track_end:
            assert tuple(res["end"]) == tuple(o["end"]), (m, n)
        assert np.array_equal(Hd[1:, 1:], o["H"][1:, 1:]), (m, n)
        assert pl.checksum(H) == oracle.checksum_h(o["H"])


@pytest.mark.parametrize("track_end", [False, True])
@pytest.mark.parametrize("scoring", [(2, -1, 1), (1, 0, 1)])
def test_sw_linear_single_multi_group(oracle, dev, LB, scoring, track_end):
    """Single-pair mode across several workgroups (cross-WG row handoff), repeated launches, full H."""
    import torch
    from cse305_parallel_sequence_alignment_amd.plan import Plan

    ma, mi, g = scoring
    rng = np.random.default_rng(11)
    for (m, n) in [(1500, 1200), (3000, 2500)]:
        A, B = rs(rng, m), rs(rng, n)
        pl = Plan(LB.SW_LINEAR, LB.CELLS_H, [m], [n], [0], [0], match=ma, mismatch=mi, gap_open=g, gap_extend=g,
                  track_end=track_end, single=True)
        assert pl.geom[0].rows_per_lane == 2  # the two-pass flow kernel
        H = torch.empty(pl.cells_elems, dtype=torch.int32, device=dev)
        dA, dB = _dev(A, dev), _dev(B, dev)
        o = oracle.sw(A, B, ma, mi, g, g, want_h=True)
        for rep in range(3):
            pl.run(dA, dB, H)
            res = pl.results()[0]
            assert res["score"] == o["score"]
            if track_end:
                assert tuple(res["end"]) == tuple(o["end"])
            assert pl.checksum(H) == oracle.checksum_h(o["H"])
        assert np.array_equal(pl.deskew(H.cpu().numpy(), 0, pl.stripe_meta())[1:, 1:], o["H"][1:, 1:])


@pytest.mark.parametrize("scoring", SW_SCORINGS)
@pytest.mark.parametrize("track_end", [False, True])
def test_sw_linear_single_score_only(oracle, dev, LB, scoring, track_end):
    """Single pair, no cell output: the two-pass plan's pass 1 alone keeps the best cell
    (score only), or the stripe kernel when the end cell is wanted."""
    from cse305_parallel_sequence_alignment_amd.plan import Plan

    ma, mi, g = scoring
    rng = np.random.default_rng(23)
    for (m, n) in [(1, 3), (64, 64), (65, 1), (300, 1200), (1300, 700), (2600, 2100)]:
        A, B = rs(rng, m), rs(rng, n)
        pl = Plan(LB.SW_LINEAR, LB.CELLS_NONE, [m], [n], [0], [0], match=ma, mismatch=mi, gap_open=g, gap_extend=g,
                  track_end=track_end, single=True)
        pl.run(_dev(A, dev), _dev(B, dev))
        res = pl.results()[0]
        o = oracle.sw(A, B, ma, mi, g, g)
        assert res["score"] == o["score"], (m, n)
        if track_end:
            assert tuple(res["end"]) == tuple(o["end"]), (m, n)


@pytest.mark.parametrize("track_end", [False, True])
def test_sw_linear_single_wide_pair_flow_kernel(oracle, dev, LB, track_end):
    """Pairs wider than the former whole-row LDS code copies (n > ~19.5k) run the two-pass flow kernel too (the
    column codes stream through LDS rings): R = 2 layout, H and the first-maximum end equal the oracle's."""
    import torch
    from cse305_parallel_sequence_alignment_amd.plan import Plan

    rng = np.random.default_rng(29)
    for (ma, mi, g), (m, n) in [((1, 0, 1), (300, 25000)), ((2, -1, 1), (200, 21000))]:
        A, B = rs(rng, m), rs(rng, n)
        pl = Plan(LB.SW_LINEAR, LB.CELLS_H, [m], [n], [0], [0], match=ma, mismatch=mi, gap_open=g, gap_extend=g,
                  track_end=track_end, single=True)
        assert pl.geom[0].rows_per_lane == 2
        H = torch.empty(pl.cells_elems, dtype=torch.int32, device=dev)
        pl.run(_dev(A, dev), _dev(B, dev), H)
        res = pl.results()[0]
        o = oracle.sw(A, B, ma, mi, g, g, want_h=True)
        assert res["score"] == o["score"]
        if track_end:
            assert tuple(res["end"]) == tuple(o["end"])
        assert pl.checksum(H) == oracle.checksum_h(o["H"])


@pytest.mark.parametrize("scoring", [(2, -1, 1), (1, 0, 1)])
def test_sw_linear_batch_ragged(oracle, dev, LB, scoring):
    import torch
    from cse305_parallel_sequence_alignment_amd.plan import Plan

    ma, mi, g = scoring
    rng = np.random.default_rng(11)
    sizes = [(1100, 1000), (600, 4000), (1300, 960), (64, 3000), (2000, 1500), (33, 17), (1, 5), (129, 1)]
    As = [rs(rng, m) for m, n in sizes]
    Bs = [rs(rng, n) for m, n in sizes]
    ao = np.cumsum([0] + [m for m, n in sizes])[:-1]
    bo = np.cumsum([0] + [n for m, n in sizes])[:-1]
    pl = Plan(LB.SW_LINEAR, LB.CELLS_H, [m for m, n in sizes], [n for m, n in sizes], ao, bo, match=ma, mismatch=mi,
              gap_open=g, gap_extend=g, track_end=True, single=False)
    H = torch.empty(pl.cells_elems, dtype=torch.int32, device=dev)
    pl.run(_dev(b"".join(As), dev), _dev(b"".join(Bs), dev), H)
    res, meta, Hh = pl.results(), pl.stripe_meta(), H.cpu().numpy()
    for k, (m, n) in enumerate(sizes):
        o = oracle.sw(As[k], Bs[k], ma, mi, g, g, want_h=True)
        assert res[k]["score"] == o["score"] and tuple(res[k]["end"]) == tuple(o["end"]), (m, n)
        assert np.array_equal(pl.deskew(Hh, k, meta)[1:, 1:], o["H"][1:, 1:]), (m, n)


def test_sw_linear_c4_shape_scores(oracle, dev, LB):
    """C4's shape (4,000 x 4,000 pairs, score only) on a 64-pair batch; spot-checked against the oracle."""
    from cse305_parallel_sequence_alignment_amd.plan import Plan

    rng = np.random.default_rng(4)
    L, K = 4000, 64
    As = [rs(rng, L) for _ in range(K)]
    B = rs(rng, L)
    pl = Plan(LB.SW_LINEAR, LB.CELLS_NONE, [L] * K, [L] * K, [k * L for k in range(K)], [0] * K, match=1,
              mismatch=0, gap_open=1, gap_extend=1, single=False)
    pl.run(_dev(b"".join(As), dev), _dev(B, dev))
    res = pl.results()
    for k in (0, 1, 31, 63):
        assert res[k]["score"] == oracle.sw(As[k], B, 1, 0, 1, 1)["score"]


# the two kernels a packed score-only batch can run (msa_capi.hip, MSA_C4_KERNEL read per plan): cflow_kernel
# (the default below two couples per CU) and the lock-step stripe kernel (batch or split mode)
C4_KERNELS = {"cflow": ("cflow",), "lockstep": ("stripe", "split")}


@pytest.mark.parametrize("c4_kernel", sorted(C4_KERNELS))
@pytest.mark.parametrize("scoring", [(1, 0, 1), (2, 1, 1), (3, 0, 2), (5, 2, 3)])
def test_sw_linear_packed_pairs(oracle, dev, LB, scoring, c4_kernel, monkeypatch):
    """Score-only batches whose pair couples (2c, 2c+1) share sizes and column sequence run two pairs per lane
    as packed int16 (MSA_ALG_SWLP): every score equals the oracle's -- couples of different shapes in one plan,
    an odd pair count (the last couple repeats its pair), similar and random pairs, sizes from 1 to 2,000 --
    on both kernels (the launch mode is asserted)."""
    from cse305_parallel_sequence_alignment_amd.plan import Plan

    monkeypatch.setenv("MSA_C4_KERNEL", c4_kernel)
    ma, mi, g = scoring
    rng = np.random.default_rng(40 + ma)
    shapes = [(700, 650), (700, 650), (64, 64), (64, 64), (1, 9), (1, 9), (2000, 1999), (2000, 1999), (130, 7),
              (130, 7), (333, 1000)]
    Bs = {}
    As, ao, bo, Bcat = [], [], [], b""
    for k, (m, n) in enumerate(shapes):
        c = k // 2
        if c not in Bs:
            Bs[c] = (len(Bcat), rs(rng, n))
            Bcat += Bs[c][1]
        B = Bs[c][1]
        A = B[:m] if (k % 4 == 1 and m <= n) else rs(rng, m)  # some similar pairs (long runs of matches)
        ao.append(sum(len(x) for x in As))
        As.append(A)
        bo.append(Bs[c][0])
    pl = Plan(LB.SW_LINEAR, LB.CELLS_NONE, [m for m, _ in shapes], [n for _, n in shapes], ao, bo, match=ma,
              mismatch=mi, gap_open=g, gap_extend=g, single=False)
    assert pl.launch_info()["mode"] in C4_KERNELS[c4_kernel]
    pl.run(_dev(b"".join(As), dev), _dev(Bcat, dev))
    res = pl.results()
    for k, (m, n) in enumerate(shapes):
        B = Bs[k // 2][1]
        assert res[k]["score"] == oracle.sw(As[k], B, ma, mi, g, g)["score"], (k, m, n)


@pytest.mark.parametrize("kind", ["packed", "packed_lockstep", "int32_H", "affine_dir"])
def test_batch_split_pairs(oracle, dev, LB, kind, monkeypatch):
    """A batch with fewer pairs than two workgroups per CU splits every pair into items chained through
    granules: packed couples run cflow_kernel by default (items of 4 stripes) and the lock-step kernel's split
    mode when forced (kp.single == 3, as every unpacked batch here); scores (and for the int32 plan the full H
    matrices, for SW affine the device traceback) equal the oracle's."""
    import torch
    from cse305_parallel_sequence_alignment_amd.plan import Plan

    rng = np.random.default_rng({"packed": 1, "packed_lockstep": 1, "int32_H": 2, "affine_dir": 3}[kind])
    if kind.startswith("packed"):
        if kind == "packed_lockstep":
            monkeypatch.setenv("MSA_C4_KERNEL", "lockstep")
        K, m, n = 37, 1500, 1400  # odd count: the last couple repeats its pair
        As = [rs(rng, m) for _ in range(K)]
        B = rs(rng, n)
        pl = Plan(LB.SW_LINEAR, LB.CELLS_NONE, [m] * K, [n] * K, [k * m for k in range(K)], [0] * K, match=1,
                  mismatch=0, gap_open=1, gap_extend=1, single=False)
        assert pl.launch_info()["mode"] == ("cflow" if kind == "packed" else "split")
        pl.run(_dev(b"".join(As), dev), _dev(B, dev))
        res = pl.results()
        for k in range(K):
            assert res[k]["score"] == oracle.sw(As[k], B, 1, 0, 1, 1)["score"], k
    elif kind == "int32_H":
        K, m = 6, 1100
        ns = [900, 1300, 1100, 700, 1250, 1000]
        As = [rs(rng, m) for _ in range(K)]
        Bs = [rs(rng, x) for x in ns]
        bo = np.cumsum([0] + ns)[:-1]
        pl = Plan(LB.SW_LINEAR, LB.CELLS_H, [m] * K, ns, [k * m for k in range(K)], bo, match=2, mismatch=-1,
                  gap_open=1, gap_extend=1, track_end=True, single=False)
        H = torch.empty(pl.cells_elems, dtype=torch.int32, device=dev)
        pl.run(_dev(b"".join(As), dev), _dev(b"".join(Bs), dev), H)
        res, meta, Hh = pl.results(), pl.stripe_meta(), H.cpu().numpy()
        for k in range(K):
            o = oracle.sw(As[k], Bs[k], 2, -1, 1, 1, want_h=True)
            assert res[k]["score"] == o["score"] and tuple(res[k]["end"]) == tuple(o["end"]), k
            assert np.array_equal(pl.deskew(Hh, k, meta)[1:, 1:], o["H"][1:, 1:]), k
    else:
        K, m, n = 5, 1300, 1250
        As = [rs(rng, m) for _ in range(K)]
        Bs = [rs(rng, n) for _ in range(K)]
        pl = Plan(LB.SW_AFFINE, LB.CELLS_DIR, [m] * K, [n] * K, [k * m for k in range(K)], [k * n for k in range(K)],
                  match=1, mismatch=0, gap_open=3, gap_extend=1, track_end=True, single=False)
        D = torch.empty(pl.cells_elems, dtype=torch.uint8, device=dev)
        pl.run(_dev(b"".join(As), dev), _dev(b"".join(Bs), dev), D)
        res = pl.results()
        for k in range(K):
            o = oracle.sw(As[k], Bs[k], 1, 0, 3, 1, want_tb=True)
            tb = pl.traceback(D, pair=k)
            assert (res[k]["score"], tuple(res[k]["end"])) == (o["score"], tuple(o["end"])), k
            assert (tuple(tb["beg"]), tb["cigar"]) == (tuple(o["beg"]), o["cigar"]), k
    assert pl.error() == 0


def test_main_alignment_kat_and_harness(oracle, dev, dataset):
    """main_alignment_function stdout (main_alignment.cpp:353-410) byte-exact on the KAT and harness pairs."""
    from cse305_parallel_sequence_alignment_amd import api

    kat = json.loads((GOLDEN / "kat.json").read_text())
    t, sc = api.main_alignment_text(b"-AGGA", b"-AGTGC", 4, 5, 3, 1, 2)
    assert t == "bp1\nbp1.2\nbp2\nbp3\nbp4\nAG-GA\nAGTGC\n"
    _, seqs = dataset
    lines = []
    for hp in kat["harness"]:
        A, B = seqs[hp["a"]][: hp["L"]], seqs[hp["b"]][: hp["L"]]
        t, sc = api.main_alignment_text(b"\0" + A, b"\0" + B, hp["L"], hp["L"], 32, 1, 2)
        assert hashlib.md5(t.encode()).hexdigest() == hp["stdout_md5"] and sc == hp["score"]
        if hp["L"] == 1000:
            lines += t.split("\n")[5:7]
    assert hashlib.md5(("\n".join(lines) + "\n").encode()).hexdigest() == kat["harness_1k_lines_md5"]
    for pr in kat["seq0_seq1_prefixes"]:
        L = pr["L"]
        t, sc = api.main_alignment_text(b"\0" + seqs[0][:L], b"\0" + seqs[1][:L], L, L, 32, 1, 2)
        l = t.split("\n")[5:7]
        assert sc == pr["score"]
        assert hashlib.md5((l[0] + "\n" + l[1] + "\n").encode()).hexdigest() == pr["lines_md5"]


def test_subproblem_fixtures(dev):
    """Subproblem::compute_tables + find_alignment on all 41 fixtures (every start/end type, g/h)."""
    from cse305_parallel_sequence_alignment_amd import api

    paths = json.loads((GOLDEN / "subproblem_paths.json").read_text())
    tabs = np.load(GOLDEN / "subproblem_tables.npz")
    for c in paths:
        A, B = c["A"].encode(), c["B"].encode()
        sp = api.Subproblem(b"\0" + A, b"\0" + B, len(A), len(B), 0, 0, 1, c["start"], c["end"], c["g"], c["h"])
        sp.compute_tables()
        if c["key"] + "_T" in tabs:
            for x, y in zip(sp._tables_int, tabs[c["key"] + "_T"]):
                assert np.array_equal(x, y), c["key"]
        sp.find_alignment()
        assert sp.alignment_list() == [tuple(x) for x in c["nodes"]], c["key"]
        assert sp.alignment_end.as_tuple() == tuple(c["end_node"]), c["key"]


def test_partial_fixtures(oracle, dev, dataset):
    """findPartialBalancedPartitionParallel (partial.cpp:149-163, int32 wrap) on the 80 fixtures + tables."""
    from cse305_parallel_sequence_alignment_amd import api

    for c in json.loads((GOLDEN / "partial.json").read_text()):
        A, B = c["A"].encode(), c["B"].encode()
        got = [a.as_tuple() for a in api.findPartialBalancedPartitionParallel(A, B, len(A), len(B), c["p"], c["g"],
                                                                               c["h"], c["start"], c["end"])]
        assert got == [tuple(x) for x in c["partition"]]
    _, seqs = dataset
    T, R = api.partial_tables(seqs[0][:40], seqs[1][:40], 40, 40, 1, 2, 1, 1)
    To, Ro = oracle.partial_tables(seqs[0][:40], seqs[1][:40], 1, 2, 1, 1)
    for a, b in zip(T + R, To + Ro):
        assert np.array_equal(a, b)


def test_partial_partition_tie_order(dev):
    """findPartialBalancedPartitionParallel with p >= 16 on the GPU: points tying on (i, j) in the order
    of the reference's std::sort (partial.cpp:141-143), all 116 fixtures of partial_ties.json."""
    from cse305_parallel_sequence_alignment_amd import api

    for c in json.loads((GOLDEN / "partial_ties.json").read_text()):
        A, B = c["A"].encode(), c["B"].encode()
        got = [a.as_tuple() for a in api.findPartialBalancedPartitionParallel(A, B, len(A), len(B), c["p"], c["g"],
                                                                               c["h"], c["start"], c["end"])]
        assert got == [tuple(x) for x in c["partition"]], (c["p"], len(A), len(B))


def test_sw_affine_traceback(oracle, dev):
    from cse305_parallel_sequence_alignment_amd import api

    rng = np.random.default_rng(3)
    for (m, n) in [(30, 40), (100, 90), (300, 257), (700, 800), (1, 1), (64, 1)]:
        A, B = rs(rng, m), rs(rng, n)
        for (ma, mi, go, ge) in [(1, 0, 1, 1), (2, -3, 5, 2), (1, -1, 3, 1)]:
            r = api.sw_align(A, B, ma, mi, go, ge)
            o = oracle.sw(A, B, ma, mi, go, ge, want_tb=True)
            assert (r["score"], r["end"], r["beg"], r["cigar"]) == (o["score"], o["end"], o["beg"], o["cigar"])


@pytest.mark.parametrize("alg,m,n,ma,mi,go,ge", [
    ("affine", 2100, 2000, 40, -30, 50, 10),   # score bound 40 x 2000 >= 2^16: unpacked tracking
    ("affine", 700, 800, 1, 0, 3, 1),          # packed (value << 15 | 32767 - step)
    ("linear", 1900, 2100, 40, -25, 30, 30),   # unpacked, SW linear
    ("linear", 900, 1000, 2, -1, 1, 1),        # packed, SW linear
])
def test_first_maximum_tracking_modes(oracle, dev, LB, alg, m, n, ma, mi, go, ge):
    """track_end plans pick the packed first-maximum mode when every score is below 2^16 and a stripe has
    fewer than 2^15 steps, else the compare-and-select mode: both must report the oracle's score and its
    first (row-major) end cell, and the affine plans' device traceback the oracle's CIGAR."""
    import torch
    from cse305_parallel_sequence_alignment_amd.plan import Plan, cigar_of

    rng = np.random.default_rng(m + n + ma)
    A, B = rs(rng, m), rs(rng, n)
    B = A[100:1100] + B[1000:]  # a long local match, so high-scoring alignments exist
    n = len(B)
    if alg == "affine":
        pl = Plan(LB.SW_AFFINE, LB.CELLS_DIR, [m], [n], [0], [0], match=ma, mismatch=mi, gap_open=go,
                  gap_extend=ge, track_end=True)
        out = torch.empty(pl.cells_elems, dtype=torch.uint8, device=dev)
    else:
        pl = Plan(LB.SW_LINEAR, LB.CELLS_H, [m], [n], [0], [0], match=ma, mismatch=mi, gap_open=go,
                  gap_extend=ge, track_end=True)
        out = torch.empty(pl.cells_elems, dtype=torch.int32, device=dev)
    pl.run(_dev(A, dev), _dev(B, dev), out)
    r = pl.results()[0]
    o = oracle.sw(A, B, ma, mi, go, ge, want_tb=(alg == "affine"))
    assert (r["score"], tuple(r["end"])) == (o["score"], tuple(o["end"]))
    if alg == "affine":
        ops = torch.empty(m + n + 2, dtype=torch.uint8, device=dev)
        info = torch.zeros(8, dtype=torch.int64, device=dev)
        pl.traceback_async(out, ops, info)
        inf = info.cpu().tolist()
        assert inf[3] == 0
        assert cigar_of(bytes(ops[:inf[0]].cpu().numpy().tobytes())) == o["cigar"]
        assert (inf[1], inf[2]) == tuple(o["beg"])


@pytest.mark.parametrize("track_end", [False, True])
def test_sw_linear_10k_c2(oracle, dev, LB, track_end):
    """C2 exactly as bench.py runs it (data.c2_pair, match 1 / mismatch 0 / gap 1, H written; track_end=False
    is the benched kernel): 25 back-to-back runs, then the sticky error word, score/end and the checksum of
    every H cell against the oracle."""
    import torch
    from cse305_parallel_sequence_alignment_amd import data
    from cse305_parallel_sequence_alignment_amd.plan import Plan

    A, B = data.c2_pair(0)
    pl = Plan(LB.SW_LINEAR, LB.CELLS_H, [10000], [10000], [0], [0], match=1, mismatch=0, gap_open=1, gap_extend=1,
              track_end=track_end)
    H = torch.empty(pl.cells_elems, dtype=torch.int32, device=dev)
    dA, dB = _dev(A, dev), _dev(B, dev)
    pl.set_timing(False)
    for _ in range(25):
        pl.run(dA, dB, H)
    assert pl.error() == 0
    o = oracle.sw(A, B, 1, 0, 1, 1, want_h=True)
    res = pl.results()[0]
    assert res["score"] == o["score"] == 9343
    if track_end:
        assert tuple(res["end"]) == tuple(o["end"])
    assert pl.checksum(H) == oracle.checksum_h(o["H"])
    # a second pair (rank 1's bench pair) through the same plan
    A1, _ = data.c2_pair(1)
    pl.run(_dev(A1, dev), dB, H)
    o1 = oracle.sw(A1, B, 1, 0, 1, 1, want_h=True)
    assert pl.results()[0]["score"] == o1["score"] and pl.checksum(H) == oracle.checksum_h(o1["H"])


def test_c4_full_batch_scores(dev, LB):
    """C4 (1024 x 4k x 4k, score only) exactly as bench.py runs it on one GPU: every score equals the
    committed oracle fixture (tests/golden/c4_scores.json)."""
    import torch
    from cse305_parallel_sequence_alignment_amd import data
    from cse305_parallel_sequence_alignment_amd.plan import Plan

    want = json.loads((GOLDEN / "c4_scores.json").read_text())["scores"]
    L, K = data.C4_LEN, data.C4_PAIRS
    qs = data.c4_queries(0, K)
    pl = Plan(LB.SW_LINEAR, LB.CELLS_NONE, [L] * K, [L] * K, [k * L for k in range(K)], [0] * K, match=1,
              mismatch=0, gap_open=1, gap_extend=1)
    pl.run(_dev(b"".join(qs), dev), _dev(data.c4_reference(), dev))
    d = torch.empty(K, dtype=torch.int32, device=dev)
    pl.scores_into(d)
    assert [r["score"] for r in pl.results()] == want
    assert d.cpu().tolist() == want


@pytest.mark.parametrize("world,rank", [(8, 0), (8, 7), (4, 3), (2, 1)])
def test_c4_rank_share_scores(dev, LB, world, rank):
    """The C4 share one rank of an N-GPU run aligns (shard.ShardedBatch's contiguous block: 128 pairs at 8
    GPUs, 256 at 4, 512 at 2) runs cflow_kernel, as bench.py's multi-GPU C4 does: every score of the share,
    over three launches of one plan (epochs), equals its slice of tests/golden/c4_scores.json."""
    import torch
    from cse305_parallel_sequence_alignment_amd import data
    from cse305_parallel_sequence_alignment_amd.plan import Plan
    from cse305_parallel_sequence_alignment_amd.shard import shard_range

    want = json.loads((GOLDEN / "c4_scores.json").read_text())["scores"]
    L = data.C4_LEN
    lo, hi = shard_range(data.C4_PAIRS, rank, world)
    assert hi - lo == data.C4_PAIRS // world
    K = hi - lo
    pl = Plan(LB.SW_LINEAR, LB.CELLS_NONE, [L] * K, [L] * K, [k * L for k in range(K)], [0] * K, match=1,
              mismatch=0, gap_open=1, gap_extend=1)
    assert pl.launch_info()["mode"] == "cflow"
    dq, dr = _dev(b"".join(data.c4_queries(lo, hi)), dev), _dev(data.c4_reference(), dev)
    d = torch.empty(K, dtype=torch.int32, device=dev)
    for _ in range(3):
        d.fill_(-1)
        pl.run(dq, dr)
        pl.scores_into(d)
        assert d.cpu().tolist() == want[lo:hi]
    assert pl.error() == 0


@pytest.mark.parametrize("m,n,w",[(300, 290, 32), (1000, 1000, 64), (1500, 1490, 512), (700, 700, 1)])
def test_nw_banded_reference_gotoh(oracle, dev, LB, m, n, w):
    """C3's kernel (banded reference Gotoh, g=1 h=2) at small sizes: every in-band H cell and the score."""
    import torch
    from cse305_parallel_sequence_alignment_amd.plan import Plan

    rng = np.random.default_rng(m + w)
    A, B = rs(rng, m), rs(rng, n)
    pl = Plan(LB.NW_BANDED, LB.CELLS_H, [m], [n], [0], [0], match=1, mismatch=0, gap_open=3, gap_extend=1, band=w)
    H = torch.empty(pl.cells_elems, dtype=torch.int32, device=dev)
    pl.run(_dev(A, dev), _dev(B, dev), H)
    score, Ho = oracle.banded_ref(A, B, w, 1.0, 2.0, want_h=True)
    Hd = pl.deskew(H.cpu().numpy(), 0, pl.stripe_meta())
    i, j = np.indices(Ho.shape)
    inb = (np.abs(i - j) <= w) & (i > 0) & (j > 0)
    assert np.array_equal(Hd[inb], Ho[inb])
    assert pl.checksum(H) == oracle.checksum_h(Ho, w)
    assert pl.results()[0]["score"] == int(score)


def test_reference_harness_linked_against_compat(tmp_path):
    """The reference's own harness (main.cpp + testing.cpp + pull_data.cpp, unmodified, built by
    oracle/Makefile into oracle/_ref/harness_msa) linked against libmsa_compat.so instead of the
    reference's alignment objects: its stdout alignment equals the reference's (golden md5)."""
    import gzip
    import shutil
    import subprocess

    from conftest import ROOT

    exe = ROOT / "oracle" / "_ref" / "harness_msa"
    if not exe.exists():
        pytest.skip("oracle/_ref/harness_msa not built (reference sources absent at build time)")
    with gzip.open(GOLDEN / "gene_sequences_test.gz", "rb") as f, open(tmp_path / "gene_sequences_test", "wb") as o:
        shutil.copyfileobj(f, o)
    r = subprocess.run([str(exe)], cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = r.stdout.split("\n")
    assert "Finished threads" in lines
    i = lines.index("bp1")
    block = "\n".join(lines[i:i + 7]) + "\n"
    kat = json.loads((GOLDEN / "kat.json").read_text())
    want = [h for h in kat["harness"] if (h["a"], h["b"], h["L"]) == (2, 15, 50)][0]
    assert hashlib.md5(block.encode()).hexdigest() == want["stdout_md5"], block


@pytest.mark.parametrize("m,n", [(65, 70), (129, 129), (1, 5), (64, 1), (193, 200), (257, 64), (70, 65)])
def test_reference_gotoh_ragged_edges(oracle, dev, m, n):
    """Shapes whose last stripe has one row (m = 64k+1) or one column: stdout, tables, partitions vs the oracle."""
    from cse305_parallel_sequence_alignment_amd import api

    rng = np.random.default_rng(m * 1000 + n)
    A, B = rs(rng, m), rs(rng, n)
    t, sc = api.main_alignment_text(b"\0" + A, b"\0" + B, m, n, 8, 1, 2)
    to, so = oracle.main_alignment_text(A, B, 1.0, 2.0)
    assert (t, sc) == (to, so)
    for st in (-1, -2, -3, 1, 2, 3):
        sp = api.Subproblem(b"\0" + A, b"\0" + B, m, n, 0, 0, 1, st, -1, 1, 2)
        sp.compute_tables()
        T1, T2, T3, _ = oracle.subproblem_tables(A, B, st, 1.0, 2.0)
        for x, y in zip((sp.T1, sp.T2, sp.T3), (T1, T2, T3)):
            assert np.array_equal(x, y), (m, n, st)
    if m >= 4 and n >= 4:
        got = [a.as_tuple() for a in api.findPartialBalancedPartitionParallel(A, B, m, n, 4, 1, 2, 1, 1)]
        assert got == oracle.partial_partition(A, B, 4, 1.0, 2.0, 1, 1)


@pytest.mark.parametrize("m,n,w", [(65, 70, 8), (129, 130, 16), (193, 193, 64)])
def test_nw_banded_single_row_stripe(oracle, dev, LB, m, n, w):
    import torch
    from cse305_parallel_sequence_alignment_amd.plan import Plan

    rng = np.random.default_rng(m + 7 * w)
    A, B = rs(rng, m), rs(rng, n)
    pl = Plan(LB.NW_BANDED, LB.CELLS_H, [m], [n], [0], [0], match=1, mismatch=0, gap_open=3, gap_extend=1, band=w)
    H = torch.empty(pl.cells_elems, dtype=torch.int32, device=dev)
    pl.run(_dev(A, dev), _dev(B, dev), H)
    score, Ho = oracle.banded_ref(A, B, w, 1.0, 2.0, want_h=True)
    assert pl.results()[0]["score"] == int(score)
    assert pl.checksum(H) == oracle.checksum_h(Ho, w)


def test_reference_fixtures_at_size(dev, LB, dataset):
    """main_alignment_function at 10k / 20k against the reference's own outputs (tests/golden/at_size.json,
    made by make_golden.py at_size from the reference's Subproblem): score, node count and the md5 of the two
    print_seq lines; plus the digest of every H = max(T1,T2,T3) cell of the reference's tables at 1k-20k."""
    import torch
    from cse305_parallel_sequence_alignment_amd import api
    from cse305_parallel_sequence_alignment_amd.plan import Plan

    _, seqs = dataset
    cases = json.loads((GOLDEN / "at_size.json").read_text())
    kat = json.loads((GOLDEN / "kat.json").read_text())
    for c in cases:
        A, B = seqs[c["a"]][:c["L"]], seqs[c["b"]][:c["L"]]
        t, sc = api.main_alignment_text(b"\0" + A, b"\0" + B, c["L"], c["L"], 32, c["g"], c["h"])
        lines = t.split("\n")[5:7]
        assert sc == c["score"], c
        assert len(lines[0]) == c["n_nodes"]
        assert hashlib.md5((lines[0] + "\n" + lines[1] + "\n").encode()).hexdigest() == c["lines_md5"], c
    digests = [(p["L"], 0, 1, 1, 2, p["h_checksum"]) for p in kat["seq0_seq1_prefixes"]]
    digests += [(c["L"], c["a"], c["b"], int(c["g"]), int(c["h"]), c["h_checksum"]) for c in cases if "h_checksum" in c]
    for L, ia, ib, g, h, want in digests:
        pl = Plan(LB.REF_GOTOH, LB.CELLS_H, [L], [L], [0], [0], match=1, mismatch=0, gap_open=g + h, gap_extend=g,
                  start_type=-1)
        H = torch.empty(pl.cells_elems, dtype=torch.int32, device=dev)
        pl.run(_dev(seqs[ia][:L], dev), _dev(seqs[ib][:L], dev), H)
        pl.results()
        assert pl.checksum(H) == int(want), (L, ia, ib)


def test_c3_full_size(oracle, dev, LB):
    """C3 as bench.py runs it: 97,403 x 97,403 banded (512) reference Gotoh, H written: score and the digest of
    every in-band H cell against the banded oracle."""
    import torch
    from cse305_parallel_sequence_alignment_amd import data
    from cse305_parallel_sequence_alignment_amd.plan import Plan

    A, B = data.c3_pair()
    m, n = len(A), len(B)
    pl = Plan(LB.NW_BANDED, LB.CELLS_H, [m], [n], [0], [0], match=1, mismatch=0, gap_open=3, gap_extend=1, band=512)
    H = torch.empty(pl.cells_elems, dtype=torch.int32, device=dev)
    pl.run(_dev(A, dev), _dev(B, dev), H)
    score, digest = oracle.banded_ref(A, B, 512, 1.0, 2.0, want_digest=True)
    assert pl.results()[0]["score"] == int(score)
    assert pl.checksum(H) == digest
    # the bench's pair converges in every chunk: the cells come from the chunked launch
    info = pl.run_info()
    assert info["mode"] == "chunked" and info["converged"] == 1 and info["chunks"] >= 4, info
    # chunks >= 1 wrote int16 cells (in-band |H| well inside int16 here), widened by the constants' add
    assert info["int16_cells"] == (0 if os.environ.get("MSA_BAND_H16") == "0" else 1), info


@pytest.mark.parametrize("which", ["synthetic", "dissimilar"])
def test_c3_other_inputs(oracle, dev, LB, which):
    """C3 beyond the bench's real pair: SURVEY §8(d)'s synthetic input (100,000 i.i.d. ACGT, B = A mutated 1% /
    0.1%, seed 0x5EED0003 -- converges in every chunk) and a dissimilar real pair (ABCB1 x KIT, 81,835 each --
    rank convergence fails, the exact launch behind the chunks recomputes it): score and the digest of every
    in-band H cell equal the banded oracle's."""
    import torch
    from cse305_parallel_sequence_alignment_amd import data
    from cse305_parallel_sequence_alignment_amd.plan import Plan

    if which == "synthetic":
        A, B = data.c3_pair(synthetic=True)
    else:
        A, B = data.bundled()[0][:81835], data.bundled()[15][:81835]
    pl = Plan(LB.NW_BANDED, LB.CELLS_H, [len(A)], [len(B)], [0], [0], match=1, mismatch=0, gap_open=3,
              gap_extend=1, band=512)
    H = torch.empty(pl.cells_elems, dtype=torch.int32, device=dev)
    pl.run(_dev(A, dev), _dev(B, dev), H)
    score, digest = oracle.banded_ref(A, B, 512, 1.0, 2.0, want_digest=True)
    assert pl.results()[0]["score"] == int(score)
    assert pl.checksum(H) == digest
    info = pl.run_info()
    assert info["mode"] == "chunked" and info["converged"] == (1 if which == "synthetic" else 0), info
    assert pl.error() == 0


def _similar(rng, m, sub=0.02, indel=0.002):
    """A random A and B = A with substitutions and short indels (length ~m)."""
    A = rs(rng, m)
    b = bytearray(A)
    for k in rng.choice(m, size=int(m * sub), replace=False):
        b[k] = ACGT[rng.integers(4)]
    for k in sorted(rng.choice(m - 16, size=int(m * indel), replace=False), reverse=True):
        if rng.integers(2):
            del b[k:k + int(rng.integers(1, 8))]
        else:
            b[k:k] = rs(rng, int(rng.integers(1, 8)))
    return A, bytes(b)


@pytest.mark.parametrize("kind,m,w", [("similar", 12000, 512), ("similar", 20011, 256), ("similar", 9001, 64),
                                      ("random", 12000, 512), ("similar_then_random", 16000, 512)])
def test_banded_chunked(oracle, dev, LB, kind, m, w):
    """Chunked banded runs (rank convergence): similar pairs converge in every chunk and the cells come from
    the chunked launch plus the per-chunk constants; a random pair (or one whose second half is random) does
    not, and the exact single-mode launch behind it recomputes the pair.  Either way the score and every
    in-band H cell equal the banded oracle's, over repeated runs of the same plan."""
    import torch
    from cse305_parallel_sequence_alignment_amd.plan import Plan

    rng = np.random.default_rng(m + w)
    if kind == "random":
        A, B = rs(rng, m), rs(rng, m + 37)
    elif kind == "similar":
        A, B = _similar(rng, m)
    else:
        A, B = _similar(rng, m // 2)
        A, B = A + rs(rng, m - m // 2), B + rs(rng, m - m // 2)
    if abs(len(A) - len(B)) > w:
        B = B[:len(A) + w // 2]
    pl = Plan(LB.NW_BANDED, LB.CELLS_H, [len(A)], [len(B)], [0], [0], match=1, mismatch=0, gap_open=3,
              gap_extend=1, band=w)
    H = torch.empty(pl.cells_elems, dtype=torch.int32, device=dev)
    score, digest = oracle.banded_ref(A, B, w, 1.0, 2.0, want_digest=True)
    for _ in range(2):
        H.fill_(7)
        pl.run(_dev(A, dev), _dev(B, dev), H)
        assert pl.results()[0]["score"] == int(score)
        assert pl.checksum(H) == digest
        info = pl.run_info()
        assert info["mode"] == "chunked" and info["chunks"] >= 4
        assert info["converged"] == (1 if kind == "similar" else 0), info
        assert info["int16_cells"] == (0 if os.environ.get("MSA_BAND_H16") == "0" else 1), info
    assert pl.error() == 0


@pytest.mark.parametrize("g,int16", [(50, 1), (60, 0)])
def test_banded_chunked_int16_bound(oracle, dev, LB, g, int16):
    """The int16 chunk cells' range bound (msa_plan_create: rows + h + g band <= 30,000): with g = 50 and band
    512 the in-band cells reach -h - g band = -25,601 and stay int16 (cells written as int16, widened by the
    add); g = 60 (30,720 past the bound) keeps int32 cells.  Either way score and every in-band cell equal
    the banded oracle's."""
    import torch
    from cse305_parallel_sequence_alignment_amd.plan import Plan

    rng = np.random.default_rng(g)
    A, B = _similar(rng, 12000)
    w = 512
    if abs(len(A) - len(B)) > w:
        B = B[:len(A) + w // 2]
    pl = Plan(LB.NW_BANDED, LB.CELLS_H, [len(A)], [len(B)], [0], [0], match=1, mismatch=0, gap_open=g + 1,
              gap_extend=g, band=w)
    H = torch.empty(pl.cells_elems, dtype=torch.int32, device=dev)
    score, digest = oracle.banded_ref(A, B, w, float(g), 1.0, want_digest=True)
    pl.run(_dev(A, dev), _dev(B, dev), H)
    assert pl.results()[0]["score"] == int(score)
    assert pl.checksum(H) == digest
    info = pl.run_info()
    assert info["mode"] == "chunked" and info["chunks"] >= 4, info
    if os.environ.get("MSA_BAND_H16") != "0":
        assert info["int16_cells"] == int16, info
    assert pl.error() == 0


def _rescore(A, B, beg, cigar, ma, mi, go, ge):
    """Score of the local alignment a CIGAR describes from beg (1-based): affine gaps go + (k-1) ge."""
    import re

    i, j, sc = beg[0] - 1, beg[1] - 1, 0
    for run, op in re.findall(r"(\d+)([MID])", cigar):
        run = int(run)
        if op == "M":
            sc += sum(ma if A[i + k] == B[j + k] else mi for k in range(run))
            i, j = i + run, j + run
        elif op == "I":
            sc -= go + (run - 1) * ge
            i += run
        else:
            sc -= go + (run - 1) * ge
            j += run
    return sc, (i, j)


@pytest.mark.parametrize("which", ["c5", "dissimilar"])
def test_c5_fill_and_device_traceback_20k(oracle, dev, LB, which):
    """C5 as bench.py runs it: 20k x 20k affine SW (open 3 / extend 1) fill + the traceback ON THE DEVICE
    (msa_plan_traceback): score, end, begin and the full CIGAR equal the oracle's; the CIGAR re-scores
    to the optimum and ends at the end cell."""
    import torch
    from cse305_parallel_sequence_alignment_amd import data
    from cse305_parallel_sequence_alignment_amd.plan import Plan

    A, B = data.c5_pair(0) if which == "c5" else (data.bundled()[5][:20000], data.bundled()[0][:20000])
    pl = Plan(LB.SW_AFFINE, LB.CELLS_DIR, [len(A)], [len(B)], [0], [0], match=1, mismatch=0, gap_open=3,
              gap_extend=1, track_end=True)
    D = torch.empty(pl.cells_elems, dtype=torch.uint8, device=dev)
    pl.run(_dev(A, dev), _dev(B, dev), D)
    tb = pl.traceback(D)
    r = pl.results()[0]
    o = oracle.sw(A, B, 1, 0, 3, 1, want_tb=True)
    assert (r["score"], tuple(r["end"])) == (o["score"], tuple(o["end"]))
    assert tuple(tb["beg"]) == tuple(o["beg"]) and tb["cigar"] == o["cigar"]
    sc, stop = _rescore(A, B, tb["beg"], tb["cigar"], 1, 0, 3, 1)
    assert sc == r["score"] and stop == tuple(r["end"])


@pytest.mark.parametrize("m,n", [(1, 1), (64, 1), (1, 300), (65, 70), (300, 257), (1000, 1300), (2600, 900)])
@pytest.mark.parametrize("scoring", [(1, 0, 3, 1), (2, -3, 5, 2), (1, -1, 1, 1), (3, -2, 0, 0), (2, 0, 5, 2), (1, 1, 0, 0)])
def test_sw_affine_flow_dir_bytes(dev, LB, m, n, scoring):
    """The two-pass affine flow kernel (single pair, direction bytes: run_info mode 1) writes the same
    direction byte as the one-pass stripe kernel (the same pair as a one-pair batch) at every cell of the
    matrix, and the same score and first-maximum end cell.  Scores >= 0 run pass 1 with the zero floor in
    its head phases only; negative mismatches with it in every step."""
    import torch
    from cse305_parallel_sequence_alignment_amd.plan import Plan

    rng = np.random.default_rng(m * 7 + n)
    A = rs(rng, m)
    B = bytes(bytearray(A[: min(m, n)]) + rs(rng, max(0, n - m)))
    b = bytearray(B)
    for k in rng.choice(len(b), size=max(1, len(b) // 10), replace=False):
        b[k] = ACGT[rng.integers(4)]
    B = bytes(b)
    ma, mi, go, ge = scoring
    out = []
    for single in (True, False):
        pl = Plan(LB.SW_AFFINE, LB.CELLS_DIR, [m], [len(B)], [0], [0], match=ma, mismatch=mi, gap_open=go,
                  gap_extend=ge, track_end=True, single=single)
        D = torch.empty(pl.cells_elems, dtype=torch.uint8, device=dev)
        pl.run(_dev(A, dev), _dev(B, dev), D)
        r = pl.results()[0]
        info = pl.run_info()
        out.append((pl.deskew_dir(D.cpu().numpy(), 0, pl.stripe_meta()), r["score"], tuple(r["end"]), info["mode"],
                    pl.geom[0].rows_per_lane))
    (d1, s1, e1, mode1, r1), (d0, s0, e0, _, _) = out
    assert mode1 == "flow" and r1 == 2  # the flow kernel's two-rows-per-lane layout
    assert (s1, e1) == (s0, e0)
    assert np.array_equal(d1[1:, 1:], d0[1:, 1:])


@pytest.mark.parametrize("m,n", [(3000, 2900), (1500, 4100), (4097, 130)])
@pytest.mark.parametrize("scoring", [(1, 0, 3, 1), (2, -3, 5, 2), (1, -1, 1, 1)])
def test_device_traceback_multi_stripe(oracle, dev, LB, m, n, scoring):
    """Device traceback across many stripes and 16-step blocks (mutated copies: long paths with gaps)."""
    import torch
    from cse305_parallel_sequence_alignment_amd.plan import Plan

    rng = np.random.default_rng(m + n)
    A = rs(rng, m)
    b = bytearray(A[:n] if n <= m else A + rs(rng, n - m))
    for k in rng.choice(len(b), size=len(b) // 20, replace=False):
        b[k] = ACGT[rng.integers(4)]
    for k in sorted(rng.choice(len(b) - 8, size=12, replace=False), reverse=True):
        if rng.integers(2):
            del b[k:k + int(rng.integers(1, 6))]
        else:
            b[k:k] = rs(rng, int(rng.integers(1, 6)))
    B = bytes(b)
    ma, mi, go, ge = scoring
    pl = Plan(LB.SW_AFFINE, LB.CELLS_DIR, [len(A)], [len(B)], [0], [0], match=ma, mismatch=mi, gap_open=go,
              gap_extend=ge, track_end=True)
    D = torch.empty(pl.cells_elems, dtype=torch.uint8, device=dev)
    pl.run(_dev(A, dev), _dev(B, dev), D)
    tb = pl.traceback(D)
    o = oracle.sw(A, B, ma, mi, go, ge, want_tb=True)
    assert (pl.results()[0]["score"], tuple(tb["beg"]), tb["cigar"]) == (o["score"], tuple(o["beg"]), o["cigar"])


def test_plan_rejects_bad_buffers(dev, LB):
    """Plan.run checks device, dtype, contiguity and sizes before handing raw pointers to the C-ABI."""
    import torch
    from cse305_parallel_sequence_alignment_amd.plan import Plan

    pl = Plan(LB.SW_LINEAR, LB.CELLS_H, [100], [120], [0], [0], match=1, mismatch=0, gap_open=1, gap_extend=1)
    dA = torch.zeros(100, dtype=torch.uint8, device=dev)
    dB = torch.zeros(120, dtype=torch.uint8, device=dev)
    H = torch.empty(pl.cells_elems, dtype=torch.int32, device=dev)
    for bad in (dict(dA=dA[:99]), dict(dB=dB.cpu()), dict(H=H[: pl.cells_elems - 1]), dict(H=H.to(torch.int64)),
                dict(dA=dA.to(torch.int32))):
        args = dict(dA=dA, dB=dB, H=H)
        args.update(bad)
        with pytest.raises(ValueError):
            pl.run(args["dA"], args["dB"], args["H"])
    pl.run(dA, dB, H)
    assert pl.results()[0]["score"] == 100  # all-equal codes: the diagonal


def test_sticky_error_word(dev, LB):
    """The plan's error word is 0 after clean runs and survives across runs until clear_error (API check)."""
    import torch
    from cse305_parallel_sequence_alignment_amd.plan import Plan

    pl = Plan(LB.SW_LINEAR, LB.CELLS_H, [3000], [2500], [0], [0], match=1, mismatch=0, gap_open=1, gap_extend=1)
    rng = np.random.default_rng(5)
    dA, dB = _dev(rs(rng, 3000), dev), _dev(rs(rng, 2500), dev)
    H = torch.empty(pl.cells_elems, dtype=torch.int32, device=dev)
    for _ in range(50):
        pl.run(dA, dB, H)
    assert pl.error() == 0
    pl.clear_error()
    assert pl.error() == 0


def _mutated(rng, m, n):
    """B = a mutated copy of A (substitutions + short indels), trimmed / extended to n."""
    A = rs(rng, m)
    b = bytearray(A[:n] if n <= m else A + rs(rng, n - m))
    for k in rng.choice(len(b), size=max(1, len(b) // 15), replace=False):
        b[k] = ACGT[rng.integers(4)]
    return A, bytes(b[:n]) + rs(rng, max(0, n - len(b)))


@pytest.mark.parametrize("gh", [(1, 2), (2, 1), (1, 0), (3, 5)])
@pytest.mark.parametrize("st,en", [(-1, -1), (-2, -3), (-3, -2), (1, 2), (3, 1), (2, -1)])
def test_gotoh_device_walk(oracle, dev, LB, gh, st, en):
    """find_alignment ON THE DEVICE (msa_plan_traceback_gotoh) over a REF_GOTOH DIR fill: the walk's ops are
    the tables of the oracle's node list (end node first), every start / end type, several (g, h), shapes
    from one row-block to many stripes and 16-step blocks."""
    import torch
    from cse305_parallel_sequence_alignment_amd.plan import Plan

    g, h = gh
    rng = np.random.default_rng(100 + 7 * g + h + 13 * st + en)
    for (m, n) in [(1, 1), (1, 40), (5, 300), (64, 64), (65, 66), (129, 700), (700, 701), (1000, 1300)]:
        A, B = _mutated(rng, m, n) if m > 100 else (rs(rng, m), rs(rng, n))
        pl = Plan(LB.REF_GOTOH, LB.CELLS_DIR, [m], [n], [0], [0], match=1, mismatch=0, gap_open=g + h,
                  gap_extend=g, start_type=st)
        D = torch.empty(pl.cells_elems, dtype=torch.uint8, device=dev)
        pl.run(_dev(A, dev), _dev(B, dev), D)
        tb = pl.traceback_gotoh(D, end_type=en)
        o = oracle.subproblem_align(A, B, st, en, float(g), float(h))
        ts = [t for (_, _, t) in o["nodes"]]
        # op k = the table step k leaves = node t's end -> start; the end node's table first
        want = "".join("MDI"[t - 1] for t in reversed(ts)) if ts else "MDI"[o["end"][2] - 1]
        assert tb["ops"].decode() == want, (m, n, st, en)
        assert tb["ops"][:1].decode() == "MDI"[o["end"][2] - 1]
        assert min(tb["stop"]) == 0 and max(tb["stop"]) >= 0, tb["stop"]


@pytest.mark.parametrize("gh", [(1, 2), (2, 1), (1, 0), (3, 5)])
@pytest.mark.parametrize("m,n", [(1, 1), (1, 40), (5, 300), (64, 64), (65, 66), (129, 700), (1000, 1300), (2600, 900)])
def test_gotoh_flow_dir_bytes(dev, LB, gh, m, n):
    """The two-pass Gotoh flow kernel (single pair, start type -1, direction bytes: run_info mode 1) writes
    the same tag byte as the one-pass stripe kernel (the same pair as a one-pair batch) at every cell, and
    the same final-cell tables (score, find_alignment's end rule)."""
    import torch
    from cse305_parallel_sequence_alignment_amd.plan import Plan

    g, h = gh
    rng = np.random.default_rng(m * 3 + n + 17 * g + h)
    A, B = _mutated(rng, m, n) if m > 100 else (rs(rng, m), rs(rng, n))
    out = []
    for single in (True, False):
        pl = Plan(LB.REF_GOTOH, LB.CELLS_DIR, [m], [n], [0], [0], match=1, mismatch=0, gap_open=g + h,
                  gap_extend=g, start_type=-1, single=single)
        D = torch.empty(pl.cells_elems, dtype=torch.uint8, device=dev)
        pl.run(_dev(A, dev), _dev(B, dev), D)
        r = pl.results()[0]
        out.append((pl.deskew_dir(D.cpu().numpy(), 0, pl.stripe_meta()), r["score"], tuple(r["fin"]),
                    pl.run_info()["mode"]))
    (d1, s1, f1, mode1), (d0, s0, f0, _) = out
    assert mode1 == "flow"
    assert (s1, f1) == (s0, f0)
    assert np.array_equal(d1[1:, 1:] & 63, d0[1:, 1:] & 63)


def _gotoh_tags(T1, T2, T3, g, h):
    """The REF1 tag byte of every cell from the reference's double tables: bits 0-1 / 2-3 / 4-5 = 4 - the table
    find_alignment's T1 / T2 / T3 branch picks (the first of T1, T2, T3 whose candidate is the maximum,
    subproblem_alignment.cpp:150-171)."""
    def first(c):
        return 4 - np.argmax(np.stack(c), axis=0).astype(np.uint8) - 1

    t1 = first([T1[:-1, :-1], T2[:-1, :-1], T3[:-1, :-1]])
    t2 = first([T1[1:, :-1] - g - h, T2[1:, :-1] - g, T3[1:, :-1] - g - h])
    t3 = first([T1[:-1, 1:] - g - h, T2[:-1, 1:] - g - h, T3[:-1, 1:] - g])
    return t1 | (t2 << 2) | (t3 << 4)


@pytest.mark.parametrize("m,n", [(130, 45000), (300, 61000), (1000, 20100), (64, 9000)])
def test_flow_kernels_wide_pairs(oracle, dev, LB, m, n):
    """Column codes stream through fixed LDS rings in the flow kernels: pairs far wider than the former
    whole-row LDS copies (SW linear n <= ~19.5k, affine / Gotoh n <= ~37k) run the flow kernels (run_info mode
    1); the ring wraps every 4 KiB of columns.  Gotoh: the tag byte of every cell equals the one derived from
    the oracle's tables, and the device walk equals the oracle's node list; affine SW: score, end, begin and
    CIGAR of the device traceback equal the oracle's; SW linear: the checksum of the whole H matrix."""
    import torch
    from cse305_parallel_sequence_alignment_amd.plan import Plan

    rng = np.random.default_rng(m + n)
    A, B = _mutated(rng, m, n)
    dA, dB = _dev(A, dev), _dev(B, dev)
    pl = Plan(LB.REF_GOTOH, LB.CELLS_DIR, [m], [n], [0], [0], match=1, mismatch=0, gap_open=3, gap_extend=1,
              start_type=-1)
    D = torch.empty(pl.cells_elems, dtype=torch.uint8, device=dev)
    pl.run(dA, dB, D)
    assert pl.run_info()["mode"] == "flow"
    r = pl.results()[0]
    tb = pl.traceback_gotoh(D, end_type=-1)
    o = oracle.subproblem_align(A, B, -1, -1, 1.0, 2.0)
    fin = tuple(float(T[m, n]) for T in (o["T1"], o["T2"], o["T3"]))
    assert tuple(float(x) for x in r["fin"]) == fin
    ts = [t for (_, _, t) in o["nodes"]]
    assert tb["ops"].decode() == "".join("MDI"[t - 1] for t in reversed(ts))
    d = pl.deskew_dir(D.cpu().numpy(), 0, pl.stripe_meta())
    assert np.array_equal(d[1:, 1:] & 63, _gotoh_tags(o["T1"], o["T2"], o["T3"], 1.0, 2.0))
    del o, d
    pl = Plan(LB.SW_AFFINE, LB.CELLS_DIR, [m], [n], [0], [0], match=2, mismatch=-3, gap_open=5, gap_extend=2,
              track_end=True)
    D = torch.empty(pl.cells_elems, dtype=torch.uint8, device=dev)
    pl.run(dA, dB, D)
    assert pl.run_info()["mode"] == "flow"
    tb = pl.traceback(D)
    o = oracle.sw(A, B, 2, -3, 5, 2, want_tb=True)
    r = pl.results()[0]
    assert (r["score"], tuple(r["end"]), tuple(tb["beg"]), tb["cigar"]) == \
        (o["score"], tuple(o["end"]), tuple(o["beg"]), o["cigar"])
    assert pl.error() == 0
    pl = Plan(LB.SW_LINEAR, LB.CELLS_H, [m], [n], [0], [0], match=1, mismatch=0, gap_open=1, gap_extend=1)
    H = torch.empty(pl.cells_elems, dtype=torch.int32, device=dev)
    pl.run(dA, dB, H)
    o = oracle.sw(A, B, 1, 0, 1, 1, want_h=True)
    assert pl.run_info()["mode"] == "flow"
    assert pl.results()[0]["score"] == o["score"]
    assert pl.checksum(H) == oracle.checksum_h(o["H"])


@pytest.mark.parametrize("kind", ["swl_h", "swl_h_end", "swa_nneg", "swa_neg", "gotoh"])
def test_flow_fill_launch_tall_pairs(oracle, dev, LB, kind):
    """Tall-narrow pairs (70,000 x 300: ~137 pass-1 items, more flow workgroups than half the CUs) take the
    separate pass-2 launch (flow_fill_kernel, launch_info fill_grid > 0), whose instantiation pick_fill
    chooses per algorithm: SW linear with H (track_end off / on), SW affine with direction bytes (scores
    >= 0, and with a negative mismatch) and the reference's Gotoh.  Checked against the oracle: H checksum
    and score; score, end, begin and CIGAR of the device traceback; the printed alignment text."""
    import torch
    from cse305_parallel_sequence_alignment_amd import api
    from cse305_parallel_sequence_alignment_amd.plan import Plan

    m, n = 70000, 300
    rng = np.random.default_rng(7000 + len(kind))
    A = rs(rng, m)
    B = bytearray(A[20000:20000 + n])  # a local match deep in A, mutated
    for k in rng.choice(n, size=n // 12, replace=False):
        B[k] = ACGT[rng.integers(4)]
    B = bytes(B)
    dA, dB = _dev(A, dev), _dev(B, dev)
    if kind.startswith("swl"):
        te = kind == "swl_h_end"
        pl = Plan(LB.SW_LINEAR, LB.CELLS_H, [m], [n], [0], [0], match=1, mismatch=0, gap_open=1, gap_extend=1,
                  track_end=te)
        info = pl.launch_info()
        assert info["mode"] == "flow" and info["fill_grid"] > 0, info
        H = torch.empty(pl.cells_elems, dtype=torch.int32, device=dev)
        pl.run(dA, dB, H)
        o = oracle.sw(A, B, 1, 0, 1, 1, want_h=True)
        r = pl.results()[0]
        assert r["score"] == o["score"]
        if te:
            assert tuple(r["end"]) == tuple(o["end"])
        assert pl.checksum(H) == oracle.checksum_h(o["H"])
    elif kind.startswith("swa"):
        sc = (1, 0, 3, 1) if kind == "swa_nneg" else (2, -3, 5, 2)
        pl = Plan(LB.SW_AFFINE, LB.CELLS_DIR, [m], [n], [0], [0], match=sc[0], mismatch=sc[1], gap_open=sc[2],
                  gap_extend=sc[3], track_end=True)
        info = pl.launch_info()
        assert info["mode"] == "flow" and info["fill_grid"] > 0, info
        D = torch.empty(pl.cells_elems, dtype=torch.uint8, device=dev)
        pl.run(dA, dB, D)
        tb = pl.traceback(D)
        o = oracle.sw(A, B, *sc, want_tb=True)
        r = pl.results()[0]
        assert (r["score"], tuple(r["end"]), tuple(tb["beg"]), tb["cigar"]) == \
            (o["score"], tuple(o["end"]), tuple(o["beg"]), o["cigar"])
    else:
        pl = Plan(LB.REF_GOTOH, LB.CELLS_DIR, [m], [n], [0], [0], match=1, mismatch=0, gap_open=3, gap_extend=1,
                  start_type=-1)
        info = pl.launch_info()
        assert info["mode"] == "flow" and info["fill_grid"] > 0, info
        D = torch.empty(pl.cells_elems, dtype=torch.uint8, device=dev)
        pl.run(dA, dB, D)
        # the oracle's Subproblem swaps a tall pair (m > n, subproblem_alignment.h:37-54); the symmetric
        # recurrence makes the unswapped tables its transposes with T2 <-> T3: T1' = T1^T, T2' = T3^T,
        # T3' = T2^T -- the tables of this (unswapped) plan
        T1, T2, T3, inv = oracle.subproblem_tables(A, B, -1, 1.0, 2.0)
        assert inv
        T1, T2, T3 = T1.T.copy(), T3.T.copy(), T2.T.copy()
        r = pl.results()[0]
        assert tuple(float(x) for x in r["fin"]) == tuple(float(T[m, n]) for T in (T1, T2, T3))
        d = pl.deskew_dir(D.cpu().numpy(), 0, pl.stripe_meta())
        assert np.array_equal(d[1:, 1:] & 63, _gotoh_tags(T1, T2, T3, 1.0, 2.0))
    assert pl.error() == 0


@pytest.mark.parametrize("how", ["batch_of_one", "g16_single"])
def test_ref1_stripe_layout_walk(oracle, dev, LB, how):
    """The tagged REF1 fill in the one-pass stripe kernel (a one-pair batch, or a single pair whose profile bytes
    4 (f + 2g) do not fit int8, g = 16) and find_alignment's device walk over the STRIPE layout (stripe starts
    read from the meta, csflow = 0): the ops equal the oracle's node list."""
    import torch
    from cse305_parallel_sequence_alignment_amd.plan import Plan

    g, h = (1, 2) if how == "batch_of_one" else (16, 3)
    rng = np.random.default_rng(77 + g)
    for (m, n) in [(1, 1), (5, 300), (65, 66), (700, 701), (1000, 1300), (900, 2600), (3000, 3100)]:
        A, B = _mutated(rng, m, n) if m > 100 else (rs(rng, m), rs(rng, n))
        pl = Plan(LB.REF_GOTOH, LB.CELLS_DIR, [m], [n], [0], [0], match=1, mismatch=0, gap_open=g + h,
                  gap_extend=g, start_type=-1, single=(how != "batch_of_one"))
        D = torch.empty(pl.cells_elems, dtype=torch.uint8, device=dev)
        pl.run(_dev(A, dev), _dev(B, dev), D)
        assert pl.run_info()["mode"] == "stripe"
        tb = pl.traceback_gotoh(D, end_type=-1)
        o = oracle.subproblem_align(A, B, -1, -1, float(g), float(h))
        ts = [t for (_, _, t) in o["nodes"]]
        want = "".join("MDI"[t - 1] for t in reversed(ts)) if ts else "MDI"[o["end"][2] - 1]
        assert tb["ops"].decode() == want, (m, n, how)


@pytest.mark.parametrize("gap", [("B", 300), ("A", 300), ("B", 700), ("A", 70), ("both", 260)])
def test_walks_across_long_gaps(oracle, dev, LB, gap):
    """Long gaps move the walk out of its stripe group on the left (horizontal gap: an on-demand group of
    the same stripe) or into a stripe far from the predicted column (vertical gap: mispredicted prefetches):
    the reference Gotoh walk (flow kernel fill) and the SW-affine walk still equal the oracle."""
    import torch
    from cse305_parallel_sequence_alignment_amd.plan import Plan

    side, L = gap
    rng = np.random.default_rng(L + len(side))
    X, Y, Z = rs(rng, 1500), rs(rng, 1200), rs(rng, L)
    # (m <= n throughout: a Plan is not swapped the way Subproblem's constructor swaps; an extra tail on B
    # keeps the vertical-gap case m <= n)
    A, B = (X + Y, X + Z + Y) if side == "B" else \
        ((X + Z + Y, X + Y + rs(rng, L + 50)) if side == "A" else (X + Z + Y, X + Y + Z))
    m, n = len(A), len(B)
    pl = Plan(LB.REF_GOTOH, LB.CELLS_DIR, [m], [n], [0], [0], match=1, mismatch=0, gap_open=3, gap_extend=1,
              start_type=-1)
    D = torch.empty(pl.cells_elems, dtype=torch.uint8, device=dev)
    pl.run(_dev(A, dev), _dev(B, dev), D)
    assert pl.run_info()["mode"] == "flow"
    tb = pl.traceback_gotoh(D, end_type=-1)
    o = oracle.subproblem_align(A, B, -1, -1, 1.0, 2.0)
    want = "".join("MDI"[t - 1] for (_, _, t) in reversed(o["nodes"]))
    assert tb["ops"].decode() == want
    pl2 = Plan(LB.SW_AFFINE, LB.CELLS_DIR, [m], [n], [0], [0], match=2, mismatch=-1, gap_open=3, gap_extend=1,
               track_end=True)
    D2 = torch.empty(pl2.cells_elems, dtype=torch.uint8, device=dev)
    pl2.run(_dev(A, dev), _dev(B, dev), D2)
    tb2 = pl2.traceback(D2)
    o2 = oracle.sw(A, B, 2, -1, 3, 1, want_tb=True)
    assert (pl2.results()[0]["score"], tuple(tb2["beg"]), tb2["cigar"]) == (o2["score"], tuple(o2["beg"]),
                                                                           o2["cigar"])


@pytest.mark.parametrize("off", [0, 1, 7])
def test_walk_ops_unaligned_and_capped(oracle, dev, LB, off):
    """The walk's decoder wave writes diagonal runs (up to 128 'M') with 16-byte stores between byte-wise head
    and tail: into an ops buffer at any byte offset, and with a capacity below the op count, the bytes written
    are the oracle's ops up to the capacity (status MSA_ERR_CAPACITY when short) and no byte outside the
    buffer changes."""
    import torch
    from cse305_parallel_sequence_alignment_amd.plan import Plan

    rng = np.random.default_rng(91 + off)
    A, B = _mutated(rng, 3000, 3050)
    m, n = len(A), len(B)
    pl = Plan(LB.REF_GOTOH, LB.CELLS_DIR, [m], [n], [0], [0], match=1, mismatch=0, gap_open=3, gap_extend=1,
              start_type=-1)
    D = torch.empty(pl.cells_elems, dtype=torch.uint8, device=dev)
    pl.run(_dev(A, dev), _dev(B, dev), D)
    o = oracle.subproblem_align(A, B, -1, -1, 1.0, 2.0)
    want = "".join("MDI"[t - 1] for (_, _, t) in reversed(o["nodes"])).encode()
    for cap in (len(want) + 5, len(want), len(want) - 37, 21):
        big = torch.full((off + cap + 64,), 0xAA, dtype=torch.uint8, device=dev)
        info = torch.zeros(8, dtype=torch.int64, device=dev)
        pl.traceback_gotoh_async(D, big[off:off + cap], info, -1)
        inf = info.cpu().tolist()
        got = big.cpu().numpy().tobytes()
        assert inf[0] == len(want), (off, cap)
        assert inf[3] == (0 if cap >= len(want) else -8), (off, cap, inf[3])
        k = min(cap, len(want))
        assert got[off:off + k] == want[:k], (off, cap)
        assert got[:off] == b"\xaa" * off and got[off + k:] == b"\xaa" * (len(got) - off - k), (off, cap)


def test_gotoh_walk_rejects_wrong_plans(dev, LB):
    """msa_plan_traceback_gotoh needs a REF_GOTOH DIR plan and a valid end type; msa_plan_traceback needs an
    SW-affine DIR plan created with track_end (its walk starts at the fill's end cell)."""
    import torch
    from cse305_parallel_sequence_alignment_amd.plan import Plan

    rng = np.random.default_rng(5)
    A, B = rs(rng, 50), rs(rng, 60)
    ref = Plan(LB.REF_GOTOH, LB.CELLS_DIR, [50], [60], [0], [0], gap_open=3, gap_extend=1)
    D = torch.empty(ref.cells_elems, dtype=torch.uint8, device=dev)
    ref.run(_dev(A, dev), _dev(B, dev), D)
    with pytest.raises(LB.MsaError) as e:
        ref.traceback_gotoh(D, end_type=0)
    assert e.value.status == -1
    with pytest.raises(LB.MsaError) as e:
        ref.traceback(D)  # the SW walk on a Gotoh plan
    assert e.value.status == -5
    sw = Plan(LB.SW_AFFINE, LB.CELLS_DIR, [50], [60], [0], [0], match=1, mismatch=0, gap_open=3, gap_extend=1,
              track_end=False)
    D2 = torch.empty(sw.cells_elems, dtype=torch.uint8, device=dev)
    sw.run(_dev(A, dev), _dev(B, dev), D2)
    with pytest.raises(LB.MsaError) as e:
        sw.traceback(D2)  # no end cell without track_end
    assert e.value.status == -5
    with pytest.raises(LB.MsaError) as e:
        sw.traceback_gotoh(D2)
    assert e.value.status == -5


@pytest.mark.parametrize("alg", ["linear", "affine"])
def test_packed_end_tracking_mismatch_above_match(oracle, dev, LB, alg):
    """The packed first-maximum key (value << 15) is chosen from max(0, match, mismatch) * min(m, n) < 2^16:
    with mismatch > match the local scores grow by the mismatch, and the plan must still report the
    oracle's score and end cell (it picks the packed or the compare-select tracking accordingly)."""
    import torch
    from cse305_parallel_sequence_alignment_amd.plan import Plan

    rng = np.random.default_rng(21)
    for (m, n, ma, mi) in [(300, 280, 1, 3), (3000, 2900, 1, 40), (700, 650, 2, 5)]:
        A, B = rs(rng, m), rs(rng, n)
        if alg == "linear":
            pl = Plan(LB.SW_LINEAR, LB.CELLS_NONE, [m], [n], [0], [0], match=ma, mismatch=mi, gap_open=1,
                      gap_extend=1, track_end=True)
            pl.run(_dev(A, dev), _dev(B, dev))
            o = oracle.sw(A, B, ma, mi, 1, 1)
        else:
            pl = Plan(LB.SW_AFFINE, LB.CELLS_NONE, [m], [n], [0], [0], match=ma, mismatch=mi, gap_open=3,
                      gap_extend=1, track_end=True)
            pl.run(_dev(A, dev), _dev(B, dev))
            o = oracle.sw(A, B, ma, mi, 3, 1)
        r = pl.results()[0]
        assert (r["score"], tuple(r["end"])) == (o["score"], tuple(o["end"])), (m, n, ma, mi)


def test_c2_plan_under_contention(oracle, dev, LB):
    """The two-pass C2 flow kernel (pass-1 / pass-2 roles by arrival ticket) while long GEMMs occupy CUs on
    another stream: the sticky error word stays 0 and the full-H checksum equals the oracle's."""
    import torch
    from cse305_parallel_sequence_alignment_amd import data
    from cse305_parallel_sequence_alignment_amd.plan import Plan

    A, B = data.c2_pair(0)
    A, B = A[:6000], B[:6000]
    pl = Plan(LB.SW_LINEAR, LB.CELLS_H, [len(A)], [len(B)], [0], [0], match=1, mismatch=0, gap_open=1,
              gap_extend=1)
    H = torch.empty(pl.cells_elems, dtype=torch.int32, device=dev)
    dA, dB = _dev(A, dev), _dev(B, dev)
    busy = torch.cuda.Stream(device=dev)
    mine = torch.cuda.Stream(device=dev)
    x = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    torch.cuda.synchronize()
    for _ in range(3):
        with torch.cuda.stream(busy):
            for _ in range(30):
                x = torch.tanh(x @ x * 1e-3)
        pl.run(dA, dB, H, stream=mine)
    torch.cuda.synchronize()
    assert pl.error() == 0
    o = oracle.sw(A, B, 1, 0, 1, 1, want_h=True)
    assert pl.results()[0]["score"] == o["score"]
    assert pl.checksum(H) == oracle.checksum_h(o["H"])
