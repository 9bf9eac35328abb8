"""GPU parity of the reference-API layer around the fill (through libmsa.so's C-ABI):
optimal_alignment over partitions (main_alignment.cpp:202-351), the partitioned
main_alignment_function, non_parallel_tables' printed text
(subproblem_alignment.cpp:357-422), one-row subproblems, and reentrant
concurrent calls (testing.cpp:145-158 calls main_alignment_function from
hardware_concurrency threads).  All comparisons are exact."""
import json
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

OPT = json.loads((GOLDEN / "optimal.json").read_text())


def test_optimal_alignment_fixtures(dev):
    """All 77 partitions of tests/golden/optimal.json (nodes reference-produced), reference
    behaviour (2-3 subproblems: only the first solved; last link never made) and fix_all."""
    from cse305_parallel_sequence_alignment_amd import api

    for c in OPT:
        A, B = c["A"].encode(), c["B"].encode()
        for key, fix in (("ref", False), ("fix_all", True)):
            text, path = api.optimal_alignment_text(b"\0" + A, b"\0" + B, c["bp"], len(A), len(B), 4, c["g"],
                                                    c["h"], fix_all=fix)
            assert text == c[key]["text"], (c["bp"], key)
            assert [list(x) for x in path] == c[key]["path"], (c["bp"], key)


@pytest.mark.parametrize("L,p", [(300, 4), (1000, 8), (1000, 16), (2000, 5)])
def test_main_alignment_partitioned(oracle, dev, dataset, L, p):
    """GPU partition (partial.cpp, wrap) -> GPU subproblems -> stitch, against the oracle chain."""
    from cse305_parallel_sequence_alignment_amd import _lib as LB
    from cse305_parallel_sequence_alignment_amd import api

    _, seqs = dataset
    for (a, b) in ((0, 1), (10, 11), (3, 4)):
        A, B = seqs[a][:L], seqs[b][:L - 7]
        part = oracle.partial_partition(A, B, p, 1.0, 2.0, -1, -1)
        mono = all(part[k + 1][0] >= part[k][0] and part[k + 1][1] >= part[k][1] and part[k + 1][:2] != part[k][:2]
                   for k in range(len(part) - 1))
        for fix in (False, True):
            if not mono:
                with pytest.raises(LB.MsaError):
                    api.main_alignment_partitioned_text(b"\0" + A, b"\0" + B, len(A), len(B), p, 1, 2, fix)
                continue
            want, _ = oracle.optimal_alignment(A, B, part, 1.0, 2.0, fix)
            got = api.main_alignment_partitioned_text(b"\0" + A, b"\0" + B, len(A), len(B), p, 1, 2, fix)
            assert got == want, (a, b, L, p, fix)


def _lf(x: int) -> str:
    return "-inf " if x == np.iinfo(np.int32).min else "%f " % float(x)


def test_non_parallel_tables_text(dev):
    """non_parallel_tables' printed tables (subproblem_alignment.cpp:401-421, printf "%lf ") equal the
    reference-produced fixture tables printed the same way."""
    from cse305_parallel_sequence_alignment_amd import api

    paths = json.loads((GOLDEN / "subproblem_paths.json").read_text())
    tabs = np.load(GOLDEN / "subproblem_tables.npz")
    done = 0
    for c in paths:
        if c["key"] + "_T" not in tabs:
            continue
        A, B = c["A"].encode(), c["B"].encode()
        sp = api.Subproblem(b"\0" + A, b"\0" + B, len(A), len(B), 0, 0, 1, c["start"], c["end"], c["g"], c["h"])
        want = "".join(f"T{v + 1}:\n" + "".join("".join(_lf(int(x)) for x in row) + "\n" for row in T)
                       for v, T in enumerate(tabs[c["key"] + "_T"]))
        assert sp.non_parallel_tables_text() == want, c["key"]
        done += 1
    assert done >= 10


@pytest.mark.parametrize("m,n", [(0, 9), (7, 0), (0, 1)])
@pytest.mark.parametrize("st,en", [(-1, -1), (1, -2), (3, -3), (2, 1), (-2, -1)])
def test_one_row_subproblem(oracle, dev, m, n, st, en):
    """lenA = 0 or lenB = 0 (partitions on the matrix edge): row-0 borders only, no path nodes
    (alignment_begin = NULL), end node from row 0 -- as the reference's Subproblem."""
    from cse305_parallel_sequence_alignment_amd import api

    A, B = b"ACGTACGTAC", b"GATTACAGAT"
    o = oracle.subproblem_align(A, B, st, en, 1.0, 2.0, idA=2, idB=1, m=m, n=n)
    sp = api.Subproblem(b"\0" + A, b"\0" + B, m, n, 2, 1, 1, st, en, 1, 2)
    sp.compute_tables()
    for x, y in zip((sp.T1, sp.T2, sp.T3), (o["T1"], o["T2"], o["T3"])):
        assert np.array_equal(x, y)
    sp.find_alignment()
    assert sp.alignment_list() == o["nodes"] == []
    assert sp.alignment_end.as_tuple() == o["end"]


def test_concurrent_main_alignment(oracle, dev, dataset):
    """Reentrancy: 8 host threads call msa_main_alignment at once (pooled streams and device
    blocks); every call's text is byte-exact."""
    from cse305_parallel_sequence_alignment_amd import api

    _, seqs = dataset
    jobs = []
    for k in range(96):
        L = (150, 400, 1000, 64, 777, 1)[k % 6]
        a, b = k % 20, (k * 7 + 3) % 20
        jobs.append((seqs[a][:L], seqs[b][:L + (k % 5)]))
    want = [oracle.main_alignment_text(A, B)[0] for A, B in jobs]

    def one(AB):
        A, B = AB
        return api.main_alignment_text(b"\0" + A, b"\0" + B, len(A), len(B), 32, 1, 2)[0]

    with ThreadPoolExecutor(max_workers=8) as ex:
        got = list(ex.map(one, jobs))
    for g, w, (A, B) in zip(got, want, jobs):
        assert g == w, (len(A), len(B))


WHOLE = json.loads((GOLDEN / "whole.json").read_text())


@pytest.mark.parametrize("c", WHOLE, ids=[f"{c['a']}x{c['b']}_{c['m']}x{c['n']}" for c in WHOLE])
def test_main_alignment_whole_sequences(oracle, dev, dataset, c):
    """main_alignment_function at the sizes its own callers use: testing.cpp:261 / :345 align WHOLE sequences of
    the bundled file (13,309-97,409 characters).  The text (bp lines, both print_seq lines) equals the 1 B/cell
    oracle's (tests/golden/whole.json, make_whole.py; the oracle reproduces the reference's own 10k / 20k
    outputs) -- whole TP53 (also against the oracle live), 48k x 47k (m > n, > 2^31 direction bytes), a
    dissimilar 40k pair, whole ABCB1 x ABCB1 (97,409 x 97,403: 9.5 GB of direction bytes) and whole CDH1."""
    import hashlib

    from cse305_parallel_sequence_alignment_amd import api

    _, seqs = dataset
    A = seqs[c["a"]] if c["La"] is None else seqs[c["a"]][:c["La"]]
    B = seqs[c["b"]] if c["Lb"] is None else seqs[c["b"]][:c["Lb"]]
    text, score = api.main_alignment_text(b"\0" + A, b"\0" + B, len(A), len(B), 64, 1, 2)
    lines = text.split("\n")[5:7]
    assert score == c["score"] and len(lines[0]) == c["n_nodes"]
    assert hashlib.md5((lines[0] + "\n" + lines[1] + "\n").encode()).hexdigest() == c["lines_md5"]
    assert hashlib.md5(text.encode("latin-1")).hexdigest() == c["text_md5"]
    if len(A) * len(B) < 3e8:
        assert text == oracle.main_alignment_text_dir(A, B, 1, 2)[0]


def test_concurrent_main_alignment_at_size(dev, dataset):
    """8 host threads call msa_main_alignment at 10k-20k at once: several two-pass flow launches share the GPU
    (pass-1 roles by arrival ticket, the first item of every XCD chunk claimed by an early arrival); every
    text equals the reference's own output (at_size.json)."""
    import hashlib

    from cse305_parallel_sequence_alignment_amd import api

    _, seqs = dataset
    cases = [c for c in json.loads((GOLDEN / "at_size.json").read_text())] * 4

    def one(c):
        A, B = seqs[c["a"]][:c["L"]], seqs[c["b"]][:c["L"]]
        t, sc = api.main_alignment_text(b"\0" + A, b"\0" + B, c["L"], c["L"], 32, c["g"], c["h"])
        lines = t.split("\n")[5:7]
        return sc, hashlib.md5((lines[0] + "\n" + lines[1] + "\n").encode()).hexdigest()

    with ThreadPoolExecutor(max_workers=8) as ex:
        got = list(ex.map(one, cases))
    for (sc, md5), c in zip(got, cases):
        assert (sc, md5) == (c["score"], c["lines_md5"]), c


def test_concurrent_main_alignment_under_budget(dev, dataset):
    """Admission control at the drop-in boundary (the reference's callers run main_alignment_function from
    hardware_concurrency threads on whole sequences, testing.cpp:269-280 / :352-358): 8 threads x 20k calls
    under a 1 GB device budget -- one call's footprint (~0.58 GB) fits, two do not -- so the calls queue on
    the budget instead of failing; every status is OK and every text equals the reference's own output."""
    import ctypes as C
    import hashlib

    from cse305_parallel_sequence_alignment_amd import _lib as LB, api

    _, seqs = dataset
    cases = [c for c in json.loads((GOLDEN / "at_size.json").read_text()) if c["L"] == 20000] * 4
    assert len(cases) >= 8
    L = LB.lib()
    budget = 1 << 30
    LB.check(L.msa_set_device_budget(budget), "msa_set_device_budget")
    try:
        def one(c):
            A, B = seqs[c["a"]][:c["L"]], seqs[c["b"]][:c["L"]]
            t, sc = api.main_alignment_text(b"\0" + A, b"\0" + B, c["L"], c["L"], 32, c["g"], c["h"])
            lines = t.split("\n")[5:7]
            return sc, hashlib.md5((lines[0] + "\n" + lines[1] + "\n").encode()).hexdigest()

        with ThreadPoolExecutor(max_workers=8) as ex:
            got = list(ex.map(one, cases))
        info = (C.c_int64 * 5)()
        LB.check(L.msa_device_budget_info(info), "msa_device_budget_info")
    finally:
        L.msa_set_device_budget(0)
    for (sc, md5), c in zip(got, cases):
        assert (sc, md5) == (c["score"], c["lines_md5"]), c
    b, inuse, peak, waits, admitted = list(info)
    assert b == budget and inuse == 0 and admitted == len(cases)
    assert peak <= budget, (peak, budget)  # never two 20k calls admitted at once
    assert waits >= 1


def test_admission_reclaims_idle_cached_memory(dev, dataset):
    """Idle cached plans and free pool blocks count against the device budget: a call admitted while
    admitted + idle bytes exceed the budget first releases the idle memory (msa_device_memory_info's
    reclaim count moves, the idle plan bytes drop), and the results stay the reference's."""
    import ctypes as C
    import hashlib

    from cse305_parallel_sequence_alignment_amd import _lib as LB, api

    _, seqs = dataset
    c20 = [c for c in json.loads((GOLDEN / "at_size.json").read_text()) if c["L"] == 20000][0]
    c10 = [c for c in json.loads((GOLDEN / "at_size.json").read_text()) if c["L"] == 10000 and c["h"] == 2.0][0]
    L = LB.lib()
    mem = (C.c_int64 * 4)()

    def run(c):
        A, B = seqs[c["a"]][:c["L"]], seqs[c["b"]][:c["L"]]
        t, sc = api.main_alignment_text(b"\0" + A, b"\0" + B, c["L"], c["L"], 32, c["g"], c["h"])
        lines = t.split("\n")[5:7]
        assert (sc, hashlib.md5((lines[0] + "\n" + lines[1] + "\n").encode()).hexdigest()) == \
            (c["score"], c["lines_md5"]), c["L"]

    LB.check(L.msa_set_device_budget(1 << 30), "msa_set_device_budget")  # one 20k call fits, 20k + 10k do not
    try:
        run(c20)  # leaves its plan cached (idle) and its blocks pooled
        LB.check(L.msa_device_memory_info(mem), "msa_device_memory_info")
        assert mem[0] == 0 and mem[1] > 0, list(mem)
        reclaims0 = mem[3]
        run(c10)  # admitted 10k + idle 20k > 1 GB: the idle memory goes first
        LB.check(L.msa_device_memory_info(mem), "msa_device_memory_info")
        assert mem[3] == reclaims0 + 1, list(mem)
        assert mem[1] < (600 << 20), list(mem)  # only the 10k plan is cached now
        run(c20)
    finally:
        L.msa_set_device_budget(0)


# ---- the reference's class Subproblem through libmsa_compat.so (C++ drop-in) ----

ROOT = GOLDEN.parent.parent
DRIVERS = {"compat_header": ROOT / "tests" / "cpp" / "subproblem_driver",
           "reference_header": ROOT / "oracle" / "_ref" / "subproblem_driver_refhdr"}
F64 = json.loads((GOLDEN / "f64_cases.json").read_text())


def _run_driver(path, lines):
    import subprocess

    r = subprocess.run([str(path)], input="".join(lines), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    cases = r.stdout.split("END_CASE\n")[:-1]
    assert len(cases) == len(lines)
    return cases


def _parse(block):
    out = dict(T=[], nodes=None, end=None, error=None)
    rows = None
    it = iter(block.splitlines())
    for ln in it:
        if ln.startswith("INV "):
            out["invert"] = int(ln[4:])
        elif ln in ("T1", "T2", "T3"):
            rows = []
            out["T"].append(rows)
        elif ln.startswith("NODES "):
            k = int(ln[6:])
            out["nodes"] = [tuple(int(x) for x in next(it).split()) for _ in range(k)]
        elif ln.startswith("END "):
            out["end"] = tuple(int(x) for x in ln[4:].split())
        elif ln.startswith("ERROR "):
            out["error"] = ln
        elif rows is not None:
            rows.append([float.fromhex(x) for x in ln.split()])
    out["T"] = [np.array(t, dtype=np.float64) for t in out["T"]]
    return out


def _line(mode, c, g, h, p=3):
    A, B = c["A"], c["B"]
    return f"{mode} {g!r} {h!r} {c['start']} {c['end']} {p} 0 0 {len(A)} {len(B)} {A} {B}\n"


def _same(x, y, what):
    """bit-exact table equality (NaN never occurs; -0.0 == 0.0 as in the reference's comparisons)"""
    assert x.shape == y.shape, (what, x.shape, y.shape)
    bad = np.argwhere(x != y)
    assert bad.size == 0, (what, bad[:4].tolist(), [(float(x[tuple(b)]).hex(), float(y[tuple(b)]).hex())
                                                      for b in bad[:4]])


def _as_f64(t):
    return np.where(t == np.iinfo(np.int32).min, -np.inf, t.astype(np.float64))


@pytest.mark.parametrize("which", list(DRIVERS))
def test_cpp_subproblem_class_fixtures(dev, which):
    """class Subproblem (ctor, compute_tables, find_alignment) from C++ on all 41 reference-produced
    fixtures: tables and node lists bit-exact.  'reference_header' is the same driver compiled against
    the reference's own subproblem_alignment.h: libmsa_compat.so is its binary drop-in."""
    drv = DRIVERS[which]
    if not drv.exists():
        pytest.skip(f"{drv.name} not built (needs /root/reference at build time)")
    paths = json.loads((GOLDEN / "subproblem_paths.json").read_text())
    tabs = np.load(GOLDEN / "subproblem_tables.npz")
    outs = _run_driver(drv, [_line("tables", c, c["g"], c["h"]) for c in paths])
    for c, blk in zip(paths, outs):
        r = _parse(blk)
        assert r["error"] is None, (c["key"], r["error"])
        if c["key"] + "_T" in tabs:
            for x, y in zip(r["T"], tabs[c["key"] + "_T"]):
                assert np.array_equal(x, _as_f64(y)), c["key"]
        assert r["nodes"] == [tuple(x) for x in c["nodes"]], c["key"]
        assert r["end"] == tuple(c["end_node"]), c["key"]


@pytest.mark.parametrize("mode", ["tables", "rows", "maps"])
def test_cpp_subproblem_double_arithmetic(dev, mode):
    """Non-integral g, h (the reference computes in double): compute_tables / compute_row(i) /
    the static MapThread bodies on three concurrent threads reproduce the reference's own
    compute_tables() cells bit for bit (tests/golden/f64_*, reference-produced), on the GPU."""
    tabs = np.load(GOLDEN / "f64_tables.npz")
    outs = _run_driver(DRIVERS["compat_header"], [_line(mode, c, c["g"], c["h"]) for c in F64])
    for c, blk in zip(F64, outs):
        r = _parse(blk)
        assert r["error"] is None or (mode == "tables" and "no predecessor" in r["error"]), (c["key"], r["error"])
        for v, (x, y) in enumerate(zip(r["T"], tabs[c["key"] + "_C"])):
            _same(x, y, (c["key"], mode, f"T{v + 1}"))


def test_cpp_non_parallel_tables_text(dev):
    """non_parallel_tables() prints exactly the reference's text (direct recurrence, %lf), for
    integral and non-integral g, h (tests/golden/f64_cases.json, reference-produced)."""
    import hashlib

    outs = _run_driver(DRIVERS["compat_header"], [_line("nonpar", c, c["g"], c["h"]) for c in F64])
    for c, blk in zip(F64, outs):
        text = blk.split("\n", 1)[1]  # after "INV x"
        if "text" in c:
            assert text == c["text"], c["key"]
        assert hashlib.md5(text.encode()).hexdigest() == c["text_md5"], c["key"]


@pytest.mark.parametrize("mode", [0, 1])
def test_subproblem_f64_c_abi(dev, mode):
    """msa_subproblem_f64 (C-ABI): mode 0 = compute_tables' prefix-max T2, 1 = non_parallel_tables'
    direct recurrence, each bit-identical to the reference's own double tables."""
    import ctypes as C

    from cse305_parallel_sequence_alignment_amd import _lib as LB

    tabs = np.load(GOLDEN / "f64_tables.npz")
    L = LB.lib()
    for c in F64:
        A, B = b"\0" + c["A"].encode(), b"\0" + c["B"].encode()
        m, n = len(c["A"]), len(c["B"])
        mm, nn = min(m, n), max(m, n)
        T = [np.empty((mm + 1, nn + 1), dtype=np.float64) for _ in range(3)]
        inv = C.c_int()
        LB.check(L.msa_subproblem_f64(A, B, m, n, 0, 0, c["start"], c["g"], c["h"], mode,
                                      *[t.ctypes.data_as(C.c_void_p) for t in T], C.byref(inv)))
        assert bool(inv.value) == c["invert"]
        for v, (x, y) in enumerate(zip(T, tabs[c["key"] + ("_C" if mode == 0 else "_N")])):
            _same(x, y, (c["key"], mode, f"T{v + 1}"))


def test_main_alignment_non_integral(oracle, dev, dataset):
    """main_alignment_function with non-integral g, h: the double row sweep + traceback over the
    double tables.  Dyadic g, h keep every table value exact, so the oracle's direct recurrence
    equals the reference's prefix-max form here (non-dyadic tables: the f64 fixtures above)."""
    from cse305_parallel_sequence_alignment_amd import api

    _, seqs = dataset
    for (g, h) in ((0.5, 1.5), (0.25, 0.5), (2.5, 0.5)):
        A, B = seqs[2][:300], seqs[7][:280]
        want, wsc = oracle.main_alignment_text(A, B, g, h)
        got, sc = api.main_alignment_text(b"\0" + A, b"\0" + B, len(A), len(B), 8, g, h)
        assert got == want and sc == wsc


def test_harness_drivers(oracle, dev, dataset, tmp_path):
    """The build-owned harness (harness.py, testing.cpp's drivers): with rand() replayed from srand(1)
    the single-threaded driver draws known pairs and prints the oracle's text for each; the threaded
    drivers write the reference's CSV layouts."""
    import io

    from cse305_parallel_sequence_alignment_amd import harness as H

    names, seqs = [], []
    assert H.read_and_store_sequences(names, seqs) == 0
    H.c_srand(1)
    picks = [(H.c_rand() % 19, H.c_rand() % 19) for _ in range(5)]
    H.c_srand(1)
    out = io.StringIO()
    assert H.test_input_size_thread(names, seqs, test_pairs=5, input_size=300, threads=1,
                                    csv_path=str(tmp_path / "in.csv"), out=out) == 0
    want = "".join(oracle.main_alignment_text(seqs[a][:300], seqs[b][:300])[0] for a, b in picks)
    assert out.getvalue() == want
    rows = (tmp_path / "in.csv").read_text().splitlines()
    assert rows[:2] == ["Testing with different input sizes", "Test number,Input size,Execution time"]
    assert [r.split(",")[:2] for r in rows[2:]] == [[str(k), "300"] for k in range(5)]
    assert H.test_similarity(names, seqs, test_pairs=8, threads=4, csv_path=str(tmp_path / "sim.csv"),
                             max_len=400, out=io.StringIO()) == 0
    rows = (tmp_path / "sim.csv").read_text().splitlines()
    assert rows[1] == "Test number,Similarity,Execution time" and len(rows) == 10
    assert H.test_n_cores_thread(names, seqs, test_pairs=6, threads=3, csv_path=str(tmp_path / "nc.csv"),
                                 max_len=200, out=io.StringIO()) == 0
    assert len((tmp_path / "nc.csv").read_text().splitlines()) == 8


# ---- the reference's main_alignment.h and partial.h through libmsa_compat.so (C++ drop-ins) ----

OPT_DRIVERS = {"compat_header": ROOT / "tests" / "cpp" / "optimal_driver",
               "reference_header": ROOT / "oracle" / "_ref" / "optimal_driver_refhdr"}
PART_DRIVERS = {"compat_header": ROOT / "tests" / "cpp" / "partial_driver",
                "reference_header": ROOT / "oracle" / "_ref" / "partial_driver_refhdr"}
PROGRESS = "bp1\nbp1.2\nbp2\nbp3\nbp4\n"


def _driver(drivers, which):
    drv = drivers[which]
    if not drv.exists():
        pytest.skip(f"{drv.name} not built (needs /root/reference at build time)")
    return drv


def _bp_args(bp):
    return f"{len(bp)} " + " ".join(f"{i} {j} {t}" for i, j, t in bp)


def _sched_expect(bp, m, n, p):
    """main_alignment.cpp:158-200 restated: omega per subproblem, its inclusive prefix sum, and
    assign_processors as optimal_alignment calls it (:244-249)."""
    import math

    omega = [max(math.ceil((b[0] - a[0]) / (m / p)), math.ceil((b[1] - a[1]) / (n / p))) for a, b in zip(bp, bp[1:])]
    sums = list(np.cumsum(omega))

    def assign(prev, cur):
        r = prev % 3
        return (cur + 2) // 3 if r == 0 else (1 + cur // 3 if r == 1 else 1 + (cur + 1) // 3)

    procs = [assign(0, omega[0])] + [assign(sums[k - 1], omega[k]) for k in range(1, len(omega))]
    return omega, [int(x) for x in sums], procs


@pytest.mark.parametrize("which", list(OPT_DRIVERS))
def test_cpp_main_alignment_api(dev, which):
    """alignment_algorithm/main_alignment.h's API from C++ (the driver compiled against the build's header,
    and against the reference's own unmodified main_alignment.h), linked against libmsa_compat.so:
    optimal_alignment's stdout for all 77 partitions of tests/golden/optimal.json (every node
    reference-produced); OptimalAlignmentMapThread + print_align on the 41 reference-produced Subproblem
    paths; the scheduler helpers (omega, ParallelPrefix, assign_processors, the block bodies)."""
    drv = _driver(OPT_DRIVERS, which)
    lines, want = [], []
    for c in OPT:
        A, B = c["A"], c["B"]
        lines.append(f"opt {c['g']!r} {c['h']!r} 4 {len(A)} {len(B)} {A} {B} {_bp_args(c['bp'])}\n")
        want.append(c["ref"]["text"])
    paths = json.loads((GOLDEN / "subproblem_paths.json").read_text())
    for c in paths:
        A, B = c["A"], c["B"]
        lines.append(f"map {c['g']!r} {c['h']!r} 3 {c['start']} {c['end']} 0 0 {len(A)} {len(B)} {A} {B}\n")
        want.append(PROGRESS + "".join(f"({i}, {j}, {t})\n" for i, j, t in c["nodes"]) +
                    "END %d %d %d\n" % tuple(c["end_node"]))
    for c in OPT[::7]:
        m, n = len(c["A"]), len(c["B"])
        for p in (1, 3, 4, 8):
            bp = c["bp"]
            omega, sums, procs = _sched_expect(bp, m, n, p)
            lines.append(f"sched {p} {m} {n} {_bp_args(bp)}\n")
            init = list(np.cumsum(omega))
            want.append("OMEGA " + " ".join(map(str, omega)) + "\nSUMS " + " ".join(map(str, sums)) +
                        "\nPROCS " + " ".join(map(str, procs)) + "\nOMEGA1 " + " ".join(map(str, omega)) +
                        "\nINIT " + " ".join(str(int(x)) for x in init) + f" | {int(init[-1])}\n" +
                        "ADD7 " + " ".join(str(int(x) + 7) for x in init) + "\n")
    outs = _run_driver(drv, lines)
    for ln, got, exp in zip(lines, outs, want):
        assert got == exp, (ln[:120], got[-300:], exp[-300:])


@pytest.mark.parametrize("which", list(PART_DRIVERS))
def test_cpp_partial_api(oracle, dev, which):
    """sequence_alignment/partial.h's API from C++ (the driver compiled against the build's header, and
    against the reference's own unmodified partial.h), linked against libmsa_compat.so: every partition
    of partial.json (80) and partial_ties.json (116, the std::sort tie order), both through
    findPartialBalancedPartitionParallel and through the step API (initialize*, fill*Parallel,
    findPartitionParallel over the caller's tables); the six filled tables against the oracle's
    restatement (pinned to the reference's partial.cpp); score()."""
    drv = _driver(PART_DRIVERS, which)
    cases = json.loads((GOLDEN / "partial.json").read_text()) + json.loads((GOLDEN / "partial_ties.json").read_text())
    lines, want = [], []
    for c in cases:
        lines.append(f"part {c['p']} {c['g']!r} {c['h']!r} {c['start']} {c['end']} {c['A']} {c['B']}\n")
        pts = " ".join(f"{i} {j} {t}" for i, j, t in c["partition"])
        want.append(f"PART {pts}\nSTEP {pts}\n")
    tab_cases = [c for c in cases[:80:9]]
    for c in tab_cases:
        lines.append(f"tabs {c['g']!r} {c['h']!r} {c['start']} {c['end']} {c['A']} {c['B']}\n")
        T, R = oracle.partial_tables(c["A"].encode(), c["B"].encode(), c["g"], c["h"], c["start"], c["end"])
        want.append("".join(f"{nm}\n" + "".join("".join(f"{int(x)} " for x in row) + "\n" for row in tab)
                            for nm, tab in zip(("T1", "T2", "T3", "TR1", "TR2", "TR3"), T + R)))
    for a, b in (("A", "A"), ("A", "C"), ("G", "T"), ("T", "T")):
        lines.append(f"score {a} {b}\n")
        want.append(f"SCORE {0 if a == b else 1}\n")
    outs = _run_driver(drv, lines)
    for ln, got, exp in zip(lines, outs, want):
        assert got == exp, (ln[:120], got[:300], exp[:300])
