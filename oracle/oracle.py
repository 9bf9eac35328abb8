"""ctypes bindings for the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, always as the checker (never as the measured or shipped path).

* ``liboracle.so``: the C restatement in ``msa_oracle.c`` (each function cites
  the reference file:line it follows).
* ``librowsweep.so``: the reference's CPU *method* (row sweep, fresh std::threads
  per phase, prefix-max T2) restated in ``cpu_rowsweep.cpp`` -- the CPU baseline.
* ``_ref/libref_sub.so`` / ``_ref/libref_partial.so``: the reference's own
  ``subproblem_alignment.cpp`` / ``partial.cpp`` compiled unmodified from
  /root/reference (``oracle/Makefile``); present only where they were built.
"""
from __future__ import annotations

import ctypes as C
import gzip
import os
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REPO = HERE.parent
NODE_DT = np.dtype([("i", np.uint64), ("j", np.uint64), ("t", np.int32), ("pad", np.int32)])

_lib = None
_ref_sub = None
_ref_partial = None


def build(quiet: bool = True) -> None:
    """Compile liboracle.so (and oracle/_ref when /root/reference exists)."""
    import subprocess

    out = subprocess.run(["make", "-C", str(HERE)], capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError("oracle build failed:\n" + out.stdout + out.stderr)
    if not quiet:
        print(out.stdout)


# MSA_ORACLE_DIR: load liboracle.so / librowsweep.so from another build of the same sources (the
# sanitizer build, oracle/_san: tests/test_host.py::test_oracle_under_sanitizers)
LIBDIR = Path(os.environ.get("MSA_ORACLE_DIR", str(HERE)))


def lib():
    global _lib
    if _lib is None:
        path = LIBDIR / "liboracle.so"
        if not path.exists():
            build()
        L = C.CDLL(str(path))
        P = C.c_void_p
        u64 = C.c_uint64
        L.orc_subproblem_tables.argtypes = [P, P, u64, u64, u64, u64, C.c_int, C.c_double, C.c_double, P, P, P, P]
        L.orc_subproblem_traceback.argtypes = [P, P, u64, u64, u64, u64, C.c_int, C.c_double, C.c_double, P, P, P,
                                               P, u64, P, P]
        L.orc_main_alignment.argtypes = [P, P, u64, u64, C.c_double, C.c_double, P, u64, P]
        L.orc_main_alignment.restype = C.c_int64
        L.orc_main_alignment_dir.argtypes = [P, P, u64, u64, C.c_int64, C.c_int64, P, u64, P]
        L.orc_main_alignment_dir.restype = C.c_int64
        L.orc_optimal_alignment.argtypes = [P, P, u64, u64, P, u64, C.c_double, C.c_double, C.c_int, P, u64, P,
                                            u64, P]
        L.orc_optimal_alignment.restype = C.c_int64
        L.orc_partial_tables.argtypes = [P, P, u64, u64, C.c_double, C.c_double, C.c_int, C.c_int, P, P, P, P, P, P]
        L.orc_partial_partition.argtypes = [P, P, P, P, P, P, u64, u64, u64, C.c_double, P, u64, P]
        L.orc_sw.argtypes = [P, P, u64, u64, C.c_int32, C.c_int32, C.c_int32, C.c_int32, P, P, P, P, P, P, P, u64]
        L.orc_banded_ref.argtypes = [P, P, u64, u64, u64, C.c_double, C.c_double, P, P]
        L.orc_banded_ref2.argtypes = [P, P, u64, u64, u64, C.c_double, C.c_double, P, P, P]
        L.orc_checksum_h.argtypes = [P, u64, u64, u64, C.c_int64]
        L.orc_checksum_h.restype = C.c_uint64
        L.orc_mix.argtypes = [u64, u64]
        L.orc_mix.restype = C.c_uint64
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


def _bytes1(s: bytes) -> np.ndarray:
    """1-based buffer like the reference harness (testing.cpp:124-128): slot 0 unused."""
    buf = np.zeros(len(s) + 2, dtype=np.uint8)
    buf[1:1 + len(s)] = np.frombuffer(s, dtype=np.uint8)
    return buf


def _bytes0(s: bytes) -> np.ndarray:
    buf = np.zeros(len(s) + 1, dtype=np.uint8)
    buf[:len(s)] = np.frombuffer(s, dtype=np.uint8)
    return buf


def subproblem_tables(A: bytes, B: bytes, start_type=-1, g=1.0, h=2.0, idA=0, idB=0, m=None, n=None):
    """Reference Subproblem tables for 0-based python strings A, B (placed 1-based).

    Returns (T1, T2, T3, invert) with shape (m'+1, n'+1) after the ctor swap."""
    a, b = _bytes1(A), _bytes1(B)
    m = len(A) - idA if m is None else m
    n = len(B) - idB if n is None else n
    mm, nn = min(m, n), max(m, n)
    T = [np.empty((mm + 1, nn + 1), dtype=np.float64) for _ in range(3)]
    inv = C.c_int(0)
    rc = lib().orc_subproblem_tables(_ptr(a), _ptr(b), m, n, idA, idB, start_type, g, h, _ptr(T[0]), _ptr(T[1]),
                                     _ptr(T[2]), C.byref(inv))
    assert rc == 0
    return T[0], T[1], T[2], bool(inv.value)


def subproblem_align(A: bytes, B: bytes, start_type=-1, end_type=-1, g=1.0, h=2.0, idA=0, idB=0, m=None, n=None):
    """Tables + find_alignment. Returns dict(nodes=[(i,j,t)...], end=(i,j,t), invert, T1,T2,T3)."""
    T1, T2, T3, inv = subproblem_tables(A, B, start_type, g, h, idA, idB, m, n)
    a, b = _bytes1(A), _bytes1(B)
    m = len(A) - idA if m is None else m
    n = len(B) - idB if n is None else n
    if inv:
        a, b, m, n, idA, idB = b, a, n, m, idB, idA
    cap = m + n + 2
    nodes = np.zeros(cap, dtype=NODE_DT)
    nn = C.c_uint64(0)
    endn = np.zeros(1, dtype=NODE_DT)
    rc = lib().orc_subproblem_traceback(_ptr(a), _ptr(b), m, n, idA, idB, end_type, g, h, _ptr(T1), _ptr(T2),
                                        _ptr(T3), _ptr(nodes), cap, C.byref(nn), _ptr(endn))
    if rc != 0:
        raise RuntimeError(f"oracle traceback rc={rc}")
    k = nn.value
    out = [(int(x["i"]), int(x["j"]), int(x["t"])) for x in nodes[:k]]
    e = endn[0]
    return dict(nodes=out, end=(int(e["i"]), int(e["j"]), int(e["t"])), invert=inv, T1=T1, T2=T2, T3=T3)


def main_alignment_text(A: bytes, B: bytes, g=1.0, h=2.0):
    """stdout of the reference main_alignment_function(A1,B1,len(A),len(B),p,g,h); returns (text, score)."""
    a, b = _bytes1(A), _bytes1(B)
    cap = 64 + 2 * (len(A) + len(B) + 4)
    out = np.zeros(cap, dtype=np.uint8)
    score = C.c_double(0)
    rc = lib().orc_main_alignment(_ptr(a), _ptr(b), len(A), len(B), g, h, _ptr(out), cap, C.byref(score))
    if rc < 0:
        raise RuntimeError(f"oracle main_alignment rc={rc}")
    return out[:rc].tobytes().decode("latin-1"), score.value


def main_alignment_text_dir(A: bytes, B: bytes, g=1, h=2):
    """main_alignment_text for integral g, h in 1 B/cell (orc_main_alignment_dir): the reference
    callers' whole-sequence sizes (13k-97k) without three (m+1)(n+1) double tables."""
    a, b = _bytes1(A), _bytes1(B)
    cap = 64 + 2 * (len(A) + len(B) + 4)
    out = np.zeros(cap, dtype=np.uint8)
    score = C.c_int64(0)
    rc = lib().orc_main_alignment_dir(_ptr(a), _ptr(b), len(A), len(B), int(g), int(h), _ptr(out), cap,
                                      C.byref(score))
    if rc < 0:
        raise RuntimeError(f"oracle main_alignment_dir rc={rc}")
    return out[:rc].tobytes().decode("latin-1"), float(score.value)


def optimal_alignment(A: bytes, B: bytes, bp, g=1.0, h=2.0, fix_all=False):
    """optimal_alignment (main_alignment.cpp:202-351) over partition bp [(i, j, t), ...] for
    0-based python strings A, B (placed 1-based).  Returns (stdout text, stitched path)."""
    a, b = _bytes1(A), _bytes1(B)
    arr = np.zeros(len(bp), dtype=NODE_DT)
    for k, (i, j, t) in enumerate(bp):
        arr[k]["i"], arr[k]["j"], arr[k]["t"] = i, j, t
    cap = 64 * len(bp) + 2 * (len(A) + len(B) + 4)
    out = np.zeros(cap, dtype=np.uint8)
    pcap = len(A) + len(B) + 2 * len(bp) + 2
    path = np.zeros(pcap, dtype=NODE_DT)
    npath = C.c_uint64(0)
    rc = lib().orc_optimal_alignment(_ptr(a), _ptr(b), len(A), len(B), _ptr(arr), len(bp), g, h,
                                     1 if fix_all else 0, _ptr(out), cap, _ptr(path), pcap, C.byref(npath))
    if rc < 0:
        raise RuntimeError(f"oracle optimal_alignment rc={rc}")
    nodes = [(int(x["i"]), int(x["j"]), int(x["t"])) for x in path[:npath.value]]
    return out[:rc].tobytes().decode("latin-1"), nodes


def partial_tables(A: bytes, B: bytes, g=1.0, h=2.0, start_type=1, end_type=1):
    a, b = _bytes0(A), _bytes0(B)
    m, n = len(A), len(B)
    T = [np.empty((m + 1, n + 1), dtype=np.int32) for _ in range(3)]
    R = [np.empty((m + 2, n + 2), dtype=np.int32) for _ in range(3)]
    rc = lib().orc_partial_tables(_ptr(a), _ptr(b), m, n, g, h, start_type, end_type, *[_ptr(x) for x in T + R])
    assert rc == 0
    return T, R


def partial_partition(A: bytes, B: bytes, p: int, g=1.0, h=2.0, start_type=1, end_type=1):
    """findPartialBalancedPartitionParallel restated; returns [(i, j, t), ...]."""
    T, R = partial_tables(A, B, g, h, start_type, end_type)
    out = np.zeros(p + 1, dtype=NODE_DT)
    nout = C.c_uint64(0)
    rc = lib().orc_partial_partition(*[_ptr(x) for x in T + R], len(A), len(B), p, h, _ptr(out), p + 1,
                                     C.byref(nout))
    assert rc == 0, rc
    return [(int(x["i"]), int(x["j"]), int(x["t"])) for x in out[:nout.value]]


def sw(A: bytes, B: bytes, match=1, mismatch=0, gap_open=1, gap_extend=1, want_h=False, want_tb=False):
    """Smith-Waterman local (build extension). Returns dict(score, end, [H], [beg, cigar])."""
    a, b = _bytes0(A), _bytes0(B)
    m, n = len(A), len(B)
    H = np.empty((m + 1, n + 1), dtype=np.int32) if want_h else None
    sc = C.c_int32(0)
    ei, ej, bi, bj = C.c_uint64(0), C.c_uint64(0), C.c_uint64(0), C.c_uint64(0)
    cig = np.zeros(4 * (m + n) + 16, dtype=np.uint8) if want_tb else None
    rc = lib().orc_sw(_ptr(a), _ptr(b), m, n, match, mismatch, gap_open, gap_extend, _ptr(H), C.byref(sc),
                      C.byref(ei), C.byref(ej), C.byref(bi) if want_tb else None, C.byref(bj) if want_tb else None,
                      _ptr(cig), 0 if cig is None else len(cig))
    assert rc == 0, rc
    r = dict(score=sc.value, end=(ei.value, ej.value))
    if want_h:
        r["H"] = H
    if want_tb:
        r["beg"] = (bi.value, bj.value)
        r["cigar"] = bytes(cig[:np.argmin(cig)]).decode()
    return r


def banded_ref(A: bytes, B: bytes, w: int, g=1.0, h=2.0, want_h=False, want_digest=False):
    """Banded reference Gotoh: score [, H] [, in-band H digest = checksum_h(H, w) without materialising H]."""
    a, b = _bytes0(A), _bytes0(B)
    m, n = len(A), len(B)
    H = np.empty((m + 1, n + 1), dtype=np.int32) if want_h else None
    sc = C.c_double(0)
    dg = C.c_uint64(0)
    rc = lib().orc_banded_ref2(_ptr(a), _ptr(b), m, n, w, g, h, _ptr(H), C.byref(sc),
                               C.byref(dg) if want_digest else None)
    assert rc == 0, rc
    out = [sc.value] + ([H] if want_h else []) + ([int(dg.value)] if want_digest else [])
    return out[0] if len(out) == 1 else tuple(out)


def checksum_h(H: np.ndarray, w: int = -1) -> int:
    H = np.ascontiguousarray(H, dtype=np.int32)
    m, n = H.shape[0] - 1, H.shape[1] - 1
    return int(lib().orc_checksum_h(_ptr(H), m, n, H.shape[1], w))


def mix_matrix(m: int, n: int) -> np.ndarray:
    """uint64 weights mix(i,j) for i in [0,m], j in [0,n] (numpy restatement of orc_mix)."""
    i = np.arange(m + 1, dtype=np.uint64)[:, None]
    j = np.arange(n + 1, dtype=np.uint64)[None, :]
    x = (i << np.uint64(32)) | j
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        x = x ^ (x >> np.uint64(31))
    return x | np.uint64(1)


_rowsweep = None


def rowsweep(A: bytes, B: bytes, p: int = 1, mode: int = 1, g=1.0, h=2.0, match=1, mismatch=0, rows=0):
    """The reference's CPU method (cpu_rowsweep.cpp): row sweep with p' fresh threads per phase.

    mode 0 = the reference's global Gotoh (double), mode 1 = SW linear int32 (C2/C4).
    Fills rows 1..rows (0 = all); returns (score, seconds)."""
    global _rowsweep
    if _rowsweep is None:
        path = LIBDIR / "librowsweep.so"
        if not path.exists():
            build()
        L = C.CDLL(str(path))
        L.cpu_rowsweep.argtypes = [C.c_int, C.c_char_p, C.c_char_p, C.c_size_t, C.c_size_t, C.c_size_t, C.c_double,
                                   C.c_double, C.c_int, C.c_int, C.c_size_t, C.POINTER(C.c_double),
                                   C.POINTER(C.c_double)]
        _rowsweep = L
    sc, secs = C.c_double(), C.c_double()
    rc = _rowsweep.cpu_rowsweep(mode, A, B, len(A), len(B), p, g, h, match, mismatch, rows, C.byref(sc),
                                C.byref(secs))
    assert rc == 0, rc
    return sc.value, secs.value


# ----------------------------------------------------------------------------
# The reference's own code (oracle/_ref) -- only where it was built.
# ----------------------------------------------------------------------------

def ref_available() -> bool:
    return (HERE / "_ref" / "libref_sub.so").exists() and (HERE / "_ref" / "libref_partial.so").exists()


def ref_sub():
    global _ref_sub
    if _ref_sub is None:
        L = C.CDLL(str(HERE / "_ref" / "libref_sub.so"))
        P = C.c_void_p
        s = C.c_size_t
        L.ref_subproblem.argtypes = [P, P, s, s, s, s, s, C.c_int, C.c_int, C.c_double, C.c_double, P, P, P, P, s,
                                     P, P, P, P, P, P, P, P]
        _ref_sub = L
    return _ref_sub


def ref_partial_lib():
    global _ref_partial
    if _ref_partial is None:
        L = C.CDLL(str(HERE / "_ref" / "libref_partial.so"))
        P = C.c_void_p
        s = C.c_size_t
        L.ref_partial.argtypes = [P, P, s, s, s, C.c_double, C.c_double, C.c_int, C.c_int, s, P, P, P, P]
        L.ref_partial_tables.argtypes = [P, P, s, s, s, C.c_double, C.c_double, C.c_int, C.c_int, P, P, P, P, P, P]
        _ref_partial = L
    return _ref_partial


def ref_subproblem(A: bytes, B: bytes, start_type=-1, end_type=-1, g=1.0, h=2.0, p=1, idA=0, idB=0, m=None,
                   n=None, tables=True, traceback=True, digest=False):
    """Run the reference's own Subproblem (compute_tables + find_alignment).

    Always returns the final cell ``fin`` = (T1, T2, T3)[m'][n']; ``digest`` adds
    ``h_digest`` = checksum_h of H = max(T1, T2, T3) computed inside the driver."""
    a, b = _bytes1(A), _bytes1(B)
    m = len(A) - idA if m is None else m
    n = len(B) - idB if n is None else n
    mm, nn = min(m, n), max(m, n)
    T = [np.empty((mm + 1, nn + 1), dtype=np.float64) for _ in range(3)] if tables else [None] * 3
    cap = (m + n + 2) if traceback else 0
    ni = np.zeros(max(cap, 1), dtype=np.uint64)
    nj = np.zeros(max(cap, 1), dtype=np.uint64)
    nt = np.zeros(max(cap, 1), dtype=np.int32)
    endn = np.zeros(3, dtype=np.uint64)
    inv = C.c_int(0)
    nn_ = C.c_size_t(0)
    secs = C.c_double(0)
    fin = np.zeros(3, dtype=np.float64)
    dg = C.c_uint64(0)
    ref_sub().ref_subproblem(_ptr(a), _ptr(b), m, n, idA, idB, p, start_type, end_type, g, h, _ptr(T[0]),
                             _ptr(T[1]), _ptr(T[2]), C.byref(inv), cap, C.byref(nn_), _ptr(ni), _ptr(nj), _ptr(nt),
                             _ptr(endn), C.byref(secs), _ptr(fin), C.byref(dg) if digest else None)
    r = dict(invert=bool(inv.value), T1=T[0], T2=T[1], T3=T[2], fill_seconds=secs.value, fin=tuple(fin.tolist()))
    if digest:
        r["h_digest"] = int(dg.value)
    if traceback:
        k = nn_.value
        r["nodes"] = [(int(ni[q]), int(nj[q]), int(nt[q])) for q in range(k)]
        r["end"] = (int(endn[0]), int(endn[1]), int(np.int64(endn[2].astype(np.int64))))
    return r


def ref_partial(A: bytes, B: bytes, p: int, g=1.0, h=2.0, start_type=1, end_type=1):
    a, b = _bytes0(A), _bytes0(B)
    cap = p + 2
    oi = np.zeros(cap, dtype=np.uint64)
    oj = np.zeros(cap, dtype=np.uint64)
    ot = np.zeros(cap, dtype=np.int32)
    nout = C.c_size_t(0)
    ref_partial_lib().ref_partial(_ptr(a), _ptr(b), len(A), len(B), p, g, h, start_type, end_type, cap,
                                  C.byref(nout), _ptr(oi), _ptr(oj), _ptr(ot))
    return [(int(oi[k]), int(oj[k]), int(ot[k])) for k in range(nout.value)]


def ref_partial_tables(A: bytes, B: bytes, g=1.0, h=2.0, start_type=1, end_type=1, p=1):
    a, b = _bytes0(A), _bytes0(B)
    m, n = len(A), len(B)
    T = [np.empty((m + 1, n + 1), dtype=np.int32) for _ in range(3)]
    R = [np.empty((m + 2, n + 2), dtype=np.int32) for _ in range(3)]
    ref_partial_lib().ref_partial_tables(_ptr(a), _ptr(b), m, n, p, g, h, start_type, end_type,
                                         *[_ptr(x) for x in T + R])
    return T, R


# ----------------------------------------------------------------------------
# dataset (tests/golden/gene_sequences_test.gz, a copy of the reference's
# bundled FASTA data file) -- FASTA parse as read_and_store_sequences
# (test_functions/pull_data.cpp:18-71)
# ----------------------------------------------------------------------------

def load_dataset():
    path = REPO / "tests" / "golden" / "gene_sequences_test.gz"
    names, seqs, cur = [], [], []
    with gzip.open(path, "rb") as f:
        for line in f.read().split(b"\n"):
            if line[:1] == b">":
                if cur:
                    seqs.append(b"".join(cur))
                    cur = []
                names.append(line.decode())
            else:
                cur.append(line)
    if cur:
        seqs.append(b"".join(cur))
    return names, seqs
