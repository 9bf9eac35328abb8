"""Python mirror of the reference's C++ interface for the hot path.

Same names and argument meanings as the reference headers; every call goes
through libmsa.so's C-ABI into the gfx950 kernels (no CPU fallback; a missing
library or GPU raises ``MsaError`` / ``ImportError``).

Reference interfaces mirrored (D-2n/CSE305_Parallel_Sequence_Alignment):
  main_alignment_function   alignment_algorithm/main_alignment.h:38, .cpp:353-410
  optimal_alignment         main_alignment.h:34, .cpp:158-351 (multi-subproblem stitch)
  Subproblem                alignment_algorithm/subproblem_alignment.h:16-97
  Align                     subproblem_alignment.h:8-13 (``align``)
  findPartialBalancedPartitionParallel  sequence_alignment/partial.h:41, partial.cpp:149-163
  partial tables            partial.h:25-35 (initialize*/fill*Parallel)

Character buffers follow the reference: ``A``/``B`` passed to
``main_alignment_function`` and ``Subproblem`` are 1-based (element 0 is
never read, testing.cpp:124-128); the partial.cpp functions read A[i-1].
"""
from __future__ import annotations

import ctypes as C
import sys
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

from . import _lib as LB


def _buf(x) -> bytes:
    if isinstance(x, str):
        x = x.encode("latin-1")
    return bytes(x)


@dataclass
class Align:
    """``align`` (subproblem_alignment.h:8-13): a path node; ``next`` links the list."""
    i: int
    j: int
    t: int
    next: Optional["Align"] = field(default=None, repr=False)

    def as_tuple(self):
        return (self.i, self.j, self.t)


def _link(nodes: List[Align]) -> Optional[Align]:
    for a, b in zip(nodes, nodes[1:]):
        a.next = b
    return nodes[0] if nodes else None


def main_alignment_text(A: bytes, B: bytes, m: int, n: int, p: int = 32, g: float = 1.0, h: float = 2.0):
    """The exact stdout of ``main_alignment_function`` and the score max(T1,T2,T3)[m][n]."""
    A, B = _buf(A), _buf(B)
    if len(A) < m + 1 or len(B) < n + 1:
        raise ValueError("A/B must be 1-based buffers of at least m+1 / n+1 bytes")
    L = LB.lib()
    need = C.c_size_t()
    score = C.c_double()
    # five progress lines + two alignment lines of at most m+n characters: one call fits
    buf = C.create_string_buffer(64 + 2 * (m + n + 2))
    LB.check(L.msa_main_alignment(A, B, m, n, p, g, h, buf, len(buf), C.byref(need), C.byref(score)),
             "msa_main_alignment")
    return buf.raw[:need.value].decode("latin-1"), score.value


def main_alignment_function(A: bytes, B: bytes, m: int, n: int, p: int, g: float, h: float) -> int:
    """Drop-in for ``int main_alignment_function(char*,char*,size_t,size_t,size_t,double,double)``:
    prints the same lines as the reference and returns 0."""
    text, _ = main_alignment_text(A, B, m, n, p, g, h)
    sys.stdout.write(text)
    sys.stdout.flush()
    return 0


class Subproblem:
    """``class Subproblem`` (subproblem_alignment.h:16-97) backed by the GPU fill.

    After ``compute_tables()`` the public ``T1``, ``T2``, ``T3`` are float64
    (m+1) x (n+1) arrays with ``-inf`` where the reference holds -infinity.
    """

    def __init__(self, A, B, m, n, id_A, id_B, p, start, end, g, h):
        A, B = _buf(A), _buf(B)
        # constructor swap (subproblem_alignment.h:37-54)
        if m <= n:
            self.A, self.B, self.m, self.n, self.id_A, self.id_B, self.invert = A, B, m, n, id_A, id_B, False
        else:
            self.A, self.B, self.m, self.n, self.id_A, self.id_B, self.invert = B, A, n, m, id_B, id_A, True
        self._orig = (A, B, m, n, id_A, id_B)
        self.p = p
        self.start_type = start
        self.end_type = end
        self.g = float(g)
        self.h = float(h)
        self.T1 = self.T2 = self.T3 = None
        self.alignment_begin: Optional[Align] = None
        self.alignment_end: Optional[Align] = None
        self._tables_int = None

    # subproblem_alignment.h:83-88
    def f(self, i: int, j: int) -> float:
        return 1.0 if self.A[self.id_A + i] == self.B[self.id_B + j] else 0.0

    # subproblem_alignment.h:91-96
    def h_prime(self, k: int) -> float:
        return self.h if (k == self.end_type and self.end_type <= -2) else 0.0

    def _call(self, tables: bool, nodes: bool):
        A, B, m, n, ida, idb = self._orig
        L = LB.lib()
        mm, nn = self.m, self.n
        T = [np.empty((mm + 1, nn + 1), dtype=np.int32) for _ in range(3)] if tables else [None] * 3
        cap = (m + n + 2) if nodes else 0
        nd = (LB.Node * max(cap, 1))()
        nn_ = C.c_size_t()
        endn = LB.Node()
        inv = C.c_int()
        tp = [t.ctypes.data_as(C.c_void_p) if t is not None else None for t in T]
        LB.check(L.msa_subproblem(A, B, m, n, ida, idb, self.start_type, self.end_type, self.g, self.h, tp[0], tp[1],
                                  tp[2], nd if nodes else None, cap, C.byref(nn_), C.byref(endn), C.byref(inv)),
                 "msa_subproblem")
        return T, [(nd[k].i, nd[k].j, nd[k].t) for k in range(nn_.value)] if nodes else None, endn

    def compute_tables(self) -> None:
        """subproblem_alignment.cpp:329-355 (the parallel row sweep) -- on the GPU."""
        T, _, _ = self._call(tables=True, nodes=False)
        self._tables_int = T
        conv = lambda t: np.where(t == np.iinfo(np.int32).min, -np.inf, t.astype(np.float64))
        self.T1, self.T2, self.T3 = (conv(t) for t in T)

    def non_parallel_tables_text(self) -> str:
        """The text subproblem_alignment.cpp:401-421 prints, from the GPU tables (msa_non_parallel_tables)."""
        A, B, m, n, ida, idb = self._orig
        L = LB.lib()
        need = C.c_size_t()
        LB.check(L.msa_non_parallel_tables(A, B, m, n, ida, idb, self.start_type, self.end_type, self.g, self.h,
                                           None, 0, C.byref(need)), "msa_non_parallel_tables")
        buf = C.create_string_buffer(need.value + 1)
        LB.check(L.msa_non_parallel_tables(A, B, m, n, ida, idb, self.start_type, self.end_type, self.g, self.h,
                                           buf, need.value + 1, C.byref(need)), "msa_non_parallel_tables")
        return buf.raw[:need.value].decode("latin-1")

    def non_parallel_tables(self) -> None:
        """subproblem_alignment.cpp:357-422: the same tables (GPU fill), printed as the reference does."""
        self.compute_tables()
        sys.stdout.write(self.non_parallel_tables_text())
        sys.stdout.flush()

    def find_alignment(self) -> None:
        """subproblem_alignment.cpp:105-172 (tie order, quirks Q1/Q2 included)."""
        _, nodes, endn = self._call(tables=False, nodes=True)
        objs = [Align(int(i), int(j), int(t)) for (i, j, t) in nodes]
        # the list runs alignment_begin -> ... -> alignment_end (the (m, n) node)
        self.alignment_begin = _link(objs)
        self.alignment_end = objs[-1] if objs else Align(int(endn.i), int(endn.j), int(endn.t))

    def alignment_list(self):
        out, a = [], self.alignment_begin
        while a is not None:
            out.append(a.as_tuple())
            a = a.next
        return out

    def print_alignment(self) -> None:
        """subproblem_alignment.cpp:174-180."""
        for (i, j, t) in self.alignment_list():
            print(f"({i}, {j}, {t})")


def _nodes_in(partial_bp):
    arr = (LB.Node * max(1, len(partial_bp)))()
    for k, a in enumerate(partial_bp):
        i, j, t = a.as_tuple() if isinstance(a, Align) else a
        arr[k].i, arr[k].j, arr[k].t = i, j, t
    return arr


def optimal_alignment_text(A, B, partial_bp, m, n, p=32, g=1.0, h=2.0, fix_all=False):
    """``optimal_alignment`` (main_alignment.cpp:202-351) over the partition ``partial_bp``
    (Align nodes or (i, j, t) tuples): returns (stdout text, stitched path as (i, j, t) tuples).

    fix_all=False keeps the reference's behaviour (2-3 subproblems: only the first is
    solved; the link into the last subproblem is never made, :344-348)."""
    A, B = _buf(A), _buf(B)
    if len(A) < m + 1 or len(B) < n + 1:
        raise ValueError("A/B must be 1-based buffers of at least m+1 / n+1 bytes")
    L = LB.lib()
    bp = _nodes_in(partial_bp)
    fl = 1 if fix_all else 0
    need, npath = C.c_size_t(), C.c_size_t()
    cap = m + n + 2 * len(partial_bp) + 2
    path = (LB.Node * cap)()
    LB.check(L.msa_optimal_alignment(A, B, m, n, p, g, h, bp, len(partial_bp), fl, None, 0, C.byref(need), path,
                                     cap, C.byref(npath)), "msa_optimal_alignment")
    buf = C.create_string_buffer(need.value + 1)
    LB.check(L.msa_optimal_alignment(A, B, m, n, p, g, h, bp, len(partial_bp), fl, buf, need.value + 1,
                                     C.byref(need), None, 0, None), "msa_optimal_alignment")
    nodes = [(int(path[k].i), int(path[k].j), int(path[k].t)) for k in range(npath.value)]
    return buf.raw[:need.value].decode("latin-1"), nodes


def optimal_alignment(A, B, partial_bp, m, n, p, g, h) -> None:
    """Drop-in for ``void optimal_alignment(char*, char*, std::vector<align>, size_t m, size_t n,
    size_t p, double g, double h)``: prints what the reference prints."""
    text, _ = optimal_alignment_text(A, B, partial_bp, m, n, p, g, h)
    sys.stdout.write(text)
    sys.stdout.flush()


def main_alignment_partitioned_text(A, B, m, n, p=4, g=1.0, h=2.0, fix_all=False) -> str:
    """main_alignment_function with its commented-out partition step enabled
    (main_alignment.cpp:365,372): GPU partition -> optimal_alignment."""
    A, B = _buf(A), _buf(B)
    if len(A) < m + 1 or len(B) < n + 1:
        raise ValueError("A/B must be 1-based buffers of at least m+1 / n+1 bytes")
    L = LB.lib()
    need = C.c_size_t()
    fl = 1 if fix_all else 0
    LB.check(L.msa_main_alignment_partitioned(A, B, m, n, p, g, h, fl, None, 0, C.byref(need)),
             "msa_main_alignment_partitioned")
    buf = C.create_string_buffer(need.value + 1)
    LB.check(L.msa_main_alignment_partitioned(A, B, m, n, p, g, h, fl, buf, need.value + 1, C.byref(need)),
             "msa_main_alignment_partitioned")
    return buf.raw[:need.value].decode("latin-1")


def print_seq(A: bytes, B: bytes, begin: Optional[Align]) -> str:
    """main_alignment.cpp:32-55 (returns the two lines instead of printing)."""
    A, B = _buf(A), _buf(B)
    l1, l2 = [], []
    a = begin
    while a is not None:
        l1.append(chr(A[a.i]) if a.t in (1, 3) and a.i < len(A) else ("?" if a.t in (1, 3) else "-"))
        l2.append(chr(B[a.j]) if a.t in (1, 2) and a.j < len(B) else ("?" if a.t in (1, 2) else "-"))
        a = a.next
    return "".join(l1) + "\n" + "".join(l2) + "\n"


def findPartialBalancedPartitionParallel(A, B, m, n, p, g, h, start_type, end_type, partition=None) -> List[Align]:
    """partial.cpp:149-163 (int32 wrap semantics, as the reference's -O0 build)."""
    A, B = _buf(A), _buf(B)
    out = (LB.Node * (p + 2))()
    nout = C.c_size_t()
    LB.check(LB.lib().msa_partial_partition(A, B, m, n, p, g, h, start_type, end_type, out, p + 2, C.byref(nout)),
             "msa_partial_partition")
    res = [Align(int(out[k].i), int(out[k].j), int(out[k].t)) for k in range(nout.value)]
    if partition is not None:
        partition.clear()
        partition.extend(res)
    return res


def partial_tables(A, B, m, n, g, h, start_type, end_type):
    """The six int32 tables partial.cpp builds (T* (m+1)x(n+1), TR* (m+2)x(n+2))."""
    A, B = _buf(A), _buf(B)
    T = [np.empty((m + 1, n + 1), dtype=np.int32) for _ in range(3)]
    R = [np.empty((m + 2, n + 2), dtype=np.int32) for _ in range(3)]
    ptr = [x.ctypes.data_as(C.c_void_p) for x in T + R]
    LB.check(LB.lib().msa_partial_tables(A, B, m, n, g, h, start_type, end_type, *ptr), "msa_partial_tables")
    return T, R


def sw_align(A, B, match=1, mismatch=0, gap_open=1, gap_extend=1, traceback=True):
    """Smith-Waterman local alignment (build extension) -> dict(score, end, beg, cigar)."""
    A, B = _buf(A), _buf(B)
    sc = C.c_int32()
    ei, ej, bi, bj = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int64()
    cap = 4 * (len(A) + len(B)) + 16
    cig = C.create_string_buffer(cap) if traceback else None
    LB.check(LB.lib().msa_sw_align(A, len(A), B, len(B), match, mismatch, gap_open, gap_extend, C.byref(sc),
                                   C.byref(ei), C.byref(ej), C.byref(bi) if traceback else None,
                                   C.byref(bj) if traceback else None, cig, cap if traceback else 0),
             "msa_sw_align")
    r = dict(score=sc.value, end=(ei.value, ej.value))
    if traceback:
        r["beg"] = (bi.value, bj.value)
        r["cigar"] = cig.value.decode()
    return r
