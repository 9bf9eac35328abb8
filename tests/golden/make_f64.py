"""Golden fixtures for the reference's DOUBLE arithmetic (any g, h), produced by the
reference's own Subproblem (alignment_algorithm/subproblem_alignment.cpp compiled
unmodified into oracle/_ref/libref_sub.so, driver oracle/ref_sub_driver.cpp):

  * compute_tables() (:329-355, T2 by omega + prefix max) -> "<key>_C" tables
  * non_parallel_tables() (:357-422, T2 by the direct recurrence) -> "<key>_N" tables,
    and the text it prints -> f64_cases.json "text" (md5 for the larger cases)

For non-integral g, h the two forms round differently, so both are pinned.
Tracebacks are not fixtures here: with non-integral g, h the reference's
find_alignment compares differently-rounded expressions and can loop forever.

    python tests/golden/make_f64.py   ->  tests/golden/f64_tables.npz, f64_cases.json
"""
from __future__ import annotations

import ctypes as C
import hashlib
import json
import sys
import tempfile
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent.parent))
from oracle import oracle as O  # noqa: E402

GH = [(0.7, 1.3), (1.1, 0.35), (0.25, 0.1), (1.0, 2.0), (0.3, -0.2)]
TYPES = [-1, -2, -3, 1, 2, 3]


def ref_non_parallel(A: bytes, B: bytes, st, en, g, h, idA=0, idB=0, m=None, n=None):
    L = O.ref_sub()
    P, s = C.c_void_p, C.c_size_t
    L.ref_non_parallel.argtypes = [P, P, s, s, s, s, s, C.c_int, C.c_int, C.c_double, C.c_double, P, P, P, P,
                                   C.c_char_p]
    a, b = O._bytes1(A), O._bytes1(B)
    m = len(A) - idA if m is None else m
    n = len(B) - idB if n is None else n
    mm, nn = min(m, n), max(m, n)
    T = [np.empty((mm + 1, nn + 1), dtype=np.float64) for _ in range(3)]
    inv = C.c_int(0)
    with tempfile.NamedTemporaryFile(suffix=".txt") as f:
        rc = L.ref_non_parallel(O._ptr(a), O._ptr(b), m, n, idA, idB, 1, st, en, g, h, O._ptr(T[0]), O._ptr(T[1]),
                                O._ptr(T[2]), C.byref(inv), f.name.encode())
        assert rc == 0
        text = Path(f.name).read_text()
    return T, text


def main():
    if not O.ref_available():
        raise SystemExit("oracle/_ref not built (needs /root/reference): make -C oracle")
    rng = np.random.default_rng(64)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    tabs, cases = {}, []
    k = 0
    for (g, h) in GH:
        for st in TYPES:
            m, n = int(rng.integers(1, 40)), int(rng.integers(1, 40))
            A, B = rng.choice(acgt, m).tobytes(), rng.choice(acgt, n).tobytes()
            en = int(rng.choice([-1, -2, -3, 1, 2, 3]))
            key = f"f{k}"
            k += 1
            r = O.ref_subproblem(A, B, st, en, g, h, p=3, tables=True, traceback=False)
            TN, text = ref_non_parallel(A, B, st, en, g, h)
            tabs[key + "_C"] = np.stack([r["T1"], r["T2"], r["T3"]])
            tabs[key + "_N"] = np.stack(TN)
            c = dict(key=key, A=A.decode(), B=B.decode(), g=g, h=h, start=st, end=en, invert=r["invert"],
                     text_md5=hashlib.md5(text.encode()).hexdigest())
            if len(text) < 6000:
                c["text"] = text
            cases.append(c)
    np.savez_compressed(HERE / "f64_tables.npz", **tabs)
    (HERE / "f64_cases.json").write_text(json.dumps(cases, indent=0) + "\n")
    diff = sum(1 for c in cases if not np.array_equal(tabs[c["key"] + "_C"], tabs[c["key"] + "_N"]))
    print(f"wrote {len(cases)} double-arithmetic cases; {diff} differ between the two T2 forms")


if __name__ == "__main__":
    main()
