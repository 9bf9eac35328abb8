"""How fast does the banded Gotoh DP (C3, band w) rank-converge on a given pair?  (CPU analysis, numpy.)

For rows r0 on a grid, run the DP from the chunked kernel's guessed row (the row-0 tent moved to the
diagonal, F = -inf) and report after how many rows its (H, F) band state is parallel to the exact one
(same -inf pattern, one constant) -- the property chunk_check_kernel tests.  Usage:
  python scripts/c3_convergence.py [real|synthetic|dissimilar] [step]
"""
import sys

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from cse305_parallel_sequence_alignment_amd import data

NI = -np.inf


def row(Hp, Fp, a, B, i, w, g, h, n):
    """Row i (1-based) of the band from row i-1's (H, F) over columns 0..n (arrays of n+1)."""
    jlo, jhi = max(1, i - w), min(n, i + w)
    H = np.full(n + 1, NI)
    F = np.full(n + 1, NI)
    js = np.arange(jlo, jhi + 1)
    f = (B[js - 1] == a).astype(np.float64)
    c1 = f + Hp[js - 1]
    c3 = np.maximum(Hp[js] - g - h, Fp[js] - g)
    x = np.maximum(c1, c3)
    if i <= w:  # column 0's T3 border
        x0 = -h - g * i
    else:
        x0 = NI
    pref = np.maximum.accumulate(np.concatenate(([x0], x)) + g * np.arange(jlo - 1, jhi + 1))[:-1]
    c2 = pref - h - g * js
    H[js] = np.maximum(np.maximum(c1, c2), c3)
    F[js] = c3
    if i <= w:
        H[0] = F[0] = -h - g * i
    return H, F


def parallel(H1, F1, H2, F2):
    a = np.concatenate((H1, F1)); b = np.concatenate((H2, F2))
    fa, fb = np.isfinite(a) & (a > -1e8), np.isfinite(b) & (b > -1e8)
    if not np.array_equal(fa, fb) or not fa.any():
        return False
    d = a[fa] - b[fa]
    return bool(np.all(d == d[0]))


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "dissimilar"
    step = int(sys.argv[2]) if len(sys.argv) > 2 else 640
    limit = int(sys.argv[3]) if len(sys.argv) > 3 else 20000
    if which == "synthetic":
        A, B = data.c3_pair(synthetic=True)
    elif which == "real":
        A, B = data.c3_pair(False)
    else:
        A, B = data.bundled()[0][:81835], data.bundled()[15][:81835]
    A = np.frombuffer(A, dtype=np.uint8); B = np.frombuffer(B, dtype=np.uint8)
    m, n, w, g, h = len(A), len(B), 512, 1.0, 2.0
    # exact rows: keep every row in a window-limited dict only at the grid, and run guesses alongside
    Hp = np.full(n + 1, NI); Fp = np.full(n + 1, NI)
    Hp[0] = 0.0
    Hp[1:w + 1] = -h - g * np.arange(1, w + 1)
    starts = list(range(step, m - 1, step))
    live = {}   # r0 -> (H, F)
    res = {}
    for i in range(1, m + 1):
        Hp, Fp = row(Hp, Fp, A[i - 1], B, i, w, g, h, n)
        if i in set(starts) and i > w + 64:
            d = np.abs(np.arange(n + 1) - i)
            Hg = np.where(d <= w, -h - g * d, NI); Hg[0] = NI if i > w else Hg[0]
            live[i] = (Hg, np.full(n + 1, NI))
            continue
        done = []
        for r0, (Hg, Fg) in live.items():
            Hg, Fg = row(Hg, Fg, A[i - 1], B, i, w, g, h, n)
            live[r0] = (Hg, Fg)
            if parallel(Hp, Fp, Hg, Fg):
                res[r0] = i - r0; done.append(r0)
            elif i - r0 >= limit:
                res[r0] = None; done.append(r0)
        for r0 in done:
            del live[r0]
    for r0 in live:
        res[r0] = None
    v = [res[r] for r in sorted(res)]
    conv = [x for x in v if x is not None]
    print(which, "m", m, "starts", len(v), "never (within", limit, "rows):", sum(x is None for x in v))
    if conv:
        print("rows to converge: median", int(np.median(conv)), "p90", int(np.percentile(conv, 90)), "max", max(conv))
    print("per start:", [(r, res[r]) for r in sorted(res)][:400])


if __name__ == "__main__":
    main()
