"""Golden fixtures for optimal_alignment (main_alignment.cpp:202-351).

main_alignment.cpp does not compile as shipped (wrong include at
:7, a merge-conflict marker at :405), so its stitching cannot be run from the
reference's own sources.  Each subproblem's node list here IS reference-produced:
the reference's own Subproblem (compute_tables + find_alignment, compiled
unmodified into oracle/_ref/libref_sub.so) runs on it.  The selection rule
(:232-341) and the stitch (:344-348) are applied to those lists by this script
and print_seq (:32-55) formats them -- so the fixture is reference-anchored on
the stitch and reference-produced on every node.

Partitions: the 80 reference-produced partitions of partial.json (p = 4 and 8),
whose subproblems include one-row ones (lenA = 0) and swapped ones (lenA > lenB),
plus hand-made partitions with 1, 2 and 3 subproblems (the reference solves
only subproblem 0 for those).  Cases with a decreasing coordinate are skipped
(the reference's size_t lengths wrap there).

    python tests/golden/make_optimal.py     ->  tests/golden/optimal.json
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent.parent))
from oracle import oracle as O  # noqa: E402


def solve_order(num, fix):
    if fix:
        return list(range(num))
    order, n3 = [], num > 3
    for r in range(3):
        if r > 0 and not n3:
            break
        i = r
        while n3 and i < num - 3:
            order.append(i)
            i += 3
        if i < num:
            order.append(i)
    return order


def reference_stitch(A, B, bp, g, h, fix):
    num = len(bp) - 1
    order = solve_order(num, fix)
    subs = {}
    for k in order:
        (i0, j0, t0), (i1, j1, t1) = bp[k], bp[k + 1]
        r = O.ref_subproblem(A, B, t0, -t1, g, h, p=1, idA=i0, idB=j0, m=i1 - i0, n=j1 - j0, tables=False)
        subs[k] = r["nodes"]
    last_link = num - 1 if fix else max(num - 2, 0)
    path = []
    for k in range(num):
        if k not in subs or not subs[k]:
            break
        path += subs[k]
        if k + 1 > last_link or k + 1 >= num:
            break
    a, b = b"\0" + A, b"\0" + B
    l1 = "".join(chr(a[i]) if t in (1, 3) and i <= len(A) else ("?" if t in (1, 3) else "-") for i, j, t in path)
    l2 = "".join(chr(b[j]) if t in (1, 2) and j <= len(B) else ("?" if t in (1, 2) else "-") for i, j, t in path)
    text = "bp1\nbp1.2\nbp2\nbp3\nbp4\n" * len(order) + l1 + "\n" + l2 + "\n"
    return dict(text=text, path=[list(x) for x in path], n_solved=len(order))


def main():
    if not O.ref_available():
        raise SystemExit("oracle/_ref not built (needs /root/reference): make -C oracle")
    cases = []
    for c in json.load(open(HERE / "partial.json")):
        bp = [tuple(x) for x in c["partition"]]
        if any(bp[k + 1][0] < bp[k][0] or bp[k + 1][1] < bp[k][1] for k in range(len(bp) - 1)):
            continue
        if any(bp[k + 1][:2] == bp[k][:2] for k in range(len(bp) - 1)):
            continue
        A, B = c["A"].encode(), c["B"].encode()
        cases.append(dict(A=c["A"], B=c["B"], g=c["g"], h=c["h"], bp=[list(x) for x in bp]))
    rng = np.random.default_rng(305)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    for parts in ([(0, 0, -1), (37, 41, 1)], [(0, 0, -1), (20, 18, 1), (37, 41, 1)],
                  [(0, 0, -1), (9, 14, 1), (20, 18, 3), (37, 41, 1)],
                  [(0, 0, -1), (9, 14, 2), (20, 25, 3), (30, 30, 1), (37, 41, 1)],
                  [(0, 0, -1), (5, 5, 1), (10, 12, 2), (15, 17, 3), (22, 20, 1), (30, 33, 1), (37, 41, 1)]):
        for g, h in ((1.0, 2.0), (2.0, 1.0)):
            A = rng.choice(acgt, 37).tobytes().decode()
            B = rng.choice(acgt, 41).tobytes().decode()
            cases.append(dict(A=A, B=B, g=g, h=h, bp=[list(x) for x in parts]))
    out = []
    for c in cases:
        A, B = c["A"].encode(), c["B"].encode()
        bp = [tuple(x) for x in c["bp"]]
        c["ref"] = reference_stitch(A, B, bp, c["g"], c["h"], False)
        c["fix_all"] = reference_stitch(A, B, bp, c["g"], c["h"], True)
        out.append(c)
    (HERE / "optimal.json").write_text(json.dumps(out, separators=(",", ":")) + "\n")
    print(f"wrote {len(out)} optimal_alignment cases")


if __name__ == "__main__":
    main()
