"""Fixtures of main_alignment_function at its callers' sizes (tests/golden/whole.json).

The reference's test_n_cores_thread / test_similarity call main_alignment_function on
WHOLE sequences of the bundled file (testing.cpp:209-287, call at :261; :295-369, call at
:345): 13,309-97,409 characters.  The reference itself cannot run them (three (m+1)(n+1)
double tables: ~226 GB at 97k), so these outputs come from the oracle's 1 B/cell
restatement orc_main_alignment_dir -- which reproduces the reference's own outputs at
10k and 20k byte for byte (tests/test_oracle_golden.py::test_oracle_dir_at_size, against
at_size.json made from the reference's Subproblem) and equals the double-table
restatement on random pairs.  So: restatement-pinned at these sizes, not reference-produced.

    python tests/golden/make_whole.py      # ~4 min, ~10 GB of RAM (the 97k pair)

Each case: sequence indices, prefix lengths (None = whole), g, h, score, node count, the
md5 of the two print_seq lines and of the whole stdout text.
"""
from __future__ import annotations

import hashlib
import json
import sys
import time
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent.parent))
from oracle import oracle as O  # noqa: E402

CASES = [
    # (a, b, La, Lb): whole TP53 pair (m < n), a 48k x 47k prefix pair (m > n: the ctor's swap; > 2^31
    # direction bytes), a dissimilar 40k pair (ABCB1 x KIT: gap-heavy path), whole ABCB1 x ABCB1 (the
    # dataset's largest pair, 97,409 x 97,403) and whole CDH1 x CDH1
    (6, 8, None, None),
    (3, 4, 48000, 47000),
    (0, 15, 40000, 40000),
    (3, 4, None, None),
    (5, 7, None, None),
]


def main():
    _, seqs = O.load_dataset()
    out = []
    for a, b, la, lb in CASES:
        A = seqs[a] if la is None else seqs[a][:la]
        B = seqs[b] if lb is None else seqs[b][:lb]
        t0 = time.time()
        text, score = O.main_alignment_text_dir(A, B, 1, 2)
        lines = text.split("\n")[5:7]
        out.append(dict(a=a, b=b, La=la, Lb=lb, m=len(A), n=len(B), g=1, h=2, score=score, n_nodes=len(lines[0]),
                        lines_md5=hashlib.md5((lines[0] + "\n" + lines[1] + "\n").encode()).hexdigest(),
                        text_md5=hashlib.md5(text.encode("latin-1")).hexdigest()))
        print(f"{a} x {b} ({len(A)} x {len(B)}): score {score}, {len(lines[0])} nodes, {time.time() - t0:.1f} s",
              flush=True)
    (HERE / "whole.json").write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main()
