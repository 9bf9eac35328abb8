"""Expected scores of the C4 batch (1024 x 4,000 x 4,000 Smith-Waterman, linear gap 1, match 1 / mismatch 0).

    python tests/golden/make_c4_scores.py

The inputs are ``cse305_parallel_sequence_alignment_amd.data.c4_queries`` /
``c4_reference`` (the bundled dataset).  Scores come from the
oracle's C restatement ``orc_sw`` -- Smith-Waterman is a build extension, so this
fixture is "reference-anchored" (the oracle's SW is checked against brute force
and shares the reference's cell recurrence), not reference-produced.
Writes tests/golden/c4_scores.json; bench.py's multi-GPU c4 run and the GPU
tests compare the all-gathered scores against it.
"""
from __future__ import annotations

import hashlib
import json
import sys
from multiprocessing import Pool
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent.parent))


def _score(k):
    from cse305_parallel_sequence_alignment_amd import data
    from oracle import oracle as O

    q = data.c4_queries(k, k + 1)[0]
    return O.sw(q, data.c4_reference(), 1, 0, 1, 1)["score"]


def digest(scores) -> str:
    return hashlib.sha256(",".join(str(int(x)) for x in scores).encode()).hexdigest()


def main():
    from cse305_parallel_sequence_alignment_amd import data
    from oracle import oracle as O

    O.build()
    with Pool(8) as p:
        scores = p.map(_score, range(data.C4_PAIRS), chunksize=8)
    out = dict(config="C4: 1024 x (4000x4000) SW linear, match 1 mismatch 0 gap 1; queries data.c4_queries, "
                      "reference data.c4_reference", scores=scores, sha256=digest(scores))
    (HERE / "c4_scores.json").write_text(json.dumps(out))
    print("wrote c4_scores.json", out["sha256"], min(scores), max(scores))


if __name__ == "__main__":
    main()
