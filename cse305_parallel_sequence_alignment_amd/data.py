"""Sequence data: the reference's FASTA reader and the benchmark workloads' inputs.

``read_and_store_sequences`` restates test_functions/pull_data.cpp:18-71 (the
reference's loader of ``gene_sequences_test``): a line starting with ``>`` opens
a new record whose name is that line; every other line is appended to the
current sequence.  Returns ``(names, sequences)`` or raises like the reference's
error returns.  The reference's bundled data file ships with the tests as
``tests/golden/gene_sequences_test.gz`` (a fixture: it is data, not code).

The workload builders give the exact inputs of BASELINE.json's configs
 so that ``bench.py``, the GPU parity tests and the fixture
generators agree byte for byte.
"""
from __future__ import annotations

import gzip
from pathlib import Path
from typing import List, Tuple

import numpy as np

REPO = Path(__file__).resolve().parent.parent
BUNDLED = REPO / "tests" / "golden" / "gene_sequences_test.gz"

C4_LEN, C4_PAIRS, C4_SEED = 4000, 1024, 0x5EED0004
C3_LEN = 97403  # the largest real pair: seq3 x seq4 truncated to the shorter


def read_and_store_sequences(filename=BUNDLED) -> Tuple[List[bytes], List[bytes]]:
    """pull_data.cpp:18-71: names (the '>' lines) and sequences (concatenated lines)."""
    path = Path(filename)
    opener = gzip.open if path.suffix == ".gz" else open
    names: List[bytes] = []
    seqs: List[bytes] = []
    cur: List[bytes] = []
    with opener(path, "rb") as f:
        for line in f.read().split(b"\n"):
            if line[:1] == b">":
                if cur:
                    seqs.append(b"".join(cur))
                    cur = []
                names.append(line)
            else:
                cur.append(line)
    if cur:
        seqs.append(b"".join(cur))
    if len(seqs) != len(names):
        raise ValueError("mismatch in sequences and names list sizes")  # pull_data.cpp:52-55
    return names, seqs


_SEQS = None


def bundled() -> List[bytes]:
    global _SEQS
    if _SEQS is None:
        _SEQS = read_and_store_sequences()[1]
    return _SEQS


def encode(s: bytes) -> np.ndarray:
    """ACGT -> codes 0..3 (the DNA map msa_encode_pair uses for every pair)."""
    return np.frombuffer(s.translate(bytes.maketrans(b"ACGT", b"\x00\x01\x02\x03")), dtype=np.uint8).copy()


def synth(n: int, seed: int) -> bytes:
    rng = np.random.default_rng(seed)
    return rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), n).tobytes()


def c2_pair(rank: int = 0, synthetic: bool = False):
    """C2: query seq(rank+1)[:10000] against the reference sequence seq0[:10000]."""
    if synthetic:
        return synth(10000, 0x5EED0001 + 1000 + rank + 1), synth(10000, 0x5EED0001 + 1000)
    s = bundled()
    return s[(rank + 1) % len(s)][:10000], s[0][:10000]


def mutate(A: bytes, seed: int, sub: float = 0.01, indel: float = 0.001, max_indel: int = 8) -> bytes:
    """A copy of A with i.i.d. substitutions (rate `sub`) and insertions / deletions of 1..max_indel
    symbols (rate `indel`), positions and symbols from numpy's generator seeded with `seed`."""
    rng = np.random.default_rng(seed)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    b = bytearray(A)
    for k in rng.choice(len(b), size=int(len(b) * sub), replace=False):
        b[k] = int(acgt[rng.integers(4)])
    for k in sorted(rng.choice(len(b) - 2 * max_indel, size=int(len(b) * indel), replace=False), reverse=True):
        ln = int(rng.integers(1, max_indel + 1))
        if rng.integers(2):
            del b[k:k + ln]
        else:
            b[k:k] = rng.choice(acgt, ln).tobytes()
    return bytes(b)


def c3_pair(synthetic: bool = False):
    """C3: seq3 x seq4 truncated to 97,403 (band 512); synthetic: A = 100,000 i.i.d.
    ACGT and B = A mutated (1% substitutions, 0.1% indels of 1..8), seed 0x5EED0003, B cut to 100,000."""
    if synthetic:
        A = synth(100000, 0x5EED0003)
        B = mutate(A, 0x5EED0003 + 1)[:100000]
        return A, B
    s = bundled()
    return s[4][:C3_LEN], s[3][:C3_LEN]


def c4_offsets() -> np.ndarray:
    rng = np.random.default_rng(C4_SEED)
    return rng.integers(0, 13309 - C4_LEN, size=C4_PAIRS)


def c4_queries(lo: int, hi: int, synthetic: bool = False) -> List[bytes]:
    """C4: 4,000-character windows seq[k % 20][off_k : off_k + 4000] for pairs k in [lo, hi)."""
    if synthetic:
        return [synth(C4_LEN, C4_SEED + k) for k in range(lo, hi)]
    s = bundled()
    offs = c4_offsets()
    return [s[k % 20][offs[k]:offs[k] + C4_LEN] for k in range(lo, hi)]


def c4_reference(synthetic: bool = False) -> bytes:
    return synth(C4_LEN, C4_SEED - 1) if synthetic else bundled()[0][:C4_LEN]


def c5_pair(rank: int = 0, synthetic: bool = False):
    """C5: seq(rank+1)[:20000] x seq0[:20000] (affine SW with traceback)."""
    if synthetic:
        return synth(20000, 0x5EED0005 + rank + 1), synth(20000, 0x5EED0005)
    s = bundled()
    return s[(rank + 1) % len(s)][:20000], s[0][:20000]
