"""Build-owned equivalents of the reference's harness (test_functions/, main.cpp).

The reference's drivers time ``main_alignment_function`` over pairs drawn from
its FASTA data and write CSV files; here they call the GPU path
(``api.main_alignment_text``: every DP cell on the MI355X) with the same
arguments and write the same files:

  read_and_store_sequences  test_functions/pull_data.cpp:18-71 (names/sequences lists, return 0/1,
                            duplicate check)
  sequence_similarity       pull_data.cpp:97-125 (matching positions in the reference's chunking,
                            divided by the LONGER length -- as the code does, not as its comment says)
  test_input_size           testing.cpp:26-80
  test_input_size_thread    testing.cpp:81-160  -> input_size_testing.csv
  test_n_cores              testing.cpp:168-207 (its core count is rand(): only printed)
  test_n_cores_thread       testing.cpp:208-281 -> n_cores_testing.csv
  test_similarity           testing.cpp:289-363 -> similarity_testing.csv
  main                      main.cpp (read the data, run test_input_size_thread)

Pair selection uses the C library's rand() through ctypes (the reference calls
rand() unseeded, i.e. srand(1)), so a single-threaded run draws the
reference's pairs; the reference's threaded drivers race on rand() and on
their index variables, so their order is not reproducible there either.  The
thread count defaults to the reference's std::thread::hardware_concurrency()
(os.cpu_count()); ``threads`` and ``test_pairs`` can be lowered.

    python -m cse305_parallel_sequence_alignment_amd.harness [input_size|n_cores|similarity] [--pairs N]
"""
from __future__ import annotations

import argparse
import ctypes
import os
import sys
import threading
import time
from typing import Callable, List, Optional

from . import api
from . import data

_libc = ctypes.CDLL(None)
_libc.rand.restype = ctypes.c_int
_rand_mu = threading.Lock()


def c_rand() -> int:
    with _rand_mu:
        return int(_libc.rand())


def c_srand(seed: int) -> None:
    _libc.srand(ctypes.c_uint(seed))


def read_and_store_sequences(names: List[bytes], sequences: List[bytes], filename=data.BUNDLED) -> int:
    """pull_data.cpp:18-71: appends to ``names`` / ``sequences``; 0 on success, 1 on error."""
    print(f"Opening data file: {filename}")
    try:
        n, s = data.read_and_store_sequences(filename)
    except OSError:
        print("Error opening file! Check the file path/name!", file=sys.stderr)
        return 1
    except ValueError:
        print("Error: mismatch in sequences and names list sizes")
        return 1
    print("File opened successfully!\nStoring sequences...")
    names.extend(n)
    sequences.extend(s)
    print("Checking for duplicate sequences...")
    if len(set(s)) != len(s):
        print("Duplicate sequence found!\nThere is at least one duplicate sequence found. Please check your data file.")
    else:
        print("No duplicate sequences found.")
    print("Dataset read successfully!")
    return 0


def sequence_similarity(seq1: bytes, seq2: bytes, num_threads: Optional[int] = None) -> float:
    """pull_data.cpp:97-125.  Chunks of iteration_size // num_threads positions, n_chunks =
    iteration_size // chunk_size of them, chunk num_threads-1 extended by the remainder (so
    positions can be counted twice); score / max(len1, len2)."""
    import numpy as np

    T = num_threads or os.cpu_count() or 1
    L = min(len(seq1), len(seq2))
    chunk = L // T
    if chunk == 0:
        raise ZeroDivisionError("sequence shorter than the thread count (the reference divides by zero here)")
    eq = np.frombuffer(seq1[:L], dtype=np.uint8) == np.frombuffer(seq2[:L], dtype=np.uint8)
    cum = np.concatenate([[0], np.cumsum(eq)])
    score = 0
    for i in range(L // chunk):
        a = i * chunk
        b = a + chunk + (L % T if i == T - 1 else 0)
        score += int(cum[b] - cum[a])
    return score / max(len(seq1), len(seq2))


def _align(seq1: bytes, seq2: bytes, size: int, p: int, out=sys.stdout) -> str:
    """One harness call: 1-based buffers of the first `size` characters (testing.cpp:124-128)."""
    text, _ = api.main_alignment_text(b"\0" + seq1[:size], b"\0" + seq2[:size], size, size, p, 1.0, 2.0)
    if out is not None:
        out.write(text)
    return text


def _pick(rng_range: int):
    return c_rand() % rng_range, c_rand() % rng_range


def _run_chunks(n_items: int, threads: int, body: Callable[[int, int, int], None]):
    """The reference's chunking: chunk = ceil(n / threads); thread t takes [t*chunk, end)."""
    chunk = (n_items + threads - 1) // threads
    ws = []
    for t in range(threads):
        start = t * chunk
        end = n_items if t == threads - 1 else start + chunk
        ws.append(threading.Thread(target=body, args=(t, start, end)))
    for w in ws:
        w.start()
    for w in ws:
        w.join()
    return chunk


def test_input_size(names, sequences, batches: int = 2, increment: int = 1000, out=sys.stdout) -> int:
    """testing.cpp:26-80."""
    print("Testing with different input sizes\n")
    rng = len(sequences) - 1
    for t in range(batches):
        print(f"Testing batch {t}\n")
        a, b = _pick(rng)
        while b == a:
            b = c_rand() % rng
        print(f"Testing sequences \n{names[a].decode()}\n and \n{names[b].decode()}\n")
        for i in range(1, batches):
            a, b = _pick(rng)
            s1, s2 = sequences[a], sequences[b]
            size = min(i * increment, min(len(s1), len(s2)))
            print(f"{size} sequence 1 length\n{size} sequence 2 length\ninput size min {size}")
            _align(s1, s2, size, 32, out)
            print("Got res")
    return 0


def test_input_size_thread(names, sequences, test_pairs: int = 1, input_size: int = 50,
                           threads: Optional[int] = None, csv_path="input_size_testing.csv", out=sys.stdout) -> int:
    """testing.cpp:81-160: pairs on `threads` host threads, each call on the GPU."""
    print("Testing with different input sizes\n")
    threads = threads or os.cpu_count() or 1
    rng = len(sequences) - 1
    sizes = [0.0] * test_pairs
    times = [0.0] * test_pairs

    def body(_t, start, end):
        for i in range(start, min(end, test_pairs)):
            a, b = _pick(rng)
            s1, s2 = sequences[a], sequences[b]
            size = min(input_size, min(len(s1), len(s2)))
            t0 = time.perf_counter()
            _align(s1, s2, size, 32, out)
            print("Got res")
            sizes[i] = size
            times[i] = time.perf_counter() - t0

    print("Starting threads")
    _run_chunks(test_pairs, threads, body)
    print("Joining threads\nFinished threads")
    with open(csv_path, "w") as f:
        f.write("Testing with different input sizes\nTest number,Input size,Execution time\n")
        for j in range(test_pairs):
            f.write(f"{j},{sizes[j]:g},{times[j]:g}\n")
    return 0


def test_n_cores(names, sequences, batches: int = 10, n_tests: int = 5) -> int:
    """testing.cpp:168-207 (the reference times nothing between its two clock reads)."""
    print("Testing with different number of cores\n")
    rng = len(sequences) - 1
    for t in range(batches):
        print(f"Testing batch {t}\n")
        a, b = _pick(rng)
        while b == a:
            b = c_rand() % rng
        print(f"Testing sequences \n{names[a].decode()}\n and \n{names[b].decode()}\n")
        for i in range(1, n_tests + 1):
            n_cores = c_rand()
            print(f"({i}/{n_tests}) Testing with number of cores: {n_cores}")
            t0 = time.perf_counter()
            print(f"Execution time: {time.perf_counter() - t0:g} seconds")
    return 0


def test_n_cores_thread(names, sequences, test_pairs: int = 2000, core_increments: int = 2,
                        threads: Optional[int] = None, csv_path="n_cores_testing.csv", max_len: Optional[int] = None,
                        out=sys.stdout) -> int:
    """testing.cpp:208-281: full-length pairs, p = the thread's core count (no effect on the result).
    max_len (not in the reference) bounds the pair length for short runs."""
    print("Testing with different input sizes\n")
    threads = threads or os.cpu_count() or 1
    rng = len(sequences) - 1
    cores = [0.0] * test_pairs
    times = [0.0] * test_pairs
    chunk = (test_pairs + threads - 1) // threads

    def body(t, start, end):
        n_cores = (((t + 1) * chunk) // core_increments) * core_increments
        for i in range(start, min(end, test_pairs)):
            a, b = _pick(rng)
            s1, s2 = sequences[a], sequences[b]
            size = min(len(s1), len(s2), max_len or 1 << 62)
            cores[i] = n_cores
            t0 = time.perf_counter()
            _align(s1, s2, size, max(1, n_cores), out)
            times[i] = time.perf_counter() - t0

    _run_chunks(test_pairs, threads, body)
    with open(csv_path, "w") as f:
        f.write("Testing with different number of cores\nTest number,Number of cores,Execution time\n")
        for j in range(test_pairs):
            f.write(f"{j},{cores[j]:g},{times[j]:g}\n")
    return 0


def test_similarity(names, sequences, test_pairs: int = 2000, threads: Optional[int] = None,
                    csv_path="similarity_testing.csv", max_len: Optional[int] = None, out=sys.stdout) -> int:
    """testing.cpp:289-363: similarity of each pair, then its alignment (p = 64) timed."""
    print("Testing with similarity computation\n")
    threads = threads or os.cpu_count() or 1
    rng = len(sequences) - 1
    sims = [0.0] * test_pairs
    times = [0.0] * test_pairs

    def body(_t, start, end):
        for i in range(start, min(end, test_pairs)):
            a, b = _pick(rng)
            s1, s2 = sequences[a], sequences[b]
            size = min(len(s1), len(s2), max_len or 1 << 62)
            sims[i] = sequence_similarity(s1, s2)
            t0 = time.perf_counter()
            _align(s1, s2, size, 64, out)
            times[i] = time.perf_counter() - t0

    _run_chunks(test_pairs, threads, body)
    with open(csv_path, "w") as f:
        f.write("Testing with similarity computation\nTest number,Similarity,Execution time\n")
        for j in range(test_pairs):
            f.write(f"{j},{sims[j]:g},{times[j]:g}\n")
    return 0


def main(argv=None) -> int:
    """main.cpp: read the data file, then run one driver (test_input_size_thread by default)."""
    ap = argparse.ArgumentParser()
    ap.add_argument("driver", nargs="?", default="input_size", choices=["input_size", "n_cores", "similarity"])
    ap.add_argument("--data", default=str(data.BUNDLED))
    ap.add_argument("--pairs", type=int, default=None)
    ap.add_argument("--threads", type=int, default=None)
    ap.add_argument("--max-len", type=int, default=None)
    a = ap.parse_args(argv)
    names: List[bytes] = []
    seqs: List[bytes] = []
    if read_and_store_sequences(names, seqs, a.data):
        return 1
    if a.driver == "input_size":
        return test_input_size_thread(names, seqs, test_pairs=a.pairs or 1, threads=a.threads)
    if a.driver == "n_cores":
        return test_n_cores_thread(names, seqs, test_pairs=a.pairs or 2000, threads=a.threads, max_len=a.max_len)
    return test_similarity(names, seqs, test_pairs=a.pairs or 2000, threads=a.threads, max_len=a.max_len)


if __name__ == "__main__":
    sys.exit(main())
