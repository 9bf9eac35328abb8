"""rocprofv3 driver: main_alignment_function's C-ABI call (host buffers in, text out) at --len, --reps times,
for a --hip-trace / --kernel-trace breakdown of where a boundary call's time goes."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cse305_parallel_sequence_alignment_amd import api, data  # noqa: E402

L = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
A, B = data.bundled()[0][:L], data.bundled()[1][:L]
for k in range(reps):
    t0 = time.perf_counter()
    text, sc = api.main_alignment_text(b"\0" + A, b"\0" + B, L, L, 32, 1.0, 2.0)
    print(f"call {k}: {1e3 * (time.perf_counter() - t0):.3f} ms score {sc}", flush=True)
