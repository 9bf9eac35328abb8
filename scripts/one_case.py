import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from cse305_parallel_sequence_alignment_amd import _lib as LB
from cse305_parallel_sequence_alignment_amd.plan import Plan
from oracle import oracle as O
ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)
def enc(s): return torch.from_numpy(np.frombuffer(s.translate(bytes.maketrans(b"ACGT", b"\x00\x01\x02\x03")), dtype=np.uint8).copy()).cuda()
rng = np.random.default_rng(7)
m, n = int(sys.argv[1]), int(sys.argv[2])
A, B = rng.choice(ACGT, m).tobytes(), rng.choice(ACGT, n).tobytes()
pl = Plan(LB.SW_LINEAR, LB.CELLS_H, [m], [n], [0], [0], match=1, mismatch=0, gap_open=1, gap_extend=1, track_end=True, single=True)
H = torch.full((pl.cells_elems,), -7, dtype=torch.int32, device="cuda")
print("plan ok", flush=True)
pl.run(enc(A), enc(B), H)
print("launched", flush=True)
torch.cuda.synchronize()
print("synced", flush=True)
try:
    res = pl.results()[0]
    print("res", res, flush=True)
except Exception as e:
    print("results error", e, flush=True)
o = O.sw(A, B, 1, 0, 1, 1, want_h=True)
Hd = pl.deskew(H.cpu().numpy(), 0, pl.stripe_meta())
print("oracle", o["score"], o["end"], "nbad", int((Hd[1:, 1:] != o["H"][1:, 1:]).sum()), flush=True)
