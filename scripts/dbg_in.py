import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from cse305_parallel_sequence_alignment_amd import _lib as LB
from cse305_parallel_sequence_alignment_amd.plan import Plan
ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)
def enc(s): return torch.from_numpy(np.frombuffer(s.translate(bytes.maketrans(b"ACGT", b"\x00\x01\x02\x03")), dtype=np.uint8).copy()).cuda()
rng = np.random.default_rng(7)
m, n = 64, 64
A, B = rng.choice(ACGT, m).tobytes(), rng.choice(ACGT, n).tobytes()
pl = Plan(LB.SW_LINEAR, LB.CELLS_H, [m], [n], [0], [0], match=1, mismatch=0, gap_open=1, gap_extend=1, track_end=False, single=True)
H = torch.full((pl.cells_elems,), -7, dtype=torch.int32, device="cuda")
pl.run(enc(A), enc(B), H)
pl.results()
f = H.cpu().numpy()
P = pl.stripe_meta()[0, 1]
for lane in (0, 1, 63):
    vals = [f[((4 * q + u) * 64 + lane) * 4 + kk] for q in range(P) for u in range(4) for kk in range(4)]
    print("lane", lane, vals)
