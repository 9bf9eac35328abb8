import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from cse305_parallel_sequence_alignment_amd import _lib as LB
from cse305_parallel_sequence_alignment_amd.plan import Plan
from oracle import oracle as O
ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)
def enc(s): return torch.from_numpy(np.frombuffer(s.translate(bytes.maketrans(b"ACGT", b"\x00\x01\x02\x03")), dtype=np.uint8).copy()).cuda()
rng = np.random.default_rng(7)
m, n = 6, 12
A, B = rng.choice(ACGT, m).tobytes(), rng.choice(ACGT, n).tobytes()
print("A", A, "B", B)
pl = Plan(LB.SW_LINEAR, LB.CELLS_H, [m], [n], [0], [0], match=1, mismatch=0, gap_open=1, gap_extend=1, track_end=True, single=True)
H = torch.full((pl.cells_elems,), -7, dtype=torch.int32, device="cuda")
pl.run(enc(A), enc(B), H)
meta = pl.stripe_meta()
print("meta", meta[:2, :3].tolist(), "geom", pl.geom[0])
Hd = pl.deskew(H.cpu().numpy(), 0, meta)
o = O.sw(A, B, 1, 0, 1, 1, want_h=True)
print("gpu\n", Hd[:, :])
print("ref\n", o["H"][:, :])
raw = H.cpu().numpy()[:2048].reshape(-1, 64, 2, 4)
print("raw group0 lane0 rows", raw[0, 0], "group1", raw[1, 0], raw[2, 0])
