"""Diagnostic: two-pass flow plans vs the oracle (score, end, full H) on small shapes; MSA_R selects rows per lane."""
import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from cse305_parallel_sequence_alignment_amd import _lib as LB
from cse305_parallel_sequence_alignment_amd.plan import Plan
from oracle import oracle as O
ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)
def enc(s): return torch.from_numpy(np.frombuffer(s.translate(bytes.maketrans(b"ACGT", b"\x00\x01\x02\x03")), dtype=np.uint8).copy()).cuda()
rng = np.random.default_rng(7)
for (ma, mi, g) in [(2, -1, 1), (1, 0, 1)]:
  for (m, n, tp) in [(64, 64, True), (128, 64, False), (1, 1, True), (2, 3, True), (130, 70, True), (257, 300, True), (700, 650, False), (1500, 1200, True)]:
    A, B = rng.choice(ACGT, m).tobytes(), rng.choice(ACGT, n).tobytes()
    pl = Plan(LB.SW_LINEAR, LB.CELLS_H, [m], [n], [0], [0], match=ma, mismatch=mi, gap_open=g, gap_extend=g, track_end=tp, single=True)
    H = torch.full((pl.cells_elems,), -7, dtype=torch.int32, device="cuda")
    pl.run(enc(A), enc(B), H)
    res = pl.results()[0]
    meta = pl.stripe_meta()
    Hd = pl.deskew(H.cpu().numpy(), 0, meta)
    o = O.sw(A, B, ma, mi, g, g, want_h=True)
    bad = np.argwhere(Hd[1:, 1:] != o["H"][1:, 1:])
    ck = pl.checksum(H) == O.checksum_h(o["H"])
    print((ma, mi, g), (m, n, tp), "R", pl.geom[0].rows_per_lane, "score", res["score"], o["score"], "end", tuple(res["end"]), tuple(o["end"]), "nbad", len(bad), "ck", ck, flush=True)
    for (i, j) in bad[:8]:
        print("   cell", i + 1, j + 1, "gpu", Hd[i + 1, j + 1], "ref", o["H"][i + 1, j + 1])
