"""Diagnostic: per-stripe start/end stamps of the pass-1 flow kernel (-DMSA_STAMPS build).
usage: MSA_LIB_PATH=variants/libmsa_stamps.so FLW=4 python scripts/stamps2.py m n"""
import sys, os, ctypes as C
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from cse305_parallel_sequence_alignment_amd import _lib as LB
from cse305_parallel_sequence_alignment_amd.plan import Plan
from oracle.oracle import load_dataset
m = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
n = int(sys.argv[2]) if len(sys.argv) > 2 else m
W = int(os.environ.get("FLW", "4"))
RR = int(os.environ.get("MSA_R", "2"))
seqs = load_dataset()[1]
enc = lambda s: torch.from_numpy(np.frombuffer(s.translate(bytes.maketrans(b"ACGT", b"\x00\x01\x02\x03")), dtype=np.uint8).copy()).cuda()
A, B = (seqs[1] * 8)[:m], (seqs[0] * 8)[:n]
pl = Plan(LB.SW_LINEAR, LB.CELLS_H, [m], [n], [0], [0], match=1, mismatch=0, gap_open=1, gap_extend=1)
out = torch.empty(max(1, pl.cells_elems), dtype=torch.int32, device="cuda")
st = torch.zeros(64 * 16 * 4096 * 4, dtype=torch.int64, device="cuda")
fn = LB.lib().msa_debug_stamps
fn.argtypes = [C.c_void_p, C.c_void_p]
dA, dB = enc(A), enc(B)
for it in range(4):
    st.zero_()
    fn(pl._h, C.c_void_p(st.data_ptr()))
    pl.run(dA, dB, out)
    torch.cuda.synchronize()
    print("kernel ms", round(pl.kernel_ms(), 4), "score", pl.results()[0]["score"])
S = (m + 64 * RR - 1) // (64 * RR)
items = (S + W - 1) // W
a = st.cpu().numpy().reshape(64, 16, 4096, 4)[:items, :W, 0, :4].reshape(-1, 4)[:S].astype(np.float64)
start, end, nslow = a[:, 0] - a[0, 0], a[:, 1] - a[0, 0], a[:, 2]
def fl_cs(k): return -((16 - (k & 15)) & 15)
def fl_P(k): return (n - fl_cs(k) + min((m - 64 * RR * k - 1) // RR, 63)) // 16 + 1
P = np.array([fl_P(k) for k in range(S)])
pt = (end - start) / P * 10.0  # ns per phase (realtime = 100 MHz)
lag = np.diff(start) * 10.0     # ns
cross = (np.arange(1, S) % W) == 0
print("stripes", S, "pass-1 span us", round(end.max() / 100, 1))
print("phase ns: stripe0 %.0f median %.0f p90 %.0f" % (pt[0], np.median(pt), np.percentile(pt, 90)))
print("lag ns: in-WG median %.0f mean %.0f | cross-WG median %.0f mean %.0f" % (
    np.median(lag[~cross]), lag[~cross].mean(), np.median(lag[cross]) if cross.any() else 0, lag[cross].mean() if cross.any() else 0))
print("lag in phases (median pt): in %.2f cross %.2f" % (np.median(lag[~cross]) / np.median(pt), (np.median(lag[cross]) / np.median(pt)) if cross.any() else 0))
print("slow-path phase fraction: median %.3f" % np.median(nslow / P))
pub = a[:, 3] - a[0, 0]
L = (start[1:] - pub[:-1]) * 10.0
print("publish->consumer start ns: in-WG median %.0f | cross-WG median %.0f" % (np.median(L[~cross]), np.median(L[cross]) if cross.any() else 0))
print("first 12 L ns", np.round(L[:12]).tolist())
print("first 12 lags ns", np.round(lag[:12]).tolist())
print("first 12 phase ns", np.round(pt[:12]).tolist())
