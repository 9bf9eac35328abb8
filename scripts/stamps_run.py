"""Diagnostic: run one C2-shaped flow-kernel plan with the -DMSA_STAMPS build and summarise per-phase stamps."""
import sys, os, ctypes as C
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from cse305_parallel_sequence_alignment_amd import _lib as LB
from cse305_parallel_sequence_alignment_amd.plan import Plan
from oracle.oracle import load_dataset
m = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
n = int(sys.argv[2]) if len(sys.argv) > 2 else m
wl_out = (sys.argv[3] if len(sys.argv) > 3 else "h")
seqs = load_dataset()[1]
enc = lambda s: torch.from_numpy(np.frombuffer(s.translate(bytes.maketrans(b"ACGT", b"\x00\x01\x02\x03")), dtype=np.uint8).copy()).cuda()
A, B = (seqs[1] * 8)[:m], (seqs[0] * 8)[:n]
pl = Plan(LB.SW_LINEAR, LB.CELLS_H if wl_out == "h" else LB.CELLS_NONE, [m], [n], [0], [0], match=1, mismatch=0, gap_open=1, gap_extend=1)
out = torch.empty(max(1, pl.cells_elems), dtype=torch.int32, device="cuda") if wl_out == "h" else None
st = torch.zeros(64 * 16 * 4096 * 4, dtype=torch.int64, device="cuda")
fn = LB.lib().msa_debug_stamps
fn.argtypes = [C.c_void_p, C.c_void_p]
dA, dB = enc(A), enc(B)
for it in range(4):
    st.zero_()
    fn(pl._h, C.c_void_p(st.data_ptr()))
    pl.run(dA, dB, out)
    torch.cuda.synchronize()
    print("kernel ms", pl.kernel_ms(), "score", pl.results()[0]["score"])
S = (m + 63) // 64
W = int(os.environ.get("FLW", "8"))
items = (S + W - 1) // W
a = st.cpu().numpy().reshape(64, 16, 4096, 4)[:items, :W + 2]
P = int(pl.stripe_meta()[0, 1])
np.savez_compressed("gpurun_out/stamps.npz", a=a[:, :, :P + 2], P=P)
t0 = a[:, :W, :P, 0].astype(np.float64)
t1 = a[:, :W, :P, 1].astype(np.float64)
rt = a[:, :W, :P, 2].astype(np.float64)
dur = np.diff(t0, axis=2)
wait = t1 - t0
print("phases", P, "items", items)
print("median phase cycles (all waves)", np.median(dur[dur > 0]), "p10/p90", np.percentile(dur[dur > 0], [10, 90]))
print("mean wait cycles per phase", wait[wait >= 0].mean(), "frac phases waiting>50cyc", (wait > 50).mean())
# stripe start (realtime, 10ns ticks) relative to the first stripe
start = rt[:, :, 0].reshape(-1)
start = start - start[0]
print("stripe start (us) first 20:", np.round(start[:20] / 100.0, 2).tolist())
lag = np.diff(start) if len(start) > 1 else np.zeros(0)
lag = np.append(lag, np.nan)
print("lag per stripe us: in-WG median", np.nanmedian(lag.reshape(items, W)[:, :W - 1]) / 100.0,
      "cross-WG median", np.nanmedian(lag.reshape(-1)[W - 1::W]) / 100.0)
for it in range(items):
    d_ = np.diff(t0[it], axis=1); w_ = t1[it] - t0[it]
    print(it, "med phase", [int(np.median(d_[w][d_[w] > 0])) if (d_[w] > 0).any() else -1 for w in range(W)],
          "wait", [int(np.mean(w_[w][w_[w] >= 0])) for w in range(W)])
endt = rt[:, :, P - 1].reshape(-1) - rt.reshape(-1)[0]
print("last stripe end (us)", endt[S - 1] / 100.0, "first stripe duration (us)", endt[0] / 100.0)
