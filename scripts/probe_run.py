"""Diagnostic: live progress of a flow-kernel launch via host-mapped probes (-DMSA_STAMPS -DFL_DBG build)."""
import sys, os, time, ctypes as C
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from cse305_parallel_sequence_alignment_amd import _lib as LB
from cse305_parallel_sequence_alignment_amd.plan import Plan
ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)
def enc(s): return torch.from_numpy(np.frombuffer(s.translate(bytes.maketrans(b"ACGT", b"\x00\x01\x02\x03")), dtype=np.uint8).copy()).cuda()
rng = np.random.default_rng(7)
m, n = int(sys.argv[1]), int(sys.argv[2])
A, B = rng.choice(ACGT, m).tobytes(), rng.choice(ACGT, n).tobytes()
pl = Plan(LB.SW_LINEAR, LB.CELLS_H, [m], [n], [0], [0], match=1, mismatch=0, gap_open=1, gap_extend=1, track_end=True, single=True)
H = torch.full((pl.cells_elems,), -7, dtype=torch.int32, device="cuda")
hip = C.CDLL("libamdhip64.so")
ptr = C.c_void_p()
nbytes = 256 * 8 * 4 * 8
assert hip.hipHostMalloc(C.byref(ptr), C.c_size_t(nbytes), C.c_uint(0)) == 0
C.memset(ptr, 0, nbytes)
arr = np.ctypeslib.as_array((C.c_uint64 * (nbytes // 8)).from_address(ptr.value)).reshape(256, 8, 4)
fn = LB.lib().msa_debug_stamps
fn.argtypes = [C.c_void_p, C.c_void_p]
fn(pl._h, ptr)
dA, dB = enc(A), enc(B)
pl_nblk = int(os.environ.get("NBLK", "1"))
pl.run(dA, dB, H)
print("launched", flush=True)
for it in range(6):
    time.sleep(1.0)
    a2 = arr.reshape(-1, 4)
    nz = np.argwhere((a2[:, 0] >= 2000) & (a2[:, 0] < 2000 + pl_nblk)).ravel()
    print("t", it, "active waves", len(nz), flush=True)
    for i in nz[:40]:
        print("   blk", i // 8, "wave", i % 8, arr.reshape(-1, 4)[i].tolist(), flush=True)
os._exit(0)
