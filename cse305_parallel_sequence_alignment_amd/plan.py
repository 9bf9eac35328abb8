"""Device-resident plans over libmsa (torch tensors as device memory/streams).

PyTorch only provides device allocation, streams and ``torch.distributed``
plumbing here; every DP cell is computed by the HIP stripe kernel.

Skewed stripe layout of per-cell outputs (H / DIR / TAB planes), per pair:
stripe s (rows 64s+1..64s+64) owns ``pmax*16*64`` elements; element
``((s*pmax*4 + t//4)*64 + r)*4 + t%4`` (DIR: ``(s*pmax + t//16)*1024 + r*16 + t%16``)
holds cell ``(i, j) = (64s + r + 1, cs_s + t - r)``, cs_s from the stripe meta.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib as LB

META_FIELDS = 12  # int32 per stripe: cs, phases, best, best_i, best_j, fin0..2, has_fin, pad*3


def _stream_ptr(stream):
    if stream is None:
        import torch

        return C.c_void_p(torch.cuda.current_stream().cuda_stream)
    if isinstance(stream, int):
        return C.c_void_p(stream)
    return C.c_void_p(stream.cuda_stream)


def _ptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())


@dataclass
class PairGeom:
    m: int
    n: int
    stripe0: int
    pmax: int
    out_off: int
    rows_per_lane: int = 1  # 2: 128-row stripes, lane r holds rows 2r+1, 2r+2 (two-pass flow plans)


class Plan:
    """One launch shape: ``n_pairs`` pairs of (m_k, n_k) codes at (a_off_k, b_off_k)."""

    def __init__(self, alg: int, cells: int, ms, ns, a_offs, b_offs, match=1, mismatch=0, gap_open=1,
                 gap_extend=1, start_type=-1, band=-1, track_end=False, single=None):
        L = LB.lib()
        self.alg, self.cells = alg, cells
        self.ms = [int(x) for x in ms]
        self.ns = [int(x) for x in ns]
        npairs = len(self.ms)
        if single is None:
            single = npairs == 1
        self._arrs = [(C.c_int64 * npairs)(*v) for v in (self.ms, self.ns, [int(x) for x in a_offs],
                                                         [int(x) for x in b_offs])]
        d = LB.PlanDesc(alg=alg, cells=cells, match=match, mismatch=mismatch, gap_open=gap_open,
                        gap_extend=gap_extend, start_type=start_type, band=band, track_end=int(bool(track_end)),
                        single=int(bool(single)), n_pairs=npairs, m=self._arrs[0], n=self._arrs[1],
                        a_off=self._arrs[2], b_off=self._arrs[3])
        self._h = C.c_void_p()
        LB.check(L.msa_plan_create(C.byref(d), C.byref(self._h)), "msa_plan_create")
        self.band = band
        self.single = bool(single)
        e = C.c_int64()
        LB.check(L.msa_plan_cells_size(self._h, C.byref(e)), "msa_plan_cells_size")
        self.cells_elems = e.value
        self.n_stripes = int(L.msa_plan_stripes(self._h))
        # per-pair layout as the C side laid it out
        self.geom = []
        lay = (C.c_int64 * 4)()
        for k, (m, n) in enumerate(zip(self.ms, self.ns)):
            LB.check(L.msa_plan_pair_layout(self._h, k, lay), "msa_plan_pair_layout")
            self.geom.append(PairGeom(m, n, int(lay[0]), int(lay[1]), int(lay[2]), max(1, int(lay[3]) >> 16)))
        self.phase_steps = int(lay[3]) & 0xFFFF

    def __del__(self):
        try:
            if self._h:
                LB.lib().msa_plan_destroy(self._h)
                self._h = C.c_void_p()
        except Exception:
            pass

    def _check_buffers(self, dA, dB, outs):
        """The C-ABI takes raw device pointers: check device, dtype, contiguity and sizes here, so an
        undersized or misplaced buffer raises instead of letting a kernel read or write out of bounds."""
        import torch

        need_a = max(o + m for o, m in zip(self._arrs[2], self.ms))
        need_b = max(o + n for o, n in zip(self._arrs[3], self.ns))
        for name, t, need in (("dA", dA, need_a), ("dB", dB, need_b)):
            if t is None or not t.is_cuda or t.dtype != torch.uint8 or not t.is_contiguous():
                raise ValueError(f"{name} must be a contiguous uint8 CUDA tensor of codes")
            if t.numel() < need:
                raise ValueError(f"{name} holds {t.numel()} codes, the plan reads {need}")
        planes = {LB.CELLS_NONE: 0, LB.CELLS_H: 1, LB.CELLS_DIR: 1, LB.CELLS_TAB: 3}[self.cells]
        want = torch.uint8 if self.cells == LB.CELLS_DIR else torch.int32
        for k, t in enumerate(outs):
            if k >= planes:
                continue
            if t is None or not t.is_cuda or t.dtype != want or not t.is_contiguous():
                raise ValueError(f"out{k} must be a contiguous {want} CUDA tensor")
            if t.numel() < self.cells_elems:
                raise ValueError(f"out{k} holds {t.numel()} elements, the plan writes {self.cells_elems}")

    def run(self, dA, dB, out0=None, out1=None, out2=None, stream=None):
        self._check_buffers(dA, dB, (out0, out1, out2))
        LB.check(LB.lib().msa_plan_run(self._h, _ptr(dA), _ptr(dB), _ptr(out0), _ptr(out1), _ptr(out2),
                                       _stream_ptr(stream)), "msa_plan_run")

    def results(self, stream=None):
        """Per-pair results; raises MsaError(TIMEOUT) if any run since creation / clear_error() had a kernel
        wait hit its spin limit (the plan's error word is sticky)."""
        n = len(self.ms)
        arr = (LB.PairResult * n)()
        LB.check(LB.lib().msa_plan_results(self._h, arr, _stream_ptr(stream)), "msa_plan_results")
        return [dict(score=r.score, status=r.status, end=(r.end_i, r.end_j), fin=tuple(r.fin)) for r in arr]

    def error(self, stream=None) -> int:
        """The sticky error word (0 = every run since creation / clear_error() completed its waits)."""
        v = C.c_int()
        LB.check(LB.lib().msa_plan_error(self._h, C.byref(v), _stream_ptr(stream)), "msa_plan_error")
        return int(v.value)

    def run_info(self, stream=None) -> dict:
        """How the last run was computed (msa_plan_run_info): launch mode, chunks, whether every chunk of a
        chunked banded run converged (else the exact launch recomputed the cells), warm-up stripes, and whether
        chunks >= 1 wrote int16 cells (widened by the add of the chunk constants)."""
        v = (C.c_int32 * 4)()
        LB.check(LB.lib().msa_plan_run_info(self._h, v, _stream_ptr(stream)), "msa_plan_run_info")
        return dict(mode={0: "stripe", 1: "flow", 2: "chunked"}[v[0]], chunks=int(v[1]), converged=int(v[2]),
                    warm_stripes=int(v[3]) & 0xffff, int16_cells=(int(v[3]) >> 16) & 1)

    def launch_info(self) -> dict:
        """How the plan launches (msa_plan_launch_info): kernel mode, grid, threads, LDS bytes, flow pass-1
        workgroups, workgroups of the separate pass-2 launch (0 = pass 2 inside the main launch), rows per
        lane, items."""
        v = (C.c_int32 * 8)()
        LB.check(LB.lib().msa_plan_launch_info(self._h, v), "msa_plan_launch_info")
        modes = {0: "stripe", 1: "flow", 2: "chunked", 3: "split", 4: "band", 5: "band_chunked", 6: "cflow"}
        return dict(mode=modes[v[0]], grid=int(v[1]), threads=int(v[2]), lds_bytes=int(v[3]), nflow=int(v[4]),
                    fill_grid=int(v[5]), rows_per_lane=int(v[6]), items=int(v[7]))

    def clear_error(self, stream=None) -> None:
        LB.check(LB.lib().msa_plan_clear_error(self._h, _stream_ptr(stream)), "msa_plan_clear_error")

    def scores_into(self, d_scores, stream=None) -> None:
        """Copy the last run's per-pair scores into a device int32 tensor (stream-ordered, no host sync)."""
        import torch

        if not d_scores.is_cuda or d_scores.dtype != torch.int32 or not d_scores.is_contiguous() or \
                d_scores.numel() < len(self.ms):
            raise ValueError("d_scores must be a contiguous int32 CUDA tensor of n_pairs elements")
        LB.check(LB.lib().msa_plan_scores(self._h, _ptr(d_scores), _stream_ptr(stream)), "msa_plan_scores")

    def stripe_meta(self, stream=None) -> np.ndarray:
        out = np.zeros((self.n_stripes, META_FIELDS), dtype=np.int32)
        LB.check(LB.lib().msa_plan_stripe_meta(self._h, out.ctypes.data_as(C.c_void_p), self.n_stripes,
                                               _stream_ptr(stream)), "msa_plan_stripe_meta")
        return out

    def checksum(self, dH, pair=0, stream=None) -> int:
        v = C.c_uint64()
        LB.check(LB.lib().msa_plan_checksum(self._h, _ptr(dH), pair, C.byref(v), _stream_ptr(stream)),
                 "msa_plan_checksum")
        return int(v.value)

    def traceback_async(self, dDir, d_ops, d_info, pair=0, stream=None) -> None:
        """Device traceback (msa_plan_traceback) of an SW-affine DIR plan, stream-ordered after run():
        d_ops (uint8, >= m+n) receives the ops end -> start, d_info (int64[4]) {n_ops, beg_i, beg_j, status}."""
        import torch

        if not (dDir.is_cuda and dDir.dtype == torch.uint8 and dDir.numel() >= self.cells_elems):
            raise ValueError("dDir must be the uint8 CUDA tensor the plan's run() wrote")
        if not (d_ops.is_cuda and d_ops.dtype == torch.uint8 and d_ops.is_contiguous()):
            raise ValueError("d_ops must be a contiguous uint8 CUDA tensor")
        if not (d_info.is_cuda and d_info.dtype == torch.int64 and d_info.numel() >= 8):
            raise ValueError("d_info must be an int64 CUDA tensor of >= 8 elements")
        LB.check(LB.lib().msa_plan_traceback(self._h, pair, _ptr(dDir), _ptr(d_ops), d_ops.numel(), _ptr(d_info),
                                             _stream_ptr(stream)), "msa_plan_traceback")

    def traceback(self, dDir, pair=0, stream=None):
        """Device traceback, fetched: dict(ops=bytes end -> start, beg=(i, j), cigar=run-length string)."""
        import torch

        dev = dDir.device
        ops = torch.empty(self.ms[pair] + self.ns[pair] + 2, dtype=torch.uint8, device=dev)
        info = torch.zeros(8, dtype=torch.int64, device=dev)
        self.traceback_async(dDir, ops, info, pair, stream)
        if stream is not None:
            # .cpu() below orders only against torch's current stream: wait for the walk's own
            (torch.cuda.ExternalStream(stream) if isinstance(stream, int) else stream).synchronize()
        inf = info.cpu().tolist()
        LB.check(int(inf[3]), "msa_plan_traceback")
        o = bytes(ops[:inf[0]].cpu().numpy().tobytes())
        return dict(ops=o, beg=(int(inf[1]), int(inf[2])), cigar=cigar_of(o),
                    stats=dict(switches=int(inf[4]), on_demand=int(inf[5]), ticks=int(inf[6]), requests=int(inf[7])))

    def traceback_gotoh_async(self, dDir, d_ops, d_info, end_type=-1, pair=0, stream=None) -> None:
        """Device find_alignment walk (msa_plan_traceback_gotoh) of a REF_GOTOH DIR plan, stream-ordered after
        run(): d_ops (uint8, >= m+n) receives one op per step end -> start ('M' T1, 'D' T2, 'I' T3), d_info
        (int64[8]) {n_ops, i+1, j+1, status, ...} with (i, j) the border cell the walk stopped at."""
        import torch

        if not (dDir.is_cuda and dDir.dtype == torch.uint8 and dDir.numel() >= self.cells_elems):
            raise ValueError("dDir must be the uint8 CUDA tensor the plan's run() wrote")
        if not (d_ops.is_cuda and d_ops.dtype == torch.uint8 and d_ops.is_contiguous()):
            raise ValueError("d_ops must be a contiguous uint8 CUDA tensor")
        if not (d_info.is_cuda and d_info.dtype == torch.int64 and d_info.numel() >= 8):
            raise ValueError("d_info must be an int64 CUDA tensor of >= 8 elements")
        LB.check(LB.lib().msa_plan_traceback_gotoh(self._h, pair, end_type, _ptr(dDir), _ptr(d_ops), d_ops.numel(),
                                                   _ptr(d_info), _stream_ptr(stream)), "msa_plan_traceback_gotoh")

    def traceback_gotoh(self, dDir, end_type=-1, pair=0):
        """Device find_alignment walk, fetched: dict(ops=bytes end -> start, stop=(i, j))."""
        import torch

        dev = dDir.device
        ops = torch.empty(self.ms[pair] + self.ns[pair] + 2, dtype=torch.uint8, device=dev)
        info = torch.zeros(8, dtype=torch.int64, device=dev)
        self.traceback_gotoh_async(dDir, ops, info, end_type, pair)
        inf = info.cpu().tolist()
        LB.check(int(inf[3]), "msa_plan_traceback_gotoh")
        return dict(ops=bytes(ops[:inf[0]].cpu().numpy().tobytes()), stop=(int(inf[1]) - 1, int(inf[2]) - 1))

    def set_timing(self, on: bool) -> None:
        """Record HIP events around the DP kernel in run() (default on; kernel_ms() needs it)."""
        LB.check(LB.lib().msa_plan_set_timing(self._h, int(bool(on))), "msa_plan_set_timing")

    def kernel_ms(self) -> float:
        v = C.c_float()
        LB.check(LB.lib().msa_plan_last_kernel_ms(self._h, C.byref(v)), "msa_plan_last_kernel_ms")
        return float(v.value)

    # ---- host-side layout helpers (tests / drop-in API) ----
    def deskew(self, flat: np.ndarray, pair: int, meta: np.ndarray, fill=0) -> np.ndarray:
        """Row-major (m+1) x (n+1) matrix of a pair's int32 cells (row/col 0 = fill)."""
        g = self.geom[pair]
        R = g.rows_per_lane
        S = (g.m + 64 * R - 1) // (64 * R)
        blk = flat[g.out_off:g.out_off + S * g.pmax * 1024 * R].reshape(S, g.pmax * 4, R, 64, 4)
        out = np.full((g.m + 1, g.n + 1), fill, dtype=flat.dtype)
        T = g.pmax * 16
        t = np.arange(T)
        r = np.arange(64)
        for s in range(S):
            cs = int(meta[g.stripe0 + s, 0])
            j = cs + t[None, :] - r[:, None]
            for rho in range(R):
                vals = blk[s, :, rho, :, :].transpose(1, 0, 2).reshape(64, T)  # [r][t]
                i = 64 * R * s + R * r + rho + 1
                ok = (i[:, None] <= g.m) & (j >= 0) & (j <= g.n)
                ii = np.broadcast_to(i[:, None], j.shape)
                out[ii[ok], j[ok]] = vals[ok]
        return out

    def deskew_dir(self, flat: np.ndarray, pair: int, meta: np.ndarray) -> np.ndarray:
        """Row-major (m+1) x (n+1) matrix of a pair's direction bytes.  Two rows per lane (the Gotoh flow
        fill): a 16-step block is 2 KiB, the wave's row-1 segments then its row-2 segments."""
        g = self.geom[pair]
        R = g.rows_per_lane
        S = (g.m + 64 * R - 1) // (64 * R)
        blk = flat[g.out_off:g.out_off + S * g.pmax * 1024 * R].reshape(S, g.pmax, R, 64, 16)
        out = np.zeros((g.m + 1, g.n + 1), dtype=np.uint8)
        T = g.pmax * 16
        t = np.arange(T)
        r = np.arange(64)
        for s in range(S):
            cs = int(meta[g.stripe0 + s, 0])
            j = cs + t[None, :] - r[:, None]
            for rho in range(R):
                vals = blk[s, :, rho].transpose(1, 0, 2).reshape(64, T)
                i = 64 * R * s + R * r + rho + 1
                ok = (i[:, None] <= g.m) & (j >= 1) & (j <= g.n)
                ii = np.broadcast_to(i[:, None], j.shape)
                out[ii[ok], j[ok]] = vals[ok]
        return out


def cigar_of(ops_end_to_start: bytes) -> str:
    """Run-length CIGAR (start -> end) of traceback ops given end -> start."""
    out, k = [], len(ops_end_to_start) - 1
    while k >= 0:
        op, run = ops_end_to_start[k], 0
        while k >= 0 and ops_end_to_start[k] == op:
            run += 1
            k -= 1
        out.append(f"{run}{chr(op)}")
    return "".join(out)


def jlo_of(i: int, band: int) -> int:
    return 1 if band < 0 else max(1, i - band)


def jhi_of(i: int, n: int, band: int) -> int:
    return n if band < 0 else min(n, i + band)


def stripe_geom(k: int, m: int, n: int, band: int, ks: int = 16):
    """Python restatement of stripe_geom() (msa_kernels.hip): (cs, P) of pair-local stripe k, P in phases of ks steps.

    Lane r of stripe k (row 64k+r+1) processes column cs + t - r at step t,
    t in [0, 16P); cs is chosen so that cs = c_lo - lead with
    lead = 1 + ((c_lo - 1 - k) mod 16), which 16-aligns producer/consumer ring I/O."""
    i0 = 64 * k + 1
    rlast = min(63, m - 64 * k - 1)
    ilast = i0 + rlast
    clo = jlo_of(i0, band)
    lead = (clo - 1 - k) % 16 + 1
    cs = clo - lead
    return cs, (jhi_of(ilast, n, band) - cs + rlast) // ks + 1


def stripe_phases(k: int, m: int, n: int, band: int, ks: int = 16) -> int:
    return stripe_geom(k, m, n, band, ks)[1]
