// msa_kernels.hip -- the DP-fill hot path as hand-written CDNA4 (gfx950) HIP.
//
// Replaces the reference's row sweep (Subproblem::compute_tables,
// subproblem_alignment.cpp:329-332; per-row T1/T3 map :229-235, T2 via the
// omega + ParallelPrefixMax scan :237-249 / :13-103) and partial.cpp's
// forward/reverse fills (:53-79) with ONE templated anti-diagonal stripe
// wavefront kernel:
//
//  * A "stripe" is 64 consecutive DP rows; one wave64 owns it, lane r = row
//    64s+r+1.  At step t lane r processes column cs + t - r (cs = the stripe's
//    start column), so the wave sweeps an anti-diagonal band.  The left
//    dependence stays in-lane (registers); the up/diag dependence comes from
//    lane r-1 through one DPP `wave_shr:1` per carried value (no LDS, no
//    __shfl).  The reference's horizontal prefix-max scan is not needed: the
//    in-lane left carry IS the scan.
//  * Lane 0 receives the row above the stripe as dedicated registers (DPP
//    `old` operand), lane 63 hands its bottom row to the next stripe through
//    an LDS ring (same workgroup) or 8-byte {tag,value} granules in HBM
//    (next workgroup; tag = launch epoch, so the data is its own flag).
//  * W compute waves per workgroup (4 = one per SIMD for a single pair, 8 in
//    batch mode) run W stripes in lock-step phases of 16 steps (one
//    s_barrier per phase); stripe k starts D_k ~ 5 phases after k-1.  A
//    separate loader wave stages the row above the workgroup's first stripe.
//  * The substitution score comes from a per-lane 8-byte profile selected by
//    v_perm_b32 with 4 column codes at a time; the byte is sign-extended into
//    the diagonal add by SDWA (no separate extract).
//  * Outputs (H / traceback bits / T1,T2,T3) are written in a skewed stripe
//    layout: one global_store_dwordx4 per lane per 4 steps, fully coalesced
//    (1 KiB per wave instruction).  Layout: element (s, t, r) of pair block
//    = ((s * pmax*4 + t/4) * 64 + r) * 4 + t%4   <->   cell (64s+r+1, cs_s+t-r).
//
// Three launch modes share the kernel:
//  * single: one pair, items = groups of W stripes, tickets in order
//    (a workgroup only ever waits on an earlier ticket -> no deadlock).
//  * batch: items = whole pairs; wave w runs stripes w, w+W, ...; the
//    wave W-1 -> wave 0 wrap link goes through a full LDS row buffer.
//  * chunked (banded single pair, rank convergence): items = chunks of
//    chunk_c consecutive stripes, each run batch-style by one workgroup, all
//    at once.  Chunk k starts chunk_warm stripes before its first stripe from a
//    GUESSED row (a tent shaped like the row-0 border) instead of waiting for
//    chunk k-1: banded max-plus DP forgets its input, so after enough rows the
//    guessed run equals the exact one up to one additive constant.  Those
//    warm-up stripes write no cells; the run's state (H, F over the band) at the
//    end of the warm-up and at the chunk's last row go to a checkpoint buffer,
//    and chunk_check/chunk_add_kernel verify the constant exactly (every band
//    entry) and add the prefix of the constants to each chunk's cells.  If any
//    chunk has not converged, the plan's exact single-mode launch (queued
//    behind, skipped otherwise) recomputes everything.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "msa_types.h"

#ifndef MSA_WAVES_SINGLE
#define MSA_WAVES_SINGLE 4  // single pair: one compute wave per SIMD (latency-bound wavefront)
#endif
#ifndef MSA_KS_SINGLE
#define MSA_KS_SINGLE 32  // steps per phase, single pair: fewer phases amortise the per-phase sync
#endif
#define MSA_KS_BATCH 16   // steps per phase, batch: fewer registers, two workgroups per CU
#ifndef MSA_KS_BATCH_SWLP
#define MSA_KS_BATCH_SWLP 16  // packed-int16 batches (C4; 32 measured: 3.55 vs 2.76 ms)
#endif
#define MSA_WAVES_BATCH 8   // batch: two per SIMD (throughput-bound, hides the step chain)
#define MSA_K 16  // output layout block: cells are stored in blocks of 16 steps (any KS is a multiple)
#define MSA_RING 256
#define MSA_ROWOFF 128
#define MSA_GOFF 128
#define MSA_NEG (-(1 << 30))
#define MSA_VIRT_CODE 7u     // SW: column code outside [1, n] (real symbols use codes 0..6)
#define MSA_NTICKET 128      // run tickets (ints): [0] stripe_kernel, [4..11] flow item chunks,
#define MSA_TK_ARRIVE 32     // flow kernel: arrival order (pass-1 / pass-2 role), own 128-B line
#define MSA_TK_BLOCK 64      // flow kernel: pass-2 blocks, own 128-B line
#define MSA_TK_BEST 96       // flow kernel, fused reduction: the best block key (u64), own 128-B line
#define MSA_TK_DONE 100      //   and the finished pass-2 blocks
#define MSA_CPAD 256         // code segment padding (bytes) on each side of a pair's columns
#define MSA_NCOPY 16         // byte-shifted code copies: every lane reads 16-byte aligned dwordx4
#define MSA_CRING 1024       // single-pair LDS code ring: columns per copy (+64 B mirror), 4 copies
#define MSA_VIRT_SCORE (-100)  // its profile byte (s + 2g space for SWL; < 0 is all that matters)

namespace msa {

template <int ALG> struct Tr;
template <> struct Tr<MSA_ALG_SWL> { static constexpr int NC = 1; };
template <> struct Tr<MSA_ALG_SWL0> { static constexpr int NC = 1; };
template <> struct Tr<MSA_ALG_SWLP> { static constexpr int NC = 1; };
// SW linear in shifted space (any of the three kernel ids)
constexpr bool swlin(int alg) { return alg == MSA_ALG_SWL || alg == MSA_ALG_SWL0 || alg == MSA_ALG_SWLP; }
// two pairs per lane: every carried value is two int16 (pair 2c low, pair 2c+1 high)
constexpr bool pk16(int alg) { return alg == MSA_ALG_SWLP; }
template <> struct Tr<MSA_ALG_SWA> { static constexpr int NC = 2; };
template <> struct Tr<MSA_ALG_NWA> { static constexpr int NC = 2; };
template <> struct Tr<MSA_ALG_REF> { static constexpr int NC = 3; };
template <> struct Tr<MSA_ALG_REF1> { static constexpr int NC = 2; };
template <> struct Tr<MSA_ALG_PART> { static constexpr int NC = 3; };

// packed int16 helpers (v_pk_add_u16 / v_pk_max_i16 on gfx950)
typedef short msa_s2 __attribute__((ext_vector_type(2)));
__host__ __device__ __forceinline__ int pk2(int v) { return (int)(((unsigned)v & 0xffffu) * 0x10001u); }
__device__ __forceinline__ int pk_add(int a, int b) {
  return __builtin_bit_cast(int, __builtin_bit_cast(msa_s2, a) + __builtin_bit_cast(msa_s2, b));
}
__device__ __forceinline__ int pk_max(int a, int b) {
  return __builtin_bit_cast(int, __builtin_elementwise_max(__builtin_bit_cast(msa_s2, a), __builtin_bit_cast(msa_s2, b)));
}
__device__ __forceinline__ int dpp_shr1(int old, int src) {
  return __builtin_amdgcn_update_dpp(old, src, 0x138, 0xf, 0xf, false);
}
// wave_shl:1 -- lane l takes lane l+1, lane 63 keeps `old`
__device__ __forceinline__ int dpp_shl1(int old, int src) {
  return __builtin_amdgcn_update_dpp(old, src, 0x130, 0xf, 0xf, false);
}
__host__ __device__ __forceinline__ int imax(int a, int b) { return a > b ? a : b; }
__device__ __forceinline__ int imax3(int a, int b, int c) { return imax(imax(a, b), c); }
// first index (1,2,3) attaining the max, the reference's tie order
// (subproblem_alignment.cpp:130-145, partial.cpp:153)
__device__ __forceinline__ int firstmax3(int a, int b, int c) {
  return (a >= b && a >= c) ? 1 : (b >= c ? 2 : 3);
}
// Wave-uniform value into an SGPR: keeps phase-level branches scalar (values
// read from LDS are otherwise treated as divergent, and every DP step ends up
// wrapped in exec-mask branching).
__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ int wrap_add(int a, int b) { return (int)((unsigned)a + (unsigned)b); }
__device__ __forceinline__ int wrap_sub(int a, int b) { return (int)((unsigned)a - (unsigned)b); }

struct StripeGeom {
  int T, P, cs, lead, mask_lo, mask_hi, c_hi, pad;
};

__host__ __device__ __forceinline__ int jlo_of(int i, int band) { return band < 0 ? 1 : imax(1, i - band); }
__host__ __device__ __forceinline__ int jhi_of(int i, int n, int band) { return band < 0 ? n : (i + band < n ? i + band : n); }

// Geometry of pair-local stripe k (rows 64k+1 .. 64k+64).
__host__ __device__ inline void stripe_geom(int k, int m, int n, int band, StripeGeom& g, int KS) {
  const int i0 = 64 * k + 1;
  const int rlast = (m - 64 * k - 1 < 63) ? (m - 64 * k - 1) : 63;
  const int ilast = i0 + rlast;
  const int clo = jlo_of(i0, band);
  int lead = (clo - 1 - k) % 16;
  if (lead < 0) lead += 16;
  lead += 1;
  g.lead = lead;
  g.cs = clo - lead;
  const int tmax_max = jhi_of(ilast, n, band) - g.cs + rlast;
  g.P = tmax_max / KS + 1;  // phases of KS steps
  g.mask_lo = jlo_of(ilast, band) - g.cs + rlast;  // max over rows of tmin
  g.mask_hi = jhi_of(i0, n, band) - g.cs - 1;      // min over rows of tmax, minus 1: every row's
                                                   // last step (final-state capture) is in a masked phase
  g.c_hi = jhi_of(ilast, n, band);
  g.T = 0;
  g.pad = 0;
}

struct KArgs {
  msa_kparams kp;
  const uint8_t* A;
  const uint8_t* B;
  const msa_pair_desc* pairs;
  msa_stripe_meta* meta;
  int* ticket;
  unsigned long long* gbuf;  // single mode: [n_items-1][NC][n + 2*GOFF] granules
  int gbuf_stride;           // granules per (item, value)
  int* err;                  // timeout / error flag
  int32_t* outH;             // O_H (or plane 0 of O_TAB)
  int32_t* outT2;            // O_TAB planes
  int32_t* outT3;
  uint8_t* outDir;           // O_DIR
  const uint8_t* cod;        // MSA_NCOPY byte-shifted copies of the padded column codes (stage_codes_kernel)
  long long cod_copy;        // bytes per copy
  unsigned long long* stamps;  // diagnostic build only (MSA_STAMPS): per-phase s_memtime
  // two-pass single pair (msa_flow.hip)
  // {epoch, value} granules: pass-2 blocks run while pass 1 is still producing
  unsigned long long* br;    // [S][brw] bottom row of every stripe
  unsigned long long* snap;  // [S][nseg][2][64] lane states at the start of every pass-2 segment
  int4* blk;                 // [S * nseg] pass-2 block bests
  const int* border;         // pass-2 blocks in expected readiness order
  int brw, nseg, nblk;
  int ps_shift;              // log2 of the phases per pass-2 segment (pass 1 saves SNAP that often)
  int nflow;                 // workgroups [0, nflow) run pass 1, the rest pass-2 blocks
  // chunked banded mode (kp.single == 2)
  int* ck;                   // [chunk][2: warm-up end, chunk end][2: H, F][ckw] band states
  int ckw;                   // entries per band row (2*band + 1, padded)
  const int* skip;           // exact single-mode launch: exit at once when *skip != 0
  // chunked banded mode with int16 chunk cells: chunks >= 1 write H relative to their guessed row as
  // int16 here ([stripe - chunk_c][pmax * 16 * 64], the outH cell order); chunk_add_kernel widens them
  int16_t* outH16;
  // two-pass SW single pair: the pass-2 blocks fold the pair result into this key themselves
  // (fl_block_result, msa_flow.hip) when set; else reduce_blocks_kernel runs after the launch
  unsigned long long* best_key;
};
#ifndef MSA_H16_PAIRED
#define MSA_H16_PAIRED 1  // int16 chunk cells: two u-blocks of a lane per 16 B (msa_band.hip)
#endif

template <int ALG>
__device__ __forceinline__ void border_top(const msa_kparams& kp, int c, int (&v)[3], int r0 = 0) {
  // Row 0 of the DP at column c (c may be < 0: unused, return NEG).  Banded Gotoh,
  // r0 > 0 (chunked mode): the GUESSED row r0 a chunk's warm-up starts from -- the
  // row-0 border's tent moved to the diagonal, H = -h - g*|c - r0| inside the band.
  if constexpr (swlin(ALG)) {
    // G(0,c) = H(0,c) + g*c = g*c; SWL0 also on the virtual columns c < 0
    v[0] = (c >= 0 || ALG == MSA_ALG_SWL0 || ALG == MSA_ALG_SWLP) ? kp.gap_open * c : MSA_NEG;
    if constexpr (pk16(ALG)) v[0] = pk2(v[0]);
    v[1] = MSA_NEG;
    v[2] = MSA_NEG;
  } else if constexpr (ALG == MSA_ALG_SWA) {
    v[0] = c >= 0 ? 0 : MSA_NEG;  // H
    v[1] = MSA_NEG;               // F
    v[2] = MSA_NEG;
  } else if constexpr (ALG == MSA_ALG_NWA) {
    if (r0 > 0) {
      const int d = c > r0 ? c - r0 : r0 - c;
      v[0] = (d <= kp.band) ? -kp.h - kp.gap_ext * d : MSA_NEG;
    } else {
      // H(0,c) = max(T1,T2,T3)(0,c): 0 at c=0, -h-g*c for 1<=c<=band; F = -inf
      const bool inb = (kp.band < 0) || (c <= kp.band);
      v[0] = (c == 0) ? 0 : ((c > 0 && inb) ? -kp.h - kp.gap_ext * c : MSA_NEG);
    }
    v[1] = MSA_NEG;
    v[2] = MSA_NEG;
  } else if constexpr (ALG == MSA_ALG_REF1) {
    // row 0 for start type -1 (:212-227): T1(0,0) = 0, T2(0,c) = -h-g*c (c >= 1), rest -inf;
    // tagged (see step<REF1>): v[0] = max(T1,T2,T3)~, v[1] = the row below's T3 candidates~
    const int GH = kp.gap_open, G = kp.gap_ext;
    if (c < 0) { v[0] = v[1] = v[2] = MSA_NEG; return; }
    if (c == 0) {
      v[0] = 3;                // T1 = 0, tag T1
      v[1] = 4 * (-GH) + 3;    // T1 - g - h
    } else {
      const int t2 = -kp.h - G * c;
      v[0] = 4 * t2 + 2;
      v[1] = 4 * (t2 - GH) + 2;
    }
    v[2] = MSA_NEG;
  } else if constexpr (ALG == MSA_ALG_REF) {
    // compute_row(0) / ComputeFirstRowMapThread (subproblem_alignment.cpp:212-227,259-280)
    const int st = kp.start_type;
    const int g = kp.gap_ext, h = kp.h;
    if (c < 0) { v[0] = v[1] = v[2] = MSA_NEG; return; }
    if (c == 0) {
      v[0] = (st == 1 || st == -1) ? 0 : MSA_NEG;
      v[1] = (st == -2) ? 0 : MSA_NEG;
      v[2] = (st == -3) ? 0 : MSA_NEG;
    } else {
      v[0] = MSA_NEG;
      v[2] = MSA_NEG;
      v[1] = (st == -2) ? -g * c : ((st == 1 || st == 3) ? MSA_NEG : -h - g * c);
    }
  } else {  // PART: initializeTables (partial.cpp:13-31), wrap semantics
    const int st = kp.start_type;
    v[0] = (c == 0 && st == 1) ? 0 : INT32_MIN;
    v[1] = (c >= 1 && st == 2) ? (int)((unsigned)(-kp.gap_open) * (unsigned)c) : INT32_MIN;
    v[2] = INT32_MIN;
  }
}

template <int ALG>
__device__ __forceinline__ void border_left(const msa_kparams& kp, int i, int (&v)[3]) {
  // Column 0 of row i (i >= 1), state order of each algorithm.
  if constexpr (swlin(ALG)) {
    v[0] = pk16(ALG) ? pk2(kp.gap_open * i) : kp.gap_open * i;  // G(i,0) = H(i,0) + g*i
    v[1] = MSA_NEG;
    v[2] = MSA_NEG;
  } else if constexpr (ALG == MSA_ALG_SWA) {
    v[0] = 0;        // H
    v[1] = MSA_NEG;  // E
    v[2] = MSA_NEG;  // F
  } else if constexpr (ALG == MSA_ALG_NWA) {
    const bool inb = (kp.band < 0) || (i <= kp.band);
    v[0] = inb ? -kp.h - kp.gap_ext * i : MSA_NEG;  // H
    v[1] = MSA_NEG;                                 // T2 (E)
    v[2] = v[0];                                    // T3 (F) = -h-g*i
  } else if constexpr (ALG == MSA_ALG_REF1) {
    // column 0 for start type -1 (:282-292): T1 = T2 = -inf, T3 = -h-g*i; state (H~, R~, D~)
    const int t3 = -kp.h - kp.gap_ext * i;
    v[0] = 4 * t3 + 1;
    v[1] = 4 * (t3 - kp.gap_open) + 1;
    v[2] = 4 * (t3 - kp.gap_ext) + 1;
  } else if constexpr (ALG == MSA_ALG_REF) {
    // compute_row(i>0) borders (subproblem_alignment.cpp:282-292)
    const int st = kp.start_type;
    v[0] = MSA_NEG;
    v[1] = MSA_NEG;
    v[2] = (st == -3) ? -kp.gap_ext * i : ((st == 1 || st == 2) ? MSA_NEG : -kp.h - kp.gap_ext * i);
  } else {
    const int st = kp.start_type;
    v[0] = INT32_MIN;
    v[1] = INT32_MIN;
    v[2] = (st == 3) ? (int)((unsigned)(-kp.gap_open) * (unsigned)i) : INT32_MIN;
  }
}

// Per-lane register state of the stripe a wave is running.
template <int ALG>
struct LaneState {
  int S[3];    // left-cell state (algorithm order, see step())
  unsigned plo2, phi2;  // SWLP: the second pair's profile
  int U[3];    // diagonal values (previous step's up values)
  int LB[3];   // left border held while t < tmin
  int tmin, tmax;
  int best, bt;  // SW best in this lane's row and the step it first occurred
  int pb;        // SWLP: max over the current phase's steps k of G - g k (both pairs, int16)
  int fin[3];
  unsigned plo, phi;  // substitution profile (8 int8 scores by column code)
  int i;              // DP row
};

// One DP step for every lane.  in[v] = value lane 0 takes from the row above.
// Returns the direction byte for O_DIR.
//
// SW linear runs in shifted space G(i,j) = H(i,j) + g*(i+j):
//   G = max(G(i-1,j-1) + s + 2g,  G(i-1,j),  G(i,j-1),  g*(i+j))
// (the 2g is folded into the substitution profile), so the loop-carried chain
// per step is DPP -> v_max3 instead of DPP -> max -> sub -> max3.  Rings and
// granules carry G; H = G - g*(i+j) is only formed for the output / best.
// TRACKPOS: 0 = best value only, 1 = best value and its first step, 2 = the same as one
// packed int (value << 15 | 32767 - step; plans with H < 2^16 and < 2^15 steps per
// stripe): one max instead of a compare and two selects per step, and a larger key is
// the larger value, then the earlier step -- the first maximum, as in mode 1.
template <int ALG, int OUT, bool MASKED, int TRACKPOS, bool FIN = false>
__device__ __forceinline__ unsigned step(const msa_kparams& kp, LaneState<ALG>& L, const int (&in)[3], int s,
                                         int t, int ct, int (&carry)[3], int& hout) {
  unsigned dir = 0;
  int nS[3];
  int fin_tab[3];  // REF1: the cell's untagged T1, T2, T3 (the final state at (m, n))
  if constexpr (ALG == MSA_ALG_SWL) {
    // ct = g*(i+j) is the same for every lane (one anti-diagonal): an SGPR
    const int up = dpp_shr1(in[0], L.S[0]);
    const int x = imax(L.U[0] + s, ct);
    nS[0] = imax3(x, up, L.S[0]);
    // opaque: keeps G a real per-step value (otherwise LLVM flattens the
    // running max3 chain and distributes the "- ct" over every term)
    asm("" : "+v"(nS[0]));
    L.U[0] = up;
  } else if constexpr (ALG == MSA_ALG_SWLP) {
    // MSA_ALG_SWL0 on two pairs at once: s holds both pairs' score + 2g as int16.  The cell above (the
    // DPP from lane r-1) enters last: the loop-carried path per step is DPP -> one v_pk_max_i16, the
    // diagonal-left max runs in the DPP's wait states
    const int up = dpp_shr1(in[0], L.S[0]);
    nS[0] = pk_max(pk_max(pk_add(L.U[0], s), L.S[0]), up);
    L.U[0] = up;
  } else if constexpr (ALG == MSA_ALG_SWL0) {
    // all scores >= 0: G(i-1,j-1) + s + 2g >= g*(i+j) whenever the diagonal
    // cell satisfies its own floor, so (by induction from the borders) the
    // zero floor never binds and is dropped.  Virtual columns score 0, which
    // keeps G = g*(i+j) (H = 0) on every cell left of column 1.
    const int up = dpp_shr1(in[0], L.S[0]);
    nS[0] = imax3(L.U[0] + s, up, L.S[0]);
    asm("" : "+v"(nS[0]));
    L.U[0] = up;
  } else if constexpr (ALG == MSA_ALG_SWA) {
    const int upH = dpp_shr1(in[0], L.S[0]);
    const int upF = dpp_shr1(in[1], L.S[2]);
    const int f = imax(upF - kp.gap_ext, upH - kp.gap_open);
    const int e = imax(L.S[1] - kp.gap_ext, L.S[0] - kp.gap_open);
    const int d = L.U[0] + s;
    const int h = imax(imax3(d, e, f), 0);
    if constexpr (OUT == MSA_OUT_DIR) {
      const unsigned hs = (h == 0) ? 0u : (h == d ? 1u : (h == e ? 2u : 3u));
      const unsigned eb = (e == L.S[0] - kp.gap_open) ? 4u : 0u;
      const unsigned fb = (f == upH - kp.gap_open) ? 8u : 0u;
      dir = hs | eb | fb;
    }
    nS[0] = h;
    nS[1] = e;
    nS[2] = f;
    L.U[0] = upH;
  } else if constexpr (ALG == MSA_ALG_NWA) {
    const int upH = dpp_shr1(in[0], L.S[0]);
    const int upF = dpp_shr1(in[1], L.S[2]);
    const int t3 = imax(upH - kp.gap_open, upF - kp.gap_ext);
    const int t2 = imax(L.S[0] - kp.gap_open, L.S[1] - kp.gap_ext);
    const int t1 = L.U[0] + s;
    nS[0] = imax3(t1, t2, t3);
    nS[1] = t2;
    nS[2] = t3;
    L.U[0] = upH;
  } else if constexpr (ALG == MSA_ALG_REF1) {
    // Start type -1: every table value of every cell with i, j >= 1 is finite (each has a
    // finite predecessor), so -inf needs no exact emulation and the three first-maximum
    // selections of find_alignment (:130-145) fold into the maxima: a value of table k is
    // carried TAGGED as 4*T + (4-k), so max() of tagged values is the maximum, ties going to
    // the lower table -- the reference's order.  Per cell the lane forms
    //   H~ = max(T1~, T2~, T3~)            -> the cell diagonally below: T1 = H + f, its tag
    //   R~ = max(T1~ - 4gh, T2~ - 4g, T3~ - 4gh)  (gh = g + h) -> T2 of the cell to the right
    //   D~ = max(T1~ - 4gh, T2~ - 4gh, T3~ - 4g)  -> T3 of the cell below
    // so only H~ and D~ cross lanes (2 DPPs), and the direction byte is three tags: the
    // diagonal's H~ (T1's predecessor), the left cell's R~ (T2's), the upper cell's D~ (T3's);
    // tag 3 / 2 / 1 = table T1 / T2 / T3.  s = 4f (profile).
    const int uH = dpp_shr1(in[0], L.S[0]);
    const int uD = dpp_shr1(in[1], L.S[2]);
    const int GH4 = 4 * kp.gap_open, G4 = 4 * kp.gap_ext;
    const int t1 = (int)((unsigned)L.U[0] | 3u) + s;  // 4(H_diag + f) + 3
    const int t2 = (int)(((unsigned)L.S[1] & ~3u) | 2u);
    const int t3 = (int)(((unsigned)uD & ~3u) | 1u);
    nS[0] = imax3(t1, t2, t3);
    nS[1] = imax(imax(t1, t3) - GH4, t2 - G4);
    nS[2] = imax(imax(t1, t2) - GH4, t3 - G4);
    if constexpr (OUT == MSA_OUT_DIR)
      dir = ((unsigned)L.U[0] & 3u) | (((unsigned)L.S[1] & 3u) << 2) | (((unsigned)uD & 3u) << 4);
    fin_tab[0] = t1 >> 2;
    fin_tab[1] = t2 >> 2;
    fin_tab[2] = t3 >> 2;
    L.U[0] = uH;
  } else if constexpr (ALG == MSA_ALG_REF) {
    const int u0 = dpp_shr1(in[0], L.S[0]);
    const int u1 = dpp_shr1(in[1], L.S[1]);
    const int u2 = dpp_shr1(in[2], L.S[2]);
    const int GH = kp.gap_open, G = kp.gap_ext;
    // exact -inf: every stored value is finite (> -2^29) or exactly MSA_NEG
    const int mx = imax3(L.U[0], L.U[1], L.U[2]);
    const int t1 = (mx == MSA_NEG) ? MSA_NEG : mx + s;
    const int a = imax(L.S[0] - GH, MSA_NEG), b = imax(L.S[1] - G, MSA_NEG), c = imax(L.S[2] - GH, MSA_NEG);
    const int t2 = imax3(a, b, c);
    const int a3 = imax(u0 - GH, MSA_NEG), b3 = imax(u1 - GH, MSA_NEG), c3 = imax(u2 - G, MSA_NEG);
    const int t3 = imax3(a3, b3, c3);
    if constexpr (OUT == MSA_OUT_DIR) {
      dir = (unsigned)firstmax3(L.U[0], L.U[1], L.U[2]) | ((unsigned)firstmax3(a, b, c) << 2) |
            ((unsigned)firstmax3(a3, b3, c3) << 4);
    }
    nS[0] = t1;
    nS[1] = t2;
    nS[2] = t3;
    L.U[0] = u0;
    L.U[1] = u1;
    L.U[2] = u2;
  } else {  // PART: fillTablesParallel (partial.cpp:53-65), int32 wrap
    const int u0 = dpp_shr1(in[0], L.S[0]);
    const int u1 = dpp_shr1(in[1], L.S[1]);
    const int u2 = dpp_shr1(in[2], L.S[2]);
    const int GH = kp.gap_open, G = kp.gap_ext;
    nS[0] = imax3(wrap_add(L.U[0], s), wrap_add(L.U[1], s), wrap_add(L.U[2], s));
    nS[1] = imax3(wrap_sub(L.S[0], GH), wrap_sub(L.S[1], G), wrap_sub(L.S[2], GH));
    nS[2] = imax3(wrap_sub(u0, GH), wrap_sub(u1, GH), wrap_sub(u2, G));
    L.U[0] = u0;
    L.U[1] = u1;
    L.U[2] = u2;
  }
  constexpr int NS = swlin(ALG) ? 1 : 3;
  (void)fin_tab;
  if constexpr (MASKED) {
    const bool before = t < L.tmin;
    const bool after = t > L.tmax;
#pragma unroll
    for (int v = 0; v < NS; ++v) nS[v] = before ? L.LB[v] : (after ? MSA_NEG : nS[v]);
    if constexpr (swlin(ALG) || ALG == MSA_ALG_SWA) {
      const int hv = swlin(ALG) ? nS[0] - ct : nS[0];
      hout = hv;
      if constexpr (TRACKPOS == 2) {
        L.best = imax(L.best, (!before && !after) ? (hv << 15) + (32767 - t) : 0);
      } else if (!before && !after) {
        if constexpr (TRACKPOS) {
          if (hv > L.best) { L.best = hv; L.bt = t; }
        } else {
          L.best = imax(L.best, hv);
        }
      }
    } else if constexpr (FIN) {  // only the stripe holding row m
      if (t == L.tmax) {
#pragma unroll
        for (int v = 0; v < 3; ++v) L.fin[v] = (ALG == MSA_ALG_REF1) ? fin_tab[v] : nS[v];
      }
    }
  } else {
    if constexpr (pk16(ALG)) {
      // ct = pk2(-g k) for step k of the phase (an SGPR fixed for the whole launch): the phase's best
      // of G - g k in both halves; the phase's g (i + j) at its step 0 is subtracted once per phase
      // (run_phase), so no scalar arithmetic runs per step
      static_assert(TRACKPOS == 0, "packed pairs: score only");
      // (KS = 16, unmasked: run_phase replaces this running max by a tree over the phase's carried
      // values, and these updates are dead code there)
      L.pb = pk_max(L.pb, pk_add(nS[0], ct));
      hout = 0;
    } else if constexpr (swlin(ALG) || ALG == MSA_ALG_SWA) {
      const int hv = swlin(ALG) ? nS[0] - ct : nS[0];
      hout = hv;
      if constexpr (TRACKPOS == 2) {
        L.best = imax(L.best, (hv << 15) + (32767 - t));
      } else if constexpr (TRACKPOS) {
        if (hv > L.best) { L.best = hv; L.bt = t; }
      } else {
        L.best = imax(L.best, hv);
      }
    }
  }
#pragma unroll
  for (int v = 0; v < NS; ++v) L.S[v] = nS[v];
  // carried values (what the lane below / next stripe needs)
  if constexpr (swlin(ALG)) {
    carry[0] = nS[0];
  } else if constexpr (ALG == MSA_ALG_SWA || ALG == MSA_ALG_NWA || ALG == MSA_ALG_REF1) {
    carry[0] = nS[0];
    carry[1] = nS[2];
  } else {
    carry[0] = nS[0];
    carry[1] = nS[1];
    carry[2] = nS[2];
  }
  return dir;
}

// Banded Gotoh (MSA_ALG_NWA) edges without per-step range masks.  A lane runs the
// bare recurrence on every step, also outside its row's band [tmin, tmax]; those
// values reach an in-band cell only through two cells, fixed up here:
//  * t == tmin - 1 (column jlo - 1: out of band, or the border column 0 when jlo = 1):
//    the state becomes the left border LB, so the row's first cell sees the exact
//    left neighbour (and the row below, whose first cell takes its diagonal from
//    column jlo - 1 only when that is the border column, the exact border value);
//  * t == tmax + 1 (column jhi + 1): H and T3 become -inf, the "up" of the row
//    below's last in-band cell (and of the next stripe's lane 0).
// Everything else a lane computes outside its band feeds only out-of-band cells (the
// row below starts and ends one column later), so in-band H, the hand-offs read at
// in-band cells and the final cell equal the masked recurrence's.  FIN captures the
// final cell at t == tmax.  Cost: 2 compares + 5 selects per step, against ~13 for
// the range masks -- and for a band the masked head phases are the chain's
// critical path (stripe k+1 starts ~9 phases into stripe k).
template <bool FIN>
__device__ __forceinline__ void band_fix(LaneState<MSA_ALG_NWA>& L, int t, int (&carry)[3]) {
  const bool fl = (t == L.tmin - 1);
#pragma unroll
  for (int v = 0; v < 3; ++v) L.S[v] = fl ? L.LB[v] : L.S[v];
  if constexpr (FIN) {
    const bool e = (t == L.tmax);
#pragma unroll
    for (int v = 0; v < 3; ++v) L.fin[v] = e ? L.S[v] : L.fin[v];
  }
  const bool fr = (t == L.tmax + 1);
  L.S[0] = fr ? MSA_NEG : L.S[0];
  L.S[2] = fr ? MSA_NEG : L.S[2];
  carry[0] = L.S[0];
  carry[1] = L.S[2];
}

// Bounded spin helper for cross-workgroup granule waits.
__device__ __forceinline__ unsigned long long gload(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gstore(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Cell-output stores (H / T2 / T3 / direction planes) are written once and
// never read back by the kernel: non-temporal stores stream them at ~64 B/clk
// per CU, where plain (write-allocate) stores saturate at ~8 B/clk per CU --
// below what four stripe waves produce (mbench/mb_store.hip measurement).
typedef int msa_v4i __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void ntstore(int4* p, int4 v) {
  const msa_v4i x = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(x, reinterpret_cast<msa_v4i*>(p));
}

enum Src { SRC_BORDER = 0, SRC_RING = 1, SRC_ROW = 2, SRC_GLOBAL = 3 };
enum Snk { SNK_NONE = 0, SNK_RING = 1, SNK_ROW = 2, SNK_GLOBAL = 3 };

// Loader wave (wave W): in single mode it pulls the row above the
// item's first stripe from the previous workgroup's granules (HBM, `sc1`)
// into the LDS staging ring one phase ahead, so no compute wave ever waits
// on a global load.

// Phase barrier.  The diagnostic build (-DMSA_STAMPS) records s_memtime just
// before and after every barrier of every wave: stamps[((item*16 + wave)*4096
// + phase)*2 + {0,1}] (phases >= 4096 and items >= 64 are not recorded).
#define MSA_BARRIER_() __syncthreads()
#ifdef MSA_STAMPS
#ifdef MSA_STAMPS_RT
#define MSA_CLOCK() __builtin_amdgcn_s_memrealtime()  // chip-wide 100 MHz: comparable across XCDs
#else
#define MSA_CLOCK() __builtin_amdgcn_s_memtime()
#endif
#define MSA_SYNC(ph_)                                                                       \
  do {                                                                                      \
    const int ph__ = (ph_);                                                                 \
    const bool rec__ = a.stamps && lane == 0 && ph__ < 4096 && item < 64;                   \
    const size_t o__ = (((size_t)item * 16 + w) * 4096 + ph__) * 4;                          \
    if (rec__) a.stamps[o__] = MSA_CLOCK();                                                 \
    MSA_BARRIER_();                                                                         \
    if (rec__) a.stamps[o__ + 1] = MSA_CLOCK();                                             \
  } while (0)
#define MSA_MARK(ph_, slot_)                                                                \
  do {                                                                                      \
    const int ph__ = (ph_);                                                                 \
    if (a.stamps && lane == 0 && ph__ < 4096 && item < 64)                                  \
      a.stamps[(((size_t)item * 16 + w) * 4096 + ph__) * 4 + (slot_)] = MSA_CLOCK();          \
  } while (0)
#else
#define MSA_SYNC(ph_) MSA_BARRIER_()
#define MSA_MARK(ph_, slot_) do {} while (0)
#endif

// c = 16-column chunk index of the item's first stripe (nch chunks in all).
template <int NC>
__device__ __forceinline__ void loader_commit(const KArgs& a, int cs0, int nch, int q, unsigned long long gv,
                                              const unsigned long long* g_in, int* stage, int chi, int n,
                                              unsigned ep, int lane) {
  const int v = lane >> 4, l = lane & 15;
  const int col = cs0 + 16 * q + l;
  const bool need = (v < NC) && (col <= chi) && (col <= n) && (q < nch);
  bool ok = !need || ((unsigned)(gv >> 32) == ep);
  unsigned spins = 0;
  while (!__all(ok)) {
    __builtin_amdgcn_s_sleep(1);
    const int cc = min(col, a.gbuf_stride - 1 - MSA_GOFF);
    const unsigned long long r = gload(g_in + (size_t)min(v, NC - 1) * a.gbuf_stride + cc + MSA_GOFF);
    gv = ok ? gv : r;
    ok = !need || ((unsigned)(gv >> 32) == ep);
    if (++spins > (1u << 24)) break;
  }
  if (spins > (1u << 24) && lane == 0) atomicExch(a.err, 1);  // (after the loop: a uniform wait loop)
  if (v < NC) stage[v * MSA_RING + ((16 * q + l) & (MSA_RING - 1))] = need ? (int)(unsigned)gv : MSA_NEG;
}

template <int NC>
__device__ __forceinline__ unsigned long long loader_issue(const KArgs& a, int cs0, int q,
                                                           const unsigned long long* g_in, int lane) {
  const int v = min(lane >> 4, NC - 1), l = lane & 15;
  const int col = min(cs0 + 16 * q + l, a.gbuf_stride - 1 - MSA_GOFF);
  return gload(g_in + (size_t)v * a.gbuf_stride + col + MSA_GOFF);
}

// SGL: single-pair variant (loader + code wave, LDS code ring, DPP shift-register hand-off)
template <int ALG, int OUT, int TRACKPOS, int W, int KS, bool SGL>
__global__ __launch_bounds__((W + 1 + (SGL ? 1 : 0)) * 64) void stripe_kernel(KArgs a) {
  static_assert(KS % 16 == 0 && KS <= 64, "phases are whole 16-step layout blocks");
  constexpr int CPP = KS / 16;  // 16-column chunks per phase
  constexpr int NC = Tr<ALG>::NC;
  // Smith-Waterman kernels never mask: columns outside [1, n] carry the
  // virtual code whose score (MSA_VIRT_SCORE) keeps every out-of-matrix cell
  // strictly below a real cell, so the plain recurrence runs over them.
  constexpr bool SWK = (swlin(ALG) || ALG == MSA_ALG_SWA);
  extern __shared__ __attribute__((aligned(16))) int smem[];
  const msa_kparams& kp = a.kp;
  const int lane = threadIdx.x & 63;
  const int w = uni(threadIdx.x >> 6);
  // the exact launch queued behind a chunked run: nothing to do when every chunk converged
  if (a.skip && uni(*(volatile const int*)a.skip)) return;

  // ---- LDS carve (int32 units, all offsets multiples of 4) ----
  int* misc = smem;  // 16 ints
  StripeGeom* sched = reinterpret_cast<StripeGeom*>(smem + 16);
  const int sched_cap = kp.sched_cap;
  // rings: [parity 2][wave W][NC][RING] + staging [NC][RING]
  int* rings = smem + 16 + sched_cap * 8;
  int* stage = rings + 2 * W * NC * MSA_RING;
  int* rowbuf = stage + NC * MSA_RING;  // NC x lds_row_words (batch wrap link)
  // single pair: 4 byte-shifted copies of a sliding column-code window, staged
  // by the loader wave two phases ahead, so compute waves never wait on vmcnt
  // (their only VMEM ops are stores).  Copy c, dword d holds columns
  // 4D+c..4D+c+3 for the live D = d (mod MSA_CRING/4); dwords [RING/4, RING/4+16)
  // mirror [0, 16) so a phase's KS/4 consecutive dwords never wrap.
  constexpr bool LDSCODE = SGL;
  constexpr int CRW = MSA_CRING / 4 + 16;  // dwords per copy
  unsigned* cring = reinterpret_cast<unsigned*>(rowbuf + NC * kp.lds_row_words);

  for (;;) {
    // ---- ticket ----
    if (threadIdx.x == 0) misc[0] = atomicAdd(a.ticket, 1);
    __syncthreads();
    const int item = uni(misc[0]);
    __syncthreads();
    if (item >= kp.n_items) break;

    int pair, k0, ns, group;
    int nwarm = 0;  // chunked: leading stripes of the item that only warm up (no cells, no meta)
    if (kp.single == 1) {
      pair = 0;
      group = item;
      k0 = item * W;
      const msa_pair_desc pd0 = a.pairs[0];
      const int S = (pd0.m + 63) / 64;
      ns = min(W, S - k0);
    } else if (kp.single == 3) {
      // a batch of equal-m pairs too small to fill the chip: every pair (SWLP: couple) is split
      // into kp.groups items of kp.chunk_c stripes (a multiple of W), consecutive tickets,
      // chained through granules; inside an item the waves cycle as in batch mode
      const int pidx = item / kp.groups;
      group = item - pidx * kp.groups;
      pair = pk16(ALG) ? 2 * pidx : pidx;
      k0 = group * kp.chunk_c;
      const int S = (a.pairs[pair].m + 63) / 64;
      ns = min(kp.chunk_c, S - k0);
    } else if (kp.single == 2) {
      pair = 0;
      group = item;
      const int S = (a.pairs[0].m + 63) / 64;
      const int ks0 = item * kp.chunk_c;  // first stripe the chunk outputs
      const int ke = min(S, ks0 + kp.chunk_c);
      int kb = ks0 - kp.chunk_warm;
      // a warm-up that would reach the matrix border (rows <= band + 64) starts at row 0
      // instead, exactly: homogeneity (the guessed run = exact + constant) needs no border
      if (kb * 64 <= kp.band + 64) kb = 0;
      k0 = kb;
      ns = ke - kb;
      nwarm = ks0 - kb;
    } else {
      pair = pk16(ALG) ? 2 * item : item;  // SWLP: item c = pairs 2c (low halves) and 2c+1 (high)
      group = 0;
      k0 = 0;
      ns = (a.pairs[pair].m + 63) / 64;
    }
    const msa_pair_desc pd = a.pairs[pair];
    // SWLP: the pair in the high halves (the last item of an odd count repeats its low pair)
    const msa_pair_desc pd2 = pk16(ALG) ? a.pairs[min(pair + 1, kp.n_pairs - 1)] : pd;
    const int m = pd.m, n = pd.n;
    const int S_pair = (m + 63) / 64;

    // ---- schedule (one lane) ----
    if (threadIdx.x == 0) {
      int total = 0;
      StripeGeom prev;
      for (int k = 0; k < ns; ++k) {
        StripeGeom g;
        stripe_geom(k0 + k, m, n, kp.band, g, KS);
        int T = 0;
        if (k > 0) {
          // the consumer's phase q reads producer columns up to cs+KS*q+KS-1,
          // computed at producer step (cs - prev.cs + 63) + KS*q + KS-1; that
          // phase must be complete (one barrier) first.  cs diff >= -15.
          const int D = (g.cs - prev.cs + 62 + KS) / KS + 1;
          T = prev.T + D;
          if (k >= W) {
            const StripeGeom& o = sched[k - W];
            T = max(T, o.T + o.P);
          }
        }
        g.T = T;
        sched[k] = g;
        prev = g;
        total = max(total, T + g.P);
      }
      misc[1] = total;
    }
    __syncthreads();
    const int total = uni(misc[1]);

    const unsigned ep = kp.epoch;

    if (LDSCODE && w == W + 1) {
      // =================== code wave (single pair) ===================
      const StripeGeom s0 = sched[0];
      // ---- column-code ring (single pair): columns needed at phase x = union over
      // the item's stripes active at x of [cs + KS(x-T) - 63, cs + KS(x-T) + KS + 3]
      auto need_hi = [&](int x) __attribute__((always_inline)) {
        int hi = INT32_MIN;
        for (int k = 0; k < ns; ++k) {
          const int T = sched[k].T, P_ = sched[k].P, c0 = sched[k].cs;
          if (T <= x && x < T + P_) hi = max(hi, c0 + KS * (x - T) + KS + 3);
        }
        return uni(hi);
      };
      const unsigned* cod_pair = reinterpret_cast<const unsigned*>(a.cod + pd.cod_off);
      const int cc = lane >> 4, ck = lane & 15;  // this lane stages copy cc, dword slot ck
      // global source of the 4 codes of columns 4D+cc..4D+cc+3 (an aligned dword of a shifted copy)
      auto code_src = [&](int D) __attribute__((always_inline)) {
        const int g = 4 * D + cc - 1 + MSA_CPAD;
        return cod_pair + ((size_t)(g & (MSA_NCOPY - 1)) * a.cod_copy + (g & ~(MSA_NCOPY - 1))) / 4;
      };
      auto code_put = [&](int D, unsigned v) __attribute__((always_inline)) {
        const int d = D & (MSA_CRING / 4 - 1);
        cring[cc * CRW + d] = v;
        if (d < 16) cring[cc * CRW + d + MSA_CRING / 4] = v;
      };
      // dword range of copy cc covering columns (a_, b_]
      auto drange = [&](int a_, int b_, int& dlo, int& dhi) __attribute__((always_inline)) {
        dlo = ((a_ + 1 - cc - 3) >> 2);
        dhi = ((b_ - cc) >> 2);
      };
      int staged = 0;  // highest column staged so far (wave-uniform)
      unsigned cval[2] = {0u, 0u};
      int cD[2] = {0, 0};
      bool cok[2] = {false, false};
      if constexpr (LDSCODE) {
        // prologue: everything phases 0 and 1 read, synchronously
        const int lo0 = s0.cs - 63 - 4;
        const int hi1 = max(need_hi(0), need_hi(1));
        int dlo, dhi;
        drange(lo0 - 1, hi1, dlo, dhi);
        for (int D = dlo + ck; D <= dhi; D += 16) code_put(D, *code_src(D));
        staged = hi1;
      }
      // issue the loads for columns needed at phase x into slot `sl`; commit later
      auto code_issue = [&](int x, int sl) __attribute__((always_inline)) {
        const int hi = need_hi(x);
        int dlo, dhi;
        drange(staged, hi, dlo, dhi);
        if (hi > staged && dhi - dlo >= 16) {  // rare big jump: stage the excess synchronously
          for (int D = dlo + ck; D <= dhi - 16; D += 16) code_put(D, *code_src(D));
          dlo = dhi - 15;
        }
        const int D = dlo + ck;
        cok[sl] = (hi > staged) && (D <= dhi);
        cD[sl] = D;
        if (cok[sl]) cval[sl] = *code_src(D);
        staged = max(staged, hi);
      };
      auto code_commit = [&](int sl) __attribute__((always_inline)) {
        if (cok[sl]) code_put(cD[sl], cval[sl]);
      };

      if constexpr (LDSCODE) {
        code_issue(2, 0);
        __syncthreads();  // phases 0, 1 staged before any compute wave reads them
        for (int ph = 0; ph < total; ph += 2) {
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            const int p = ph + s;
            if (p < total) {
              // slot s holds the loads for phase p+2 (issued two iterations ago, or
              // in the prologue): commit them (visible after this phase's barrier),
              // then prefetch phase p+4... p+3 into the freed slot
              code_commit(s);
              code_issue(p + 3, s);
              MSA_SYNC(p);
            }
          }
        }
      }
      continue;
    }

    if (w == W) {
      // =================== loader wave ===================
      const bool act = (kp.single == 1 || kp.single == 3) && group > 0;
      StripeGeom s0 = sched[0];
      s0.cs = uni(s0.cs);
      s0.P = uni(s0.P);
      int chi = n;
      if (k0 > 0) {
        StripeGeom gp;
        stripe_geom(k0 - 1, m, n, kp.band, gp, KS);
        chi = gp.c_hi;
      }
      // (single: item == group; mode 3: a pair's groups are consecutive items)
      const unsigned long long* g_in = act ? a.gbuf + (size_t)(item - 1) * NC * a.gbuf_stride : a.gbuf;
      // the item holds the pair's first stripe: stage the DP's row 0; chunked: the guessed
      // row above the chunk's first (warm-up) stripe
      const bool border = (k0 == 0) || kp.single == 2;
      const int brow = (kp.single == 2) ? 64 * k0 : 0;
      // all staging / sinking works in 16-column chunks; phase p = chunks [CPP*p, CPP*p + CPP)
      const int nch0 = s0.P * CPP;
      auto commit_border = [&](int c) __attribute__((always_inline)) {
        const int v = lane >> 4, l = lane & 15;
        int bv[3];
        border_top<ALG>(kp, s0.cs + 16 * c + l, bv, brow);
        const int val = (v == 0) ? bv[0] : (v == 1 ? bv[1] : bv[2]);
        if (v < NC) stage[v * MSA_RING + ((16 * c + l) & (MSA_RING - 1))] = val;
      };
      // Sink: the item's last stripe hands its bottom row to the next
      // workgroup.  Its compute wave only writes its LDS ring; this wave
      // publishes the KS columns of each phase as {epoch, value} granules
      // one phase later (after the barrier that completes them).
      const int sl_idx = ns - 1;
      // (with the DPP shift register the compute wave publishes itself)
      const bool sink = (kp.single == 1 || kp.single == 3) && (k0 + sl_idx) < S_pair - 1 && !(NC == 1 && SGL);
      StripeGeom sl = sched[sl_idx];
      sl.T = uni(sl.T); sl.P = uni(sl.P); sl.cs = uni(sl.cs);
      int sl_out_cs = 0;
      if (sink) {
        StripeGeom gn;
        stripe_geom(k0 + sl_idx + 1, m, n, kp.band, gn, KS);
        sl_out_cs = uni(gn.cs);
      }
      const int* ring_last = rings + ((((sl_idx / W) & 1) * W + sl_idx % W) * NC) * MSA_RING;
      unsigned long long* g_out = a.gbuf + (size_t)item * NC * a.gbuf_stride;
      auto sink_phase = [&](int q) __attribute__((always_inline)) {
        if (!sink || q < 0 || q >= sl.P) return;
        const int v = lane >> 4, l = lane & 15;
        if (v < NC) {
#pragma unroll
          for (int h = 0; h < CPP; ++h) {
            const int x = sl.cs + KS * q + 16 * h - 63 - sl_out_cs + l;
            const int col = sl.cs + KS * q + 16 * h - 63 + l;
            if (col + MSA_GOFF >= 0 && col + MSA_GOFF < a.gbuf_stride) {
              const int val = ring_last[v * MSA_RING + (x & (MSA_RING - 1))];
              gstore(g_out + (size_t)v * a.gbuf_stride + col + MSA_GOFF,
                     ((unsigned long long)ep << 32) | (unsigned)val);
            }
          }
        }
      };
      // Staging runs one phase ahead of the compute waves: phase 0 before
      // the first barrier, phase p+1 during phase p.
      if (border) {
#pragma unroll
        for (int h = 0; h < CPP; ++h) commit_border(h);
      }
      // Just-in-time staging: during phase p the loader issues the granule
      // loads of phase p+1, then waits for them (one global round trip fits
      // in a phase) and commits -- the producer only has to be one phase plus
      // the store->load visibility ahead.
      unsigned long long G[CPP];
      if (act) {
        {
          // phase 0's columns published before anything is loaded
          const int colw = min(min(s0.cs + 16 * (CPP - 1) + 15, chi), n);
          unsigned spins = 0;
          while (uni((int)(unsigned)(gload(g_in + colw + MSA_GOFF) >> 32)) != (int)ep) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > (1u << 24)) break;
          }
          if (spins > (1u << 24) && lane == 0) atomicExch(a.err, 1);
        }
#pragma unroll
        for (int h = 0; h < CPP; ++h) G[h] = loader_issue<NC>(a, s0.cs, h, g_in, lane);
#pragma unroll
        for (int h = 0; h < CPP; ++h) loader_commit<NC>(a, s0.cs, nch0, h, G[h], g_in, stage, chi, n, ep, lane);
      }
      __syncthreads();  // phase 0 staged before any compute wave reads it
      for (int p = 0; p < total; ++p) {
        if (act) {
          if (p + 1 < s0.P) {
#pragma unroll
            for (int h = 0; h < CPP; ++h) G[h] = loader_issue<NC>(a, s0.cs, (p + 1) * CPP + h, g_in, lane);
            sink_phase(p - 1 - sl.T);
#pragma unroll
            for (int h = 0; h < CPP; ++h)
              loader_commit<NC>(a, s0.cs, nch0, (p + 1) * CPP + h, G[h], g_in, stage, chi, n, ep, lane);
          } else {
            sink_phase(p - 1 - sl.T);
          }
        } else {
          if (border && p + 1 < s0.P) {
#pragma unroll
            for (int h = 0; h < CPP; ++h) commit_border((p + 1) * CPP + h);
          }
          sink_phase(p - 1 - sl.T);  // the last stripe's phase completed by the previous barrier
        }
        MSA_SYNC(p);
      }
      sink_phase(total - 1 - sl.T);
      continue;
    }

    // =================== compute waves ===================
    // Wave w runs stripes w, w+W, ...  Every wave passes exactly `total`
    // barriers (one per phase): idle phases before a stripe's start T, then
    // the stripe's P phases as three loops -- masked head, unmasked body (no
    // per-step range checks, no per-phase bookkeeping), masked tail.
    __syncthreads();  // pairs with the loader's post-staging barrier
    int ph = 0;
    for (int cur = w; cur < ns; cur += W) {
      StripeGeom sg = sched[cur];
      sg.T = uni(sg.T); sg.P = uni(sg.P); sg.cs = uni(sg.cs); sg.lead = uni(sg.lead);
      sg.mask_lo = uni(sg.mask_lo); sg.mask_hi = uni(sg.mask_hi); sg.c_hi = uni(sg.c_hi);
      // row code of this lane: a cold HBM load, issued before the idle phases
      // (on the critical path of the wavefront if it waited for the stripe start)
      const int ks = k0 + cur;  // pair-local stripe index
      const int row_i = 64 * ks + lane + 1;
      const unsigned ac = (row_i <= m) ? (a.A[pd.a_off + row_i - 1] & 7u) : 0u;
      const unsigned ac2 = (pk16(ALG) && row_i <= m) ? (a.A[pd2.a_off + row_i - 1] & 7u) : 0u;
      for (; ph < sg.T; ++ph) MSA_SYNC(ph);
      // ---- stripe init ----
      LaneState<ALG> L;
      L.i = row_i;
      const int ivalid = min(L.i, m);
      L.tmin = jlo_of(L.i, kp.band) - sg.cs + lane;
      L.tmax = (L.i <= m) ? jhi_of(L.i, n, kp.band) - sg.cs + lane : -1;
      {
        int lb[3];
        border_left<ALG>(kp, ivalid, lb);
        if (kp.band >= 0 && jlo_of(L.i, kp.band) > 1) lb[0] = lb[1] = lb[2] = MSA_NEG;
#pragma unroll
        for (int v = 0; v < 3; ++v) { L.LB[v] = lb[v]; L.S[v] = lb[v]; L.U[v] = MSA_NEG; L.fin[v] = 0; }
      }
      L.best = 0;
      L.bt = -1;
      L.pb = (int)0x80008000u;
      const int gdiag = kp.gap_open * (64 * ks + 1 + sg.cs);  // SWL: g*(i+j) at step 0, same for all lanes
      // SWLP: pk2(-g k) per step k of a phase, wave-uniform and fixed for the launch (opaque: computed
      // once per stripe instead of rematerialized at every step)
      int gkp[KS];
#pragma unroll
      for (int k = 0; k < KS; ++k) {
        gkp[k] = pk16(ALG) ? pk2(-kp.gap_open * k) : 0;
        if constexpr (pk16(ALG)) asm("" : "+s"(gkp[k]));
      }
      // SWL: the lane starts left of the matrix on virtual cells with H = 0,
      // i.e. G = g*(i+j); its left neighbour at step 0 is G = gdiag - g
      if constexpr (swlin(ALG)) {
        L.S[0] = gdiag - kp.gap_open;      // G(i, cs-r-1)
        L.U[0] = gdiag - 2 * kp.gap_open;  // G(i-1, cs-r-1)
        if constexpr (pk16(ALG)) {
          L.S[0] = pk2(L.S[0]);
          L.U[0] = pk2(L.U[0]);
        }
      }
      // substitution profile of this row (codes 0..7)
      {
        int sm, sx;
        if constexpr (ALG == MSA_ALG_REF || ALG == MSA_ALG_NWA) { sm = 1; sx = 0; }
        else if constexpr (ALG == MSA_ALG_REF1) { sm = 4; sx = 0; }  // 4f: tagged values
        else if constexpr (ALG == MSA_ALG_PART) { sm = 0; sx = 1; }
        else if constexpr (swlin(ALG)) { sm = kp.match + 2 * kp.gap_open; sx = kp.mismatch + 2 * kp.gap_open; }
        else { sm = kp.match; sx = kp.mismatch; }
        const unsigned bx = (unsigned)(sx & 0xff) * 0x01010101u;
        auto table = [&](unsigned c, unsigned& plo_, unsigned& phi_) __attribute__((always_inline)) {
          unsigned lo = bx, hi = bx;
          const unsigned bm = (unsigned)(sm & 0xff);
          if (c < 4) lo = (lo & ~(0xffu << (8 * c))) | (bm << (8 * c));
          else hi = (hi & ~(0xffu << (8 * (c - 4)))) | (bm << (8 * (c - 4)));
          // virtual columns: SWL0 scores them 0, so (floor-free) G = g*(i+j), i.e.
          // H = 0, holds exactly on every cell left of column 1 -- the border
          // column itself; right of column n they never beat a real cell
          if constexpr (ALG == MSA_ALG_SWL0 || ALG == MSA_ALG_SWLP)
            hi = (hi & 0x00ffffffu) | ((unsigned)((2 * kp.gap_open) & 0xff) << 24);
          else if constexpr (SWK) hi = (hi & 0x00ffffffu) | ((unsigned)(MSA_VIRT_SCORE & 0xff) << 24);
          plo_ = lo;
          phi_ = hi;
        };
        table(ac, L.plo, L.phi);
        L.plo2 = L.phi2 = 0;
        if constexpr (pk16(ALG)) table(ac2, L.plo2, L.phi2);
      }
      // code stream: lane r needs columns cs - r + t; column c sits in copy
      // (c-1+CPAD)&15 at byte (c-1+CPAD) & ~15, so every read is an aligned dwordx4
      const unsigned* cptr;
      {
        const int b0 = sg.cs - lane - 1 + MSA_CPAD;  // > 0
        cptr = reinterpret_cast<const unsigned*>(a.cod + (size_t)(b0 & (MSA_NCOPY - 1)) * a.cod_copy + pd.cod_off +
                                                 (b0 & ~(MSA_NCOPY - 1)));
      }
      // batch: codes of phase q+1 are loaded during phase q (global loads);
      // single pair: read from the loader-staged LDS ring at phase start
      unsigned cwn[KS / 4];
      // packed batches (C4): codes two phases ahead (cwn = phase q+1, cwn2 = phase q+2): one phase of
      // lock-step computing did not cover a global load's latency (stamps: ~0.3 us of a 1.04 us phase
      // waited for the codes)
      constexpr bool CPF2 = pk16(ALG) && !LDSCODE;
      unsigned cwn2[KS / 4];
      const int cj0 = sg.cs - lane;                // column of this lane at step 0
      const unsigned* cr_base = cring + (cj0 & 3) * CRW;
      const int cd0 = cj0 >> 2;                    // floor: absolute dword index at step 0
      auto load_codes = [&](const int q) __attribute__((always_inline)) {
        if constexpr (LDSCODE) {
          const unsigned* cp = cr_base + ((cd0 + (KS / 4) * q) & (MSA_CRING / 4 - 1));
#pragma unroll
          for (int u = 0; u < KS / 4; ++u) cwn[u] = cp[u];
        } else if constexpr (CPF2) {
          // (a phase past the stripe's last reads the padded copy: the padding covers KS/4 dwords)
#pragma unroll
          for (int u = 0; u < KS / 4; ++u) cwn[u] = cwn2[u];
#pragma unroll
          for (int u = 0; u < KS / 4; u += 4) {
            const uint4 c4 = *reinterpret_cast<const uint4*>(cptr + (KS / 4) * (q + 1) + u);
            cwn2[u] = c4.x; cwn2[u + 1] = c4.y; cwn2[u + 2] = c4.z; cwn2[u + 3] = c4.w;
          }
        } else {
#pragma unroll
          for (int u = 0; u < KS / 4; u += 4) {
            const uint4 c4 = *reinterpret_cast<const uint4*>(cptr + (KS / 4) * q + u);
            cwn[u] = c4.x; cwn[u + 1] = c4.y; cwn[u + 2] = c4.z; cwn[u + 3] = c4.w;
          }
        }
      };
      if constexpr (CPF2) {
#pragma unroll
        for (int u = 0; u < KS / 4; u += 4) {
          const uint4 c4 = *reinterpret_cast<const uint4*>(cptr + u);
          cwn2[u] = c4.x; cwn2[u + 1] = c4.y; cwn2[u + 2] = c4.z; cwn2[u + 3] = c4.w;
        }
        load_codes(0);  // cwn = phase 0, cwn2 = phase 1
      } else if constexpr (!LDSCODE) {
        load_codes(0);
      }
      // input: the loader's staging ring (row 0 or the previous workgroup),
      // the wrap row buffer (batch), or the ring of the previous wave
      const int* in_ptr;
      int in_vs, in_mask;
      const int par_in = ((cur - 1) / W) & 1;  // round parity of the producer stripe
      if (cur == 0) {
        in_ptr = stage; in_vs = MSA_RING; in_mask = MSA_RING - 1;
      } else if (cur % W == 0) {
        in_ptr = rowbuf + MSA_ROWOFF; in_vs = kp.lds_row_words; in_mask = 0x3fffffff;
      } else {
        in_ptr = rings + ((par_in * W + (w - 1)) * NC) * MSA_RING; in_vs = MSA_RING; in_mask = MSA_RING - 1;
      }
      int snk;
      if (cur == ns - 1) snk = ((kp.single == 1 || kp.single == 3) && ks < S_pair - 1) ? SNK_GLOBAL : SNK_NONE;
      else snk = (cur % W == W - 1) ? SNK_ROW : SNK_RING;
      int* const ring_out = rings + (((cur / W) & 1) * W + w) * NC * MSA_RING;
      int* out_ptr;
      int out_vs, out_mask, out_add, out_lim;
      if (snk == SNK_ROW) {
        out_ptr = rowbuf; out_vs = kp.lds_row_words; out_mask = 0x3fffffff; out_add = MSA_ROWOFF;
        out_lim = kp.lds_row_words - 4;
      } else {
        out_ptr = ring_out; out_vs = MSA_RING; out_mask = MSA_RING - 1; out_add = 0; out_lim = 1 << 30;
      }
      int out_cs = 0;
      if (snk != SNK_NONE) {
        StripeGeom gn;
        stripe_geom(ks + 1, m, n, kp.band, gn, KS);
        out_cs = gn.cs;
      }
      int out_chi = n;  // c_hi of the producer row above (input masking, banded)
      if (ks > 0) {
        StripeGeom gp;
        stripe_geom(ks - 1, m, n, kp.band, gp, KS);
        out_chi = gp.c_hi;
      }
      snk = uni(snk); out_cs = uni(out_cs); out_chi = uni(out_chi);
      unsigned long long* const g_out = a.gbuf + (size_t)item * NC * a.gbuf_stride;
      const size_t obase = (size_t)pd.out_off + (size_t)ks * pd.pmax * MSA_K * 64;  // pmax: 16-step blocks
      // chunked mode: warm-up stripes store no cells and no meta (another chunk owns them);
      // the warm-up's last stripe and the chunk's last stripe save lane 63's (H, F) row
      const bool outp = uni(cur >= nwarm);
      int ckslot = -1;
      if constexpr (ALG == MSA_ALG_NWA) {
        if (kp.single == 2) {
          if (cur == nwarm - 1) ckslot = 2 * item;
          else if (cur == ns - 1 && ks < S_pair - 1) ckslot = 2 * item + 1;
        }
      }
      ckslot = uni(ckslot);
      const int ckrow = 64 * ks + 64;  // lane 63's row

      // MASKED_: 0 no range checks; 1 per-lane start/end checks; 2..5 banded Gotoh in the
      // regular middle of the band, head (2, 3) or tail (4, 5) fix-ups by v_writelane, fix-up
      // steps of parity MODE & 1 (see band_fix / the range split below)
      int fix_base = 0;  // lane fixed up at the phase's first fix-up step (modes 2..5)
      auto run_phase = [&](const int q, auto MASKED_, auto INMASK_, auto FIN_) __attribute__((always_inline)) {
        constexpr int MMODE = (int)decltype(MASKED_)::value;
        constexpr bool MASKED = MMODE != 0;
        constexpr bool INMASK = decltype(INMASK_)::value;  // input columns beyond the producer's last
        constexpr bool FIN = decltype(FIN_)::value;        // capture the state at each row's last column
        // ---- all LDS reads of the phase up front (one exposed latency per phase) ----
        int IN[NC][KS];
        {
          const int* base = in_ptr + ((KS * q) & in_mask);
#pragma unroll
          for (int v = 0; v < NC; ++v) {
#pragma unroll
            for (int u = 0; u < KS / 4; ++u) {
              const int4 x = *reinterpret_cast<const int4*>(base + v * in_vs + 4 * u);
              IN[v][4 * u + 0] = x.x; IN[v][4 * u + 1] = x.y; IN[v][4 * u + 2] = x.z; IN[v][4 * u + 3] = x.w;
            }
          }
          if constexpr (INMASK) {
            if (sg.cs + KS * q + KS - 1 > out_chi) {  // uniform: only the phases past the producer's end
#pragma unroll
              for (int k = 0; k < KS; ++k) {
                const bool o = sg.cs + KS * q + k > out_chi;
#pragma unroll
                for (int v = 0; v < NC; ++v) IN[v][k] = o ? (pk16(ALG) ? (int)0x80008000u : MSA_NEG) : IN[v][k];
              }
            }
          }
        }
        unsigned cw[KS / 4];
        if constexpr (LDSCODE) load_codes(q);
#pragma unroll
        for (int u = 0; u < KS / 4; ++u) {
          cw[u] = cwn[u];
        }
#ifdef MSA_STAMPS
        {
          int z = IN[0][0] ^ (int)cw[0];
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          asm volatile("" ::"v"(z));
          MSA_MARK(ph + q, 3);
        }
#endif
        if constexpr (!LDSCODE) load_codes(q + 1);
        int hist[NC][KS];
        int hv[KS];
        unsigned dirw[KS / 4];
        // NC == 1: lane 63's carried value is collected by a DPP shift register
        // (one wave_shl per step: after KS steps lane 64-KS+k holds step k),
        // so the hand-off is ONE ds_write_b32 of KS lanes per phase instead of
        // KS/4 single-lane b128 writes that all waves issue at once.
        // (single-pair kernels only: in batch the SIMDs are saturated and the
        // extra DPP per step costs more than the lockstep writes)
        constexpr bool SHREG = (NC == 1) && SGL;
        int shreg = 0;
        int4* hrow = reinterpret_cast<int4*>(a.outH + obase) + (size_t)((KS / 4) * q) * 64 + lane;
        int4* t2row = reinterpret_cast<int4*>(a.outT2 + obase) + (size_t)((KS / 4) * q) * 64 + lane;
        int4* t3row = reinterpret_cast<int4*>(a.outT3 + obase) + (size_t)((KS / 4) * q) * 64 + lane;
#pragma unroll
        for (int u = 0; u < KS / 4; ++u) {
          const unsigned s4 = __builtin_amdgcn_perm(L.phi, L.plo, cw[u]);
          const unsigned s4b = pk16(ALG) ? __builtin_amdgcn_perm(L.phi2, L.plo2, cw[u]) : 0u;
          unsigned dq = 0;
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) {
            const int k = 4 * u + kk;
            const int t = KS * q + k;
            // SWLP: {s4 byte kk, 0, s4b byte kk, 0} = both pairs' score + 2g as int16 (>= 0)
            const int s = pk16(ALG) ? (int)__builtin_amdgcn_perm(s4b, s4, 0x0c000c00u | ((4u + kk) << 16) | (unsigned)kk)
                                    : ((int)(s4 << (24 - 8 * kk))) >> 24;
            int inv[3];
#pragma unroll
            for (int v = 0; v < NC; ++v) inv[v] = IN[v][k];
            int cr[3];
            int ct = pk16(ALG) ? gkp[k] : gdiag + kp.gap_open * t;
            if constexpr (swlin(ALG) && !pk16(ALG)) asm("" : "+s"(ct));  // one SGPR feeds both the floor and H
            unsigned d;
            if constexpr (ALG == MSA_ALG_NWA && MMODE >= 2) {
              d = step<ALG, OUT, false, TRACKPOS, false>(kp, L, inv, s, t, ct, cr, hv[k]);
              // one lane per two steps sits on the band's edge: its index is wave-uniform
              constexpr int PAR = MMODE & 1;
              if (((k - PAR) & 1) == 0) {
                const int rr = fix_base + ((k - PAR) >> 1);
                // the lane select goes through M0 (one SGPR source per VALU op: the value is
                // the other), saved and restored around the writes (M0 is reserved to the
                // compiler); s_nop 3 covers the SALU-write -> lane-select wait states
                const int negv = MSA_NEG;
                if constexpr (MMODE <= 3) {  // head: the row's left neighbour is -inf
                  int keep;
                  asm("s_mov_b32 %2, m0\n\ts_mov_b32 m0, %4\n\ts_nop 3\n\tv_writelane_b32 %0, %3, m0\n\t"
                      "v_writelane_b32 %1, %3, m0\n\ts_mov_b32 m0, %2"
                      : "+v"(L.S[0]), "+v"(L.S[1]), "=&s"(keep) : "s"(negv), "s"(rr));
                } else {  // tail: the row below's (and the hand-off's) up value is -inf
                  int keep;
                  asm("s_mov_b32 %2, m0\n\ts_mov_b32 m0, %4\n\ts_nop 3\n\tv_writelane_b32 %0, %3, m0\n\t"
                      "v_writelane_b32 %1, %3, m0\n\ts_mov_b32 m0, %2"
                      : "+v"(L.S[0]), "+v"(L.S[2]), "=&s"(keep) : "s"(negv), "s"(rr));
                  cr[0] = L.S[0];
                  cr[1] = L.S[2];
                }
              }
            } else if constexpr (ALG == MSA_ALG_NWA && MASKED) {
              d = step<ALG, OUT, false, TRACKPOS, false>(kp, L, inv, s, t, ct, cr, hv[k]);
              band_fix<FIN>(L, t, cr);
            } else {
              d = step<ALG, OUT, MASKED, TRACKPOS, FIN>(kp, L, inv, s, t, ct, cr, hv[k]);
            }
#pragma unroll
            for (int v = 0; v < NC; ++v) hist[v][k] = cr[v];
            if constexpr (SHREG) shreg = dpp_shl1(cr[0], shreg);
            dq |= d << (8 * kk);
          }
          dirw[u] = dq;
          if constexpr (!SHREG) {
            // lane 63 hands this quad's carried values to the next stripe right
            // away (keeps only 4 steps of history live: no register spills at NC=3)
            if (snk != SNK_NONE && lane == 63) {
              const int x = (sg.cs + KS * q + 4 * u - 63 - out_cs + out_add) & out_mask;  // multiple of 4
              if (x >= 0 && x <= out_lim) {
#pragma unroll
                for (int v = 0; v < NC; ++v)
                  *reinterpret_cast<int4*>(out_ptr + x + v * out_vs) =
                      make_int4(hist[v][4 * u], hist[v][4 * u + 1], hist[v][4 * u + 2], hist[v][4 * u + 3]);
              }
            }
          }
          if constexpr (ALG == MSA_ALG_NWA) {
            // chunked mode: lane 63's band state of this quad into the checkpoint row (two
            // stripes per chunk take this branch)
            if (ckslot >= 0 && lane == 63) {
#pragma unroll
              for (int kk = 0; kk < 4; ++kk) {
                const int col = sg.cs + KS * q + 4 * u + kk - 63;
                const int e = col - (ckrow - kp.band);
                if (e >= 0 && e <= 2 * kp.band && col >= 1 && col <= n) {
                  a.ck[(size_t)(2 * ckslot) * a.ckw + e] = hist[0][4 * u + kk];
                  a.ck[(size_t)(2 * ckslot + 1) * a.ckw + e] = hist[1][4 * u + kk];
                }
              }
            }
          }
          // cell outputs: one 1 KiB coalesced store per wave per 4 steps
          if (!outp) {
          } else if constexpr (OUT == MSA_OUT_H) {
            int4 h4;
            if constexpr (ALG == MSA_ALG_REF || ALG == MSA_ALG_PART) {
              h4 = make_int4(imax3(hist[0][4 * u], hist[1][4 * u], hist[2][4 * u]),
                             imax3(hist[0][4 * u + 1], hist[1][4 * u + 1], hist[2][4 * u + 1]),
                             imax3(hist[0][4 * u + 2], hist[1][4 * u + 2], hist[2][4 * u + 2]),
                             imax3(hist[0][4 * u + 3], hist[1][4 * u + 3], hist[2][4 * u + 3]));
            } else if constexpr (swlin(ALG) || ALG == MSA_ALG_SWA) {
              h4 = make_int4(hv[4 * u], hv[4 * u + 1], hv[4 * u + 2], hv[4 * u + 3]);
            } else {
              h4 = make_int4(hist[0][4 * u], hist[0][4 * u + 1], hist[0][4 * u + 2], hist[0][4 * u + 3]);
            }
            ntstore(hrow + u * 64, h4);
          } else if constexpr (OUT == MSA_OUT_TAB) {
            ntstore(hrow + u * 64, make_int4(hist[0][4 * u], hist[0][4 * u + 1], hist[0][4 * u + 2], hist[0][4 * u + 3]));
            ntstore(t2row + u * 64, make_int4(hist[1][4 * u], hist[1][4 * u + 1], hist[1][4 * u + 2], hist[1][4 * u + 3]));
            ntstore(t3row + u * 64, make_int4(hist[2][4 * u], hist[2][4 * u + 1], hist[2][4 * u + 2], hist[2][4 * u + 3]));
          }
        }
        if (outp && OUT == MSA_OUT_DIR) {
#pragma unroll
          for (int h = 0; h < CPP; ++h)
            ntstore(reinterpret_cast<int4*>(a.outDir + obase) + (size_t)(CPP * q + h) * 64 + lane,
                    make_int4((int)dirw[4 * h], (int)dirw[4 * h + 1], (int)dirw[4 * h + 2], (int)dirw[4 * h + 3]));
        }
        if constexpr (pk16(ALG)) {
          // both pairs' H = G - g (i + j): the phase's best of G - g k, minus g (i + j) at its step 0.
          // KS = 16, unmasked: max over k of G_k - g k as a four-level tree over the carried values
          // (independent ops, no serial chain of 16 dependent max with their wait states)
          if constexpr (KS == 16 && !MASKED) {
            int r8[8], r4[4], r2[2];
#pragma unroll
            for (int j = 0; j < 8; ++j) r8[j] = pk_max(hist[0][2 * j], pk_add(hist[0][2 * j + 1], gkp[1]));
#pragma unroll
            for (int j = 0; j < 4; ++j) r4[j] = pk_max(r8[2 * j], pk_add(r8[2 * j + 1], gkp[2]));
#pragma unroll
            for (int j = 0; j < 2; ++j) r2[j] = pk_max(r4[2 * j], pk_add(r4[2 * j + 1], gkp[4]));
            L.pb = pk_max(r2[0], pk_add(r2[1], gkp[8]));
          }
          L.best = pk_max(L.best, pk_add(L.pb, pk2(-(gdiag + kp.gap_open * KS * q))));
          L.pb = (int)0x80008000u;
        }
        MSA_MARK(ph + q, 2);
        // hand the bottom row to the next stripe: lane 63, once per phase
        if constexpr (SHREG) {
          if (snk != SNK_NONE && lane >= 64 - KS) {
            const int kk_ = lane - (64 - KS);
            if (snk == SNK_GLOBAL) {
              // last stripe of the item: publish straight to the next workgroup
              const int col = sg.cs + KS * q - 63 + kk_;
              if (col + MSA_GOFF >= 0 && col + MSA_GOFF < a.gbuf_stride)
                gstore(g_out + col + MSA_GOFF, ((unsigned long long)ep << 32) | (unsigned)shreg);
            } else {
              const int x = sg.cs + KS * q - 63 - out_cs + out_add + kk_;
              const int xm = x & out_mask;
              if (x >= 0 && xm < out_lim + 4) out_ptr[xm] = shreg;
            }
          }
        }
      };
      using T_ = std::true_type;
      using F_ = std::false_type;
      // phase q needs no range checks iff KS*q >= mask_lo (every lane has
      // started), KS*q+KS-1 <= mask_hi (none has finished) and every input
      // column cs+KS*q+KS-1 <= out_chi
      const int P = sg.P;
      const int lim = min(sg.mask_hi, out_chi - sg.cs) - (KS - 1);
      const int qa = uni(min(P, sg.mask_lo <= 0 ? 0 : (sg.mask_lo + KS - 1) / KS));
      const int qb = uni(max(qa, min(P, lim >= 0 ? lim / KS + 1 : 0)));
      auto run_range = [&](const int qb_, const int qe_, auto MASKED_, auto INMASK_, auto FIN_) __attribute__((always_inline)) {
        for (int q = qb_; q < qe_; ++q) {
          run_phase(q, MASKED_, INMASK_, FIN_);
          MSA_SYNC(ph + q);
        }
      };
      const bool fin_stripe = uni(ks == S_pair - 1);
      if constexpr (SWK) {
        // no state masking; only the inputs past the producer's last column
        // (never written into the ring / granules) are replaced by -inf
        const int li = out_chi - sg.cs - (KS - 1);
        const int qi = uni(min(P, li >= 0 ? li / KS + 1 : 0));
        run_range(0, qi, F_{}, F_{}, F_{});
        run_range(qi, P, F_{}, T_{}, F_{});
      } else if (fin_stripe) {
        run_range(0, qa, T_{}, T_{}, T_{});
        run_range(qa, qb, F_{}, F_{}, F_{});
        run_range(qb, P, T_{}, T_{}, T_{});
      } else {
        // banded Gotoh, a full stripe away from the matrix borders: lane r's first step is
        // A0 + 2r and its last C0 + 2r, so at a step of the right parity exactly one lane
        // needs the head (or tail) fix-up, at an index the wave knows in a scalar register.
        // Phases whose every fix-up lane is in [0, 63] take the v_writelane path (2 lane
        // writes per two steps instead of 2 compares and 5 selects per step); the others,
        // and every other stripe, band_fix.
        bool regular = false;
        int A0 = 0, C0 = 0;
        if constexpr (ALG == MSA_ALG_NWA) {
          const int i0 = 64 * ks + 1;
          regular = uni(kp.band >= 64 && i0 + 63 <= m && i0 - kp.band > 1 && i0 + 63 + kp.band < n);
          A0 = uni(jlo_of(i0, kp.band) - sg.cs);
          C0 = uni(jhi_of(i0, n, kp.band) - sg.cs);
        }
        if (regular) {
          const int par = (A0 - 1) & 1;
          const int h0 = min(qa, max(0, (A0 - 1 + 15) / 16));
          const int h1 = min(qa, max(h0, (A0 + 110) / 16 + 1));
          const int t0 = min(P, max(qb, (C0 + 1 + 15) / 16));
          const int t1 = min(P, max(t0, (C0 + 112) / 16 + 1));
          using H0 = std::integral_constant<int, 2>;
          using H1 = std::integral_constant<int, 3>;
          using E0 = std::integral_constant<int, 4>;
          using E1 = std::integral_constant<int, 5>;
          // fix_base: lane of the phase's first fix-up step, (16q + par - (A0 - 1)) / 2 (head)
          // or (16q + par - (C0 + 1)) / 2 (tail)
          auto run_fast = [&](const int qb_, const int qe_, auto MODE_, const int edge) __attribute__((always_inline)) {
            for (int q = qb_; q < qe_; ++q) {
              fix_base = uni((KS * q + par - edge) >> 1);
              run_phase(q, MODE_, T_{}, F_{});
              MSA_SYNC(ph + q);
            }
          };
          run_range(0, h0, T_{}, T_{}, F_{});
          if (par) run_fast(h0, h1, H1{}, A0 - 1); else run_fast(h0, h1, H0{}, A0 - 1);
          run_range(h1, qa, T_{}, T_{}, F_{});
          run_range(qa, qb, F_{}, F_{}, F_{});
          run_range(qb, t0, T_{}, T_{}, F_{});
          if (par) run_fast(t0, t1, E1{}, C0 + 1); else run_fast(t0, t1, E0{}, C0 + 1);
          run_range(t1, P, T_{}, T_{}, F_{});
        } else {
          run_range(0, qa, T_{}, T_{}, F_{});
          run_range(qa, qb, F_{}, F_{}, F_{});
          run_range(qb, P, T_{}, T_{}, F_{});
        }
      }
      ph += P;
      // ---- stripe finalize ----
      msa_stripe_meta* md = a.meta + pd.stripe0 + ks;
      if (!outp) continue;  // a warm-up stripe: its meta belongs to the chunk that outputs it
      if constexpr (pk16(ALG)) {
        // each half separately: pair 2c's best (low halves), then pair 2c+1's (high halves)
        msa_stripe_meta* md2 = a.meta + pd2.stripe0 + ks;
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          const int bv = half ? (L.best >> 16) : (int)(short)(L.best & 0xffff);
          int b = (L.i <= m) ? bv : INT32_MIN;
          int bi = L.i;
#pragma unroll
          for (int off = 32; off >= 1; off >>= 1) {
            const int ob = __shfl_xor(b, off);
            const int oi = __shfl_xor(bi, off);
            if (ob > b || (ob == b && oi < bi)) { b = ob; bi = oi; }
          }
          if (lane == 0) {
            msa_stripe_meta* mh = half ? md2 : md;
            mh->best = b;
            mh->best_i = bi;
            mh->best_j = -1;
            mh->cs = sg.cs;
            mh->phases = sg.P * CPP;
          }
        }
      } else if constexpr (swlin(ALG) || ALG == MSA_ALG_SWA) {
        // first max in row-major order: max best, then min row
        const int bv = (TRACKPOS == 2) ? (L.best >> 15) : L.best;
        const int bt = (TRACKPOS == 2) ? 32767 - (L.best & 32767) : L.bt;
        int b = (L.i <= m) ? bv : INT32_MIN;
        int bi = L.i;
        int bj = sg.cs + bt - lane;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
          const int ob = __shfl_xor(b, off);
          const int oi = __shfl_xor(bi, off);
          const int oj = __shfl_xor(bj, off);
          if (ob > b || (ob == b && oi < bi)) { b = ob; bi = oi; bj = oj; }
        }
        if (lane == 0) {
          md->best = b;
          md->best_i = bi;
          md->best_j = TRACKPOS ? bj : -1;
        }
      } else {
        if (L.i == m) {
          md->fin[0] = L.fin[0];
          md->fin[1] = L.fin[1];
          md->fin[2] = L.fin[2];
          md->has_fin = 1;
        }
      }
      if (lane == 0) {
        md->cs = sg.cs;
        md->phases = sg.P * CPP;  // in 16-step layout blocks
      }
    }
    for (; ph < total; ++ph) MSA_SYNC(ph);
  }
}

// ---------------------------------------------------------------------------
// Column codes -> MSA_NCOPY byte-shifted, padded copies (one thread per output dword):
// copy c, byte x of pair p = code of column x + c - CPAD + 1 (virt outside [1, n]).
// ---------------------------------------------------------------------------
__global__ void stage_codes_kernel(const uint8_t* B, const msa_pair_desc* pairs, int n_pairs, uint8_t* cod,
                                   long long cod_copy, unsigned virt, int* ticket) {
  // the run's ticket counters and error word start at 0 (this launch precedes the DP kernel)
  if (ticket && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x < MSA_NTICKET) ticket[threadIdx.x] = 0;
  const int p = blockIdx.y;
  if (p >= n_pairs) return;
  const msa_pair_desc pd = pairs[p];
  const int seg = ((pd.n + 2 * MSA_CPAD) + 15) & ~15;  // bytes per copy of this pair (multiple of 16)
  for (int d = blockIdx.x * blockDim.x + threadIdx.x; d < MSA_NCOPY * (seg / 4); d += gridDim.x * blockDim.x) {
    const int c = d / (seg / 4), x = 4 * (d - c * (seg / 4));
    unsigned word = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int col = x + b + c - MSA_CPAD + 1;
      const unsigned code = (col >= 1 && col <= pd.n) ? (B[pd.b_off + col - 1] & 7u) : virt;
      word |= code << (8 * b);
    }
    *reinterpret_cast<unsigned*>(cod + (size_t)c * cod_copy + pd.cod_off + x) = word;
  }
}

// ---------------------------------------------------------------------------
// Per-pair reduction of the stripe results.
// ---------------------------------------------------------------------------
struct PairResult {
  int32_t score, status;
  int64_t end_i, end_j;
  int32_t fin[3];
  int32_t pad;
};

// A two-pass SW plan's best-cell key (fl_block_result, msa_flow.hip): score ^ 2^31 in the high word,
// ~(i (n + 1) + j) of the first best cell in row-major order in the low word; a score <= 0 keeps the
// end at (0, 0), reduce_blocks_kernel's rule.
__host__ __device__ inline PairResult best_key_decode(unsigned long long k, long long n) {
  PairResult r;
  r.score = (int32_t)((uint32_t)(k >> 32) ^ 0x80000000u);
  r.status = 0;
  const unsigned long long lin = (unsigned long long)(~(uint32_t)k);
  r.end_i = r.score > 0 ? (int64_t)(lin / (unsigned long long)(n + 1)) : 0;
  r.end_j = r.score > 0 ? (int64_t)(lin % (unsigned long long)(n + 1)) : 0;
  r.fin[0] = r.fin[1] = r.fin[2] = 0;
  r.pad = 0;
  return r;
}
__global__ void best_key_kernel(const unsigned long long* key, long long n, PairResult* out) {
  if (threadIdx.x == 0) out[0] = best_key_decode(*key, n);
}

// ---------------------------------------------------------------------------
// Chunked banded mode (kp.single == 2), after the chunk launch.
// chunk_check_kernel, one workgroup per chunk k >= 1: chunk k's run from its guessed
// row reached the band row above its first output row with state (H, F) = `warm`;
// chunk k-1 ended on the same row with `end`.  The guessed run is exact up to one
// constant iff end - warm is the same number d_k at every finite entry and both are
// -inf at the same entries (<= MSA_NEG/2: -inf may drift by a few gap costs).  Then
// every later row of chunk k is its computed value + d_k (the recurrence is max-plus
// homogeneous: it has no border term there) -- exact, not approximate.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void chunk_check_kernel(const int* __restrict__ ck, int ckw, int* dk, int* okk) {
  const int k = blockIdx.x;
  if (k == 0) {
    if (threadIdx.x == 0) { dk[0] = 0; okk[0] = 1; }
    return;
  }
  const int* end = ck + (size_t)(2 * (2 * (k - 1) + 1)) * ckw;  // slot 2(k-1)+1, planes H then F
  const int* warm = ck + (size_t)(2 * (2 * k)) * ckw;           // slot 2k
  __shared__ int first, bad;
  if (threadIdx.x == 0) { first = 0x7fffffff; bad = 0; }
  __syncthreads();
  constexpr int NH = MSA_NEG / 2;
  int mybad = 0, myfirst = 0x7fffffff;  // (one LDS atomic per thread, not per finite entry)
  for (int e = threadIdx.x; e < 2 * ckw; e += 256) {
    const int x = end[e], y = warm[e];
    if ((x > NH) != (y > NH)) mybad = 1;
    else if (x > NH && myfirst == 0x7fffffff) myfirst = e;  // e grows: the thread's first is its least
  }
  if (myfirst != 0x7fffffff) atomicMin(&first, myfirst);
  if (mybad) atomicOr(&bad, 1);
  __syncthreads();
  const int f = first;
  const int ref = (f < 2 * ckw) ? end[f] - warm[f] : 0;
  mybad = (f >= 2 * ckw);  // no finite entry: nothing pins the constant
  for (int e = threadIdx.x; e < 2 * ckw; e += 256) {
    const int x = end[e], y = warm[e];
    if (x > NH && x - y != ref) mybad = 1;
  }
  if (mybad) atomicOr(&bad, 1);
  __syncthreads();
  if (threadIdx.x == 0) {
    dk[k] = ref;
    okk[k] = bad ? 0 : 1;
  }
}

// grid (x, n_chunks): chunk k adds e_k = d_1 + ... + d_k to the cells it output (stripes
// [k*chunk_c, (k+1)*chunk_c), contiguous in the layout) and, for the stripe holding row m,
// to the final state.  If any chunk did not converge nothing is added, *skip = 0 and the
// tickets are reset: the exact single-mode launch queued next recomputes the pair.
// H16 (band_kernel's int16 chunk cells, KArgs::outH16): chunk k >= 1's cells are read from there
// (2 B per cell) and written widened to H (4 B) -- 6 B per cell instead of the in-place 8 B.
__global__ __launch_bounds__(256) void chunk_add_kernel(int32_t* H, const int16_t* H16, const msa_pair_desc* pairs,
                                                        msa_stripe_meta* meta, const int* dk, const int* okk,
                                                        int n_chunks, int chunk_c, int* skip, int* ticket) {
  const int k = blockIdx.y;
  const msa_pair_desc pd = pairs[0];
  const int S = (pd.m + 63) / 64;
  __shared__ int sh_e, sh_ok;
  // the prefix of chunk constants and the all-converged flag, over the block's threads (a serial
  // loop of 2 x n_chunks dependent global loads in thread 0 cost each block microseconds)
  {
    int e = 0, ok = 1;
    for (int j = threadIdx.x; j < n_chunks; j += blockDim.x) {
      ok &= okk[j];
      if (j <= k) e += dk[j];
    }
    const int all_ok = __syncthreads_and(ok);
    if (threadIdx.x == 0) sh_e = 0;
    __syncthreads();
    if (e != 0) atomicAdd(&sh_e, e);
    __syncthreads();
    e = sh_e;
    ok = all_ok;
    if (threadIdx.x == 0) sh_ok = ok;
  }
  if (threadIdx.x == 0) {
    const int e = sh_e, ok = sh_ok;
    if (blockIdx.x == 0 && k == 0) {
      *skip = ok;
      if (!ok)
        for (int t = 0; t < MSA_NTICKET; ++t) ticket[t] = 0;
    }
    if (ok && blockIdx.x == 0 && k == n_chunks - 1) {
      msa_stripe_meta* md = meta + pd.stripe0 + S - 1;
#pragma unroll
      for (int v = 0; v < 3; ++v)
        if (md->fin[v] > MSA_NEG / 2) md->fin[v] += e;
    }
  }
  __syncthreads();
  const int e = sh_e;
  const bool wide = (H16 != nullptr && k >= 1);  // this chunk's cells are int16 in H16
  if (!sh_ok || H == nullptr || (e == 0 && !wide)) return;
  const int ks0 = k * chunk_c, ke = min(S, ks0 + chunk_c);
  const size_t per = (size_t)pd.pmax * MSA_K * 64;  // int32 cells per stripe
  msa_v4i* p = reinterpret_cast<msa_v4i*>(H + pd.out_off + (size_t)ks0 * per);
  const size_t nv = (size_t)(ke - ks0) * per / 4;  // per is a multiple of 1024: nv of 256
  const size_t step = (size_t)gridDim.x * 1024;
  if (wide) {
    // every load and every store instruction covers whole 128-B lines (16-B loads feeding two 16-B stores
    // 32 B apart wrote every other 16 B of a line per instruction: 190 vs 145 us for C3's in-place int32
    // add); plain loads, the int16 cells were just written and are partly in the MALL.
    // MSA_H16_PAIRED: int16 16-B group G = (b, lane) holds the lane's 4 cells of u-blocks 2b and 2b + 1
    // (int32 16-B groups (2b, lane) and (2b + 1, lane), 64 groups per u-block); else 8-B group x = the
    // int32 16-B group x.
    typedef int v2i_t __attribute__((ext_vector_type(2)));
    auto widen = [&](int lo, int hi) __attribute__((always_inline)) {
      return msa_v4i{(lo << 16 >> 16) + e, (lo >> 16) + e, (hi << 16 >> 16) + e, (hi >> 16) + e};
    };
    if constexpr (MSA_H16_PAIRED) {
      // one 8-B half of a pair group per thread (8-B loads, as below: 16-B loads feeding two stores 1 KB
      // apart took 146 vs 134 us): half h of group (b, lane) -> int32 group (2b + h, lane); a wave's
      // store covers 32 lanes' 16 B of two u-blocks, whole lines
      const v2i_t* q = reinterpret_cast<const v2i_t*>(H16 + (size_t)(ks0 - chunk_c) * per);
      for (size_t x0 = (size_t)blockIdx.x * 1024 + threadIdx.x; x0 < nv; x0 += step) {  // 4 loads in flight
        v2i_t v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (x0 + 256 * u < nv) v[u] = q[x0 + 256 * u];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const size_t x = x0 + 256 * u;
          if (x < nv) {
            const size_t G = x >> 1;
            const size_t o = 2 * G - (G & 63) + 64 * (x & 1);  // (2b + h) * 64 + lane
            __builtin_nontemporal_store(widen(v[u].x, v[u].y), p + o);
          }
        }
      }
    } else {
      const v2i_t* q = reinterpret_cast<const v2i_t*>(H16 + (size_t)(ks0 - chunk_c) * per);
      for (size_t x0 = (size_t)blockIdx.x * 1024 + threadIdx.x; x0 < nv; x0 += step) {  // 4 loads in flight
        v2i_t v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (x0 + 256 * u < nv) v[u] = q[x0 + 256 * u];
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (x0 + 256 * u < nv) __builtin_nontemporal_store(widen(v[u].x, v[u].y), p + x0 + 256 * u);
      }
    }
    return;
  }
  // Plain loads: the band the chunk launch just streamed out is partly still in the MALL, so
  // they read ~3% faster than non-temporal ones (C3 0.649 vs 0.674 ms); measured the same or
  // slower: 8 loads in flight, plain stores, the last-written cells first.
  for (size_t x0 = (size_t)blockIdx.x * 1024 + threadIdx.x; x0 < nv; x0 += step) {  // 4 loads in flight
    msa_v4i v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (x0 + 256 * u < nv) v[u] = p[x0 + 256 * u];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (x0 + 256 * u < nv) __builtin_nontemporal_store(v[u] + e, p + x0 + 256 * u);
  }
}

__global__ __launch_bounds__(64) void reduce_pairs_kernel(const msa_pair_desc* pairs, const msa_stripe_meta* meta,
                                                         int n_pairs, int sw, PairResult* out) {
  // one wave per pair: lanes stride over the pair's stripes (a serial loop of
  // dependent meta loads took ~27 us for a 157-stripe pair)
  const int p = blockIdx.x;
  if (p >= n_pairs) return;
  const int lane = threadIdx.x;
  const msa_pair_desc pd = pairs[p];
  const int S = (pd.m + 63) / 64;
  PairResult r;
  r.status = 0;
  r.pad = 0;
  r.fin[0] = r.fin[1] = r.fin[2] = 0;
  if (sw) {
    // first max in row-major order; the empty alignment (score 0 at (0,0))
    // wins unless some stripe has a positive best
    int b = 0, bi = 0, bj = 0;
    for (int s = lane; s < S; s += 64) {
      const msa_stripe_meta& md = meta[pd.stripe0 + s];
      if (md.best > b) { b = md.best; bi = md.best_i; bj = md.best_j; }  // strided: rows increase with s
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      const int ob = __shfl_xor(b, off), oi = __shfl_xor(bi, off), oj = __shfl_xor(bj, off);
      if (ob > b || (ob == b && ob > 0 && oi < bi)) { b = ob; bi = oi; bj = oj; }
    }
    r.score = b;
    r.end_i = bi;
    r.end_j = bj;
  } else {
    const msa_stripe_meta md = meta[pd.stripe0 + S - 1];
    r.fin[0] = md.fin[0];
    r.fin[1] = md.fin[1];
    r.fin[2] = md.fin[2];
    r.score = max(max(md.fin[0], md.fin[1]), md.fin[2]);
    r.end_i = pd.m;
    r.end_j = pd.n;
    r.status = md.has_fin ? 0 : -1;
  }
  if (lane == 0) out[p] = r;
}

// ---------------------------------------------------------------------------
// Order-independent digest of an H output in the skewed layout (matches
// oracle orc_checksum_h): sum mix(i,j) * (uint32)H(i,j) over valid cells.
// ---------------------------------------------------------------------------
__device__ __forceinline__ unsigned long long splitmix64(unsigned long long x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// R rows per lane (two-pass flow plans may use R = 2): element
// ((s*pmax*4 + t/4)*R + rho)*256 + r*4 + t%4 <-> cell (64Rs + Rr + rho + 1, cs_s + t - r)
__global__ void checksum_kernel(const int32_t* H, const msa_pair_desc* pairs, const msa_stripe_meta* meta, int pair,
                                int band, int R, unsigned long long* out) {
  const msa_pair_desc pd = pairs[pair];
  const int S = (pd.m + 64 * R - 1) / (64 * R);
  const long long per_stripe = (long long)pd.pmax * MSA_K * 64 * R;
  const long long total = per_stripe * S;
  unsigned long long acc = 0;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const int s = (int)(e / per_stripe);
    const long long rem = e - (long long)s * per_stripe;
    const int quad = (int)((rem >> 8) / R);  // /(256R)
    const int rho = (int)((rem >> 8) - (long long)quad * R);
    const int r = (int)((rem >> 2) & 63);
    const int t = quad * 4 + (int)(rem & 3);
    const int i = 64 * R * s + R * r + rho + 1;
    const int j = meta[pd.stripe0 + s].cs + t - r;
    if (i > pd.m || j < 1 || j > pd.n) continue;
    if (band >= 0 && (i - j > band || j - i > band)) continue;
    const unsigned long long mix = splitmix64(((unsigned long long)i << 32) | (unsigned)j) | 1ull;
    acc += mix * (unsigned long long)(unsigned)H[pd.out_off + e];
  }
  // wave reduce
  for (int off = 32; off >= 1; off >>= 1) {
    const unsigned lo = __shfl_xor((unsigned)acc, off), hi = __shfl_xor((unsigned)(acc >> 32), off);
    acc += ((unsigned long long)hi << 32) | lo;
  }
  if ((threadIdx.x & 63) == 0) atomicAdd(out, acc);
}

}  // namespace msa

namespace msa {

// ---------------------------------------------------------------------------
// findPartitionParallel (partial.cpp:81-146) on device.  For every k in
// [1,p) it reduces max(T1+R1, T2+R2+h, T3+R3+h) (int32 wrap) over the row band
// rows [k*bm, (k+1)*bm) (scan order i, then j) and the column band columns
// [k*bn, (k+1)*bn) (scan order j, then i); the first maximum in scan order
// wins (the reference's strict '>').  Key = (val ^ 0x80000000) << 32 |
// (~scan_idx & 0x3fffffff) << 2 | type, reduced with 64-bit atomicMax.
// Forward planes F* and reverse planes R' (reverse fill = forward fill of the
// reversed strings) are read in the skewed stripe layout (msa_partial_partition), or
// the six tables row-major as the caller of findPartitionParallel holds them
// (msa_partition_tables).
// ---------------------------------------------------------------------------
__device__ __forceinline__ int skew_get(const int32_t* plane, const msa_pair_desc& pd, const msa_stripe_meta* meta,
                                        int i, int j) {
  const int s = (i - 1) >> 6, r = (i - 1) & 63;
  const int t = j - meta[pd.stripe0 + s].cs + r;
  const size_t e = (size_t)pd.out_off + (((size_t)s * pd.pmax * 4 + (t >> 2)) * 64 + r) * 4 + (t & 3);
  return plane[e];
}

// row-major tables as the reference holds them (findPartitionParallel's own inputs, host
// vector<vector<int>> flattened): T* (m+1) x (n+1), TR* (m+2) x (n+2), TR[i][j] at (m+1-i', n+1-j')
struct PartSkew {
  const int32_t *F1, *F2, *F3, *R1, *R2, *R3;
  const msa_pair_desc *pdf, *pdr;
  const msa_stripe_meta *mf, *mr;
  __device__ void get(int m, int n, int i, int j, int f[3], int r[3]) const {
    const msa_pair_desc f0 = pdf[0], r0 = pdr[0];
    f[0] = skew_get(F1, f0, mf, i, j), f[1] = skew_get(F2, f0, mf, i, j), f[2] = skew_get(F3, f0, mf, i, j);
    const int ri = m + 1 - i, rj = n + 1 - j;  // reverse fill = forward fill of the reversed strings
    r[0] = skew_get(R1, r0, mr, ri, rj), r[1] = skew_get(R2, r0, mr, ri, rj), r[2] = skew_get(R3, r0, mr, ri, rj);
  }
};
struct PartRowMajor {
  const int32_t *F1, *F2, *F3, *R1, *R2, *R3;
  __device__ void get(int m, int n, int i, int j, int f[3], int r[3]) const {
    const size_t ef = (size_t)i * (n + 1) + j, er = (size_t)i * (n + 2) + j;
    f[0] = F1[ef], f[1] = F2[ef], f[2] = F3[ef];
    r[0] = R1[er], r[1] = R2[er], r[2] = R3[er];
  }
};

template <class TABS>
__global__ void partition_kernel(TABS tabs, int m, int n, int p, int hh, unsigned long long* keys) {
  const int bm = m / p, bn = n / p;
  const long long rowcells = (long long)bm * n, colcells = (long long)bn * m;
  const long long total = (long long)(p - 1) * (rowcells + colcells);
  // thread-local best per slot; flushed when the (monotone) slot changes
  int cur_slot = -1;
  unsigned long long cur_key = 0;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    int k, i, j, slot;
    long long idx;
    if (e < (long long)(p - 1) * rowcells) {
      k = 1 + (int)(e / rowcells);
      idx = e - (long long)(k - 1) * rowcells;
      i = k * bm + (int)(idx / n);
      j = 1 + (int)(idx % n);
      if (i > m) continue;
      slot = 2 * k;
    } else {
      const long long e2 = e - (long long)(p - 1) * rowcells;
      k = 1 + (int)(e2 / colcells);
      idx = e2 - (long long)(k - 1) * colcells;
      j = k * bn + (int)(idx / m);
      i = 1 + (int)(idx % m);
      if (j > n) continue;
      slot = 2 * k + 1;
    }
    int f[3], r[3];
    tabs.get(m, n, i, j, f, r);
    const int val = imax3(wrap_add(f[0], r[0]), wrap_add(wrap_add(f[1], r[1]), hh), wrap_add(wrap_add(f[2], r[2]), hh));
    if (val == INT32_MIN) continue;  // can never beat the reference's INT_MIN start
    const unsigned type = (unsigned)firstmax3(f[0], f[1], f[2]);
    const unsigned long long key = ((unsigned long long)((unsigned)val ^ 0x80000000u) << 32) |
                                   ((unsigned long long)((~(unsigned)idx) & 0x3fffffffu) << 2) | type;
    if (slot != cur_slot) {
      if (cur_slot >= 0 && cur_key) atomicMax(keys + cur_slot, cur_key);
      cur_slot = slot;
      cur_key = 0;
    }
    cur_key = key > cur_key ? key : cur_key;
  }
  if (cur_slot >= 0 && cur_key) atomicMax(keys + cur_slot, cur_key);
}

}  // namespace msa
