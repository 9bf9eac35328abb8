// msa_flow.hip -- single-pair Smith-Waterman (linear gap) in two passes: the
// latency-bound DP chain, then a chip-wide recompute that writes H (config C2:
// one 10k x 10k pair on one GPU).  Replaces, for this configuration, the
// reference's row sweep Subproblem::compute_tables (subproblem_alignment.cpp:
// 329-332; per-row T1/T3 :229-235, the omega prefix-max scan :237-249, :13-103).
//
// Pass 1 (flow_kernel) runs stripe_kernel's geometry (64-row stripes, lane r =
// row 64s+r+1 at column cs+t-r in step t) as a flag-synchronised pipeline cut
// down to the loop-carried chain.  Per DP step a compute wave issues one DPP
// wave_shr:1 (the cell above, from lane r-1; lane 0 takes the producer's value
// through the DPP `old` operand), one SDWA byte add (diagonal + score from a
// v_perm'd profile word) and one v_max3:
//     G(i,j) = max3(G(i-1,j-1) + s + 2g, G(i-1,j), G(i,j-1)),   G = H + g(i+j)
// (X-space, X = H - g with a zero floor, when scores can be negative).  The
// step time is the DPP -> v_max3 latency (~21 cycles measured on one wave);
// nothing else sits on the chain:
//   * waves 0..W-1 compute (one per SIMD), wave W io-in, wave W+1 io-out;
//   * no s_barrier: a producer's lane 63 writes each 16-column block of its
//     bottom row to an LDS ring and then bumps its phase counter; the consumer
//     reads the counter, then the block (LDS executes one wave's DS
//     instructions in issue order), half a phase ahead of use.  A slot is
//     re-used once the consumer and io-out have passed it;
//   * io-in: column codes into LDS (8 byte-shifted copies, one ds_read2_b64
//     per lane per phase) ahead of the blocks it publishes, and the row above
//     the workgroup (the previous workgroup's {epoch, value} granules, or row 0);
//   * io-out: every link's blocks -> the bottom-row array BR (pass 2's input),
//     the last link's also -> {epoch, value} granules for the next workgroup;
//   * every segment (FL_PS phases, FL_PS_FILL for a separate pass-2 launch) each lane's state -> SNAP;
//   * items (W stripes) come from 8 per-XCD ticket chunks: consecutive items
//     share an L2, and an item only ever waits on an earlier one.
// Pass 2 (fill_kernel): every (stripe, segment) block restarts
// from SNAP and BR, recomputes its cells with the same instructions, writes
// int32 H in the skewed stripe layout (coalesced non-temporal 1 KiB stores)
// and reduces its best cell.  Thousands of independent blocks fill the chip,
// so H streams at HBM rate instead of stalling the chain (a 1 KiB store
// stalls its wave ~40 cycles, longer than a DP step).
#pragma once

namespace msa {

#ifndef FL_W
#define FL_W 4          // compute waves per workgroup: one per SIMD (8, two per SIMD, measured: C2
                        // 0.576 vs 0.455 ms, C5 2.78 vs 1.91, ref 1.73 vs 1.12 -- a chain wave keeps its
                        // SIMD's issue busy, so a second wave on it slows both)
#endif
#define FL_RINGB 16     // ring blocks of 16 columns per link (256 columns)
#define FL_OFF 95       // LDS code copy x, byte y <-> column y + x - FL_OFF (== CPAD-1 mod 16)
#define FL_NCOPY 8      // byte-shifted LDS code copies (8-byte aligned 8-code reads)
#define FL_FLAGS 128    // ints of flags at the start of LDS
// Column codes stream through an LDS ring per copy: copy-local byte y sits at y mod FL_CRING,
// and the 16 bytes at ring position 0 are mirrored past the end (FL_CSTR = ring + guard), so
// every 16-byte read at any ring position is contiguous.  io-in refills a slot once every
// compute wave has passed it, so the kernel runs any n (whole-row copies capped SW linear at
// n <= ~19.5k and affine / Gotoh at ~37k).
#define FL_CRING 4096
#define FL_CSTR (FL_CRING + 16)
// When a copy's whole code row fits the LDS budget (kp.code_whole, msa_capi.hip), the copies are
// linear (stride L8 + 16, no wrap) and io-in never holds blocks back for ring space: the ring's
// refill bookkeeping measured +6 us on C2 (10k, 0.459 -> 0.465 ms).
#ifndef FL_PS
#define FL_PS 8         // phases per pass-2 segment of the in-launch pass 2 (pass 1 saves its state every
#endif                  // segment: KArgs::ps_shift, the plan's segment length)
#ifndef FL_PS_FILL
#define FL_PS_FILL 32   // ... of the separate pass-2 launch (flow_fill_kernel, long pairs): fewer, longer
#endif                  // blocks stage SNAP + BR less often (97k ref: 15.70 -> 13.02 ms at 32, 13.36 at 16)
// A pass-2 wave's LDS area (p2_stage): two value streams of fl_p2vs(PS) ints (the row above the block's
// 16 PS columns), then the column codes its phases read, one staged dword per lane and round.
// Lane r of phase k reads code dwords (63 - r + 16 k) / 4 + [0, 5), i.e. up to (63 + 16 (PS - 1)) / 4
// + 4: 48 dwords at PS = 8, 144 at 32.  Round 5 staged a fixed 64 dwords, so a 16-phase build read
// its last phases' codes from the next wave's area (a wrong direction-byte plane, a wrong 97k walk
// with the right score); the span now follows the segment length.
constexpr int fl_ps(int caller) { return caller ? FL_PS_FILL : FL_PS; }
constexpr int fl_p2vs(int ps) { return 16 * ps > 256 ? 16 * ps : 256; }     // ints per value stream
constexpr int fl_p2codw(int ps) { return (63 + 16 * (ps - 1)) / 4 + 5; }  // code dwords a block's phases read
constexpr int fl_p2cod(int ps) { return (fl_p2codw(ps) + 63) / 64 * 64; } // staged: whole rounds of 64 lanes
constexpr int fl_p2ints(int ps) { return 2 * fl_p2vs(ps) + fl_p2cod(ps); } // 576 at PS = 8, 1216 at 32
static_assert(fl_p2ints(FL_PS) == 576 || FL_PS != 8, "in-launch pass-2 LDS area");
static_assert(16 * FL_PS <= fl_p2vs(FL_PS) && 16 * FL_PS_FILL <= fl_p2vs(FL_PS_FILL),
              "a value stream holds the row above a segment's 16-column phases");
static_assert(fl_p2codw(FL_PS_FILL) <= fl_p2cod(FL_PS_FILL), "the staged code span covers every code dword read");
static_assert((FL_PS & (FL_PS - 1)) == 0 && (FL_PS_FILL & (FL_PS_FILL - 1)) == 0, "segments: powers of two");
#define FL_FILLW 4      // waves per workgroup of the separate pass-2 launch (flow_fill_kernel)
#define FL_SPIN_MAX (1u << 26)  // a spin limit sets err = the site's code (10..15) instead of hanging
#ifndef FL_PF
#define FL_PF 12        // step of a phase at which the next phase's inputs are read
#endif
#ifndef FL_FSLEEP
#define FL_FSLEEP 32    // s_sleep between a pass-2 wave's polls of its block's last granule
#endif
// Affine / Gotoh pass-2 waves claim their blocks in readiness order but long before pass 1 reaches
// them (pass 1 is the chain): after FL_FSLONG polls a wave polls every FL_FSLEEP2 x 64 cycles instead
// (ref 10k: ~4 of the kernel's ~32 VALU lane-ops per cell were such polls)
#ifndef FL_FSLEEP2
#define FL_FSLEEP2 96
#endif
#ifndef FL_FSLONG
#define FL_FSLONG 8
#endif
__device__ __forceinline__ void fl_poll_sleep(int polls) {
  if (polls < FL_FSLONG) __builtin_amdgcn_s_sleep(FL_FSLEEP);
  else __builtin_amdgcn_s_sleep(FL_FSLEEP2);
}
#ifndef FL_IOSLEEP
#define FL_IOSLEEP 1    // s_sleep of an idle io wave
#endif
// Diagnostic builds only (-DMSA_ABL=mask; results are wrong): 1 no pass-2 work, 2 no SNAP
// stores, 4 io-out stores no bottom rows (granules still), 8 R = 2 pass-2 blocks store no cells, 16 SW-linear compute waves never wait on their producer
// or consumers (each stripe runs at its own speed), 32 never on the producer, 64 never on consumers
#ifndef MSA_ABL
#define MSA_ABL 0
#endif
// v_max3_i32 as one opaque instruction: the compiler re-associates three max3 that share an operand
// (h, R~, D~ of one cell) into a max + two max + a max3 -- four VALU instead of three
__device__ __forceinline__ int vmax3(int a, int b, int c) {
  int d;
  asm("v_max3_i32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}

__host__ __device__ __forceinline__ int fl_cs(int k) { return -((16 - (k & 15)) & 15); }  // -((-k) mod 16)
// R rows per lane: stripe k holds rows 64Rk+1 .. 64R(k+1); rlast = last lane with a row
__host__ __device__ __forceinline__ int fl_P(int k, int m, int n, int R = 1) {
  const int rl = (m - 64 * R * k - 1) / R;
  const int rlast = (rl < 63) ? rl : 63;
  return (n - fl_cs(k) + rlast) / 16 + 1;
}
// link k-1 -> k: ring block b holds columns cs_k + 16b .. +15 of row 64k;
// producer phase q writes block q - fl_dq(k); its last block is fl_bmax(k)
__host__ __device__ __forceinline__ int fl_delta(int kc) { return fl_cs(kc - 1) + 1 - fl_cs(kc); }
__host__ __device__ __forceinline__ int fl_dq(int kc) { return 4 - fl_delta(kc) / 16; }
__host__ __device__ __forceinline__ int fl_bmax(int kc, int m, int n, int R = 1) {
  return fl_P(kc - 1, m, n, R) - 1 - fl_dq(kc);
}
// bytes per LDS code copy for n columns (covers the prefetch one phase past a stripe's last)
__host__ __device__ __forceinline__ int fl_code_bytes(int n) { return ((n + 208) + 15) & ~15; }

// LDS accesses through explicit address-space-3 pointers: a generic pointer
// would become a FLAT access (counted in vmcnt AND lgkmcnt, forcing full waits)
typedef __attribute__((address_space(3))) int lds_int;
typedef int fl_v4i __attribute__((ext_vector_type(4)));
typedef unsigned fl_v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) fl_v4i lds_int4;
__device__ __forceinline__ lds_int* L(int* p) { return (lds_int*)(p); }
__device__ __forceinline__ lds_int* L(lds_int* p) { return p; }
__device__ __forceinline__ int lds_vload(const int* p) { return *(volatile lds_int*)(p); }
__device__ __forceinline__ void lds_vstore(int* p, int v) { *(volatile lds_int*)(p) = v; }
#define FL_CBAR() asm volatile("" ::: "memory")
// Diagnostic build (-DMSA_STAMPS): stamps[((item*16 + w)*4096 + q)*4 + slot], q = 0:
//   slot 0: s_memrealtime at the stripe's start, 1: at its end, 2: slow-path phases
#ifdef MSA_STAMPS
#define FL_STAMP(q_, slot_, v_)                                                                        \
  do {                                                                                              \
    if (a.stamps && lane == 0 && (q_) < 4096 && item < 64)                                           \
      a.stamps[(((size_t)item * 16 + w) * 4096 + (q_)) * 4 + (slot_)] = (v_);                        \
  } while (0)
#else
#define FL_STAMP(q_, slot_, v_) do {} while (0)
#endif
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)(p);
}
// Inline-asm DS ops: the compiler does not count them, so every wait below is
// explicit (s_waitcnt lgkmcnt(N), N = DS ops issued after the awaited one), and
// every output stays live (named "+v" by its wait) until it has landed.
__device__ __forceinline__ int ds_read_b32(unsigned a) {
  int v;
  asm volatile("ds_read_b32 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}
template <int OFF>
__device__ __forceinline__ fl_v4i ds_read_b128(unsigned a) {
  fl_v4i v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(a), "i"(OFF) : "memory");
  return v;
}
__device__ __forceinline__ fl_v4u ds_read2_b64(unsigned a) {
  fl_v4u v;
  asm volatile("ds_read2_b64 %0, %1 offset1:1" : "=v"(v) : "v"(a) : "memory");
  return v;
}
// slow path: re-read a block into the same registers (tied operands: no copies on the fast path)
__device__ __forceinline__ void ds_reread_b128x4(unsigned a, fl_v4i (&in)[4]) {
  asm volatile(
      "ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:16\n\t"
      "ds_read_b128 %2, %4 offset:32\n\tds_read_b128 %3, %4 offset:48\n\ts_waitcnt lgkmcnt(0)"
      : "+v"(in[0]), "+v"(in[1]), "+v"(in[2]), "+v"(in[3])
      : "v"(a)
      : "memory");
}
template <int N = 0>
__device__ __forceinline__ void lgkm_wait(int& v) { asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(v) : "i"(N) : "memory"); }
// A stripe's end: every phase already waited for its prefetched inputs, so only the hand-off writes
// may be in flight -- a plain wait, tying no registers.  (Tying the ring-input arrays here, as before,
// kept the second buffer of the ping-pong live out of the phase loop, and the compiler then copied
// every DPP input of the odd phases to a temporary: 32-40 extra v_mov per odd phase.)
__device__ __forceinline__ void lgkm_drain() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
template <int N = 0>
__device__ __forceinline__ void lgkm_wait_v(fl_v4i (&in)[4], fl_v4u& cw) {
  asm volatile("s_waitcnt lgkmcnt(%5)" : "+v"(in[0]), "+v"(in[1]), "+v"(in[2]), "+v"(in[3]), "+v"(cw) : "i"(N) : "memory");
}
// Lane 63 alone: its 16 bottom-row values -> ring block as 16 ds_write_addtid_b32
// (LDS[M0 + offset + 4*lane]; lane 63: M0 = slot - 252; cheaper to issue than
// four single-lane b128 writes), then the phase counter (DS ops of one wave
// execute in order: the block lands first).  s_nop 4: an SALU exec write needs
// 5 wait states before a DPP op.
__device__ __forceinline__ void ds_handoff_tid(unsigned long long m63, unsigned m0v, const int (&x)[16], unsigned pa,
                                               int pv) {
  unsigned long long sv;
  asm volatile(
      "s_mov_b64 %[sv], exec\n\ts_mov_b64 exec, %[m]\n\ts_nop 0\n\t"
      "ds_write_addtid_b32 %[x0] offset:0\n\tds_write_addtid_b32 %[x1] offset:4\n\t"
      "ds_write_addtid_b32 %[x2] offset:8\n\tds_write_addtid_b32 %[x3] offset:12\n\t"
      "ds_write_addtid_b32 %[x4] offset:16\n\tds_write_addtid_b32 %[x5] offset:20\n\t"
      "ds_write_addtid_b32 %[x6] offset:24\n\tds_write_addtid_b32 %[x7] offset:28\n\t"
      "ds_write_addtid_b32 %[x8] offset:32\n\tds_write_addtid_b32 %[x9] offset:36\n\t"
      "ds_write_addtid_b32 %[x10] offset:40\n\tds_write_addtid_b32 %[x11] offset:44\n\t"
      "ds_write_addtid_b32 %[x12] offset:48\n\tds_write_addtid_b32 %[x13] offset:52\n\t"
      "ds_write_addtid_b32 %[x14] offset:56\n\tds_write_addtid_b32 %[x15] offset:60\n\t"
      "ds_write_b32 %[pa], %[pv]\n\t"
      "s_mov_b64 exec, %[sv]\n\ts_nop 4"
      : [sv] "=&s"(sv)
      : [m] "s"(m63), "{m0}"(m0v), [x0] "v"(x[0]), [x1] "v"(x[1]), [x2] "v"(x[2]), [x3] "v"(x[3]), [x4] "v"(x[4]),
        [x5] "v"(x[5]), [x6] "v"(x[6]), [x7] "v"(x[7]), [x8] "v"(x[8]), [x9] "v"(x[9]), [x10] "v"(x[10]),
        [x11] "v"(x[11]), [x12] "v"(x[12]), [x13] "v"(x[13]), [x14] "v"(x[14]), [x15] "v"(x[15]), [pa] "v"(pa),
        [pv] "v"(pv)
      : "memory");
}




// Affine hand-off: lane 63 alone writes its 16 Z and 16 F~ of the phase as 8 b128 writes
// (the F~ half of a link's ring sits 1 KiB after the Z half), then the phase counter.
__device__ __forceinline__ void ds_handoff_aff(unsigned long long m63, unsigned addr, const fl_v4i (&z)[4],
                                               const fl_v4i (&f)[4], unsigned pa, int pv) {
  unsigned long long sv;
  asm volatile(
      "s_mov_b64 %[sv], exec\n\ts_mov_b64 exec, %[m]\n\ts_nop 0\n\t"
      "ds_write_b128 %[a], %[z0]\n\tds_write_b128 %[a], %[z1] offset:16\n\t"
      "ds_write_b128 %[a], %[z2] offset:32\n\tds_write_b128 %[a], %[z3] offset:48\n\t"
      "ds_write_b128 %[a], %[f0] offset:1024\n\tds_write_b128 %[a], %[f1] offset:1040\n\t"
      "ds_write_b128 %[a], %[f2] offset:1056\n\tds_write_b128 %[a], %[f3] offset:1072\n\t"
      "ds_write_b32 %[pa], %[pv]\n\t"
      "s_mov_b64 exec, %[sv]\n\ts_nop 4"
      : [sv] "=&s"(sv)
      : [m] "s"(m63), [a] "v"(addr), [z0] "v"(z[0]), [z1] "v"(z[1]), [z2] "v"(z[2]), [z3] "v"(z[3]), [f0] "v"(f[0]),
        [f1] "v"(f[1]), [f2] "v"(f[2]), [f3] "v"(f[3]), [pa] "v"(pa), [pv] "v"(pv)
      : "memory");
}
typedef unsigned fl_v2u __attribute__((ext_vector_type(2)));
// 16 code bytes from a 4-byte aligned LDS address: two ds_read2_b32
__device__ __forceinline__ void ds_read_codes16(unsigned a, fl_v2u& lo, fl_v2u& hi) {
  asm volatile("ds_read2_b32 %0, %2 offset1:1\n\tds_read2_b32 %1, %2 offset0:2 offset1:3"
               : "=&v"(lo), "=&v"(hi)
               : "v"(a)
               : "memory");
}
template <int N = 0>
__device__ __forceinline__ void lgkm_wait_aff(fl_v4i (&z)[4], fl_v4i (&f)[4], fl_v2u& lo, fl_v2u& hi) {
  asm volatile("s_waitcnt lgkmcnt(%10)"
               : "+v"(z[0]), "+v"(z[1]), "+v"(z[2]), "+v"(z[3]), "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]),
                 "+v"(lo), "+v"(hi)
               : "i"(N)
               : "memory");
}
// Affine profile: score + 2e + oe for codes 0..6 (int8); the virtual code 7 gets 0, i.e. s =
// -(2e + oe) <= 0, which keeps H = 0 left of column 1 and never lifts a cell right of n
// above the real cell it came from.
__device__ __forceinline__ void fl_profile_aff(int match, int mismatch, int e, int oe, unsigned ac, unsigned& plo,
                                               unsigned& phi) {
  const int sm = match + 2 * e + oe, sx = mismatch + 2 * e + oe;
  const unsigned bx = (unsigned)(sx & 0xff) * 0x01010101u;
  unsigned lo = bx, hi = bx;
  const unsigned bm = (unsigned)(sm & 0xff);
  if (ac < 4) lo = (lo & ~(0xffu << (8 * ac))) | (bm << (8 * ac));
  else hi = (hi & ~(0xffu << (8 * (ac - 4)))) | (bm << (8 * (ac - 4)));
  plo = lo;
  phi = hi & 0x00ffffffu;
}

// Gotoh profile (tagged, shifted): 4 (f + 2g), f = 1 on a match, 0 otherwise (the reference's
// f, main_alignment.cpp); the virtual code 7 (columns past n) gets 0.
__device__ __forceinline__ void fl_profile_got(int g, unsigned ac, unsigned& plo, unsigned& phi) {
  const int sm = 4 * (1 + 2 * g), sx = 8 * g;
  const unsigned bx = (unsigned)(sx & 0xff) * 0x01010101u;
  unsigned lo = bx, hi = bx;
  const unsigned bm = (unsigned)(sm & 0xff);
  if (ac < 4) lo = (lo & ~(0xffu << (8 * ac))) | (bm << (8 * ac));
  else hi = (hi & ~(0xffu << (8 * (ac - 4)))) | (bm << (8 * (ac - 4)));
  plo = lo;
  phi = hi & 0x00ffffffu;
}

// Substitution profile of a row: score + g (X-space) or + 2g (G-space) for
// codes 0..7; code 7 = virtual column (outside [1, n]): score 0 without the
// floor (keeps H = 0 left of column 1, never above a real cell right of n),
// -100 with it.
template <bool GS, bool FLOOR>
__device__ __forceinline__ void fl_profile(int match, int mismatch, int g, unsigned ac, unsigned& plo, unsigned& phi) {
  const int sh = GS ? 2 * g : g;
  const int sm = match + sh, sx = mismatch + sh;
  const unsigned bx = (unsigned)(sx & 0xff) * 0x01010101u;
  unsigned lo = bx, hi = bx;
  const unsigned bm = (unsigned)(sm & 0xff);
  if (ac < 4) lo = (lo & ~(0xffu << (8 * ac))) | (bm << (8 * ac));
  else hi = (hi & ~(0xffu << (8 * (ac - 4)))) | (bm << (8 * (ac - 4)));
  const int sv = (FLOOR ? MSA_VIRT_SCORE : 0) + sh;
  hi = (hi & 0x00ffffffu) | ((unsigned)(sv & 0xff) << 24);
  plo = lo;
  phi = hi;
}

// One DP step of every lane; returns the cell's G (G-space) or H (X-space).
template <bool GS, bool FLOOR>
__device__ __forceinline__ int fl_step(int in, int s, int& X, int& U, int g) {
  const int up = dpp_shr1(in, X);
  int h = imax3(U + s, up, X);
  if constexpr (FLOOR) h = imax(h, 0);
  asm("" : "+v"(h));  // keeps the chain a real per-step value
  U = up;
  X = GS ? h : h - g;
  return h;
}

// FLOOR: scores may be negative (zero floor, X-space); otherwise G-space.  Affine SW: the
// floor in every pass-1 step; otherwise (scores >= 0) only in the head phases.
// BEST: track the best cell in pass 1 (score-only plans: no pass 2).
// SAVE: write BR and SNAP for pass 2.
// AFF: Smith-Waterman with affine gaps (config C5), pass 2 writing direction bytes.  Values
// run shifted by e(i+j) (e = gap_extend, o = gap_open, oe = o - e):
//   H~ = H + e(i+j),  E~ = E + e(i+j),  F~ = F + e(i+j),  Z = H~ - oe
//   E~(i,j) = max(E~(i,j-1), Z(i,j-1))      F~(i,j) = max(F~(i-1,j), Z(i-1,j))
//   H~(i,j) = max(Z(i-1,j-1) + s + 2e + oe,  E~,  F~,  e(i+j))
// so no gap constant sits between a DPP and its max; the floor e(i+j) is wave-uniform per
// step (i+j is constant along a step).  Lanes hand Z and F~ down (2 DPPs per step), links
// carry both (two values per column in the rings, granules and bottom rows), a lane's state
// is (Z left, E~, F~, diagonal Z).  The direction byte is stripe_kernel's MSA_ALG_SWA byte:
// every tie test compares values at one cell, which the shift leaves exact.
// GOT: the reference's Gotoh recurrence, start type -1, in stripe_kernel's tagged form
// (MSA_ALG_REF1: value x 4 + tag, max() = the reference's first-maximum table order) and
// shifted by g(i+j) as above:
//   t1 = (H~diag | 3) + 4(f + 2g),  t2 = (R~left & ~3) | 2,  t3 = (D~up & ~3) | 1
//   H~ = max(t1, t2, t3),  R~ = max(t1 - 4h, t2, t3 - 4h),  D~ = max(t1 - 4h, t2 - 4h, t3)
// (R~ / D~ = T2 of the cell to the right / T3 of the cell below; the gap extension g is
// absorbed by the shift, so the borders are constants: row 0 (3, 3 - 4h) at column 0 and
// (2 - 4h, 2 - 8h) right of it, column 0 (1 - 4h, 1 - 8h, 1 - 4h)).  Links carry H~ and D~,
// a lane's state is (H~, R~, D~, diagonal H~); the first 6 phases hold lanes still left of
// column 1 at the column-0 border (stripe_kernel's LB masking).  Pass 2 writes the tag bytes
// traceback_kernel<TB_REF_TAG> walks and the (m, n) tables find_alignment's end rule reads.
// What a pass-2 block needs, by value (a reference to the kernel's KArgs would
// put them on the stack of the pass-1 path too).
struct FillArgs {
  const uint8_t* A;
  const uint8_t* cod;
  const unsigned long long* br;
  const unsigned long long* snap;
  int32_t* outH;
  int4* blk;
  int* err;
  long long cod_copy, a_off, cod_off, out_off;
  int m, n, pmax, nseg, brw, match, mismatch, g;
  unsigned ep;
  uint8_t* outDir;  // affine / Gotoh: direction bytes
  int oe;           // affine: gap_open - gap_extend (g = gap_extend); Gotoh: h
  msa_stripe_meta* meta;  // Gotoh: the final cell's tables go to the last stripe's meta
  int stripe0;
  unsigned long long* best_key;  // SW: the pair's best-cell key (fl_block_result), or nullptr
#ifdef MSA_STAMPS
  unsigned long long* stamps;  // diagnostic: pass-2 block tick totals (FL_P2STAT)
#endif
};
#ifdef MSA_STAMPS
// pass-2 totals (diagnostic build): [0] ticks waiting for the block's last granule, [1] ticks loading and
// checking its inputs, [2] ticks computing + storing, [3] blocks, at item 62 / wave 15's stamp area
#define FL_P2STAT(a_, k_, v_) \
  do { if ((a_).stamps && lane == 0) atomicAdd((a_).stamps + ((size_t)(62 * 16 + 15) * 4096) * 4 + (k_), (unsigned long long)(v_)); } while (0)
#else
#define FL_P2STAT(a_, k_, v_) do {} while (0)
#endif
// Pass-2 block functions read their arguments from the kernel's own argument segment (scalar loads,
// FillArgs built in SGPRs) and get their wave's LDS area as an LDS pointer: no by-value struct on the
// stack, so the kernel needs no scratch (a stack copy of FillArgs per call cost the launch its scratch
// setup and every access a private-memory load).
// The pair result of a two-pass SW plan, folded by the pass-2 blocks themselves when best_key is set
// (msa_plan_create: (m + 1)(n + 1) < 2^32): lane 0 of a block folds the block's best into one 64-bit key
// with a non-returning atomicMax -- score, then the first cell in row-major order, reduce_blocks_kernel's
// rule -- instead of storing it for a reduce_blocks_kernel launch (that launch, ~5 us, and its dispatch
// gap, ~6 us, leave C2's step).  Readers decode the key (best_key_decode).  Measured and not kept: the
// last block writing the PairResult itself -- a done counter and two __threadfence, which made every
// pass-2 wave wait for its cell stores: C2 kernel 0.466 -> 0.477 ms.
__device__ __forceinline__ void fl_block_result(int4* blk_out, unsigned long long* best_key, int blk, int lane, int bb,
                                                int bi, int bj, int n) {
  if (lane != 0) return;
  if (best_key) {
    const unsigned lo = bb > 0 ? ~(unsigned)((unsigned long long)bi * (unsigned)(n + 1) + (unsigned)bj) : 0xffffffffu;
    atomicMax(best_key, ((unsigned long long)((unsigned)bb ^ 0x80000000u) << 32) | lo);
  } else {
    blk_out[blk] = make_int4(bb, bi, bj, 0);
  }
}
typedef const __attribute__((address_space(4))) struct KArgs kargs_c;
__device__ __forceinline__ FillArgs fill_args_of(kargs_c* k) {
  // (measured: the pointer made wave-uniform -- scalar loads of the arguments instead of vector loads --
  // made C2 slower, 0.466 -> 0.476 ms)
  const msa_pair_desc pd = k->pairs[0];
  return FillArgs{k->A, k->cod, k->br, k->snap, k->outH, k->blk, k->err, k->cod_copy, pd.a_off, pd.cod_off,
                  pd.out_off, pd.m, pd.n, pd.pmax, k->nseg, k->brw, k->kp.match, k->kp.mismatch, k->kp.gap_ext,
                  k->kp.epoch, k->outDir, k->kp.gap_open - k->kp.gap_ext, k->meta, pd.stripe0, k->best_key
#ifdef MSA_STAMPS
                  , k->stamps
#endif
  };
}
// Pass-2 block functions, one instantiation per calling kernel (CALLER 0: flow_kernel's in-launch pass 2,
// 1: flow_fill_kernel): a non-inlined function shared by two kernels gets the tighter register budget of
// the two (flow_fill_kernel's four waves per SIMD = 128 VGPRs), and spilled there -- fill_block_aff2 188 B
// and fill_block_got2 68 B of scratch per lane, which was C5's and ref's unexplained HBM traffic
template <bool FLOOR, bool TRACKPOS, int R, int CALLER>
// SW-linear pass-2 blocks take their arguments by value (C2 0.4646 -> 0.4604 ms against the kernarg pointer)
__device__ __attribute__((noinline)) void fill_block(const FillArgs fa, int blk, int lane, lds_int* lds);
template <int CALLER> __device__ __attribute__((noinline)) void fill_block_aff(kargs_c* ka, int blk, int lane, lds_int* lds);
template <int CALLER> __device__ __attribute__((noinline)) void fill_block_aff2(kargs_c* ka, int blk, int lane, lds_int* lds);
template <int CALLER> __device__ __attribute__((noinline)) void fill_block_got(kargs_c* ka, int blk, int lane, lds_int* lds);
template <int CALLER> __device__ __attribute__((noinline)) void fill_block_got2(kargs_c* ka, int blk, int lane, lds_int* lds);

template <bool FLOOR, bool BEST, bool SAVE, bool TRACKPOS, int R = 1, int FK = 0>
#ifndef FL_WPE
#define FL_WPE 2  // waves per SIMD the register budget is sized for (3: no faster for 97k pairs, C5 3% slower: spills)
#endif
__global__ __launch_bounds__((FL_W + 2) * 64) __attribute__((amdgpu_waves_per_eu(FL_WPE, 8))) void flow_kernel(KArgs a) {
  constexpr bool GS = !FLOOR;
  constexpr bool AFF = FK != 0;  // two values per link column (affine SW, Gotoh)
  constexpr bool GOT = FK == 2;  // the reference's Gotoh, tagged
  static_assert(R == 1 || (R == 2 && !BEST), "two rows per lane: pass-2 plans only");
  static_assert(!AFF || (SAVE && !BEST), "affine / Gotoh: two-pass");
  constexpr int NV = AFF ? 2 : 1;                  // values per column on a link (Z, F~)
  constexpr int NCP = AFF ? 4 : FL_NCOPY;          // LDS code copies (affine: 4-byte aligned reads)
  extern __shared__ __attribute__((aligned(16))) int smem[];
  const msa_kparams& kp = a.kp;
  const int lane = threadIdx.x & 63;
  const int w = uni(threadIdx.x >> 6);
  constexpr int W = FL_W;
  // flags: [0] item; prog[l] 32+l (l = 0: io-in's published blocks, l = c+1:
  // compute wave c's finished phases); rcons[l] 64+l (io-out: blocks of link l
  // taken); dummy sink 96..127
  int* flags = smem;
  int* rings = smem + FL_FLAGS;                                               // [W+1 links][NV][256]
  uint8_t* codes = reinterpret_cast<uint8_t*>(rings + (W + 1) * 256 * NV);  // [NCP][cstr] rings / rows
  const int L8 = kp.lds_code_bytes;  // bytes of a copy's whole (linear) code row
  const bool cwhole = kp.code_whole != 0;
  const int cstr = cwhole ? L8 + 16 : FL_CSTR;               // bytes per LDS copy
  const unsigned cmask = cwhole ? 0xffffffffu : (unsigned)(FL_CRING - 1);
  const msa_pair_desc pd = a.pairs[0];
  const int m = pd.m, n = pd.n;
  const int S = (m + 64 * R - 1) / (64 * R);
  const int g = kp.gap_ext;
  const int oe = kp.gap_open - kp.gap_ext;  // affine
  const unsigned ep = kp.epoch;
  const int chunk = kp.sched_cap;  // G: items per XCD run (msa_plan_create)

#ifdef MSA_STAMPS
  // workgroup lifetimes: item 63 / wave 15's area, q = blockIdx.x: slot 0 start, 1 end, 2 role
  auto wg_stamp = [&](int slot, unsigned long long v) {
    if (a.stamps && threadIdx.x == 0 && blockIdx.x < 4096)
      a.stamps[(((size_t)63 * 16 + 15) * 4096 + blockIdx.x) * 4 + slot] = v;
  };
  wg_stamp(0, __builtin_amdgcn_s_memrealtime());
#endif
  // Role by arrival, not by blockIdx: the first nflow workgroups to START run pass 1,
  // the later ones pass-2 blocks.  A pass-2 block waits only on pass-1 outputs, and
  // every pass-1 role is held by a workgroup that is already running (and stays
  // resident until every item is claimed), so progress does not depend on the order
  // in which the hardware dispatches workgroups, or on CUs held by other kernels.
  if (threadIdx.x == 0) smem[1] = atomicAdd(a.ticket + MSA_TK_ARRIVE, 1);
  __syncthreads();
  const int arrival = uni(smem[1]);
  // Pass-1 items come from 8 chunks, a workgroup's own chunk first: blockIdx & 7 (round-robin
  // placement puts workgroup b on XCD b % 8, so a chunk's consecutive items share an L2),
  // except that the first 8 arrivals take chunk = arrival: every chunk's first item is then
  // claimed by a running workgroup even if the workgroup with blockIdx c is not resident (CUs
  // held by other launches), and a chunk's later items wait only on claimed ones.
  const int grp = arrival < 8 ? arrival : (int)(blockIdx.x & 7);  // (blockIdx & 7 alone: C2 0.539 vs 0.459 ms)
  if constexpr (SAVE) {
#ifdef MSA_STAMPS
    if (a.stamps && threadIdx.x == 0 && blockIdx.x < 2048)
      a.stamps[(((size_t)63 * 16 + 15) * 4096 + 2048 + blockIdx.x) * 4 + 0] = __builtin_amdgcn_s_memrealtime();
#endif
    if (arrival >= a.nflow) {
#ifdef MSA_STAMPS
      wg_stamp(2, 2);
#endif
      if constexpr ((MSA_ABL & 1) != 0) return;
      // pass-2 workgroup: every wave takes blocks on its own, in expected readiness order
      for (;;) {
        // (a separate, non-inlined block function keeps this loop's control flow
        // uniform: inlined, the structurizer re-entered it without the ticket)
        int t = 0;
        if (lane == 0) t = atomicAdd(a.ticket + MSA_TK_BLOCK, 1);
        t = __builtin_amdgcn_readlane(t, 0);
        if (t >= a.nblk) break;
        kargs_c* ka = (kargs_c*)__builtin_amdgcn_kernarg_segment_ptr();  // (a is the only argument)
        lds_int* wl = L(smem + w * fl_p2ints(FL_PS));
        if constexpr (GOT && R == 2) fill_block_got2<0>(ka, a.border[t], lane, wl);
        else if constexpr (GOT) fill_block_got<0>(ka, a.border[t], lane, wl);
        else if constexpr (AFF && R == 2) fill_block_aff2<0>(ka, a.border[t], lane, wl);
        else if constexpr (AFF) fill_block_aff<0>(ka, a.border[t], lane, wl);
        else fill_block<FLOOR, TRACKPOS, R, 0>(fill_args_of(ka), a.border[t], lane, wl);
      }
#ifdef MSA_STAMPS
      wg_stamp(1, __builtin_amdgcn_s_memrealtime());
#endif
      return;
    }
  }
  // pass-1 waves issue ahead of any pass-2 waves sharing their CU (long pairs: two workgroups per CU)
#ifndef FL_P1PRIO
#define FL_P1PRIO 3
#endif
  __builtin_amdgcn_s_setprio(FL_P1PRIO);

  for (;;) {
    if (threadIdx.x == 0) {
      // own chunk first, then the others': every item is claimed by a running
      // workgroup before any workgroup turns to pass-2 blocks (which wait on items)
      // (XCD gg's t-th item: run t / G of its runs, which are runs gg, gg + 8, ... of G items)
      int it = kp.n_items;
      for (int d = 0; d < 8; ++d) {
        const int gg = (grp + d) & 7;
        if (gg * chunk >= kp.n_items) continue;
        const int t = atomicAdd(a.ticket + 4 + gg, 1);
        const int x = ((t / chunk) * 8 + gg) * chunk + t % chunk;
        if (x < kp.n_items) {
          it = x;
          break;
        }
      }
      flags[0] = it;
    }
    if (threadIdx.x >= 16 && threadIdx.x < 128) flags[threadIdx.x] = 0;
    __syncthreads();
    const int item = uni(flags[0]);
#ifdef MSA_STAMPS
    if (a.stamps && threadIdx.x == 0 && blockIdx.x < 2048 && item < kp.n_items) {
      a.stamps[(((size_t)63 * 16 + 15) * 4096 + 2048 + blockIdx.x) * 4 + 1] = __builtin_amdgcn_s_memrealtime();
      a.stamps[(((size_t)63 * 16 + 15) * 4096 + 2048 + blockIdx.x) * 4 + 2] = item + 1;
    }
#endif
    if (item >= kp.n_items) break;
    const int k0 = item * W;

    if (w == W) {
      // =================== io-in: codes + the row above stripe k0 ===================
      int* ring = rings;
      int* pub = flags + 32;
      const int* cons = flags + 33;  // compute wave 0's finished phases = blocks it no longer needs
      const int cs_c = fl_cs(k0);
      const int Pc = fl_P(k0, m, n, R);
      const int Bmax = (k0 == 0) ? Pc - 1 : min(Pc - 1, fl_bmax(k0, m, n, R));
      const uint8_t* gcod = a.cod + pd.cod_off;
      int Yr = 0;  // bytes [0, Yr) of every copy's code row have been loaded into the rings
      const int nact = min(W, S - k0);  // compute waves with a stripe in this item
      // Ring slots are free below byte 16 c + FL_CRING - 32 of every copy, c = the slowest active
      // compute wave's finished phases: a wave past phase c - 1 reads (phase >= c) bytes >= cs -
      // 63 + FL_OFF - 7 + 16 c >= 16 c + 10, and loading chunk y overwrites chunk y - FL_CRING
      // (and, at ring position 0, the guard that mirrors it).
      auto code_cap = [&]() __attribute__((always_inline)) {
        if (cwhole) return 1 << 30;
        int c = 1 << 30;
#pragma unroll
        for (int w2 = 0; w2 < W; ++w2)
          if (w2 < nact) c = min(c, lds_vload(flags + 33 + w2));
        FL_CBAR();
        return 16 * uni(c) + FL_CRING - 32;
      };
      auto load_codes = [&](int Y1) __attribute__((always_inline)) {
        Y1 = min(Y1, L8);
        if (Y1 <= Yr) return;
        Y1 = min(Y1, code_cap());
        const int tot = NCP * ((Y1 - Yr) / 16);  // 16-byte chunks over all copies
        for (int c0 = 0; c0 < tot; c0 += 4 * 64) {     // 4 loads in flight per lane
          int4 v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int c = min(c0 + r * 64 + lane, tot - 1);
            const int x = c & (NCP - 1), y = Yr + 16 * (c / NCP);
            v[r] = *reinterpret_cast<const int4*>(gcod + (size_t)x * a.cod_copy + (y + MSA_CPAD - 1 - FL_OFF));
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int c = c0 + r * 64 + lane;
            const int x = c & (NCP - 1), y = Yr + 16 * (c / NCP);
            const int pos = (int)((unsigned)y & cmask);
            const fl_v4i d{v[r].x, v[r].y, v[r].z, v[r].w};
            if (c < tot) {
              *(lds_int4*)(codes + x * cstr + pos) = d;
              if (!cwhole && pos == 0) *(lds_int4*)(codes + x * cstr + FL_CRING) = d;  // the guard
            }
          }
        }
        Yr = max(Yr, Y1);
      };
      load_codes(1024);
#ifdef MSA_STAMPS
      __builtin_amdgcn_s_waitcnt(0);
      FL_STAMP(0, 0, __builtin_amdgcn_s_memrealtime());
#endif
      const unsigned long long* g_in = a.gbuf + (size_t)(item > 0 ? item - 1 : 0) * NV * a.gbuf_stride;
      int b = 0;
      int consv = 0;
      unsigned spins = 0;
      while (b <= Bmax) {
        if (Yr < L8 && Yr < 16 * b + 768) load_codes(Yr + 1024);
        // up to 16 blocks (256 columns) per round trip: lane l, load r -> block b + 4r + l/16
        int val[4], valf[4];
        int nb = 0;
        if (k0 == 0) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int col = cs_c + 16 * b + 64 * r + lane;
            val[r] = AFF ? g * col - oe : (GS ? g * col : -g);  // row 0: H = 0 (affine: Z; F~ = -inf)
            valf[r] = MSA_NEG;
            if constexpr (GOT) {  // row 0, tagged and shifted (oe = h)
              val[r] = col < 0 ? MSA_NEG : (col == 0 ? 3 : 2 - 4 * oe);
              valf[r] = col < 0 ? MSA_NEG : (col == 0 ? 3 : 2 - 4 * oe);  // D~ + 4h (pass-1 convention)
            }
          }
          nb = min(16, Bmax - b + 1);
        } else {
          unsigned long long gv[4], gf[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int col = cs_c + 16 * b + 64 * r + lane;
            const int ci = min(max(col + MSA_GOFF, 0), a.gbuf_stride - 1);
            gv[r] = gload(g_in + ci);
            if constexpr (AFF) gf[r] = gload(g_in + a.gbuf_stride + ci);
          }
          bool run = true;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            val[r] = (int)(unsigned)gv[r];
            const int blk = b + 4 * r + (lane >> 4);
            bool ok = (blk > Bmax) || ((unsigned)(gv[r] >> 32) == ep);
            if constexpr (AFF) {
              valf[r] = (int)(unsigned)gf[r];
              ok = ok && ((blk > Bmax) || ((unsigned)(gf[r] >> 32) == ep));
            }
            const unsigned long long bal = __ballot(ok);
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
              run = run && (((bal >> (16 * jj)) & 0xffffull) == 0xffffull);
              if (run) nb = 4 * r + jj + 1;
            }
          }
          nb = uni(min(nb, Bmax - b + 1));
        }
        // ring slots: block x is free once the consumer has passed x - 16
        if (consv < b + nb - FL_RINGB) consv = uni(lds_vload(cons));
        nb = min(nb, consv + FL_RINGB - b);
        if (nb <= 0) {
          if (k0 == 0 || consv + FL_RINGB <= b) __builtin_amdgcn_s_sleep(FL_IOSLEEP);  // (granule polls pace themselves)
          if (++spins > FL_SPIN_MAX) break;
          continue;
        }
        // codes for the blocks' next phases must be in LDS before they are published (a full
        // code ring -- the last compute wave far behind -- holds the blocks back)
        if (Yr < L8 && Yr < 16 * (b + nb) + 192) {
          load_codes(16 * (b + nb) + 1024);
          if (Yr < L8) nb = min(nb, (Yr - 192) / 16 - b);
          if (nb <= 0) {
            __builtin_amdgcn_s_sleep(FL_IOSLEEP);
            if (++spins > FL_SPIN_MAX) break;
            continue;
          }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int blk = b + 4 * r + (lane >> 4);
          if (blk < b + nb) {
            *L(ring + (blk & (FL_RINGB - 1)) * 16 + (lane & 15)) = val[r];
            if constexpr (AFF) *L(ring + 256 + (blk & (FL_RINGB - 1)) * 16 + (lane & 15)) = valf[r];
          }
        }
        FL_CBAR();
        if (lane == 0) lds_vstore(pub, b + nb);
        b += nb;
      }
      // (a spin limit ends the loop; reported after it: a divergent store inside a wait loop makes the
      // loop's control flow exec-mask based -- tests/test_host.py::test_wait_loops_are_wave_uniform)
      if (b <= Bmax && lane == 0) atomicExch(a.err, 10);
    } else if (w == W + 1) {
      // ============ io-out: links' blocks -> BR (pass 2), last link -> granules ============
      int bl[W + 1], bmx[W + 1];
#pragma unroll
      for (int l = 0; l <= W; ++l) {
        bl[l] = 0;
        bmx[l] = (l >= 1 && k0 + l < S && (SAVE || l == W)) ? fl_bmax(k0 + l, m, n, R) : -1;
      }
      unsigned long long* g_out = a.gbuf + (size_t)item * NV * a.gbuf_stride;
      const int S_br = (m + 64 * R - 1) / (64 * R);  // affine: F~ bottom rows follow the Z rows
      unsigned spins = 0;
      for (;;) {
        bool left = false, any = false;
#pragma unroll
        for (int l = 1; l <= W; ++l) {
          if (bl[l] > bmx[l]) continue;
          left = true;
          const int kc = k0 + l;
          const int avail = min(uni(lds_vload(flags + 32 + l)) - fl_dq(kc), bmx[l] + 1);
          FL_CBAR();
          if (avail <= bl[l]) continue;
          any = true;
          const int nb = min(4, avail - bl[l]);
          const int j = lane >> 4, c = lane & 15;
          if (j < nb) {
            const int blk = bl[l] + j;
            const int v = *(const lds_int*)(rings + l * 256 * NV + (blk & (FL_RINGB - 1)) * 16 + c);
            const int vf = AFF ? *(const lds_int*)(rings + l * 256 * NV + 256 + (blk & (FL_RINGB - 1)) * 16 + c) : 0;
            if (SAVE && (MSA_ABL & 4) == 0) {
              gstore(a.br + (size_t)(kc - 1) * a.brw + 16 * blk + c, ((unsigned long long)ep << 32) | (unsigned)v);
              if constexpr (AFF)  // (Gotoh: D~ + 4h on the links, D~ for pass 2)
                gstore(a.br + (size_t)(S_br + kc - 1) * a.brw + 16 * blk + c,
                       ((unsigned long long)ep << 32) | (unsigned)(GOT ? vf - 4 * oe : vf));
            }
            if (l == W) {
              const int col = fl_cs(kc) + 16 * blk + c;
              if (col + MSA_GOFF >= 0 && col + MSA_GOFF < a.gbuf_stride) {
                gstore(g_out + col + MSA_GOFF, ((unsigned long long)ep << 32) | (unsigned)v);
                if constexpr (AFF)
                  gstore(g_out + a.gbuf_stride + col + MSA_GOFF, ((unsigned long long)ep << 32) | (unsigned)vf);
              }
            }
          }
          bl[l] += nb;
          FL_CBAR();
          if (lane == 0) lds_vstore(flags + 64 + l, bl[l]);
        }
        if (!left) break;
        if (!any) {
          // (a longer sleep after empty rounds -- s_sleep 4 after two -- cut the polls' VALU but cost C2
          // 2.7%: 0.4691 vs 0.4565 ms; the last link's granules and BR wait on this wave)
          __builtin_amdgcn_s_sleep(FL_IOSLEEP);
          if (++spins > FL_SPIN_MAX) break;
        }
      }
      if (spins > FL_SPIN_MAX && lane == 0) atomicExch(a.err, 11);  // (after the loop, as io-in)
    } else if (k0 + w < S) {
     // (two-value kinds: affine SW and Gotoh share this wave's protocol; the one-value SW-linear
     // wave follows in the else branch)
     if constexpr (AFF) {
      // =================== compute wave (affine / Gotoh): stripe k ===================
      const int k = k0 + w;
      const int cs = fl_cs(k);
      const int P = fl_P(k, m, n, R);
      const int row_i = 64 * R * k + R * lane + 1;  // (R = 2, Gotoh: rows row_i, row_i + 1)
      const unsigned ac = (row_i <= m) ? (a.A[pd.a_off + row_i - 1] & 7u) : 0u;
      const unsigned ac2 = (R == 2 && row_i + 1 <= m) ? (a.A[pd.a_off + row_i] & 7u) : 0u;
      const bool has_out = (k < S - 1);
      const int Bin = (k == 0) ? P - 1 : min(P - 1, fl_bmax(k, m, n, R));
      const int dq_in = (w == 0) ? 0 : fl_dq(k);
      const int dq = has_out ? fl_dq(k + 1) : 0;
      const unsigned a_ring_in = lds_addr(rings + w * 512);
      const unsigned a_prog_in = lds_addr(flags + 32 + w);
      const unsigned a_ring_out = lds_addr(rings + (w + 1) * 512);
      int* const prog_me = flags + 32 + w + 1;
      const unsigned a_prog_me = lds_addr(prog_me);
      const unsigned a_cons1 = lds_addr(w + 1 < W ? flags + 32 + w + 2 : flags + 64 + W);
      const unsigned a_cons2 = lds_addr(flags + 64 + w + 1);
      unsigned plo, phi, plo2 = 0, phi2 = 0;
      if constexpr (GOT) fl_profile_got(g, ac, plo, phi);
      else fl_profile_aff(kp.match, kp.mismatch, g, oe, ac, plo, phi);
      if constexpr (R == 2 && GOT) fl_profile_got(g, ac2, plo2, phi2);
      if constexpr (R == 2 && !GOT) fl_profile_aff(kp.match, kp.mismatch, g, oe, ac2, plo2, phi2);
      // LDS code address of phase q: ring of copy x, byte (y_lane + 16 q) mod FL_CRING
      unsigned a_cring, y_code;
      {
        const int c0 = cs - lane + FL_OFF;
        const int x = c0 & (NCP - 1);
        a_cring = lds_addr(reinterpret_cast<int*>(codes + x * cstr));
        y_code = (unsigned)(c0 - x);
      }
      // step 0: lane r at column cs - r (virtual, H = 0): its left cell's Z, the diagonal Z
      // (Gotoh: Zl / E / Fo / U hold H~ / R~ / D~ / diagonal H~, the column-0 border)
      const int flr0 = g * (64 * k + 1 + cs);  // e(i+j) at step 0, every lane
      int Zl = g * (row_i + cs - lane - 1) - oe;
      int U = Zl - g;
      int E = MSA_NEG, Fo = MSA_NEG;
      const int tmin = 1 - cs + lane;  // Gotoh: the lane's first step at column >= 1
      if constexpr (GOT) {  // (E / Fo carry R~ + 4h / D~ + 4h in pass 1: see the step)
        Zl = 1 - 4 * oe;
        E = 1 - 4 * oe;
        Fo = 1;
        U = MSA_NEG;
      }
      // R = 2 (Gotoh): row 2's H~, R~ + 4h and D~ + 4h (Zl / E / U hold row 1's; row 2's diagonal is
      // row 1's previous H~, its cell above row 1's new one -- no state of their own); the next lane's
      // row 1 takes the cell above from row 2 (Zl2, Fo2) through the DPP.  Affine: row 2's Z left, E~,
      // F~ (virtual cells left of column 1: H = 0, Z = e(i+j) - oe), the lane's floor e(i+j) row 1
      int Zl2 = 1 - 4 * oe, E2 = 1 - 4 * oe, Fo2 = 1;
      const int flb = g * (128 * k + 1 + cs + lane);  // affine R = 2: e(i+j) of row 1 at step 0
      if constexpr (R == 2 && !GOT) {
        Zl2 = Zl + g;
        E2 = MSA_NEG;
        Fo2 = MSA_NEG;
      }
      int pubv = 0, consv = 0;
      unsigned spins = 0;
      fl_v4i ZA[4], FA[4], ZB[4], FB[4];
      fl_v2u CAl, CAh, CBl, CBh;
      const unsigned long long m63 = 1ull << 63;
      auto issue_reads = [&](int q, fl_v4i (&Z)[4], fl_v4i (&F)[4], fl_v2u& Cl, fl_v2u& Ch, int& pubn)
          __attribute__((always_inline)) {
        const unsigned ra = a_ring_in + (unsigned)((q & (FL_RINGB - 1)) * 64);
        pubn = ds_read_b32(a_prog_in);
        Z[0] = ds_read_b128<0>(ra);
        Z[1] = ds_read_b128<16>(ra);
        Z[2] = ds_read_b128<32>(ra);
        Z[3] = ds_read_b128<48>(ra);
        F[0] = ds_read_b128<1024>(ra);
        F[1] = ds_read_b128<1040>(ra);
        F[2] = ds_read_b128<1056>(ra);
        F[3] = ds_read_b128<1072>(ra);
        ds_read_codes16(a_cring + ((y_code + 16u * (unsigned)q) & cmask), Cl, Ch);
      };
      auto wait_flag = [&](unsigned addr, int& val, int need) __attribute__((always_inline)) {
        while (val < need) {
          int v = ds_read_b32(addr);
          lgkm_wait<0>(v);
          val = uni(v);
          if (val < need) {
            __builtin_amdgcn_s_sleep(0);
            if (++spins > FL_SPIN_MAX) break;
          }
        }
        // (reported after the loop: a divergent store inside it would make the loop's
        // values divergent, i.e. VGPRs and exec-mask branches on the hot path)
        if (val < need && lane == 0) atomicExch(a.err, 12);
      };
      auto refresh_cons = [&](int need) __attribute__((always_inline)) {
        while (consv < need) {
          int c1 = ds_read_b32(a_cons1);
          int c2 = ds_read_b32(a_cons2);
          lgkm_wait<0>(c1);
          lgkm_wait<0>(c2);
          consv = uni(min(c1, c2));
          if (consv < need) {
            __builtin_amdgcn_s_sleep(0);
            if (++spins > FL_SPIN_MAX) break;
          }
        }
        if (consv < need && lane == 0) atomicExch(a.err, 13);
      };
      auto mask_in = [&](int q, fl_v4i (&Z)[4], fl_v4i (&F)[4]) __attribute__((always_inline)) {
        if (q > Bin) {  // past the producer's last column (all > n)
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            Z[u] = fl_v4i{MSA_NEG, MSA_NEG, MSA_NEG, MSA_NEG};
            F[u] = fl_v4i{MSA_NEG, MSA_NEG, MSA_NEG, MSA_NEG};
          }
        }
      };
#ifdef MSA_STAMPS
      int nslow = 0;
#endif
      wait_flag(a_prog_in, pubv, min(1, Bin + 1) + dq_in);
      FL_STAMP(0, 0, __builtin_amdgcn_s_memrealtime());
      {
        int pub0;
        issue_reads(0, ZA, FA, CAl, CAh, pub0);
        lgkm_wait_aff<0>(ZA, FA, CAl, CAh);
        lgkm_wait<0>(pub0);
        mask_in(0, ZA, FA);
      }
      auto run_phase = [&](const int q, fl_v4i (&Z)[4], fl_v4i (&F)[4], fl_v2u& Cl, fl_v2u& Ch, fl_v4i (&Zn)[4],
                           fl_v4i (&Fn)[4], fl_v2u& Cln, fl_v2u& Chn, auto MASK_, auto HEAD_)
          __attribute__((always_inline)) {
        constexpr bool MASK = decltype(MASK_)::value;
        constexpr bool HEAD = decltype(HEAD_)::value;  // Gotoh: lanes left of column 1 hold the border
        const int need = MASK ? min(q + 1, Bin + 1) : q + 1;
        if (pubv - dq_in < need) {
#ifdef MSA_STAMPS
          ++nslow;
#endif
          wait_flag(a_prog_in, pubv, need + dq_in);
          const unsigned ra = a_ring_in + (unsigned)((q & (FL_RINGB - 1)) * 64);
          ds_reread_b128x4(ra, Z);
          ds_reread_b128x4(ra + 1024u, F);
          if constexpr (MASK) mask_in(q, Z, F);
        }
        if ((q & ((1 << a.ps_shift) - 1)) == 0) {  // pass 2 restarts here: each lane's (Z left, E~, F~, diagonal Z)
          if constexpr (R == 2) {  // rows 1 and 2: H~, R~, diagonal H~ / H~, R~, D~ (pass 2: unshifted)
            // (affine: Z left, E~, diagonal Z / Z left, E~, F~)
            constexpr int SH = GOT ? 1 : 0;
            unsigned long long* sp = a.snap + ((size_t)k * a.nseg + (q >> a.ps_shift)) * 384 + lane;
            gstore(sp, ((unsigned long long)ep << 32) | (unsigned)Zl);
            gstore(sp + 64, ((unsigned long long)ep << 32) | (unsigned)(E - SH * 4 * oe));
            gstore(sp + 128, ((unsigned long long)ep << 32) | (unsigned)U);
            gstore(sp + 192, ((unsigned long long)ep << 32) | (unsigned)Zl2);
            gstore(sp + 256, ((unsigned long long)ep << 32) | (unsigned)(E2 - SH * 4 * oe));
            gstore(sp + 320, ((unsigned long long)ep << 32) | (unsigned)(Fo2 - SH * 4 * oe));
          } else {
            unsigned long long* sp = a.snap + ((size_t)k * a.nseg + (q >> a.ps_shift)) * 256 + lane;
            gstore(sp, ((unsigned long long)ep << 32) | (unsigned)Zl);
            gstore(sp + 64, ((unsigned long long)ep << 32) | (unsigned)(GOT ? E - 4 * oe : E));  // pass 2: R~, D~
            gstore(sp + 128, ((unsigned long long)ep << 32) | (unsigned)(GOT ? Fo - 4 * oe : Fo));
            gstore(sp + 192, ((unsigned long long)ep << 32) | (unsigned)U);
          }
        }
        int xz[16], xf[16];
        int pubn = 0;
        const int flq = flr0 + 16 * g * q;
        const unsigned cw[4] = {Cl.x, Cl.y, Ch.x, Ch.y};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const unsigned s4 = __builtin_amdgcn_perm(phi, plo, cw[u]);
          const unsigned s4b = (R == 2) ? __builtin_amdgcn_perm(phi2, plo2, cw[u]) : 0u;
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) {
            const int kx = 4 * u + kk;
            if (kx == FL_PF) issue_reads(q + 1, Zn, Fn, Cln, Chn, pubn);
            const int sc = ((int)(s4 << (24 - 8 * kk))) >> 24;
            if constexpr (GOT && R == 2) {
              // row 1: the cell above is the previous lane's row 2 (lane 0: the link)
              const int uH = dpp_shr1(Z[kx >> 2][kx & 3], Zl2);
              const int uD = dpp_shr1(F[kx >> 2][kx & 3], Fo2);
              int h1, rr1, dd1;
              if (kx == 15) {  // row 1 on tag-carrying values only at a phase's last step (its hand-off)
                const int t1 = (int)((unsigned)U | 3u) + sc;
                const int t2p = (int)(((unsigned)E & ~3u) | 2u);
                const int t3p = (int)(((unsigned)uD & ~3u) | 1u);
                const int t2 = t2p - 4 * oe, t3 = t3p - 4 * oe;
                h1 = vmax3(t1, t2, t3);
                rr1 = vmax3(t1, t2p, t3);
                dd1 = vmax3(t1, t2, t3p);
              } else {
                // Pass 1 never reads a tag: every consumer of a cell re-tags it (t1 = (U | 3) + s, the
                // and-or of t2p / t3p), so row 1's candidates keep their inputs' tag bits (values are
                // 4v + tag, tag in 1..3: the maxima and every value are exact).  Row 1's tags are only
                // exported through SNAP, i.e. by a phase's last step (kx 15, tagged above); row 2 feeds
                // the hand-off (BR) at every step and stays tagged.  3 VALU per step fewer.
                const int t1 = U + sc;
                const int t2 = E - 4 * oe, t3 = uD - 4 * oe;
                h1 = vmax3(t1, t2, t3);
                rr1 = vmax3(t1, E, t3);
                dd1 = vmax3(t1, t2, uD);
              }
              asm("" : "+v"(h1));
              // row 2: diagonal = row 1's previous H~, above = row 1's new cell
              const int sb = ((int)(s4b << (24 - 8 * kk))) >> 24;
              const int s1 = (int)((unsigned)Zl | 3u) + sb;
              const int s2p = (int)(((unsigned)E2 & ~3u) | 2u);
              const int s2 = s2p - 4 * oe;
              int h2, rr2, dd2;
              if constexpr (HEAD) {
                const bool before = 16 * q + kx < tmin;
                h1 = before ? 1 - 4 * oe : h1;
                rr1 = before ? 1 - 4 * oe : rr1;
                dd1 = before ? 1 : dd1;
                const int s3p = (int)(((unsigned)dd1 & ~3u) | 1u), s3 = s3p - 4 * oe;
                h2 = vmax3(s1, s2, s3);
                rr2 = vmax3(s1, s2p, s3);
                dd2 = vmax3(s1, s2, s3p);
                h2 = before ? 1 - 4 * oe : h2;
                rr2 = before ? 1 - 4 * oe : rr2;
                dd2 = before ? 1 : dd2;
              } else {
                const int s3p = (int)(((unsigned)dd1 & ~3u) | 1u), s3 = s3p - 4 * oe;
                h2 = vmax3(s1, s2, s3);
                rr2 = vmax3(s1, s2p, s3);
                dd2 = vmax3(s1, s2, s3p);
              }
              asm("" : "+v"(h2));
              U = uH;
              Zl = h1;
              E = rr1;
              Zl2 = h2;
              E2 = rr2;
              Fo2 = dd2;
              xz[kx] = h2;
              xf[kx] = dd2;
            } else if constexpr (GOT) {
              // R~ and D~ are carried + 4h (E = R~ + 4h, Fo / F = D~ + 4h): then
              //   R~ + 4h = max3(t1, t2 + 4h, t3),  D~ + 4h = max3(t1, t2, t3 + 4h)
              // and t2 = t2' - 4h, t3 = t3' - 4h (4h keeps the tag bits): 11 VALU per step, not 12.
              // SNAP and io-out's BR copy hand pass 2 the unshifted values; granules and rings keep
              // this convention.
              const int uH = dpp_shr1(Z[kx >> 2][kx & 3], Zl);
              const int uD = dpp_shr1(F[kx >> 2][kx & 3], Fo);
              const int t1 = (int)((unsigned)U | 3u) + sc;
              const int t2p = (int)(((unsigned)E & ~3u) | 2u);
              const int t3p = (int)(((unsigned)uD & ~3u) | 1u);
              const int t2 = t2p - 4 * oe, t3 = t3p - 4 * oe;
              int h = imax3(t1, t2, t3);
              int rr = imax3(t1, t2p, t3);
              int dd = imax3(t1, t2, t3p);
              asm("" : "+v"(h));
              if constexpr (HEAD) {
                const bool before = 16 * q + kx < tmin;
                h = before ? 1 - 4 * oe : h;
                rr = before ? 1 - 4 * oe : rr;
                dd = before ? 1 : dd;
              }
              U = uH;
              Zl = h;
              E = rr;
              Fo = dd;
              xz[kx] = h;
              xf[kx] = dd;
            } else if constexpr (R == 2) {
              // affine, two rows: row 1 takes the cell above from the previous lane's row 2, row 2
              // from row 1 (Z and F~ at the same column), its diagonal from row 1's previous Z
              const int upZ = dpp_shr1(Z[kx >> 2][kx & 3], Zl2);
              const int upF = dpp_shr1(F[kx >> 2][kx & 3], Fo2);
              const int sb = ((int)(s4b << (24 - 8 * kk))) >> 24;
              const int flr1 = flb + g * (16 * q + kx);
              const int e1 = imax(E, Zl);
              const int f1 = imax(upF, upZ);
              const int d1 = (FLOOR || HEAD) ? imax(U + sc, flr1) : U + sc;
              int h1 = imax3(d1, e1, f1);
              asm("" : "+v"(h1));
              const int zprev = Zl;
              U = upZ;
              E = e1;
              Zl = h1 - oe;
              const int e2 = imax(E2, Zl2);
              const int f2 = imax(f1, Zl);
              const int d2 = (FLOOR || HEAD) ? imax(zprev + sb, flr1 + g) : zprev + sb;
              int h2 = imax3(d2, e2, f2);
              asm("" : "+v"(h2));
              E2 = e2;
              Fo2 = f2;
              Zl2 = h2 - oe;
              xz[kx] = Zl2;
              xf[kx] = f2;
            } else {
              const int upZ = dpp_shr1(Z[kx >> 2][kx & 3], Zl);
              const int upF = dpp_shr1(F[kx >> 2][kx & 3], Fo);
              const int e = imax(E, Zl);
              const int f = imax(upF, upZ);
              // the floor e(i+j) (H = 0, a local start): with scores >= 0 (!FLOOR) the diagonal
              // term of every real cell is already >= it (H~diag + s + 2e >= e(i+j)), so only the
              // head phases, where lanes still hold virtual columns left of column 1, need it
              const int d = (FLOOR || HEAD) ? imax(U + sc, flq + g * kx) : U + sc;
              int h = imax3(d, e, f);
              asm("" : "+v"(h));
              U = upZ;
              E = e;
              Fo = f;
              Zl = h - oe;
              xz[kx] = Zl;
              xf[kx] = f;
            }
          }
        }
        lgkm_wait<10>(pubn);  // the counter read (oldest of the eleven) has landed
        pubv = uni(pubn);
        lgkm_wait_aff<0>(Zn, Fn, Cln, Chn);  // phase q+1's inputs (before the hand-off writes)
        const int bq = q - dq;
        if (has_out && bq >= 0) {
          if (consv < bq - (FL_RINGB - 1)) refresh_cons(bq - (FL_RINGB - 1));
          const fl_v4i z4[4] = {{xz[0], xz[1], xz[2], xz[3]}, {xz[4], xz[5], xz[6], xz[7]},
                                {xz[8], xz[9], xz[10], xz[11]}, {xz[12], xz[13], xz[14], xz[15]}};
          const fl_v4i f4[4] = {{xf[0], xf[1], xf[2], xf[3]}, {xf[4], xf[5], xf[6], xf[7]},
                                {xf[8], xf[9], xf[10], xf[11]}, {xf[12], xf[13], xf[14], xf[15]}};
          ds_handoff_aff(m63, a_ring_out + (unsigned)((bq & (FL_RINGB - 1)) * 64), z4, f4, a_prog_me, q + 1);
        } else {
          FL_CBAR();
          if (lane == 0) lds_vstore(prog_me, q + 1);
        }
        if constexpr (MASK) mask_in(q + 1, Zn, Fn);
      };
      using T_ = std::true_type;
      using F_ = std::false_type;
      const int qa = max(0, min(P, Bin));
      int q = 0;
      bool done = false;
      if constexpr (GOT || (AFF && !FLOOR)) {
        // head: phases 0..5 (steps < 96 > every lane's tmin <= 79) hold the column-0 border
        // (affine SW without the floor: the phases that still need it)
        if (qa >= 6) {
          for (; q < 6; q += 2) {
            run_phase(q, ZA, FA, CAl, CAh, ZB, FB, CBl, CBh, F_{}, T_{});
            run_phase(q + 1, ZB, FB, CBl, CBh, ZA, FA, CAl, CAh, F_{}, T_{});
          }
        } else {  // a short stripe: every phase masked both ways
          for (; q + 1 < P; q += 2) {
            run_phase(q, ZA, FA, CAl, CAh, ZB, FB, CBl, CBh, T_{}, T_{});
            run_phase(q + 1, ZB, FB, CBl, CBh, ZA, FA, CAl, CAh, T_{}, T_{});
          }
          if (q < P) run_phase(q, ZA, FA, CAl, CAh, ZB, FB, CBl, CBh, T_{}, T_{});
          done = true;
        }
      }
      if (!done) {  // (the SW-linear wave's loop shape below)
      for (; q + 1 < qa; q += 2) {
        run_phase(q, ZA, FA, CAl, CAh, ZB, FB, CBl, CBh, F_{}, F_{});
        run_phase(q + 1, ZB, FB, CBl, CBh, ZA, FA, CAl, CAh, F_{}, F_{});
      }
      if (q < qa) {
        run_phase(q, ZA, FA, CAl, CAh, ZB, FB, CBl, CBh, F_{}, F_{});
        ++q;
        for (; q + 1 < P; q += 2) {
          run_phase(q, ZB, FB, CBl, CBh, ZA, FA, CAl, CAh, T_{}, F_{});
          run_phase(q + 1, ZA, FA, CAl, CAh, ZB, FB, CBl, CBh, T_{}, F_{});
        }
        if (q < P) run_phase(q, ZB, FB, CBl, CBh, ZA, FA, CAl, CAh, T_{}, F_{});
      } else {
        for (; q + 1 < P; q += 2) {
          run_phase(q, ZA, FA, CAl, CAh, ZB, FB, CBl, CBh, T_{}, F_{});
          run_phase(q + 1, ZB, FB, CBl, CBh, ZA, FA, CAl, CAh, T_{}, F_{});
        }
        if (q < P) run_phase(q, ZA, FA, CAl, CAh, ZB, FB, CBl, CBh, T_{}, F_{});
      }
      }
      lgkm_drain();
      FL_STAMP(0, 1, __builtin_amdgcn_s_memrealtime());
      FL_STAMP(0, 2, (unsigned long long)nslow);
      msa_stripe_meta* md = a.meta + pd.stripe0 + k;
      if (lane == 0) {
        md->cs = cs;
        md->phases = P;
      }
     } else {
      // =================== compute wave: stripe k ===================
      const int k = k0 + w;
      const int cs = fl_cs(k);
      const int P = fl_P(k, m, n, R);
      const int row_i = 64 * R * k + R * lane + 1;  // (R = 2: rows row_i, row_i + 1)
      const unsigned ac = (row_i <= m) ? (a.A[pd.a_off + row_i - 1] & 7u) : 0u;
      const unsigned ac2 = (R == 2 && row_i + 1 <= m) ? (a.A[pd.a_off + row_i] & 7u) : 0u;
      const bool has_out = (k < S - 1);
      const int Bin = (k == 0) ? P - 1 : min(P - 1, fl_bmax(k, m, n, R));
      const int dq_in = (w == 0) ? 0 : fl_dq(k);  // producer's counter counts phases (io-in: blocks)
      const int dq = has_out ? fl_dq(k + 1) : 0;  // phase q writes out block q - dq
      // LDS byte addresses (32-bit, for the inline-asm DS ops)
      const unsigned a_ring_in = lds_addr(rings + w * 256);
      const unsigned a_prog_in = lds_addr(flags + 32 + w);
      const unsigned a_ring_out = lds_addr(rings + (w + 1) * 256);
      const unsigned a_prog_me = lds_addr(flags + 32 + w + 1);
      // out-ring consumers: the next compute wave (or io-out for the last link) and io-out's BR copy
      const unsigned a_cons1 = lds_addr(w + 1 < W ? flags + 32 + w + 2 : flags + 64 + W);
      const unsigned a_cons2 = lds_addr(flags + 64 + w + 1);
      const bool two_cons = SAVE || (w + 1 == W);
      const unsigned a_dummy = lds_addr(flags + 96 + 8 * (w & 1));  // sink for a phase with nothing to hand off
      unsigned plo, phi, plo2 = 0, phi2 = 0;
      fl_profile<GS, FLOOR>(kp.match, kp.mismatch, g, ac, plo, phi);
      if constexpr (R == 2) fl_profile<GS, FLOOR>(kp.match, kp.mismatch, g, ac2, plo2, phi2);
      // LDS code address: column cs - lane + t, copy x = (cs - lane + OFF) & 7, ring byte
      // (y_lane + 16 q) mod FL_CRING in phase q
      unsigned a_cring, y_code;
      {
        const int c0 = cs - lane + FL_OFF;
        const int x = c0 & (FL_NCOPY - 1);
        a_cring = lds_addr(reinterpret_cast<int*>(codes + x * cstr));
        y_code = (unsigned)(c0 - x);
      }
      // G-space: H = G - g(i+j), i+j = 64k + 1 + cs + t for every lane of step t
      const int negct0 = -g * (64 * k + 1 + cs);
      int gk[16];
#pragma unroll
      for (int kx = 0; kx < 16; ++kx) {
        gk[kx] = -g * kx;
        if constexpr (BEST) asm("" : "+v"(gk[kx]));  // VGPR constants: H = v_add3(G, -ct_q, -g k)
      }

      // left neighbour and diagonal at step 0 (virtual cells, H = 0); R = 2: X/U row
      // row_i, X2 row row_i + 1 (its diagonal is row row_i's left neighbour, its up
      // row row_i's new value: no state of its own)
      int X = GS ? g * (64 * R * k + (R - 1) * lane + cs) : -g;
      int U = GS ? g * (64 * R * k + (R - 1) * lane + cs - 1) : -g;
      int X2 = GS ? X + g : -g;
      int best = 0;
      int pubv = 0, consv = 0;
      unsigned spins = 0;
      fl_v4i INa[4], INb[4];
      fl_v4u CWa, CWb;
      const unsigned long long m63 = 1ull << 63;

      // all LDS traffic of the loop is inline asm with hand-placed waits
      auto issue_reads = [&](int q, fl_v4i (&IN)[4], fl_v4u& CW, int& pubn) __attribute__((always_inline)) {
        const unsigned ra = a_ring_in + (unsigned)((q & (FL_RINGB - 1)) * 64);
        pubn = ds_read_b32(a_prog_in);
        IN[0] = ds_read_b128<0>(ra);
        IN[1] = ds_read_b128<16>(ra);
        IN[2] = ds_read_b128<32>(ra);
        IN[3] = ds_read_b128<48>(ra);
        CW = ds_read2_b64(a_cring + ((y_code + 16u * (unsigned)q) & cmask));
      };
      auto reread_in = [&](int q, fl_v4i (&IN)[4]) __attribute__((always_inline)) {
        ds_reread_b128x4(a_ring_in + (unsigned)((q & (FL_RINGB - 1)) * 64), IN);
      };
#ifdef MSA_STAMPS
      unsigned long long tw_in = 0, tw_cons = 0;  // s_memtime ticks in the two wait loops
      int ncons = 0;
#endif
      auto wait_flag = [&](unsigned addr, int& val, int need) __attribute__((always_inline)) {
#ifdef MSA_STAMPS
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#endif
        while (val < need) {
          int v = ds_read_b32(addr);
          lgkm_wait<0>(v);
          val = uni(v);
          if (val < need) {
            __builtin_amdgcn_s_sleep(0);
            if (++spins > FL_SPIN_MAX) break;
          }
        }
        // (reported after the loop: a divergent store inside it would make the loop's
        // values divergent, i.e. VGPRs and exec-mask branches on the hot path)
        if (val < need && lane == 0) atomicExch(a.err, 12);
#ifdef MSA_STAMPS
        tw_in += __builtin_amdgcn_s_memtime() - t0;
#endif
      };
      auto refresh_cons = [&](int need) __attribute__((always_inline)) {
#ifdef MSA_STAMPS
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
        ++ncons;
#endif
        while (consv < need) {
          int c1 = ds_read_b32(a_cons1);
          int c2 = ds_read_b32(a_cons2);
          lgkm_wait<0>(c1);
          lgkm_wait<0>(c2);
          consv = uni(two_cons ? min(c1, c2) : c1);
          if (consv < need) {
            __builtin_amdgcn_s_sleep(0);
            if (++spins > FL_SPIN_MAX) break;
          }
        }
        if (consv < need && lane == 0) atomicExch(a.err, 13);
#ifdef MSA_STAMPS
        tw_cons += __builtin_amdgcn_s_memtime() - t0;
#endif
      };
      auto mask_in = [&](int q, fl_v4i (&IN)[4]) __attribute__((always_inline)) {
        if (q > Bin) {  // past the producer's last column (all > n)
#pragma unroll
          for (int u = 0; u < 4; ++u) IN[u] = fl_v4i{MSA_NEG, MSA_NEG, MSA_NEG, MSA_NEG};
        }
      };
#ifdef MSA_STAMPS
      int nslow = 0;
#endif
      // phase 0 inputs, synchronously
      wait_flag(a_prog_in, pubv, min(1, Bin + 1) + dq_in);
      FL_STAMP(0, 0, __builtin_amdgcn_s_memrealtime());
      {
        int pub0;
        issue_reads(0, INa, CWa, pub0);
        lgkm_wait_v<0>(INa, CWa);
        lgkm_wait<0>(pub0);
        mask_in(0, INa);
      }

      auto run_phase = [&](const int q, fl_v4i (&IN)[4], fl_v4u& CW, fl_v4i (&INn)[4], fl_v4u& CWn, auto MASK_)
          __attribute__((always_inline)) {
        constexpr bool MASK = decltype(MASK_)::value;  // phase q+1 may lie past the producer's last block
        const int need = MASK ? min(q + 1, Bin + 1) : q + 1;
        if (__builtin_expect((MSA_ABL & 48) == 0 && pubv - dq_in < need, 0)) {
#ifdef MSA_STAMPS
          ++nslow;
#endif
          wait_flag(a_prog_in, pubv, need + dq_in);
          reread_in(q, IN);
          if constexpr (MASK) mask_in(q, IN);
        }
        if constexpr (SAVE && (MSA_ABL & 2) == 0) {
          if ((q & ((1 << a.ps_shift) - 1)) == 0) {  // pass 2 restarts here: each lane's left and diagonal values
            unsigned long long* sp = a.snap + ((size_t)k * a.nseg + (q >> a.ps_shift)) * (128 * R) + lane;
            gstore(sp, ((unsigned long long)ep << 32) | (unsigned)X);
            gstore(sp + 64, ((unsigned long long)ep << 32) | (unsigned)U);
            if constexpr (R == 2) gstore(sp + 128, ((unsigned long long)ep << 32) | (unsigned)X2);
          }
        }
        int hv[16];
        int xo[16];  // lane 63's values of the phase are the hand-off
        int pubn = 0;
        const int negct = negct0 - 16 * g * q;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const unsigned s4 = __builtin_amdgcn_perm(phi, plo, CW[u]);
          const unsigned s4b = (R == 2) ? __builtin_amdgcn_perm(phi2, plo2, CW[u]) : 0u;
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) {
            const int kx = 4 * u + kk;
            if (kx == FL_PF) issue_reads(q + 1, INn, CWn, pubn);  // prefetch phase q+1 (6 DS ops)
            const int s = ((int)(s4 << (24 - 8 * kk))) >> 24;
            if constexpr (R == 1) {
              const int h = fl_step<GS, FLOOR>(IN[kx >> 2][kx & 3], s, X, U, g);
              xo[kx] = X;
              if constexpr (BEST) hv[kx] = GS ? h + negct + gk[kx] : h;
            } else {
              // row 1's up = the previous lane's row 2 (lane 0: the producer's value);
              // row 2's up = row 1's new value, its diagonal = row 1's previous value
              const int sb = ((int)(s4b << (24 - 8 * kk))) >> 24;
              const int up = dpp_shr1(IN[kx >> 2][kx & 3], X2);
              int h1 = imax3(U + s, up, X);
              if constexpr (FLOOR) h1 = imax(h1, 0);
              asm("" : "+v"(h1));
              U = up;
              const int xprev = X;
              X = GS ? h1 : h1 - g;
              int h2 = imax3(xprev + sb, X, X2);
              if constexpr (FLOOR) h2 = imax(h2, 0);
              asm("" : "+v"(h2));
              X2 = GS ? h2 : h2 - g;
              xo[kx] = X2;
            }
          }
        }
        if constexpr (BEST) {
#pragma unroll
          for (int kx = 0; kx < 16; kx += 2) best = imax3(best, hv[kx], hv[kx + 1]);
        }
        lgkm_wait<5>(pubn);  // the counter read (oldest of the six) has landed
        pubv = uni(pubn);
        // hand-off: lane 63's 16 values of this phase = block q - dq of the out ring
        const int bq = q - dq;
        const bool wr = has_out && bq >= 0;
        if (__builtin_expect((MSA_ABL & 80) == 0 && wr && consv < bq - (FL_RINGB - 1), 0))
          refresh_cons(bq - (FL_RINGB - 1));
        const unsigned wa = wr ? a_ring_out + (unsigned)((bq & (FL_RINGB - 1)) * 64) : a_dummy;
        // lane 63 alone: 16 ds_write_addtid_b32 + the counter (measured 6.5% faster on C2 than four
        // single-lane b128 writes; 8 b64 writes, every-lane b128 writes into a sink and a DPP shift
        // register were slower -- DESIGN.md section 5)
        ds_handoff_tid(m63, wa - 252u, xo, a_prog_me, q + 1);
#ifdef MSA_STAMPS
        if (q == dq) FL_STAMP(0, 3, __builtin_amdgcn_s_memrealtime());
#endif
        lgkm_wait_v<5>(INn, CWn);  // phase q+1's prefetched inputs have landed (the writes may fly)
        if constexpr (MASK) mask_in(q + 1, INn);
      };
      using T_ = std::true_type;
      using F_ = std::false_type;
      // phases q < qa prefetch a block q+1 <= Bin: no masking code
      const int qa = max(0, min(P, Bin));
      int q = 0;
      for (; q + 1 < qa; q += 2) {
        run_phase(q, INa, CWa, INb, CWb, F_{});
        run_phase(q + 1, INb, CWb, INa, CWa, F_{});
      }
      if (q < qa) {
        run_phase(q, INa, CWa, INb, CWb, F_{});
        ++q;
        for (; q + 1 < P; q += 2) {
          run_phase(q, INb, CWb, INa, CWa, T_{});
          run_phase(q + 1, INa, CWa, INb, CWb, T_{});
        }
        if (q < P) run_phase(q, INb, CWb, INa, CWa, T_{});
      } else {
        for (; q + 1 < P; q += 2) {
          run_phase(q, INa, CWa, INb, CWb, T_{});
          run_phase(q + 1, INb, CWb, INa, CWa, T_{});
        }
        if (q < P) run_phase(q, INa, CWa, INb, CWb, T_{});
      }
      lgkm_drain();
      FL_STAMP(0, 1, __builtin_amdgcn_s_memrealtime());
      FL_STAMP(0, 2, (unsigned long long)nslow);
      FL_STAMP(1, 0, tw_in);
      FL_STAMP(1, 1, tw_cons);
      FL_STAMP(1, 2, (unsigned long long)ncons);
      // ---- stripe finalize ----
      msa_stripe_meta* md = a.meta + pd.stripe0 + k;
      if constexpr (BEST) {
        int bb = (row_i <= m) ? best : INT32_MIN;
        int bi = row_i;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
          const int ob = __shfl_xor(bb, off);
          const int oi = __shfl_xor(bi, off);
          if (ob > bb || (ob == bb && oi < bi)) { bb = ob; bi = oi; }
        }
        if (lane == 0) {
          md->best = bb;
          md->best_i = bi;
          md->best_j = -1;
        }
      }
      if (lane == 0) {
        md->cs = cs;
        md->phases = P;
      }
     }
    }
    __syncthreads();
  }
#ifdef MSA_STAMPS
  wg_stamp(2, 1);
  wg_stamp(1, __builtin_amdgcn_s_memrealtime());
#endif
}

// A pass-2 block's inputs are staged in its wave's LDS area (fl_p2ints(PS) ints) before the phase loop:
// the row above its PS phases, value stream k at lds + fl_p2vs(PS) k (columns [0, nv) from the bottom-row
// granules the caller loaded, row 0 for stripe 0, -inf past the producer's last block), and the column
// codes the block reads -- columns cs - 63 + 16 q0 + [0, 4 fl_p2cod(PS)), one dword per lane and round
// from an aligned staged copy -- at lds + 2 fl_p2vs(PS).  The phase loop then issues no global load: a load in flight (codes
// prefetched phases ahead) made every phase wait for the previous phases' H / direction stores too --
// one vmcnt counter for both -- i.e. ~1 us per phase.  2.3 KiB per wave: pass-2 workgroups fit beside
// a pass-1 one on a CU.
template <int NV, int PS, class ROW0>
__device__ __forceinline__ void p2_stage(lds_int* lds, int s, int nv, int ntot, int lane, ROW0 row0, const uint8_t* cod,
                                         long long cod_copy, int cs, int q0) {
  constexpr int VS = fl_p2vs(PS), COD = fl_p2cod(PS);
  const int b = cs - 63 + 16 * q0 - 1 + MSA_CPAD;  // byte of that first column in copy 0 (>= 0: CPAD 256)
  const int c = b & (MSA_NCOPY - 1);              // copy c holds it at the 16-aligned byte b - c
  unsigned w[COD / 64];
#pragma unroll
  for (int d = 0; d < COD / 64; ++d) {
    // (round 0 stays inside the copy: b + 256 <= the padded row; later rounds -- PS > 12 -- are clamped
    // to it, the dwords past the row's end are never read by a phase < P)
    const long long o = (b - c) + 4 * (64 * d + lane);
    w[d] = *reinterpret_cast<const unsigned*>(cod + (size_t)c * cod_copy + (d == 0 ? o : min(o, cod_copy - 4)));
  }
#pragma unroll
  for (int k = 0; k < NV; ++k)
    for (int v = (s == 0 ? 0 : nv) + lane; v < ntot; v += 64) *L(lds + VS * k + v) = (s == 0) ? row0(v, k) : MSA_NEG;
#pragma unroll
  for (int d = 0; d < COD / 64; ++d) *L(lds + 2 * VS + 64 * d + lane) = (int)w[d];
  FL_CBAR();  // (one wave's LDS ops execute in order: the phase loop's reads see these writes)
}
// Lane r's 16 column codes of the block's phase k (columns cs - r + 16 (q0 + k) + [0, 16)): five dwords
// of the staged span and four byte-aligns (the shift (63 - r) mod 4 is the lane's for every phase).
template <int PS>
__device__ __forceinline__ fl_v4u p2_codes(lds_int* lds, int k, int lane) {
  const int o = (63 - lane) + 16 * k;
  const lds_int* p = L(lds + 2 * fl_p2vs(PS) + (o >> 2));
  const unsigned d0 = p[0], d1 = p[1], d2 = p[2], d3 = p[3], d4 = p[4];
  const unsigned sh = (unsigned)o & 3u;
  return fl_v4u{__builtin_amdgcn_alignbyte(d1, d0, sh), __builtin_amdgcn_alignbyte(d2, d1, sh),
                __builtin_amdgcn_alignbyte(d3, d2, sh), __builtin_amdgcn_alignbyte(d4, d3, sh)};
}

// Pass 2: block (stripe s, segment seg) of PS phases, one wave.  Its inputs
// are {epoch, value} granules that pass 1 may still be writing: the wave waits
// for the block's last bottom-row granule, then loads and checks them all.
// R = 2: lane r holds rows 128s+2r+1 (X/U) and 128s+2r+2 (X2); cells go to the
// R = 2 layout (per 4 steps: the wave's row-1 int4s, then its row-2 int4s).
template <bool FLOOR, bool TRACKPOS, int R, int CALLER>
__device__ __attribute__((noinline)) void fill_block(const FillArgs a, int blk, int lane, lds_int* lds) {
  constexpr int PS = fl_ps(CALLER);
  constexpr bool GS = !FLOOR;
  const unsigned ep = a.ep;
  const int m = a.m, n = a.n, S = (m + 64 * R - 1) / (64 * R), g = a.g;
  const int s = blk / a.nseg, seg = blk - s * a.nseg;
  int bb = INT32_MIN, bi = 0, bj = 0;
  if (s < S) {
    const int P = fl_P(s, m, n, R);
    const int q0 = seg * PS;
    if (q0 < P) {
      int q1 = min(P, q0 + PS);
      const int cs = fl_cs(s);
      const int row_i = 64 * R * s + R * lane + 1;
      const unsigned ac = (row_i <= m) ? (a.A[a.a_off + row_i - 1] & 7u) : 0u;
      const unsigned ac2 = (R == 2 && row_i + 1 <= m) ? (a.A[a.a_off + row_i] & 7u) : 0u;
      unsigned plo, phi, plo2 = 0, phi2 = 0;
      fl_profile<GS, FLOOR>(a.match, a.mismatch, g, ac, plo, phi);
      if constexpr (R == 2) fl_profile<GS, FLOOR>(a.match, a.mismatch, g, ac2, plo2, phi2);
      const int Bin = (s == 0) ? P - 1 : min(P - 1, fl_bmax(s, m, n, R));
      const unsigned long long* sp = a.snap + ((size_t)s * a.nseg + seg) * (128 * R) + lane;
      const unsigned long long* brow = a.br + (size_t)(s > 0 ? s - 1 : 0) * a.brw;
      // bottom-row blocks [q0, qb) of the row above come from pass 1 (s > 0)
      const int qb = (s > 0) ? min(q1, Bin + 1) : q0;
      const int nv = 16 * max(0, qb - q0);  // granules, lane l holds l, l+64, ...
      int X = 0, U = 0, X2 = 0;
      // uniform waits (ballots) and no early exits: the compiler keeps the wave whole
      bool ready = (nv == 0);
      for (int t2 = 0; !ready && t2 < (int)(FL_SPIN_MAX >> 2); ++t2) {  // the block's last granule first
        const unsigned long long gl = gload(brow + 16 * q0 + nv - 1);
        ready = __ballot((unsigned)(gl >> 32) != ep) == 0;
        if (!ready) __builtin_amdgcn_s_sleep(FL_FSLEEP);
      }
      if (ready) {
        ready = false;
        for (int tries = 0; !ready && tries < (int)FL_SPIN_MAX; ++tries) {
          const unsigned long long x0 = gload(sp), u0 = gload(sp + 64);
          bool ok = ((unsigned)(x0 >> 32) == ep) && ((unsigned)(u0 >> 32) == ep);
          X = (int)(unsigned)x0;
          U = (int)(unsigned)u0;
          if constexpr (R == 2) {
            const unsigned long long x2 = gload(sp + 128);
            ok = ok && ((unsigned)(x2 >> 32) == ep);
            X2 = (int)(unsigned)x2;
          }
          for (int v = lane; v < nv; v += 64) {
            const unsigned long long gv = gload(brow + 16 * q0 + v);
            ok = ok && ((unsigned)(gv >> 32) == ep);
            *L(lds + v) = (int)(unsigned)gv;
          }
          ready = __ballot(!ok) == 0;
          if (!ready) __builtin_amdgcn_s_sleep(8);
        }
      }
      if (!ready) {
        if (lane == 0) atomicExch(a.err, 15);
        q1 = q0;  // nothing computed; the block reports no cell
      }
      // row 0 (stripe 0): H = 0 left of and on the top border
      p2_stage<1, PS>(lds, s, nv, 16 * (q1 - q0), lane,
                  [&](int v, int) { return GS ? g * (cs + 16 * q0 + v) : -g; }, a.cod + a.cod_off, a.cod_copy, cs, q0);
      // H = G - g(i+j); i+j = 64Rs + 1 + cs + t + (R-1) lane on row 1, +1 on row 2
      const int negct0 = -g * (64 * R * s + 1 + cs + (R - 1) * lane);
      int gk[16];
#pragma unroll
      for (int kx = 0; kx < 16; ++kx) {
        gk[kx] = -g * kx;
        asm("" : "+v"(gk[kx]));
      }
      int best = INT32_MIN, bt = -1, best2 = INT32_MIN, bt2 = -1;
      msa_v4i* hp = reinterpret_cast<msa_v4i*>(a.outH + (size_t)a.out_off + (size_t)s * a.pmax * MSA_K * 64 * R) + lane;
      for (int q = q0; q < q1; ++q) {
        int IN[16];
        {
          const lds_int4* src = reinterpret_cast<const lds_int4*>(L(lds + 16 * (q - q0)));
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const fl_v4i v = src[u];
            IN[4 * u] = v.x; IN[4 * u + 1] = v.y; IN[4 * u + 2] = v.z; IN[4 * u + 3] = v.w;
          }
        }
        const fl_v4u c4 = p2_codes<PS>(lds, q - q0, lane);
        const unsigned cw[4] = {c4.x, c4.y, c4.z, c4.w};
        const int negct = negct0 - 16 * g * q;
        int hv[16], hv2[16];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const unsigned s4 = __builtin_amdgcn_perm(phi, plo, cw[u]);
          const unsigned s4b = (R == 2) ? __builtin_amdgcn_perm(phi2, plo2, cw[u]) : 0u;
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) {
            const int kx = 4 * u + kk;
            const int sc = ((int)(s4 << (24 - 8 * kk))) >> 24;
            if constexpr (R == 1) {
              const int h = fl_step<GS, FLOOR>(IN[kx], sc, X, U, g);
              hv[kx] = GS ? h + negct + gk[kx] : h;
            } else {
              const int sb = ((int)(s4b << (24 - 8 * kk))) >> 24;
              const int up = dpp_shr1(IN[kx], X2);
              int h1 = imax3(U + sc, up, X);
              if constexpr (FLOOR) h1 = imax(h1, 0);
              asm("" : "+v"(h1));
              U = up;
              const int xprev = X;
              X = GS ? h1 : h1 - g;
              int h2 = imax3(xprev + sb, X, X2);
              if constexpr (FLOOR) h2 = imax(h2, 0);
              asm("" : "+v"(h2));
              X2 = GS ? h2 : h2 - g;
              hv[kx] = GS ? h1 + negct + gk[kx] : h1;
              hv2[kx] = GS ? h2 + negct + gk[kx] - g : h2;
            }
            if constexpr (TRACKPOS) {
              if (hv[kx] > best) { best = hv[kx]; bt = 16 * q + kx; }
              if (R == 2 && hv2[kx] > best2) { best2 = hv2[kx]; bt2 = 16 * q + kx; }
            }
          }
          __builtin_nontemporal_store(msa_v4i{hv[4 * u], hv[4 * u + 1], hv[4 * u + 2], hv[4 * u + 3]},
                                      hp + (size_t)(4 * q + u) * 64 * R);
          if constexpr (R == 2)  // (each store: one contiguous 1 KiB)
            __builtin_nontemporal_store(msa_v4i{hv2[4 * u], hv2[4 * u + 1], hv2[4 * u + 2], hv2[4 * u + 3]},
                                        hp + (size_t)(4 * q + u) * 128 + 64);
        }
        if constexpr (!TRACKPOS) {
#pragma unroll
          for (int kx = 0; kx < 16; kx += 2) best = imax3(best, hv[kx], hv[kx + 1]);
          if constexpr (R == 2) {
#pragma unroll
            for (int kx = 0; kx < 16; kx += 2) best2 = imax3(best2, hv2[kx], hv2[kx + 1]);
          }
        }
      }
      bb = (row_i <= m) ? best : INT32_MIN;
      bi = row_i;
      bj = TRACKPOS ? cs + bt - lane : -1;
      if (R == 2 && row_i + 1 <= m && best2 > bb) {  // ties keep the upper row
        bb = best2;
        bi = row_i + 1;
        bj = TRACKPOS ? cs + bt2 - lane : -1;
      }
    }
  }
  // first max in row-major order: max score, then min row, then min column
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const int ob = __shfl_xor(bb, off), oi = __shfl_xor(bi, off), oj = __shfl_xor(bj, off);
    if (ob > bb || (ob == bb && (oi < bi || (oi == bi && oj < bj)))) { bb = ob; bi = oi; bj = oj; }
  }
  fl_block_result(a.blk, a.best_key, blk, lane, bb, bi, bj, a.n);
}

// Pass 2, affine (config C5): block (stripe s, segment seg) recomputes its PS phases from
// SNAP (Z left, E~, F~, diagonal Z per lane) and the stripe above's bottom row (Z and F~
// granules), writes the direction bytes in the skewed stripe layout -- lane r's 16 bytes of a
// phase are one 16-byte store, a wave's phase one contiguous 1 KiB -- and reduces its first
// maximum H = H~ - e(i+j).  The bytes are stripe_kernel's MSA_ALG_SWA bytes (the walk
// traceback_kernel<TB_SW> reads them unchanged).
template <int CALLER>
__device__ __attribute__((noinline)) void fill_block_aff(kargs_c* ka, int blk, int lane, lds_int* lds) {
  constexpr int PS = fl_ps(CALLER);
  const FillArgs a = fill_args_of(ka);
  const unsigned ep = a.ep;
  const int m = a.m, n = a.n, S = (m + 63) / 64, g = a.g, oe = a.oe;
  const int s = blk / a.nseg, seg = blk - s * a.nseg;
  int bb = INT32_MIN, bi = 0, bj = 0;
  if (s < S) {
    const int P = fl_P(s, m, n, 1);
    const int q0 = seg * PS;
    if (q0 < P) {
      int q1 = min(P, q0 + PS);
      const int cs = fl_cs(s);
      const int row_i = 64 * s + lane + 1;
      const unsigned ac = (row_i <= m) ? (a.A[a.a_off + row_i - 1] & 7u) : 0u;
      unsigned plo, phi;
      fl_profile_aff(a.match, a.mismatch, g, oe, ac, plo, phi);
      const int Bin = (s == 0) ? P - 1 : min(P - 1, fl_bmax(s, m, n, 1));
      const unsigned long long* sp = a.snap + ((size_t)s * a.nseg + seg) * 256 + lane;
      const unsigned long long* brz = a.br + (size_t)(s > 0 ? s - 1 : 0) * a.brw;
      const unsigned long long* brf = a.br + (size_t)(S + (s > 0 ? s - 1 : 0)) * a.brw;
      const int qb = (s > 0) ? min(q1, Bin + 1) : q0;
      const int nv = 16 * max(0, qb - q0);  // granules per value, lane l holds l, l+64, ...
      int Zl = 0, E = 0, Fo = 0, U = 0;
      bool ready = (nv == 0);
      for (int t2 = 0; !ready && t2 < (int)(FL_SPIN_MAX >> 2); ++t2) {  // the block's last granules first
        const unsigned long long gz = gload(brz + 16 * q0 + nv - 1), gf = gload(brf + 16 * q0 + nv - 1);
        ready = __ballot((unsigned)(gz >> 32) != ep || (unsigned)(gf >> 32) != ep) == 0;
        if (!ready) fl_poll_sleep(t2);
      }
      if (ready) {
        ready = false;
        for (int tries = 0; !ready && tries < (int)FL_SPIN_MAX; ++tries) {
          const unsigned long long x0 = gload(sp), x1 = gload(sp + 64), x2 = gload(sp + 128), x3 = gload(sp + 192);
          bool ok = ((unsigned)(x0 >> 32) == ep) && ((unsigned)(x1 >> 32) == ep) && ((unsigned)(x2 >> 32) == ep) &&
                    ((unsigned)(x3 >> 32) == ep);
          Zl = (int)(unsigned)x0;
          E = (int)(unsigned)x1;
          Fo = (int)(unsigned)x2;
          U = (int)(unsigned)x3;
          for (int v = lane; v < nv; v += 64) {
            const unsigned long long gz = gload(brz + 16 * q0 + v), gf = gload(brf + 16 * q0 + v);
            ok = ok && ((unsigned)(gz >> 32) == ep) && ((unsigned)(gf >> 32) == ep);
            *L(lds + v) = (int)(unsigned)gz;
            *L(lds + fl_p2vs(PS) + v) = (int)(unsigned)gf;
          }
          ready = __ballot(!ok) == 0;
          if (!ready) __builtin_amdgcn_s_sleep(8);
        }
      }
      if (!ready) {
        if (lane == 0) atomicExch(a.err, 15);
        q1 = q0;
      }
      // row 0 (stripe 0): Z = g col - oe (H = 0), F~ = -inf
      p2_stage<2, PS>(lds, s, nv, 16 * (q1 - q0), lane,
                  [&](int v, int k) { return k == 0 ? g * (cs + 16 * q0 + v) - oe : MSA_NEG; }, a.cod + a.cod_off,
                  a.cod_copy, cs, q0);
      const int flr0 = g * (64 * s + 1 + cs);
      int best = INT32_MIN, bt = -1;
      fl_v4u* dp = reinterpret_cast<fl_v4u*>(a.outDir + (size_t)a.out_off + (size_t)s * a.pmax * 1024) + lane;
      for (int q = q0; q < q1; ++q) {
        int INZ[16], INF[16];
        {
          const lds_int4* srz = reinterpret_cast<const lds_int4*>(L(lds + 16 * (q - q0)));
          const lds_int4* srf = reinterpret_cast<const lds_int4*>(L(lds + fl_p2vs(PS) + 16 * (q - q0)));
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const fl_v4i vz = srz[u], vf = srf[u];
            INZ[4 * u] = vz.x; INZ[4 * u + 1] = vz.y; INZ[4 * u + 2] = vz.z; INZ[4 * u + 3] = vz.w;
            INF[4 * u] = vf.x; INF[4 * u + 1] = vf.y; INF[4 * u + 2] = vf.z; INF[4 * u + 3] = vf.w;
          }
        }
        const fl_v4u c4 = p2_codes<PS>(lds, q - q0, lane);
        const unsigned cw[4] = {c4.x, c4.y, c4.z, c4.w};
        const int flq = flr0 + 16 * g * q;
        unsigned dw[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const unsigned s4 = __builtin_amdgcn_perm(phi, plo, cw[u]);
          unsigned word = 0;
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) {
            const int kx = 4 * u + kk;
            const int sc = ((int)(s4 << (24 - 8 * kk))) >> 24;
            const int flr = flq + g * kx;
            const int upZ = dpp_shr1(INZ[kx], Zl);
            const int upF = dpp_shr1(INF[kx], Fo);
            const int e = imax(E, Zl);
            const int f = imax(upF, upZ);
            const int draw = U + sc;
            int h = imax3(imax(draw, flr), e, f);
            asm("" : "+v"(h));
            // stripe_kernel's SWA byte: H's source (0 local start, 1 diagonal, 2 E, 3 F), bit 2
            // E opened from H(i, j-1), bit 3 F opened from H(i-1, j)
            const unsigned hs = (h == flr) ? 0u : (h == draw ? 1u : (h == e ? 2u : 3u));
            const unsigned dir = hs | ((e == Zl) ? 4u : 0u) | ((f == upZ) ? 8u : 0u);
            word |= dir << (8 * kk);
            const int hv = h - flr;
            if (hv > best) { best = hv; bt = 16 * q + kx; }
            U = upZ;
            E = e;
            Fo = f;
            Zl = h - oe;
          }
          dw[u] = word;
        }
        __builtin_nontemporal_store(fl_v4u{dw[0], dw[1], dw[2], dw[3]}, dp + (size_t)q * 64);
      }
      bb = (row_i <= m) ? best : INT32_MIN;
      bi = row_i;
      bj = cs + bt - lane;
    }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const int ob = __shfl_xor(bb, off), oi = __shfl_xor(bi, off), oj = __shfl_xor(bj, off);
    if (ob > bb || (ob == bb && (oi < bi || (oi == bi && oj < bj)))) { bb = ob; bi = oi; bj = oj; }
  }
  fl_block_result(a.blk, a.best_key, blk, lane, bb, bi, bj, a.n);
}

// Pass 2, affine, two rows per lane (R = 2: 128-row stripes, lane r holds rows 128s+2r+1 and
// 128s+2r+2 at column cs + t - r): as fill_block_aff, both rows per step -- row 1 takes the cell
// above (Z, F~) from the previous lane's row 2 (lane 0: the stripe above's bottom row), row 2 from
// row 1 at the same column and its diagonal from row 1's previous Z.  A phase's bytes go out as
// one 2 KiB block (row-1 segments, then row-2 segments: traceback_kernel<TB_SW, 2>'s layout).
template <int CALLER>
__device__ __attribute__((noinline)) void fill_block_aff2(kargs_c* ka, int blk, int lane, lds_int* lds) {
  constexpr int PS = fl_ps(CALLER);
  const FillArgs a = fill_args_of(ka);
  const unsigned ep = a.ep;
  const int m = a.m, n = a.n, S = (m + 127) / 128, g = a.g, oe = a.oe;
  const int s = blk / a.nseg, seg = blk - s * a.nseg;
  int bb = INT32_MIN, bi = 0, bj = 0;
  if (s < S) {
    const int P = fl_P(s, m, n, 2);
    const int q0 = seg * PS;
    if (q0 < P) {
      int q1 = min(P, q0 + PS);
      const int cs = fl_cs(s);
      const int row_i = 128 * s + 2 * lane + 1;
      const unsigned ac = (row_i <= m) ? (a.A[a.a_off + row_i - 1] & 7u) : 0u;
      const unsigned ac2 = (row_i + 1 <= m) ? (a.A[a.a_off + row_i] & 7u) : 0u;
      unsigned plo, phi, plo2, phi2;
      fl_profile_aff(a.match, a.mismatch, g, oe, ac, plo, phi);
      fl_profile_aff(a.match, a.mismatch, g, oe, ac2, plo2, phi2);
      const int Bin = (s == 0) ? P - 1 : min(P - 1, fl_bmax(s, m, n, 2));
      const unsigned long long* sp = a.snap + ((size_t)s * a.nseg + seg) * 384 + lane;
      const unsigned long long* brz = a.br + (size_t)(s > 0 ? s - 1 : 0) * a.brw;
      const unsigned long long* brf = a.br + (size_t)(S + (s > 0 ? s - 1 : 0)) * a.brw;
      const int qb = (s > 0) ? min(q1, Bin + 1) : q0;
      const int nv = 16 * max(0, qb - q0);
      int Zl = 0, E = 0, U = 0, Zl2 = 0, E2 = 0, Fo2 = 0;
      bool ready = (nv == 0);
      for (int t2 = 0; !ready && t2 < (int)(FL_SPIN_MAX >> 2); ++t2) {
        const unsigned long long gz = gload(brz + 16 * q0 + nv - 1), gf = gload(brf + 16 * q0 + nv - 1);
        ready = __ballot((unsigned)(gz >> 32) != ep || (unsigned)(gf >> 32) != ep) == 0;
        if (!ready) fl_poll_sleep(t2);
      }
      if (ready) {
        ready = false;
        for (int tries = 0; !ready && tries < (int)FL_SPIN_MAX; ++tries) {
          const unsigned long long x0 = gload(sp), x1 = gload(sp + 64), x2 = gload(sp + 128), x3 = gload(sp + 192),
                                   x4 = gload(sp + 256), x5 = gload(sp + 320);
          bool ok = ((unsigned)(x0 >> 32) == ep) && ((unsigned)(x1 >> 32) == ep) && ((unsigned)(x2 >> 32) == ep) &&
                    ((unsigned)(x3 >> 32) == ep) && ((unsigned)(x4 >> 32) == ep) && ((unsigned)(x5 >> 32) == ep);
          Zl = (int)(unsigned)x0;
          E = (int)(unsigned)x1;
          U = (int)(unsigned)x2;
          Zl2 = (int)(unsigned)x3;
          E2 = (int)(unsigned)x4;
          Fo2 = (int)(unsigned)x5;
          for (int v = lane; v < nv; v += 64) {
            const unsigned long long gz = gload(brz + 16 * q0 + v), gf = gload(brf + 16 * q0 + v);
            ok = ok && ((unsigned)(gz >> 32) == ep) && ((unsigned)(gf >> 32) == ep);
            *L(lds + v) = (int)(unsigned)gz;
            *L(lds + fl_p2vs(PS) + v) = (int)(unsigned)gf;
          }
          ready = __ballot(!ok) == 0;
          if (!ready) __builtin_amdgcn_s_sleep(8);
        }
      }
      if (!ready) {
        if (lane == 0) atomicExch(a.err, 15);
        q1 = q0;
      }
      // row 0 (stripe 0): Z = g col - oe (H = 0), F~ = -inf
      p2_stage<2, PS>(lds, s, nv, 16 * (q1 - q0), lane,
                  [&](int v, int k) { return k == 0 ? g * (cs + 16 * q0 + v) - oe : MSA_NEG; }, a.cod + a.cod_off,
                  a.cod_copy, cs, q0);
      const int flb = g * (128 * s + 1 + cs + lane);  // e(i+j) of row 1 at step 0 (row 2: + g)
      int best = INT32_MIN, bt = -1, best2 = INT32_MIN, bt2 = -1;
      fl_v4u* dp = reinterpret_cast<fl_v4u*>(a.outDir + (size_t)a.out_off + (size_t)s * a.pmax * 2048) + lane;
      for (int q = q0; q < q1; ++q) {
        int INZ[16], INF[16];
        {
          const lds_int4* srz = reinterpret_cast<const lds_int4*>(L(lds + 16 * (q - q0)));
          const lds_int4* srf = reinterpret_cast<const lds_int4*>(L(lds + fl_p2vs(PS) + 16 * (q - q0)));
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const fl_v4i vz = srz[u], vf = srf[u];
            INZ[4 * u] = vz.x; INZ[4 * u + 1] = vz.y; INZ[4 * u + 2] = vz.z; INZ[4 * u + 3] = vz.w;
            INF[4 * u] = vf.x; INF[4 * u + 1] = vf.y; INF[4 * u + 2] = vf.z; INF[4 * u + 3] = vf.w;
          }
        }
        const fl_v4u c4 = p2_codes<PS>(lds, q - q0, lane);
        const unsigned cw[4] = {c4.x, c4.y, c4.z, c4.w};
        const int flq = flb + 16 * g * q;
        unsigned dw1[4], dw2[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const unsigned s4 = __builtin_amdgcn_perm(phi, plo, cw[u]);
          const unsigned s4b = __builtin_amdgcn_perm(phi2, plo2, cw[u]);
          unsigned word1 = 0, word2 = 0;
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) {
            const int kx = 4 * u + kk;
            const int sc = ((int)(s4 << (24 - 8 * kk))) >> 24;
            const int sb = ((int)(s4b << (24 - 8 * kk))) >> 24;
            const int flr = flq + g * kx, flr2 = flr + g;
            // row 1
            const int upZ = dpp_shr1(INZ[kx], Zl2);
            const int upF = dpp_shr1(INF[kx], Fo2);
            const int e1 = imax(E, Zl);
            const int f1 = imax(upF, upZ);
            const int d1 = U + sc;
            int h1 = imax3(imax(d1, flr), e1, f1);
            asm("" : "+v"(h1));
            const unsigned hs1 = (h1 == flr) ? 0u : (h1 == d1 ? 1u : (h1 == e1 ? 2u : 3u));
            word1 |= (hs1 | ((e1 == Zl) ? 4u : 0u) | ((f1 == upZ) ? 8u : 0u)) << (8 * kk);
            if (h1 - flr > best) { best = h1 - flr; bt = 16 * q + kx; }
            const int zprev = Zl;
            U = upZ;
            E = e1;
            Zl = h1 - oe;
            // row 2: diagonal = row 1's previous Z, above = row 1's new cell
            const int e2 = imax(E2, Zl2);
            const int f2 = imax(f1, Zl);
            const int d2 = zprev + sb;
            int h2 = imax3(imax(d2, flr2), e2, f2);
            asm("" : "+v"(h2));
            const unsigned hs2 = (h2 == flr2) ? 0u : (h2 == d2 ? 1u : (h2 == e2 ? 2u : 3u));
            word2 |= (hs2 | ((e2 == Zl2) ? 4u : 0u) | ((f2 == Zl) ? 8u : 0u)) << (8 * kk);
            if (h2 - flr2 > best2) { best2 = h2 - flr2; bt2 = 16 * q + kx; }
            E2 = e2;
            Fo2 = f2;
            Zl2 = h2 - oe;
          }
          dw1[u] = word1;
          dw2[u] = word2;
        }
        if constexpr ((MSA_ABL & 8) == 0) {
          __builtin_nontemporal_store(fl_v4u{dw1[0], dw1[1], dw1[2], dw1[3]}, dp + (size_t)q * 128);
          __builtin_nontemporal_store(fl_v4u{dw2[0], dw2[1], dw2[2], dw2[3]}, dp + (size_t)q * 128 + 64);
        }
      }
      bb = (row_i <= m) ? best : INT32_MIN;
      bi = row_i;
      bj = cs + bt - lane;
      if (row_i + 1 <= m && best2 > bb) {  // ties keep the upper row
        bb = best2;
        bi = row_i + 1;
        bj = cs + bt2 - lane;
      }
    }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const int ob = __shfl_xor(bb, off), oi = __shfl_xor(bi, off), oj = __shfl_xor(bj, off);
    if (ob > bb || (ob == bb && (oi < bi || (oi == bi && oj < bj)))) { bb = ob; bi = oi; bj = oj; }
  }
  fl_block_result(a.blk, a.best_key, blk, lane, bb, bi, bj, a.n);
}

// Pass 2, Gotoh (the reference's main_alignment_function path): block (stripe s, segment
// seg) recomputes its PS phases from SNAP (H~, R~, D~, diagonal H~ per lane) and the
// stripe above's bottom row (H~ and D~ granules) and writes the tag bytes (T1's, T2's, T3's
// predecessor: the diagonal H~'s, the left R~'s and the upper D~'s tag) in the skewed stripe
// layout.  The block holding cell (m, n) stores its three tables, unshifted, as the last
// stripe's final state (reduce_pairs_kernel turns it into the pair result, the walk reads
// find_alignment's end rule from it).
template <int CALLER>
__device__ __attribute__((noinline)) void fill_block_got(kargs_c* ka, int blk, int lane, lds_int* lds) {
  constexpr int PS = fl_ps(CALLER);
  const FillArgs a = fill_args_of(ka);
  const unsigned ep = a.ep;
  const int m = a.m, n = a.n, S = (m + 63) / 64, g = a.g, h4 = 4 * a.oe;
  const int s = blk / a.nseg, seg = blk - s * a.nseg;
  if (s < S) {
    const int P = fl_P(s, m, n, 1);
    const int q0 = seg * PS;
    if (q0 < P) {
      int q1 = min(P, q0 + PS);
      const int cs = fl_cs(s);
      const int row_i = 64 * s + lane + 1;
      const unsigned ac = (row_i <= m) ? (a.A[a.a_off + row_i - 1] & 7u) : 0u;
      unsigned plo, phi;
      fl_profile_got(g, ac, plo, phi);
      const int Bin = (s == 0) ? P - 1 : min(P - 1, fl_bmax(s, m, n, 1));
      const unsigned long long* sp = a.snap + ((size_t)s * a.nseg + seg) * 256 + lane;
      const unsigned long long* brz = a.br + (size_t)(s > 0 ? s - 1 : 0) * a.brw;
      const unsigned long long* brf = a.br + (size_t)(S + (s > 0 ? s - 1 : 0)) * a.brw;
      const int qb = (s > 0) ? min(q1, Bin + 1) : q0;
      const int nv = 16 * max(0, qb - q0);
      int Hs = 0, Rs = 0, Ds = 0, U = 0;
#ifdef MSA_STAMPS
      const unsigned long long tp0 = __builtin_amdgcn_s_memtime();
      unsigned long long tp1 = tp0;
#endif
      bool ready = (nv == 0);
      for (int t2 = 0; !ready && t2 < (int)(FL_SPIN_MAX >> 2); ++t2) {
        const unsigned long long gz = gload(brz + 16 * q0 + nv - 1), gf = gload(brf + 16 * q0 + nv - 1);
        ready = __ballot((unsigned)(gz >> 32) != ep || (unsigned)(gf >> 32) != ep) == 0;
        if (!ready) fl_poll_sleep(t2);
      }
#ifdef MSA_STAMPS
      tp1 = __builtin_amdgcn_s_memtime();
#endif
      if (ready) {
        ready = false;
        for (int tries = 0; !ready && tries < (int)FL_SPIN_MAX; ++tries) {
          const unsigned long long x0 = gload(sp), x1 = gload(sp + 64), x2 = gload(sp + 128), x3 = gload(sp + 192);
          bool ok = ((unsigned)(x0 >> 32) == ep) && ((unsigned)(x1 >> 32) == ep) && ((unsigned)(x2 >> 32) == ep) &&
                    ((unsigned)(x3 >> 32) == ep);
          Hs = (int)(unsigned)x0;
          Rs = (int)(unsigned)x1;
          Ds = (int)(unsigned)x2;
          U = (int)(unsigned)x3;
          for (int v = lane; v < nv; v += 64) {
            const unsigned long long gz = gload(brz + 16 * q0 + v), gf = gload(brf + 16 * q0 + v);
            ok = ok && ((unsigned)(gz >> 32) == ep) && ((unsigned)(gf >> 32) == ep);
            *L(lds + v) = (int)(unsigned)gz;
            *L(lds + fl_p2vs(PS) + v) = (int)(unsigned)gf;
          }
          ready = __ballot(!ok) == 0;
          if (!ready) __builtin_amdgcn_s_sleep(8);
        }
      }
      if (!ready) {
        if (lane == 0) atomicExch(a.err, 15);
        q1 = q0;
      }
      // row 0 (stripe 0), tagged and shifted: H~ 3 at column 0, 2 - 4h right of it; D~ 3 - 4h, 2 - 8h
      p2_stage<2, PS>(lds, s, nv, 16 * (q1 - q0), lane,
                  [&](int v, int k) {
                    const int col = cs + 16 * q0 + v;
                    return col < 0 ? MSA_NEG : (k == 0 ? (col == 0 ? 3 : 2 - h4) : (col == 0 ? 3 - h4 : 2 - 2 * h4));
                  },
                  a.cod + a.cod_off, a.cod_copy, cs, q0);
#ifdef MSA_STAMPS
      const unsigned long long tp2 = __builtin_amdgcn_s_memtime();
#endif
      const int tmin = 1 - cs + lane;
      // the final cell (m, n): the lane of row m at step n - cs + lane of the last stripe
      const int tf = (row_i == m) ? n - cs + lane : -1;
      fl_v4u* dp = reinterpret_cast<fl_v4u*>(a.outDir + (size_t)a.out_off + (size_t)s * a.pmax * 1024) + lane;
      auto phase = [&](const int q, auto HEAD_, auto CAP_) __attribute__((always_inline)) {
        constexpr bool HEAD = decltype(HEAD_)::value;  // lanes left of column 1 hold the border
        constexpr bool CAP = decltype(CAP_)::value;    // the phase holds cell (m, n)
        int INZ[16], INF[16];
        {
          const lds_int4* srz = reinterpret_cast<const lds_int4*>(L(lds + 16 * (q - q0)));
          const lds_int4* srf = reinterpret_cast<const lds_int4*>(L(lds + fl_p2vs(PS) + 16 * (q - q0)));
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const fl_v4i vz = srz[u], vf = srf[u];
            INZ[4 * u] = vz.x; INZ[4 * u + 1] = vz.y; INZ[4 * u + 2] = vz.z; INZ[4 * u + 3] = vz.w;
            INF[4 * u] = vf.x; INF[4 * u + 1] = vf.y; INF[4 * u + 2] = vf.z; INF[4 * u + 3] = vf.w;
          }
        }
        const fl_v4u c4 = p2_codes<PS>(lds, q - q0, lane);
        const unsigned cw[4] = {c4.x, c4.y, c4.z, c4.w};
        unsigned dw[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const unsigned s4 = __builtin_amdgcn_perm(phi, plo, cw[u]);
          unsigned word = 0;
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) {
            const int kx = 4 * u + kk;
            const int sc = ((int)(s4 << (24 - 8 * kk))) >> 24;
            const int uH = dpp_shr1(INZ[kx], Hs);
            const int uD = dpp_shr1(INF[kx], Ds);
            const int t1 = (int)((unsigned)U | 3u) + sc;
            const int t2 = (int)(((unsigned)Rs & ~3u) | 2u);
            const int t3 = (int)(((unsigned)uD & ~3u) | 1u);
            const unsigned dir = ((unsigned)U & 3u) | (((unsigned)Rs & 3u) << 2) | (((unsigned)uD & 3u) << 4);
            word |= dir << (8 * kk);
            const int t1h = t1 - h4;
            int hh = imax3(t1, t2, t3);
            int rr = imax3(t1h, t2, t3 - h4);
            int dd = imax3(t1h, t2 - h4, t3);
            asm("" : "+v"(hh));
            if constexpr (HEAD) {
              const bool before = 16 * q + kx < tmin;
              hh = before ? 1 - h4 : hh;
              rr = before ? 1 - 2 * h4 : rr;
              dd = before ? 1 - h4 : dd;
            }
            if constexpr (CAP) {
              if (16 * q + kx == tf) {
                const int gmn = g * (m + n);  // unshift
                msa_stripe_meta* md = a.meta + a.stripe0 + S - 1;
                md->fin[0] = (t1 >> 2) - gmn;
                md->fin[1] = (t2 >> 2) - gmn;
                md->fin[2] = (t3 >> 2) - gmn;
                md->has_fin = 1;
              }
            }
            U = uH;
            Hs = hh;
            Rs = rr;
            Ds = dd;
          }
          dw[u] = word;
        }
        __builtin_nontemporal_store(fl_v4u{dw[0], dw[1], dw[2], dw[3]}, dp + (size_t)q * 64);
      };
      using T_ = std::true_type;
      using F_ = std::false_type;
      for (int q = q0; q < q1; ++q) {
        const bool cap = __ballot(tf >= 16 * q && tf < 16 * q + 16) != 0ull;
        if (cap) phase(q, T_{}, T_{});
        else if (q < 6) phase(q, T_{}, F_{});
        else phase(q, F_{}, F_{});
      }
#ifdef MSA_STAMPS
      const unsigned long long tp3 = __builtin_amdgcn_s_memtime();
      if ((blk & 15) == 0) {  // a sample of the blocks (the atomics would serialize all of them)
        FL_P2STAT(a, 0, tp1 - tp0);
        FL_P2STAT(a, 1, tp2 - tp1);
        FL_P2STAT(a, 2, tp3 - tp2);
        FL_P2STAT(a, 3, 1);
      }
#endif
    }
  }
  if (lane == 0) a.blk[blk] = make_int4(0, 0, 0, 0);
}

// Pass 2, Gotoh, two rows per lane (R = 2: 128-row stripes, lane r holds rows 128s+2r+1 and
// 128s+2r+2 at column cs + t - r): as fill_block_got, both rows per step -- row 1 takes the cell above
// from the previous lane's row 2 (lane 0: the stripe above's bottom row), row 2 from row 1 at the same
// column, its diagonal from row 1's previous cell.  A phase's bytes go out as one 2 KiB block: the
// wave's row-1 16-byte segments, then its row-2 segments (traceback_kernel's R = 2 layout).
template <int CALLER>
__device__ __attribute__((noinline)) void fill_block_got2(kargs_c* ka, int blk, int lane, lds_int* lds) {
  constexpr int PS = fl_ps(CALLER);
  const FillArgs a = fill_args_of(ka);
  const unsigned ep = a.ep;
  const int m = a.m, n = a.n, S = (m + 127) / 128, g = a.g, h4 = 4 * a.oe;
  const int s = blk / a.nseg, seg = blk - s * a.nseg;
  if (s < S) {
    const int P = fl_P(s, m, n, 2);
    const int q0 = seg * PS;
    if (q0 < P) {
      int q1 = min(P, q0 + PS);
      const int cs = fl_cs(s);
      const int row_i = 128 * s + 2 * lane + 1;
      const unsigned ac = (row_i <= m) ? (a.A[a.a_off + row_i - 1] & 7u) : 0u;
      const unsigned ac2 = (row_i + 1 <= m) ? (a.A[a.a_off + row_i] & 7u) : 0u;
      unsigned plo, phi, plo2, phi2;
      fl_profile_got(g, ac, plo, phi);
      fl_profile_got(g, ac2, plo2, phi2);
      const int Bin = (s == 0) ? P - 1 : min(P - 1, fl_bmax(s, m, n, 2));
      const unsigned long long* sp = a.snap + ((size_t)s * a.nseg + seg) * 384 + lane;
      const unsigned long long* brz = a.br + (size_t)(s > 0 ? s - 1 : 0) * a.brw;
      const unsigned long long* brf = a.br + (size_t)(S + (s > 0 ? s - 1 : 0)) * a.brw;
      const int qb = (s > 0) ? min(q1, Bin + 1) : q0;
      const int nv = 16 * max(0, qb - q0);
      int U = 0, Hs1 = 0, Rs1 = 0, Hs2 = 0, Rs2 = 0, Ds2 = 0;
      bool ready = (nv == 0);
      for (int t2 = 0; !ready && t2 < (int)(FL_SPIN_MAX >> 2); ++t2) {
        const unsigned long long gz = gload(brz + 16 * q0 + nv - 1), gf = gload(brf + 16 * q0 + nv - 1);
        ready = __ballot((unsigned)(gz >> 32) != ep || (unsigned)(gf >> 32) != ep) == 0;
        if (!ready) fl_poll_sleep(t2);
      }
      if (ready) {
        ready = false;
        for (int tries = 0; !ready && tries < (int)FL_SPIN_MAX; ++tries) {
          const unsigned long long x0 = gload(sp), x1 = gload(sp + 64), x2 = gload(sp + 128), x3 = gload(sp + 192),
                                   x4 = gload(sp + 256), x5 = gload(sp + 320);
          bool ok = ((unsigned)(x0 >> 32) == ep) && ((unsigned)(x1 >> 32) == ep) && ((unsigned)(x2 >> 32) == ep) &&
                    ((unsigned)(x3 >> 32) == ep) && ((unsigned)(x4 >> 32) == ep) && ((unsigned)(x5 >> 32) == ep);
          // R~ and D~ carried + 4h, as in pass 1 (the tag bits are unchanged): 2 subtractions per
          // row-step instead of 3
          Hs1 = (int)(unsigned)x0;
          Rs1 = (int)(unsigned)x1 + h4;
          U = (int)(unsigned)x2;
          Hs2 = (int)(unsigned)x3;
          Rs2 = (int)(unsigned)x4 + h4;
          Ds2 = (int)(unsigned)x5 + h4;
          for (int v = lane; v < nv; v += 64) {
            const unsigned long long gz = gload(brz + 16 * q0 + v), gf = gload(brf + 16 * q0 + v);
            ok = ok && ((unsigned)(gz >> 32) == ep) && ((unsigned)(gf >> 32) == ep);
            *L(lds + v) = (int)(unsigned)gz;
            *L(lds + fl_p2vs(PS) + v) = (int)(unsigned)gf + h4;
          }
          ready = __ballot(!ok) == 0;
          if (!ready) __builtin_amdgcn_s_sleep(8);
        }
      }
      if (!ready) {
        if (lane == 0) atomicExch(a.err, 15);
        q1 = q0;
      }
      // row 0 (stripe 0), tagged and shifted: H~ 3 at column 0, 2 - 4h right of it; D~ + 4h 3, 2 - 4h
      p2_stage<2, PS>(lds, s, nv, 16 * (q1 - q0), lane,
                  [&](int v, int k) {
                    const int col = cs + 16 * q0 + v;
                    return col < 0 ? MSA_NEG : (k == 0 ? (col == 0 ? 3 : 2 - h4) : (col == 0 ? 3 : 2 - h4));
                  },
                  a.cod + a.cod_off, a.cod_copy, cs, q0);
      const int tmin = 1 - cs + lane;
      // the final cell (m, n): row m is row 1 or row 2 of one lane of the last stripe
      const int tf1 = (row_i == m) ? n - cs + lane : -1;
      const int tf2 = (row_i + 1 == m) ? n - cs + lane : -1;
      const int tf = max(tf1, tf2);
      fl_v4u* dp = reinterpret_cast<fl_v4u*>(a.outDir + (size_t)a.out_off + (size_t)s * a.pmax * 2048) + lane;
      auto phase = [&](const int q, auto HEAD_, auto CAP_) __attribute__((always_inline)) {
        constexpr bool HEAD = decltype(HEAD_)::value;  // lanes left of column 1 hold the border
        constexpr bool CAP = decltype(CAP_)::value;    // the phase holds cell (m, n)
        int INZ[16], INF[16];
        {
          const lds_int4* srz = reinterpret_cast<const lds_int4*>(L(lds + 16 * (q - q0)));
          const lds_int4* srf = reinterpret_cast<const lds_int4*>(L(lds + fl_p2vs(PS) + 16 * (q - q0)));
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const fl_v4i vz = srz[u], vf = srf[u];
            INZ[4 * u] = vz.x; INZ[4 * u + 1] = vz.y; INZ[4 * u + 2] = vz.z; INZ[4 * u + 3] = vz.w;
            INF[4 * u] = vf.x; INF[4 * u + 1] = vf.y; INF[4 * u + 2] = vf.z; INF[4 * u + 3] = vf.w;
          }
        }
        const fl_v4u c4 = p2_codes<PS>(lds, q - q0, lane);
        const unsigned cw[4] = {c4.x, c4.y, c4.z, c4.w};
        unsigned dw1[4], dw2[4];
        // four cells' direction bytes, tags of their inputs H~ diag | R~ left << 2 | D~ up << 4: the
        // low bytes of the four H~, R~ and D~ gathered by v_perm (3 each), then two byte-wise bfi
        // merges and one mask -- 14 ops per 4 cells instead of 5 per cell
        auto gather4 = [](const int* b) __attribute__((always_inline)) {
          const unsigned lo = __builtin_amdgcn_perm((unsigned)b[1], (unsigned)b[0], 0x0c0c0400u);
          const unsigned hi = __builtin_amdgcn_perm((unsigned)b[3], (unsigned)b[2], 0x0c0c0400u);
          return __builtin_amdgcn_perm(hi, lo, 0x05040100u);
        };
        auto dword = [&](const int* h, const int* r, const int* d) __attribute__((always_inline)) {
          const unsigned HT = gather4(h), RT = gather4(r), DT = gather4(d), M = 0x03030303u;
          unsigned x, y;
          asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(x) : "s"(M), "v"(RT), "v"(DT << 2));
          asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(y) : "s"(M), "v"(HT), "v"(x << 2));
          return y & 0x3f3f3f3fu;
        };
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const unsigned s4 = __builtin_amdgcn_perm(phi, plo, cw[u]);
          const unsigned s4b = __builtin_amdgcn_perm(phi2, plo2, cw[u]);
          int h1t[4], r1t[4], d1t[4], h2t[4], r2t[4], d2t[4];
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) {
            const int kx = 4 * u + kk;
            const int sc = ((int)(s4 << (24 - 8 * kk))) >> 24;
            const int sb = ((int)(s4b << (24 - 8 * kk))) >> 24;
            // row 1 (R~ / D~ carried + 4h: Rs1, uD, and the results rr, dd)
            const int uH = dpp_shr1(INZ[kx], Hs2);
            const int uD = dpp_shr1(INF[kx], Ds2);
            const int t1 = (int)((unsigned)U | 3u) + sc;
            const int t2p = (int)(((unsigned)Rs1 & ~3u) | 2u);
            const int t3p = (int)(((unsigned)uD & ~3u) | 1u);
            h1t[kk] = U; r1t[kk] = Rs1; d1t[kk] = uD;
            const int t2 = t2p - h4, t3 = t3p - h4;
            int hh1 = vmax3(t1, t2, t3);
            int rr1 = vmax3(t1, t2p, t3);
            int dd1 = vmax3(t1, t2, t3p);
            // row 2: diagonal = row 1's previous H~, above = row 1's new cell
            const bool before = HEAD && (16 * q + kx < tmin);
            if constexpr (HEAD) {
              hh1 = before ? 1 - h4 : hh1;
              rr1 = before ? 1 - h4 : rr1;
              dd1 = before ? 1 : dd1;
            }
            const int s1 = (int)((unsigned)Hs1 | 3u) + sb;
            const int s2p = (int)(((unsigned)Rs2 & ~3u) | 2u);
            const int s3p = (int)(((unsigned)dd1 & ~3u) | 1u);
            h2t[kk] = Hs1; r2t[kk] = Rs2; d2t[kk] = dd1;
            const int s2 = s2p - h4, s3 = s3p - h4;
            int hh2 = vmax3(s1, s2, s3);
            int rr2 = vmax3(s1, s2p, s3);
            int dd2 = vmax3(s1, s2, s3p);
            if constexpr (HEAD) {
              hh2 = before ? 1 - h4 : hh2;
              rr2 = before ? 1 - h4 : rr2;
              dd2 = before ? 1 : dd2;
            }
            if constexpr (CAP) {
              if (16 * q + kx == tf) {
                const int gmn = g * (m + n);  // unshift
                // (the slot reduce_pairs_kernel reads: the last 64-row stripe's meta)
                msa_stripe_meta* md = a.meta + a.stripe0 + (m + 63) / 64 - 1;
                md->fin[0] = ((tf1 >= 0 ? t1 : s1) >> 2) - gmn;
                md->fin[1] = ((tf1 >= 0 ? t2 : s2) >> 2) - gmn;
                md->fin[2] = ((tf1 >= 0 ? t3 : s3) >> 2) - gmn;
                md->has_fin = 1;
              }
            }
            U = uH;
            Hs1 = hh1;
            Rs1 = rr1;
            Hs2 = hh2;
            Rs2 = rr2;
            Ds2 = dd2;
          }
          dw1[u] = dword(h1t, r1t, d1t);
          dw2[u] = dword(h2t, r2t, d2t);
        }
        if constexpr ((MSA_ABL & 8) == 0) {
          __builtin_nontemporal_store(fl_v4u{dw1[0], dw1[1], dw1[2], dw1[3]}, dp + (size_t)q * 128);
          __builtin_nontemporal_store(fl_v4u{dw2[0], dw2[1], dw2[2], dw2[3]}, dp + (size_t)q * 128 + 64);
        }
      };
      using T_ = std::true_type;
      using F_ = std::false_type;
      for (int q = q0; q < q1; ++q) {
        const bool cap = __ballot(tf >= 16 * q && tf < 16 * q + 16) != 0ull;
        if (cap) phase(q, T_{}, T_{});
        else if (q < 6) phase(q, T_{}, F_{});
        else phase(q, F_{}, F_{});
      }
    }
  }
  if (lane == 0) a.blk[blk] = make_int4(0, 0, 0, 0);
}

// Pass 2 as a launch of its own, queued behind the pass-1 launch, for long pairs (msa_plan_create:
// pass 1 needs most CUs -- ~n / (W lag) items in flight -- and the flow kernel's register budget
// (~220 VGPRs for affine / Gotoh) leaves no room for a pass-2 workgroup beside a pass-1 one, so
// in-launch pass-2 workgroups only started once pass 1 was done, at 1.5 waves per SIMD).  Here
// every input is complete when the blocks start, and the pass-2 code alone sets the register
// budget: several waves per SIMD hide each other's LDS and store latency.
template <bool FLOOR, bool TRACKPOS, int R, int FK>
#ifndef FL_FILL_WPE
#define FL_FILL_WPE 4  // waves per SIMD the pass-2 launch is sized for
#endif
__global__ __launch_bounds__(FL_FILLW * 64) __attribute__((amdgpu_waves_per_eu(FL_FILL_WPE, 8))) void flow_fill_kernel(KArgs a) {
  extern __shared__ __attribute__((aligned(16))) int smem[];
  const int lane = threadIdx.x & 63;
  const int w = uni(threadIdx.x >> 6);
  kargs_c* ka = (kargs_c*)__builtin_amdgcn_kernarg_segment_ptr();  // (a is the only argument)
  lds_int* wl = L(smem + w * fl_p2ints(FL_PS_FILL));
  for (;;) {
    int t = 0;
    if (lane == 0) t = atomicAdd(a.ticket + MSA_TK_BLOCK, 1);
    t = __builtin_amdgcn_readlane(t, 0);
    if (t >= a.nblk) break;
    if constexpr (FK == 2 && R == 2) fill_block_got2<1>(ka, a.border[t], lane, wl);
    else if constexpr (FK == 2) fill_block_got<1>(ka, a.border[t], lane, wl);
    else if constexpr (FK == 1 && R == 2) fill_block_aff2<1>(ka, a.border[t], lane, wl);
    else if constexpr (FK == 1) fill_block_aff<1>(ka, a.border[t], lane, wl);
    else fill_block<FLOOR, TRACKPOS, R, 1>(fill_args_of(ka), a.border[t], lane, wl);
  }
}

// Pair result of a two-pass plan from the pass-2 block bests: every thread folds
// a strided share (loads all in flight), then wave shuffles, then 4 wave results.
__global__ __launch_bounds__(1024) void reduce_blocks_kernel(const int4* blk, int nblk, PairResult* out) {
  __shared__ int4 sh[16];
  // empty alignment: score 0 at (0, 0); first maximum in row-major order
  auto better = [](int vb, int vi, int vj, int b_, int i_, int j_) {
    return vb > b_ || (vb == b_ && vb > 0 && (vi < i_ || (vi == i_ && vj < j_)));
  };
  int b = 0, bi = 0, bj = 0;
  for (int x0 = threadIdx.x; x0 < nblk; x0 += 4096) {  // four loads in flight per thread
    int4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = (x0 + 1024 * u < nblk) ? blk[x0 + 1024 * u] : make_int4(0, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (better(v[u].x, v[u].y, v[u].z, b, bi, bj)) { b = v[u].x; bi = v[u].y; bj = v[u].z; }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const int ob = __shfl_xor(b, off), oi = __shfl_xor(bi, off), oj = __shfl_xor(bj, off);
    if (better(ob, oi, oj, b, bi, bj)) { b = ob; bi = oi; bj = oj; }
  }
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = make_int4(b, bi, bj, 0);
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int x = 1; x < 16; ++x) {
      const int4 v = sh[x];
      if (better(v.x, v.y, v.z, b, bi, bj)) { b = v.x; bi = v.y; bj = v.z; }
    }
    PairResult r;
    r.score = b;
    r.status = 0;
    r.end_i = bi;
    r.end_j = bj;
    r.fin[0] = r.fin[1] = r.fin[2] = 0;
    r.pad = 0;
    out[0] = r;
  }
}

}  // namespace msa
