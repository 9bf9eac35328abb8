// msa_traceback.hip -- on-device traceback walks over direction bytes.
//
//  * SW affine (config C5): the fill (stripe_kernel or the affine flow kernel,
//    MSA_ALG_SWA, MSA_OUT_DIR) leaves one byte per cell -- bits 0-1: where H came
//    from (0 = local start, 1 = diagonal, 2 = E / horizontal gap, 3 = F / vertical
//    gap); bit 2: E here opened from H(i, j-1); bit 3: F here opened from H(i-1, j).
//    The walk is the tie order of oracle orc_sw (first maximum), from the pair's end
//    cell.
//  * Reference Gotoh (MSA_ALG_REF / REF1, MSA_OUT_DIR: main_alignment_function /
//    Subproblem::find_alignment, subproblem_alignment.cpp:105-172): bits 0-1 = T1's
//    predecessor table, 2-3 = T2's, 4-5 = T3's (REF: table numbers 1..3, the first
//    table in the reference's order T1, T2, T3 whose value reproduces the cell by
//    exact equality; REF1: tags 4 - table).  The walk starts at (m, n) in the end
//    node's table (the reference's end-type rule, :112-146, from the fill's final
//    state) and stops when i == 0 or j == 0 (:147).  One op per step = the table the
//    step leaves from ('M' T1 / diagonal, 'D' T2 / consumes B, 'I' T3 / consumes
//    A); the host turns them into the reference's align list (node coordinates,
//    quirks Q1/Q2).
//
// Both layouts are the skewed stripe layout: cell (64s + r + 1, cs_s + t - r) at
// byte (s*pmax + t/16)*1024 + r*16 + t%16 of the pair's block -- a 16-step x
// 64-row block is 1 KiB, one 16-byte row segment per lane.
//
// One wave walks the path from the pair's end cell (read from the reduction's
// PairResult on the same stream, no host round trip).  Its state is uniform
// (SGPRs).  Inside a stripe t only decreases (every move lowers it by 1 or 2), so
// the walk needs, per stripe, the bytes left of where it enters: a GROUP of 16
// blocks (256 steps x 64 rows, 16 KiB) ending a little right of the entry point.
// A diagonal path crosses a stripe in 64 steps (t drops by 128), so one group per
// stripe usually serves.  Groups are staged in LDS by LDS-DMA, one slot per stripe
// modulo 4, by a second wave of the workgroup (the loader): when the walk enters
// stripe s the loader prefetches stripe s-3's group at the column a diagonal path
// would enter it (a misprediction -- after gaps -- costs an on-demand load), and
// publishes each group once it has landed; the walker only reads LDS.  A third
// wave decodes the walk's step words into op bytes while the walk goes on (round
// 6: the walker used to issue the 16-32 loads per stripe itself, ~1,400 ticks of
// issue stalls per stripe, and to decode at the end: 31% and 8% of its time).
// Inside a group:
//  * in state T1 / H, one LDS gather gives lane q the byte of cell (i - q, j - q);
//    a ballot of "diagonal move, staying in T1 / H" and a find-first-zero give the
//    length of the diagonal run ahead (up to 64 steps in ~10 instructions, 128 with
//    two cells per lane in the 128-row layouts: C5's optimal path is 15 diagonal
//    runs of ~1,300 cells between 14 gaps);
//  * otherwise an 8 x 8 window: one LDS read gives lane (a, b) the byte of cell
//    (i - a, j - b), turned into a transition word, and up to 7 steps are resolved
//    from it with v_readlane.
// Steps are recorded in an LDS ring (window words of nibbles, run words) that the
// decoder wave turns into op bytes, one word per lane (no scalar-cache writes).
// Output: ops from the end cell back to the start ('M' diagonal, 'D' a gap
// consuming B, 'I' a gap consuming A), info = {n_ops, beg_i, beg_j, status,
// stripes entered, groups staged on demand (first, mispredicted, left on the left),
// s_memtime ticks of the walk, times the walker waited for the loader}.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace msa {

// Group loads are LDS-DMA (global_load_lds_dwordx4: each lane's 16 bytes land at
// M0 + 16 * lane, no VGPR destination), issued as inline asm so that the
// compiler's wait-count pass does not see them (it would drain them with vmcnt(0)
// in front of unrelated work); they are waited for explicitly (s_waitcnt vmcnt(N),
// memory clobber) before a slot is read.  M0 is written in the statement that uses
// it (an SALU M0 write needs one wait state before the load).
__device__ __forceinline__ void glds16(const uint8_t* gsrc, unsigned lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_dst)
               : "memory");
}
// 16 consecutive 1 KiB blocks (lane base pointer g) into 16 KiB of LDS at lds_dst: 16 loads.
// The instruction offset moves the LDS destination as well as the source (measured:
// mbench/mb_glds.hip), so four loads share one base and one M0 (offsets 0..3 KiB) and M0
// steps by 4 KiB per base.
__device__ __forceinline__ void glds16x16(const uint8_t* g, unsigned lds_dst) {
  const uint8_t* g1 = g + 4096;
  const uint8_t* g2 = g + 8192;
  const uint8_t* g3 = g + 12288;
  unsigned keep;
#define TB_L4(v)                                                                                 \
  "global_load_lds_dwordx4 " v ", off\n\tglobal_load_lds_dwordx4 " v ", off offset:1024\n\t"     \
  "global_load_lds_dwordx4 " v ", off offset:2048\n\tglobal_load_lds_dwordx4 " v ", off offset:3072\n\t"
#define TB_M0 "s_add_u32 m0, m0, 0x1000\n\ts_nop 0\n\t"
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %5\n\ts_nop 0\n\t" TB_L4("%1") TB_M0 TB_L4("%2") TB_M0 TB_L4("%3")
                   TB_M0 TB_L4("%4") "s_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(g), "v"(g1), "v"(g2), "v"(g3), "s"(lds_dst)
               : "memory");
#undef TB_L4
#undef TB_M0
}
// Transitions of the walk (oracle orc_sw tie order), by state:
//  H: the low two bits hs of the byte -- 0 local start (stop), 1 diagonal ('M', stay in H),
//     2 from E (no op, go to E), 3 from F (no op, go to F);
//  E: 'D' (a gap consuming B), back to H if bit 2 (E opened from H(i, j-1)), else stay;
//  F: 'I' (a gap consuming A), back to H if bit 3 (F opened from H(i-1, j)), else stay.
// A transition field is (10 x next state, 30 = stop) | (lane step: 9 M / 1 D / 8 I / 0 none)
// << 6; TB_FH holds the four H fields at 16-bit spacing, indexed by hs.
constexpr unsigned long long TB_FH = 30ull | ((9ull << 6) << 16) | (10ull << 32) | (20ull << 48);

__device__ __forceinline__ void vm_wait_all() { asm volatile("s_waitcnt vmcnt(0)" : : : "memory"); }
// wait until at most n VMEM ops are outstanding, n rounded down to 0, 16, 32 or 48
__device__ __forceinline__ void vm_wait_le(int n) {
  if (n >= 48) asm volatile("s_waitcnt vmcnt(48)" : : : "memory");
  else if (n >= 32) asm volatile("s_waitcnt vmcnt(32)" : : : "memory");
  else if (n >= 16) asm volatile("s_waitcnt vmcnt(16)" : : : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" : : : "memory");
}

// find_alignment's end node table (subproblem_alignment.cpp:112-146) from the final
// state fin = (T1, T2, T3)(m, n), MSA_NEG = -inf: end_type > 0 names it; otherwise
// the first of T1, T2 + h', T3 + h' that is >= the others (h' = h for the table
// end_type <= -2 names).  Returns 0, 1, 2 for T1, T2, T3.
__device__ __forceinline__ int ref_end_state(const int32_t (&fin)[3], int end_type, int h) {
  if (end_type > 0) return end_type - 1;
  const long long NI = -(1ll << 62);  // -inf: absorbs + h
  auto v = [&](int k) {
    const long long x = fin[k];
    return x == (long long)MSA_NEG ? NI : x + ((k + 1 == -end_type && end_type <= -2) ? h : 0);
  };
  const long long t1 = v(0), t2 = v(1), t3 = v(2);
  if (t1 >= t2 && t1 >= t3) return 0;
  if (t2 >= t1 && t2 >= t3) return 1;
  return 2;
}

// Walk kinds: Smith-Waterman affine; the reference's Gotoh walk over table numbers (REF
// fill) or over tags (REF1 fill, tag = 4 - table).
enum { TB_SW = 0, TB_REF = 1, TB_REF_TAG = 2 };

// The transition word of a cell (see the window comment in traceback_kernel): three 10-bit
// fields, field s (bits 10s..) = 10 x the next state (30 = stop) | the lane step of leaving
// state s << 6, and bits 30-31 = 10b.  A step shifts the 64-bit {7, word} right by the current
// field's position and takes the low 6 bits of the result as the next position (the 64-bit
// shift reads only those 6 bits of its shift operand: no mask op), bits 6-9 as the lane step.
// Bits 30-35 of {7, word} read 30: the stop state is absorbing (lane step 0, stay at 30), so
// the steps after a stop are no-ops and a window needs no branch per step.
template <int KIND>
__device__ __forceinline__ unsigned tb_word(unsigned dv) {
  if constexpr (KIND == TB_REF_TAG) {
    // table s leaves by its fixed move (T1 diagonal 9, T2 left 1, T3 up 8) into table 4 - x, x
    // = the tag in bits 2s..2s+1: next state 10 (3 - x), and x = 0 (no predecessor) gives 30
    // (stop) -- one formula, 30 - 10x, for every x.  The three 2-bit tags spread to 10-bit
    // spacing by one multiply (copies at bits 0, 8, 16 never overlap), then the word is
    // C - 10 x spread (each field 30 - 10x >= 0: no borrow between fields).
    constexpr unsigned C = (30u | (9u << 6)) | ((30u | (1u << 6)) << 10) | ((30u | (8u << 6)) << 20) | (1u << 31);
    const unsigned sp = (dv * 0x10101u) & 0x300C03u;
    return C - 10u * sp;
  } else if constexpr (KIND == TB_REF) {
    // table numbers x = 1..3 (0: no predecessor): next state 10 (x - 1), or 30
    auto fld = [](unsigned step, unsigned x) { return (x ? 10u * (x - 1u) : 30u) | (step << 6); };
    return fld(9u, dv & 3u) | (fld(1u, (dv >> 2) & 3u) << 10) | (fld(8u, (dv >> 4) & 3u) << 20) | (1u << 31);
  } else {
    const unsigned fH = (unsigned)(TB_FH >> (16 * (dv & 3u))) & 0x3ffu;
    const unsigned fE = (1u << 6) | ((dv & 4u) ? 0u : 10u);
    const unsigned fF = (8u << 6) | ((dv & 8u) ? 0u : 20u);
    return fH | (fE << 10) | (fF << 20) | (1u << 31);
  }
}
// State 0 (T1 / H) continues diagonally and stays in state 0 at a cell with byte dv.
template <int KIND>
__device__ __forceinline__ bool tb_diag_stay(unsigned dv) {
  if constexpr (KIND == TB_REF_TAG) return (dv & 3u) == 3u;  // T1's predecessor T1 (tag 3)
  else return (dv & 3u) == 1u;                             // T1 from T1 / H from the diagonal
}

// Hand-off words between the walk's three waves (LDS; see traceback_kernel).
struct TbCtl {
  unsigned long long ready[4];  // per slot: the group that has landed there, (b0 << 32) | stripe
  int req_seq[4], req_s[4], req_t[4];  // walker -> loader s & 3: stage stripe s's group covering step t
  int ent_seq, ent_s, ent_col;  // walker -> loader: entered stripe s at column j - r (the prefetch hint)
  int consumed;                 // decoder -> walker: ring words decoded (their entries are free again)
  int done, nw_total;           // walker: finished, after nw_total words
  int n_demand[4];              // loaders: groups staged because a request found none covering
  long long nops, t_dec;        // decoder: ops decoded; busy ticks (diagnostic build)
  int wi, wj, wstatus, n_switch, n_req;  // walker: where it stopped, status, stripes entered, requests
  long long t_walk, wst[5];              // walker: ticks; diagnostic build: wait, runs, windows, in groups, in runs
  long long lst[4];                      // loader (diagnostic build): ticks issuing, waiting, issue-to-publish, groups
};
// Hand-off accesses: relaxed workgroup-scope atomics on the LDS words (plain ds_read / ds_write that
// the compiler neither drops nor merges; a volatile access through a generic pointer would be a flat
// op, counted on vmcnt beside the loader's LDS-DMA).  One wave's LDS ops execute in order; the
// compiler barriers keep the hand-off accesses in program order.
template <class T>
__device__ __forceinline__ T tb_ld(T& x) {
  const T v = __hip_atomic_load(&x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  asm volatile("" : : : "memory");
  return v;
}
template <class T, class U>
__device__ __forceinline__ void tb_st(T& x, U v) {
  __hip_atomic_store(&x, (T)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  asm volatile("" : : : "memory");
}
// a hand-off word read by a whole wave, kept uniform (an LDS value is otherwise "divergent": VGPRs)
__device__ __forceinline__ int tb_u(int& x) { return __builtin_amdgcn_readfirstlane(tb_ld(x)); }
__device__ __forceinline__ unsigned long long tb_u64(unsigned long long& x) {
  const unsigned long long v = tb_ld(x);
  return ((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((int)(v >> 32)) << 32) |
         (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)v);
}
// spin bound of the walker's waits on the other two waves (MSA_ERR_TIMEOUT past it; ~1 s)
constexpr int TB_SPIN_MAX = 1 << 24;

// KIND TB_SW: Smith-Waterman affine walk; TB_REF / TB_REF_TAG: the reference's Gotoh walk
// (end_type, h: find_alignment's end rule).  RL = rows per lane of the layout: 1, or 2 for the
// two-rows-per-lane Gotoh flow fill (128-row stripes, lane r holds rows 2r+1 and 2r+2 at column
// cs + t - r; a 16-step block is 2 KiB: the row-1 segments, then the row-2 segments).
//
// One workgroup of six waves.  Wave 1 walks; its state is uniform (SGPRs) and it touches LDS
// only.  Waves 0, 3, 4, 5 stage stripe groups into LDS, one slot (stripe mod 4) each (each its own
// vmcnt and issue stalls: a loader stages one group per four stripes): on the walker's request (stripe s, step t: the
// group covering t) and, each time the walker enters a stripe, the next three stripes' predicted
// groups; a loader publishes a group in ready[slot] once its loads have landed (its own
// s_waitcnt), so the issue stalls of 16-32 KiB of LDS-DMA per stripe and the load latency stay off
// the walk (an LDS-DMA lane writes M0 + 16 x its lane: mbench/mb_dma.hip).  Wave 2 decodes the
// walker's LDS ring of step words into op bytes while the walk goes on.  Every wave's loop ends:
// the walker's waits are bounded (TB_SPIN_MAX), and the other waves leave after the walker's
// `done`, the loaders with none of their loads in flight.
template <int KIND, int RL = 1>
__global__ __launch_bounds__(384) void traceback_kernel(const uint8_t* __restrict__ dir,
                                                        const msa_pair_desc* __restrict__ pairs,
                                                        const msa_stripe_meta* __restrict__ meta,
                                                        const PairResult* __restrict__ res, int pair, int end_type,
                                                        int hpen, uint8_t* __restrict__ ops, long long cap,
                                                        long long* __restrict__ info, int csflow,
                                                        const unsigned long long* __restrict__ best_key) {
  constexpr bool REF = KIND != TB_SW;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const msa_pair_desc pd = pairs[pair];
  const uint8_t* base = dir + pd.out_off + lane * 16;
  const int pmax = pd.pmax;
  // Group slots: 4 x 16 KiB behind a guard (window lanes whose cell lies outside the group
  // read an unused byte there -- down to 2,270 B below a slot -- and hold frozen words).
  constexpr int GB = 16, GT = 16 * GB, GBYTES = 1024 * RL * GB, NSLOT = 4;
  constexpr int SR = 64 * RL;  // rows per stripe
  constexpr int TB_GUARD = 2304;
  __shared__ __attribute__((aligned(16))) uint8_t stage_raw[TB_GUARD + NSLOT * GBYTES];
  typedef __attribute__((address_space(3))) uint8_t lds_u8;
  // (a flat pointer to LDS holds the LDS address in its low 32 bits)
  const unsigned stage_lds = (unsigned)(uintptr_t)&stage_raw[TB_GUARD];
  // every stripe's start column, staged in LDS once (a stripe change then costs an LDS
  // read, not a ~1 us dependent global load); pairs with more stripes read the rest from HBM
  constexpr int TB_CSL = RL == 1 ? 8192 : 1;  // (RL = 2: flow layouts only, stripe starts computed)
  __shared__ int csl[TB_CSL];
  const int S = (pd.m + SR - 1) / SR;
  // The walk records one word per window -- nibble q (from the top) = the lane step of step q
  // (9 'M', 1 'D', 8 'I', 0 no op), the step count in bits 28-31 -- or per diagonal run --
  // 15 in bits 28-31, the run length below -- into an LDS ring (all lanes store the same word:
  // no per-lane branch in the walk).  No word is 0: a 0 entry is free.
  constexpr int TB_RAW = 4096;
  __shared__ unsigned rawl[TB_RAW];
  __shared__ TbCtl ctl_s;
  if (!csflow)
    for (int k = threadIdx.x; k < S && k < TB_CSL; k += 384) csl[k] = meta[pd.stripe0 + k].cs;
  for (int k = threadIdx.x; k < TB_RAW; k += 384) rawl[k] = 0u;
  if (threadIdx.x == 0) {
    for (int k = 0; k < NSLOT; ++k) ctl_s.ready[k] = ~0ull;  // stripe -1: empty
    for (int k = 0; k < 4; ++k) ctl_s.req_seq[k] = ctl_s.n_demand[k] = 0;
    ctl_s.ent_seq = ctl_s.consumed = ctl_s.done = ctl_s.nw_total = 0;
    ctl_s.nops = ctl_s.t_dec = 0;
  }
  __syncthreads();
  auto cs_of = [&](int k) {  // wave-uniform (readfirstlane: an LDS value is otherwise "divergent")
    // the flow kernels' stripes start at fl_cs(k) = -((-k) mod 16): no LDS round trip
    if (csflow) return -((16 - (k & 15)) & 15);
    return k < TB_CSL ? __builtin_amdgcn_readfirstlane(csl[k]) : meta[pd.stripe0 + k].cs;
  };
  // the group of stripe s ending a little right of step t (blocks b0 .. b0 + 15 of the stripe)
  auto group_b0 = [&](int t) __attribute__((always_inline)) {
    int b0 = ((t + 16) >> 4) - (GB - 1);
    b0 = b0 < pmax - GB ? b0 : pmax - GB;
    return b0 > 0 ? b0 : 0;
  };
  auto sel4 = [](int k, int a, int b, int c, int d) __attribute__((always_inline)) {
    const int lo = (k & 1) ? b : a, hi = (k & 1) ? d : c;  // (three selects, no branches)
    return (k & 2) ? hi : lo;
  };
  auto set4 = [](int k, int v, int& a, int& b, int& c, int& d) __attribute__((always_inline)) {
    a = k == 0 ? v : a;
    b = k == 1 ? v : b;
    c = k == 2 ? v : c;
    d = k == 3 ? v : d;
  };

  if (wave != 1 && wave != 2) {
    // ---- loaders: stage groups, publish them once landed; wave 0 the stripes s = 0 mod 4 (slot 0),
    // waves 3, 4, 5 those of slots 1, 2, 3 (each its own vmcnt and issue stalls: a loader stages one
    // group per four stripes) ----
    const int par = __builtin_amdgcn_readfirstlane(wave == 0 ? 0 : wave - 2);  // (uniform: M0 and the SGPR operands)
    // slot bookkeeping (slot = stripe & 3): the stripe staged there, its first block, the count
    // of loads issued up to its own (its loads are complete once at most `issued - end` later
    // loads are outstanding), and whether it has been published
    int sl_s0 = -1, sl_s1 = -1, sl_s2 = -1, sl_s3 = -1;
    int sl_b0 = 0, sl_b1 = 0, sl_b2 = 0, sl_b3 = 0;
    int sl_e0 = 0, sl_e1 = 0, sl_e2 = 0, sl_e3 = 0;
    int pub = 15, issued = 0, last_req = 0, last_ent = 0, n_demand = 0;
#ifdef MSA_TB_STATS
    long long t_iss = 0, t_lw = 0, t_lat = 0, n_grp = 0, ti0 = 0, ti1 = 0, ti2 = 0, ti3 = 0;
#endif
    // stage stripe s, blocks b0.. into slot s & 3 (always 16 loads: a stripe with fewer blocks
    // loads its last one again, so the outstanding-load arithmetic stays exact)
    auto stage_group = [&](int s, int b0) __attribute__((always_inline)) {
      const int k = s & (NSLOT - 1);
#ifdef MSA_TB_STATS
      const long long a = (long long)__builtin_amdgcn_s_memtime();
#endif
      const unsigned dst = stage_lds + (unsigned)GBYTES * (unsigned)k;
      const uint8_t* g = base + ((long long)s * pmax + b0) * (1024 * RL);
      if (pmax >= GB) {
        glds16x16(g, dst);
        if constexpr (RL == 2) glds16x16(g + 16384, dst + 16384u);
      } else {
#pragma unroll
        for (int q = 0; q < GB * RL; ++q) {
          const int qb = q / RL < pmax ? q / RL : pmax - 1;  // (a short stripe loads its last block again)
          glds16(base + ((long long)s * pmax + qb) * (1024 * RL) + 1024 * (q % RL), dst + 1024u * q);
        }
      }
      issued += GB * RL;
#ifdef MSA_TB_STATS
      {
        const long long e = (long long)__builtin_amdgcn_s_memtime();
        t_iss += e - a;
        ++n_grp;
        ti0 = k == 0 ? e : ti0;
        ti1 = k == 1 ? e : ti1;
        ti2 = k == 2 ? e : ti2;
        ti3 = k == 3 ? e : ti3;
      }
#endif
      set4(k, s, sl_s0, sl_s1, sl_s2, sl_s3);
      set4(k, b0, sl_b0, sl_b1, sl_b2, sl_b3);
      set4(k, issued, sl_e0, sl_e1, sl_e2, sl_e3);
      pub &= ~(1 << k);
    };
    // wait until the loads of slot k have landed, then publish every slot whose loads have
    auto land = [&](int k) __attribute__((always_inline)) {
      const int n = issued - sel4(k, sl_e0, sl_e1, sl_e2, sl_e3);
      const int lvl = n >= 48 ? 48 : n >= 32 ? 32 : n >= 16 ? 16 : 0;
#ifdef MSA_TB_STATS
      const long long a = (long long)__builtin_amdgcn_s_memtime();
#endif
      vm_wait_le(n);
#ifdef MSA_TB_STATS
      const long long e = (long long)__builtin_amdgcn_s_memtime();
      t_lw += e - a;
#endif
      for (int q = 0; q < NSLOT; ++q)
        if (!((pub >> q) & 1) && sel4(q, sl_e0, sl_e1, sl_e2, sl_e3) <= issued - lvl) {
          tb_st(ctl_s.ready[q], ((unsigned long long)(unsigned)sel4(q, sl_b0, sl_b1, sl_b2, sl_b3) << 32) |
                          (unsigned)sel4(q, sl_s0, sl_s1, sl_s2, sl_s3));
          pub |= 1 << q;
#ifdef MSA_TB_STATS
          t_lat += e - (q == 0 ? ti0 : q == 1 ? ti1 : q == 2 ? ti2 : ti3);
#endif
        }
    };
    for (;;) {
      const int rq = tb_u(ctl_s.req_seq[par]);
      if (rq != last_req) {
        // the walker waits for stripe s's group covering step t
        last_req = rq;
        const int s = tb_u(ctl_s.req_s[par]), t = tb_u(ctl_s.req_t[par]);
        const int k = s & (NSLOT - 1);
        const int b0 = sel4(k, sl_b0, sl_b1, sl_b2, sl_b3);
        if (sel4(k, sl_s0, sl_s1, sl_s2, sl_s3) != s || t < 16 * b0 || t >= 16 * b0 + GT) {
          stage_group(s, group_b0(t));
          ++n_demand;
        }
        land(k);
        continue;
      }
      const int ev = tb_u(ctl_s.ent_seq);
      if (ev != last_ent) {
        // the walker entered stripe s (it is done with s + 1, whose slot s - 3 now takes): prefetch
        // the next three stripes' groups (only s - 3 is new in steady state).  A diagonal path from
        // (i, j) enters stripe s - d at column j - r - 64d + 63, step t_d = j - r - 64d + 126 -
        // cs(s - d) (RL = 2: row 128 (s - d) + 128, lane 63, column j - r - 128d + 127); the group
        // ends 16 steps right of it.  A stripe already staged is never restaged here, so no slot
        // the walker may be reading is overwritten.
        last_ent = ev;
        const int s = tb_u(ctl_s.ent_s), col = tb_u(ctl_s.ent_col);
        for (int d = 1; d <= NSLOT - 1; ++d) {
          const int sd = s - d;
          if (sd < 0) break;
          if ((sd & 3) != par) continue;  // (another loader's stripe)
          if (sel4(sd & (NSLOT - 1), sl_s0, sl_s1, sl_s2, sl_s3) == sd) continue;
          stage_group(sd, group_b0(RL == 2 ? col - 128 * d + 190 - cs_of(sd) : col - 64 * d + 126 - cs_of(sd)));
        }
        continue;
      }
      if (pub != 15) {
        // publish the oldest group still in flight
        int ko = -1, eo = 0;
        for (int q = 0; q < NSLOT; ++q) {
          const int e = sel4(q, sl_e0, sl_e1, sl_e2, sl_e3);
          if (!((pub >> q) & 1) && (ko < 0 || e < eo)) { ko = q; eo = e; }
        }
        land(ko);
        continue;
      }
      if (tb_u(ctl_s.done)) break;
      __builtin_amdgcn_s_sleep(1);
    }
    vm_wait_all();  // no load left in flight when the wave ends
    tb_st(ctl_s.n_demand[par], n_demand);
#ifdef MSA_TB_STATS
    tb_st(ctl_s.lst[0], t_iss);
    tb_st(ctl_s.lst[1], t_lw);
    tb_st(ctl_s.lst[2], t_lat);
    tb_st(ctl_s.lst[3], n_grp);
#endif
  } else if (wave == 2) {
    // ---- decoder: ring words -> op bytes, one word per lane, a wave prefix sum of the op counts ----
    int pos = 0;
    long long nops = 0;
#ifdef MSA_TB_STATS
    long long t_dec = 0;
#endif
    for (;;) {
      const int dn = tb_u(ctl_s.done);
      const unsigned w0 = tb_ld(rawl[(pos + lane) & (TB_RAW - 1)]);
      const unsigned long long bal = __ballot(w0 != 0u);
      const int nq = ~bal == 0ull ? 64 : (int)__builtin_ctzll(~bal);  // the written words from pos on
      if (nq == 0) {
        if (dn && pos >= tb_u(ctl_s.nw_total)) break;
        __builtin_amdgcn_s_sleep(2);
        continue;
      }
#ifdef MSA_TB_STATS
      const long long td0 = (long long)__builtin_amdgcn_s_memtime();
#endif
      const unsigned w = lane < nq ? w0 : 0u;
      const int k = (int)(w >> 28);
      int c = 0;
      if (k == 15) c = (int)(w & 0xffffu);
      else
        for (int q = 0; q < k; ++q) c += ((w >> (4 * q)) & 15u) != 0u;
      int incl = c;  // inclusive prefix sum over the lanes
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(incl, off);
        if (lane >= off) incl += y;
      }
      long long o = nops + incl - c;
      if (k == 15) {
        // a run of c 'M' (up to 128): bytes up to a 16-byte boundary, 16-byte stores, bytes
        const long long e = o + c < cap ? o + c : cap;
        for (; o < e && ((uintptr_t)(ops + o) & 15u); ++o) ops[o] = 'M';
        for (; o + 16 <= e; o += 16) *(uint4*)(ops + o) = make_uint4(0x4d4d4d4du, 0x4d4d4d4du, 0x4d4d4d4du, 0x4d4d4d4du);
        for (; o < e; ++o) ops[o] = 'M';
      } else {
        for (int q = 0; q < k; ++q) {
          const unsigned dl = (w >> (4 * (k - 1 - q))) & 15u;  // step 0 in the top nibble
          if (dl != 0u) {
            if (o < cap) ops[o] = dl == 9u ? 'M' : (dl == 1u ? 'D' : 'I');
            ++o;
          }
        }
      }
      nops += __shfl(incl, 63);
      if (lane < nq) tb_st(rawl[(pos + lane) & (TB_RAW - 1)], 0u);  // free the entries, then say so
      pos += nq;
      tb_st(ctl_s.consumed, pos);
#ifdef MSA_TB_STATS
      t_dec += (long long)__builtin_amdgcn_s_memtime() - td0;
#endif
    }
    tb_st(ctl_s.nops, nops);
#ifdef MSA_TB_STATS
    tb_st(ctl_s.t_dec, t_dec);
#endif
  } else {
    // ---- walker ----
    int i = 0, j = 0, status = 0, n_switch = 0, n_req = 0;
#ifdef MSA_TB_STATS
    long long n_run = 0, n_win = 0, t_win = 0, t_run = 0, t_wait = 0;  // diagnostic build
#endif
    const long long t_begin = (long long)__builtin_amdgcn_s_memtime();
    // (a two-pass SW plan whose pass-2 blocks folded the result into the best-cell key: no PairResult)
    const PairResult r0 = (!REF && best_key) ? best_key_decode(*best_key, pd.n) : res[pair];
    // plans hold m, n < 2^26
    i = REF ? pd.m : (int)r0.end_i;
    j = REF ? pd.n : (int)r0.end_j;
    // SW: 0 in H, 1 in E (horizontal gap), 2 in F (vertical gap); REF: 0, 1, 2 = T1, T2, T3
    int st = 0;
    if constexpr (REF) st = ref_end_state(r0.fin, end_type, hpen);
    int nw = 0, rseq = 0, eseq = 0;
    auto record = [&](unsigned w) __attribute__((always_inline)) {
      if ((nw & (TB_RAW / 2 - 1)) == 0 && nw >= TB_RAW) {
        // entering a ring half: its words of the previous lap must have been decoded
        for (int spin = 0; tb_u(ctl_s.consumed) < nw - TB_RAW / 2; ++spin)
          if (spin > TB_SPIN_MAX) { status = MSA_ERR_TIMEOUT; return; }
      }
      tb_st(rawl[nw & (TB_RAW - 1)], w);  // every lane stores the same word
      ++nw;
    };
    // the group of stripe s covering step t: published by the loader in ready[s & 3], or requested
    auto covers = [&](unsigned long long v, int s, int t) __attribute__((always_inline)) {
      const int vb = (int)(v >> 32);
      return (int)(unsigned)v == s && t >= 16 * vb && t < 16 * vb + GT;
    };
    auto need_group = [&](int s, int t) __attribute__((always_inline)) {
      unsigned long long v = tb_u64(ctl_s.ready[s & (NSLOT - 1)]);
      if (!covers(v, s, t)) {
#ifdef MSA_TB_STATS
        const long long a = (long long)__builtin_amdgcn_s_memtime();
#endif
        ++n_req;
        tb_st(ctl_s.req_s[s & 3], s);
        tb_st(ctl_s.req_t[s & 3], t);
        tb_st(ctl_s.req_seq[s & 3], ++rseq);  // (one counter: a channel's values still change on every request)
        for (int spin = 0; !covers(v, s, t); ++spin) {
          if (spin > TB_SPIN_MAX) { status = MSA_ERR_TIMEOUT; break; }
          v = tb_u64(ctl_s.ready[s & (NSLOT - 1)]);
        }
#ifdef MSA_TB_STATS
        t_wait += (long long)__builtin_amdgcn_s_memtime() - a;
#endif
      }
      asm volatile("" : : : "memory");  // (the group's bytes are read after its ready word)
      return (int)(v >> 32);
    };
    // Windows.  One LDS read gives lane (a, b) = (lane >> 3, lane & 7) the direction byte of
    // cell (i - a, j - b) -- (r - a, tg - a - b) in the group -- and the lane turns it into its
    // transition word (tb_word).  A step is then a v_readlane of the word at the walk's lane
    // index plus a few scalar ops; seven steps stay inside the 8 x 8 window.  A lane whose cell
    // lies outside the group or on the matrix border (i - a < 1 or j - b < 1) holds the FROZEN
    // word instead (every state: lane step 0, stay), so a window needs no step budget: a walk
    // that reaches such a cell stops there, and the next group takes over.
    // The byte of (rr, tt) sits at ((tt >> 4) << 10) | (rr << 4) | (tt & 15) of the group.
    // With u = tg & 15 and d = u - (a + b) in [-14, 15]: tt >> 4 = (tg >> 4) + (d >> 4) and
    // tt & 15 = d & 15, so the address is a uniform part plus d + 1008 (d >> 4) - 16a.
    const int wa = lane >> 3, wb = lane & 7;
    const int wc = wa + wb, wa16 = 16 * wa;
    constexpr unsigned FROZEN = (10u << 10) | (20u << 20) | (1u << 31);
    if (REF || r0.score > 0) {
      bool stopped = false;
      int s_cur = -1, cs = 0;
      // outer iteration: the walk entered a stripe, or left its group on the left
      while (i > 0 && j > 0 && !stopped && status == 0) {
        const int s = (i - 1) / SR;
        int r = (i - 1) - SR * s;  // row in the stripe (RL = 2: lane r >> 1, half r & 1)
        if (s != s_cur) {
          cs = cs_of(s);
          s_cur = s;
          ++n_switch;
          // tell the loader (its prefetch hint; it is done with stripe s + 1's slot)
          tb_st(ctl_s.ent_col, j - r);
          tb_st(ctl_s.ent_s, s);
          tb_st(ctl_s.ent_seq, ++eseq);
        }
        const int t = j - cs + (RL == 2 ? (r >> 1) : r);
        const int b0 = need_group(s, t);
        if (status != 0) break;
        const unsigned grp_lds = stage_lds + (unsigned)GBYTES * (unsigned)(s & (NSLOT - 1));
        int tg = t - 16 * b0;
#ifdef MSA_TB_STATS
        const long long tw0 = (long long)__builtin_amdgcn_s_memtime();
#endif
        int sh = 10 * st;
        for (;;) {
          if (sh == 0) {
#ifdef MSA_TB_STATS
            const long long tr0 = (long long)__builtin_amdgcn_s_memtime();
#endif
            // diagonal run: lane q reads cell (i - q, j - q) (inside the group and the matrix
            // for q <= qmax); the run is the number of leading lanes that continue diagonally
            // in state 0, the walk moves that many cells at once.  RL = 2: lane q also reads cell
            // q + 64 (a 128-row stripe in one run; both reads in flight together).
            constexpr int RUNMAX = 64 * RL;
            int q;
            if constexpr (RL == 2) {  // cell (i - q, j - q): step t - q - (r/2 - rr/2), 2 KiB blocks
              const int lim = min(min(r, i - 1), j - 1);
              unsigned long long bal[2];
#pragma unroll
              for (int h = 0; h < 2; ++h) {
                const int qq = lane + 64 * h, rr = r - qq;
                const int tt = tg - qq - ((r >> 1) - (rr >> 1));
                const bool valid = qq <= lim && tt >= 0;
                const unsigned go = (unsigned)(((tt >> 4) << 11) + ((rr & 1) << 10) + ((rr >> 1) << 4) + (tt & 15));
                const unsigned dv = *(const lds_u8*)(uintptr_t)(grp_lds + (valid ? go : 0u));
                bal[h] = __ballot(valid && tb_diag_stay<KIND>(dv));
              }
              // leading "diagonal, stay" cells
              q = ~bal[0] != 0ull ? (int)__builtin_ctzll(~bal[0])
                                  : 64 + (~bal[1] == 0ull ? 64 : (int)__builtin_ctzll(~bal[1]));
            } else {
              int qmax = r < (tg >> 1) ? r : (tg >> 1);
              qmax = qmax < i - 1 ? qmax : i - 1;
              qmax = qmax < j - 1 ? qmax : j - 1;
              const bool valid = lane <= qmax;
              const int tt = tg - 2 * lane, rr = r - lane;
              const unsigned go = (unsigned)(((tt >> 4) << 10) + (rr << 4) + (tt & 15));
              const unsigned dv = *(const lds_u8*)(uintptr_t)(grp_lds + (valid ? go : 0u));
              const unsigned long long bal = __ballot(valid && tb_diag_stay<KIND>(dv));
              q = ~bal == 0ull ? 64 : (int)__builtin_ctzll(~bal);  // leading "diagonal, stay" cells
            }
#ifdef MSA_TB_STATS
            ++n_run;
#endif
            if (q > 0) {
              record((15u << 28) | (unsigned)q);
              if constexpr (RL == 2) tg -= q + ((r >> 1) - ((r - q) >> 1));
              else tg -= 2 * q;
              r -= q;
              i -= q;
              j -= q;
#ifdef MSA_TB_STATS
              t_run += (long long)__builtin_amdgcn_s_memtime() - tr0;
#endif
              if (r < 0 || tg < 0 || i <= 0 || j <= 0) break;
              // every cell read continues: the one after them is unread -- another run, not a
              // window (round 6: a window of seven diagonal steps, ~1,000 ticks, followed the
              // first of the two 64-cell runs of every 128-row stripe)
              if (q == RUNMAX) continue;
            }
          }
          // a window of seven steps
          int wt;
          {
            unsigned ga;
            bool live;
            if constexpr (RL == 2) {  // lane (a, b): cell (i - a, j - b), row r - a, step tg - b - (r/2 - (r-a)/2)
              const int rr = r - wa, tt = tg - wb - ((r >> 1) - (rr >> 1));
              live = wa <= min(r, i - 1) && wb <= j - 1 && tt >= 0;
              ga = grp_lds + (live ? (unsigned)(((tt >> 4) << 11) + ((rr & 1) << 10) + ((rr >> 1) << 4) + (tt & 15)) : 0u);
            } else {
              const int d = (tg & 15) - wc;
              ga = grp_lds + (unsigned)(((tg >> 4) << 10) + (r << 4)) + (unsigned)(d + 1008 * (d >> 4) - wa16);
              live = wa <= min(r, i - 1) && wb <= j - 1 && wc <= tg;
            }
            const unsigned dv = *(const lds_u8*)(uintptr_t)ga;
            const unsigned w = tb_word<KIND>(dv);  // (evaluated for every lane: a select, no branch)
            wt = (int)(live ? w : FROZEN);
          }
          int idx = 0;
          unsigned wcode = 0;
          // seven steps, unrolled and branch-free: per step a v_readlane, a 64-bit shift (the
          // absorbing stop, tb_word), a bit-field extract, an add and the record
#pragma unroll
          for (int kk = 0; kk < 7; ++kk) {
            const unsigned long long w64 = (7ull << 32) | (unsigned)__builtin_amdgcn_readlane(wt, idx);
            const unsigned f = (unsigned)(w64 >> (sh & 63));
            const unsigned dl = (f >> 6) & 15u;
            sh = (int)f;
            idx += (int)dl;
            wcode = (wcode << 4) + dl;
          }
          sh &= 31;
          record(wcode | (7u << 28));
          const int da = idx >> 3, db = idx & 7;
          if constexpr (RL == 2) tg -= db + ((r >> 1) - ((r - da) >> 1));
          else tg -= da + db;
          r -= da;
          i -= da;
          j -= db;
#ifdef MSA_TB_STATS
          ++n_win;
#endif
          // stop; or the walk left the group (top row or left edge) or reached the border
          if (sh == 30 || r < 0 || tg < 0 || i <= 0 || j <= 0) break;
        }
#ifdef MSA_TB_STATS
        t_win += (long long)__builtin_amdgcn_s_memtime() - tw0;
#endif
        st = (sh == 30) ? 3 : sh / 10;
        if constexpr (REF) {
          // a cell without a predecessor table (cannot happen for a complete fill)
          if (st == 3) { status = -9; stopped = true; }  // MSA_ERR_NOMATCH
          // find_alignment stops at the matrix border (:147): the border cells' frozen words end
          // the walk exactly there
        } else if (st == 3) {  // local start (H came from 0): the walk ends at this cell
          st = 0;
          stopped = true;
        }
      }
    }
    tb_st(ctl_s.t_walk, (long long)__builtin_amdgcn_s_memtime() - t_begin);
    tb_st(ctl_s.wi, i);
    tb_st(ctl_s.wj, j);
    tb_st(ctl_s.wstatus, status);
    tb_st(ctl_s.n_switch, n_switch);
    tb_st(ctl_s.n_req, n_req);
#ifdef MSA_TB_STATS
    tb_st(ctl_s.wst[0], t_wait);
    tb_st(ctl_s.wst[1], n_run);
    tb_st(ctl_s.wst[2], n_win);
    tb_st(ctl_s.wst[3], t_win);
    tb_st(ctl_s.wst[4], t_run);
#endif
    tb_st(ctl_s.nw_total, nw);
    tb_st(ctl_s.done, 1);
  }
  __syncthreads();  // (waves 0 and 2 have left their loops: the ops are written, no load in flight)
  if (threadIdx.x == 0) {
    // info[0..3] (ops, begin, status) in every build: the callers check the status word
    const long long nops = ctl_s.nops;
    int status = ctl_s.wstatus;
    if (nops > cap && status == 0) status = -8;  // MSA_ERR_CAPACITY
    info[0] = nops;
    info[1] = ctl_s.wi + 1;
    info[2] = ctl_s.wj + 1;
    info[3] = status;
#ifdef MSA_TB_STATS
    // diagnostic build (scripts/tb_stats.py; the caller passes 18 words)
    info[4] = ctl_s.wst[0];
    info[5] = ctl_s.wst[1];
    info[6] = ctl_s.wst[2];
    info[7] = ctl_s.wst[3];
    info[8] = ctl_s.t_walk;
    info[9] = ctl_s.n_demand[0] + ctl_s.n_demand[1] + ctl_s.n_demand[2] + ctl_s.n_demand[3];
    info[10] = ctl_s.wst[4];
    info[11] = ctl_s.t_dec;
    info[12] = ctl_s.n_switch;
    info[13] = ctl_s.n_req;
    info[14] = ctl_s.lst[0];
    info[15] = ctl_s.lst[1];
    info[16] = ctl_s.lst[2];
    info[17] = ctl_s.lst[3];
#else
    info[4] = ctl_s.n_switch;
    info[5] = ctl_s.n_demand[0] + ctl_s.n_demand[1] + ctl_s.n_demand[2] + ctl_s.n_demand[3];  // groups staged on request (the first, mispredictions, walks leaving a group)
    info[6] = ctl_s.t_walk;    // s_memtime ticks, the walk's start to its last step
    info[7] = ctl_s.n_req;     // times the walker waited for the loader
#endif
  }
}

}  // namespace msa
