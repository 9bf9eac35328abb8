// msa_traceback.hip -- on-device traceback walks over direction bytes.
//
//  * SW affine (config C5): the fill (stripe_kernel, MSA_ALG_SWA, MSA_OUT_DIR)
//    leaves one byte per cell -- bits 0-1: where H came from (0 = local start,
//    1 = diagonal, 2 = E / horizontal gap, 3 = F / vertical gap); bit 2: E here
//    opened from H(i, j-1); bit 3: F here opened from H(i-1, j).  The walk is the
//    tie order of oracle orc_sw (first maximum), from the pair's end cell.
//  * Reference Gotoh (MSA_ALG_REF, MSA_OUT_DIR: main_alignment_function /
//    Subproblem::find_alignment, subproblem_alignment.cpp:105-172): bits 0-1 =
//    T1's predecessor table, 2-3 = T2's, 4-5 = T3's (1..3, the first table in
//    the reference's order T1, T2, T3 whose value reproduces the cell by exact
//    equality).  The walk starts at (m, n) in the end node's table (the
//    reference's end-type rule, :112-146, from the fill's final state) and stops
//    when i == 0 or j == 0 (:147).  One op per step = the table the step leaves
//    from ('M' T1 / diagonal, 'D' T2 / consumes B, 'I' T3 / consumes A); the host
//    turns them into the reference's align list (node coordinates, quirks Q1/Q2).
//
// Both layouts are the skewed stripe layout: cell (64s + r + 1, cs_s + t - r) at
// byte (s*pmax + t/16)*1024 + r*16 + t%16 of the pair's block -- a 16-step x
// 64-row block is 1 KiB, one 16-byte row segment per lane.
//
// One wave walks the path from the pair's end cell (read from the reduction's
// PairResult on the same stream, no host round trip).  Its state is uniform
// (SGPRs); the 4 KiB group of blocks under the walk sits in LDS and a step
// reads its byte there at a wave-uniform address.  While walking, the wave
// prefetches the group it will need next (the stripe above, at the column the
// path will leave through, or the group to the left, whichever boundary comes
// first) into a second staging buffer, so most group switches find their bytes
// already loaded.  Inside a group, one LDS read fetches an 8x8 window of bytes
// (one per lane) and up to 7 steps are resolved from it with v_readlane.
// Steps are recorded as nibbles, one word per window, in an LDS ring that is
// decoded into op bytes by the whole wave in parallel (no scalar-cache writes).
// Output: ops from the end cell back to the start ('M' diagonal, 'D' a gap
// consuming B, 'I' a gap consuming A), info = {n_ops, beg_i, beg_j, status,
// group switches, of them fetched on demand (mispredicted), s_memtime ticks of
// the walk, of them waiting for group loads}.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace msa {

// A "group" is 4 consecutive 16-step blocks of one stripe: steps [64g, 64g + 64)
// of all 64 rows, 4 KiB contiguous (blocks of a stripe are consecutive in
// memory).  Lane r holds its row's 64 bytes in 16 dwords; dword k covers steps
// 64g + 4k .. +3.  A diagonal step lowers t by 2 and r by 1, so a group serves
// ~32 diagonal steps and a 64-row stripe takes 1-3 groups.
// Group loads are LDS-DMA (global_load_lds_dwordx4: each lane's 16 bytes land
// at LDS base + 16 * lane, no VGPR destination) into the second of two 4 KiB
// staging buffers; the walk reads its byte from the current one.  They are
// issued as inline asm so that
// the compiler's wait-count pass does not see them -- it would otherwise drain
// them with vmcnt(0) in front of unrelated work.  At most one group load is in
// flight; it is waited for explicitly (s_waitcnt vmcnt(0), memory clobber, so
// the LDS reads that follow cannot move above it) before the staging buffer is
// read or refilled.  M0 is written in the same statement that uses it.
__device__ __forceinline__ void glds16(const uint8_t* gsrc, unsigned lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_dst)
               : "memory");
}
// Transitions of the walk (oracle orc_sw tie order), by state:
//  H: the low two bits hs of the byte -- 0 local start (stop), 1 diagonal ('M', stay in H),
//     2 from E (no op, go to E), 3 from F (no op, go to F);
//  E: 'D' (a gap consuming B), back to H if bit 2 (E opened from H(i, j-1)), else stay;
//  F: 'I' (a gap consuming A), back to H if bit 3 (F opened from H(i-1, j)), else stay.
// A transition field is (lane step: 9 M / 1 D / 8 I / 0 none) | (9 x next state, 27 = stop)
// << 4; TB_FH holds the four H fields at 16-bit spacing, indexed by hs.
constexpr unsigned long long TB_FH = (27ull << 4) | (9ull << 16) | ((9ull << 4) << 32) | ((18ull << 4) << 48);

__device__ __forceinline__ void vm_wait_all() { asm volatile("s_waitcnt vmcnt(0)" : : : "memory"); }

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

// The transition word of a cell (see the window comment in traceback_kernel): three 9-bit
// fields, field s = the lane step of leaving state s | 9 x the next state << 4 (27 = stop),
// and bit 31 set.  With bit 31 set and 13 as the high word of the 64-bit shift in a step, the
// stop state is absorbing: shifting by 27 yields lane step 0 and next state 27 again, so the
// steps after a stop are no-ops and a window needs no branch per step.
template <int KIND>
__device__ __forceinline__ unsigned tb_word(unsigned dv) {
  if constexpr (KIND == TB_REF_TAG) {
    // table s leaves by its fixed move (T1 diagonal 9, T2 left 1, T3 up 8) into table 4 - x, x
    // = the tag in bits 2s..2s+1: next state 9 x (3 - x), and x = 0 (no predecessor) gives 27
    // (stop) -- one formula, 27 - 9x, for every x.  The three 2-bit tags spread to 9-bit
    // spacing by one multiply (copies at bits 0, 7, 14 never overlap), then the word is
    // C - 144 x spread (each field 27 - 9x >= 0: no borrow between fields).
    constexpr unsigned C = 9u | (1u << 9) | (8u << 18) | (27u << 4) | (27u << 13) | (27u << 22) | (1u << 31);
    const unsigned sp = (dv * 0x4081u) & 0xC0603u;
    return C - 144u * sp;
  } else if constexpr (KIND == TB_REF) {
    // table numbers x = 1..3 (0: no predecessor): next state 9 (x - 1), or 27
    auto fld = [](unsigned step, unsigned x) { return step | ((x ? 9u * (x - 1u) : 27u) << 4); };
    return fld(9u, dv & 3u) | (fld(1u, (dv >> 2) & 3u) << 9) | (fld(8u, (dv >> 4) & 3u) << 18) | (1u << 31);
  } else {
    const unsigned fH = (unsigned)(TB_FH >> (16 * (dv & 3u))) & 0x1ffu;
    const unsigned fE = 1u | ((dv & 4u) ? 0u : (9u << 4));
    const unsigned fF = 8u | ((dv & 8u) ? 0u : (18u << 4));
    return fH | (fE << 9) | (fF << 18) | (1u << 31);
  }
}

// KIND TB_SW: Smith-Waterman affine walk; TB_REF / TB_REF_TAG: the reference's Gotoh walk
// (end_type, h: find_alignment's end rule).
template <int KIND>
__global__ __launch_bounds__(64) void traceback_kernel(const uint8_t* __restrict__ dir,
                                                       const msa_pair_desc* __restrict__ pairs,
                                                       const msa_stripe_meta* __restrict__ meta,
                                                       const PairResult* __restrict__ res, int pair, int end_type,
                                                       int hpen, uint8_t* __restrict__ ops, long long cap,
                                                       long long* __restrict__ info) {
  constexpr bool REF = KIND != TB_SW;
  const int lane = threadIdx.x;
  const msa_pair_desc pd = pairs[pair];
  const PairResult r0 = res[pair];
  const uint8_t* base = dir + pd.out_off + lane * 16;
  const int pmax = pd.pmax;
  // plans hold m, n < 2^26
  int i = REF ? pd.m : (int)r0.end_i, j = REF ? pd.n : (int)r0.end_j;
  int nops = 0;
  // SW: 0 in H, 1 in E (horizontal gap), 2 in F (vertical gap); REF: 0, 1, 2 = T1, T2, T3
  int st = 0;
  if constexpr (REF) st = ref_end_state(r0.fin, end_type, hpen);
  int status = 0;
  // current group / the one being fetched, behind a guard: a window lane whose cell lies
  // outside the group reads an unused byte (down to 1,136 B before a buffer), never another
  // variable (its word is never reached: the step budget keeps the walk inside the group)
  constexpr int TB_GUARD = 1280;
  __shared__ __attribute__((aligned(16))) uint8_t stage_raw[TB_GUARD + 2 * 4096];
  uint8_t (*stage)[4096] = reinterpret_cast<uint8_t (*)[4096]>(stage_raw + TB_GUARD);
  typedef __attribute__((address_space(3))) uint8_t lds_u8;
  const unsigned stage_lds = (unsigned)(uintptr_t)(lds_u8*)&stage[0][0];
  int cb = 0;  // stage[cb] holds the current group, stage[cb ^ 1] receives the next
  long long cur_key = -1, nxt_key = -1;  // s * 2^32 + g
  bool pend = false;                     // a group load into `stage` is in flight
  int s_cached = -1;
  int cs = 0, cs_up = 0;
  // every stripe's start column, staged in LDS once (a stripe change then costs an LDS
  // read, not a ~1 us dependent global load); pairs with more stripes read the rest from HBM
  constexpr int TB_CSL = 8192;
  __shared__ int csl[TB_CSL];
  const int S = (pd.m + 63) / 64;
  for (int k = lane; k < S && k < TB_CSL; k += 64) csl[k] = meta[pd.stripe0 + k].cs;
  auto cs_of = [&](int k) {  // wave-uniform (readfirstlane: an LDS value is otherwise "divergent")
    return k < TB_CSL ? __builtin_amdgcn_readfirstlane(csl[k]) : meta[pd.stripe0 + k].cs;
  };
  // The walk records, per window of <= 7 steps, one word: nibble k = the lane step of
  // step k (9 'M', 1 'D', 8 'I', 0 no op), steps in bits 28-31.  The words go to an LDS
  // ring (all lanes store the same word: no per-lane branch in the walk); when it is
  // full, and at the end, decode() turns them into op bytes in parallel (one word per
  // lane, a wave prefix sum of the op counts) and appends them to `ops`.
  constexpr int TB_RAW = 4096;
  __shared__ unsigned rawl[TB_RAW];
  int nw = 0;
  auto decode = [&]() {
    for (int b0 = 0; b0 < nw; b0 += 64) {
      const unsigned w = (b0 + lane < nw) ? rawl[b0 + lane] : 0u;
      const int k = (int)(w >> 28);
      int c = 0;
      for (int q = 0; q < k; ++q) c += ((w >> (4 * q)) & 15u) != 0u;
      int incl = c;  // inclusive prefix sum over the lanes
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(incl, off);
        if (lane >= off) incl += y;
      }
      long long o = nops + incl - c;
      for (int q = 0; q < k; ++q) {
        const unsigned dl = (w >> (4 * q)) & 15u;
        if (dl != 0u) {
          if (o < cap) ops[o] = dl == 9u ? 'M' : (dl == 1u ? 'D' : 'I');
          ++o;
        }
      }
      nops += __shfl(incl, 63);
    }
    nw = 0;
  };
  auto key_of = [](int s, int g) { return ((long long)s << 32) | (unsigned)g; };
  // issue the 4 block loads of group (s, g) into stage[cb ^ 1] (blocks past the stripe's
  // pmax are not loaded, so no read leaves the pair's direction bytes)
  auto issue_group = [&](int s, int g) {
    const long long blk0 = (long long)s * pmax + 4ll * g;
    const unsigned dst = stage_lds + 4096u * (unsigned)(cb ^ 1);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (4 * g + q < pmax) glds16(base + (blk0 + q) * 1024, dst + 1024u * q);
  };
  int n_switch = 0, n_sync = 0;               // group switches, of them fetched on demand
#ifdef MSA_TB_STATS
  long long n_outer = 0, n_win = 0, t_win = 0;  // diagnostic build: outer iterations, windows, ticks in windows
#endif
  long long t_wait = 0;  // diagnostic build: clock ticks spent waiting for group loads
  const long long t_begin = (long long)__builtin_amdgcn_s_memtime();
  auto timed_wait = [&]() {
#ifdef MSA_TB_STATS
    const long long a = (long long)__builtin_amdgcn_s_memtime();
    vm_wait_all();
    t_wait += (long long)__builtin_amdgcn_s_memtime() - a;
#else
    vm_wait_all();
#endif
  };
  if (REF || r0.score > 0) {
    bool stopped = false;
    // outer iteration: make the group under (i, j) current, keep the next one in flight,
    // then run the steps that provably stay inside the group without any further checks
    while (i > 0 && j > 0 && !stopped) {
      const int s = (i - 1) >> 6;
      int r = (i - 1) & 63;
      if (s != s_cached) {
        cs = cs_of(s);
        cs_up = s > 0 ? cs_of(s - 1) : 0;
        s_cached = s;
      }
      int t = j - cs + r;
      const int g = t >> 6;
      const long long key = key_of(s, g);
      if (key != cur_key) {
        ++n_switch;
        if (pend) {
          timed_wait();
          pend = false;
          if (key != nxt_key) issue_group(s, g), timed_wait(), ++n_sync;  // mispredicted: fetch now
        } else {
          issue_group(s, g);
          timed_wait();
          ++n_sync;
        }
        nxt_key = -1;
        cb ^= 1;  // the fetched group becomes current
        cur_key = key;
      }
      // steps that stay in this group (each lowers r by <= 1 and t by <= 2) and inside the
      // matrix (i and j drop by <= 1 per step)
      const int to_top = r + 1, to_left = ((t & 63) >> 1) + 1;
      int budget = to_top < to_left ? to_top : to_left;
      budget = budget < i ? budget : i;
      budget = budget < j ? budget : j;
      // prefetch the group the walk leaves into: the stripe above (at the column a
      // diagonal path exits through) if the top row comes first, else the group to the left
      long long want = -1;
      int ws = 0, wg = 0;
      if (to_top <= to_left) {
        const int tu = (j - r) - cs_up + 63;
        if (s > 0 && tu >= 0) {
          ws = s - 1;
          wg = tu >> 6;
          want = key_of(ws, wg);
        }
      } else if (g > 0) {
        ws = s;
        wg = g - 1;
        want = key_of(ws, wg);
      }
      if (want >= 0 && want != nxt_key && want != cur_key) {
        if (pend) timed_wait();  // stage[cb ^ 1] is about to be refilled
        issue_group(ws, wg);
        nxt_key = want;
        pend = true;
      }
      const int r_in = r, t_in = t;
      // The budget's steps run in windows of up to 7.  One LDS read gives lane (a, b) =
      // (lane >> 3, lane & 7) the direction byte of cell (i - a, j - b) -- (r - a, t - a - b) in
      // the group -- and the lane turns it into its transition word (tb_word).  A step is then
      // a v_readlane of the word at the walk's lane index plus a few scalar ops; seven steps
      // stay inside the 8 x 8 window, the budget keeps them inside the group.
      // The byte of (rr, tt) sits at ((tt >> 4) << 10) | (rr << 4) | (tt & 15) of the group.
      // With u = t & 15 and d = u - (a + b) in [-14, 15]: tt >> 4 = (t >> 4) + (d >> 4) and
      // tt & 15 = d & 15, so the address is a uniform part plus d + 1008 (d >> 4) - 16a (lanes
      // outside the group land in the guard or an unused byte, never reached).
      const unsigned grp_lds = stage_lds + 4096u * (unsigned)cb;
      const int wc = (lane >> 3) + (lane & 7), wa16 = 16 * (lane >> 3);
      bool stop = false;
#ifdef MSA_TB_STATS
      ++n_outer;
      const long long tw0 = (long long)__builtin_amdgcn_s_memtime();
#endif
      int sh = 9 * st;
      while (budget > 0 && !stop) {
        const int kmax = budget < 7 ? budget : 7;
        const int tg = t & 63;
        const int d = (tg & 15) - wc;
        const unsigned ga = grp_lds + (unsigned)(((tg >> 4) << 10) + (r << 4)) + (unsigned)(d + 1008 * (d >> 4) - wa16);
        const unsigned dv = *(const lds_u8*)(uintptr_t)ga;
        const int wt = (int)tb_word<KIND>(dv);
        int idx = 0, k = 0;
        unsigned wcode = 0;
        if (kmax == 7) {
          // a full window (the common case), unrolled and branch-free: per step a v_readlane,
          // a 64-bit shift (the absorbing stop, tb_word) and five scalar ops
#pragma unroll
          for (int kk = 0; kk < 7; ++kk) {
            const unsigned long long w64 = (13ull << 32) | (unsigned)__builtin_amdgcn_readlane(wt, idx);
            const unsigned f = (unsigned)(w64 >> sh);
            const unsigned dl = f & 15u;
            sh = (int)((f >> 4) & 31u);
            idx += (int)dl;
            wcode |= dl << (4 * kk);
          }
          k = 7;
        } else {
          for (; k < kmax; ++k) {
            const unsigned long long w64 = (13ull << 32) | (unsigned)__builtin_amdgcn_readlane(wt, idx);
            const unsigned f = (unsigned)(w64 >> sh);
            const unsigned dl = f & 15u;
            sh = (int)((f >> 4) & 31u);
            idx += (int)dl;
            wcode |= dl << (4 * k);
          }
        }
        stop = sh == 27;  // the steps after a stop recorded no-op nibbles
        rawl[nw] = wcode | ((unsigned)k << 28);  // every lane stores the same word
        if (++nw == TB_RAW) decode();
        const int da = idx >> 3, db = idx & 7;
        r -= da;
        t -= da + db;
        budget -= k;
#ifdef MSA_TB_STATS
        ++n_win;
#endif
      }
#ifdef MSA_TB_STATS
      t_win += (long long)__builtin_amdgcn_s_memtime() - tw0;
#endif
      st = stop ? 3 : sh / 9;
      i -= r_in - r;                  // rows consumed
      j -= (t_in - t) - (r_in - r);   // columns consumed
      if constexpr (REF) {
        // a cell without a predecessor table (cannot happen for a complete fill)
        if (st == 3) { status = -9; stopped = true; }  // MSA_ERR_NOMATCH
        // find_alignment stops at the matrix border (:147); the budget (<= min(i, j)) makes
        // a window end exactly there
      } else if (st == 3) {  // local start (H came from 0): the walk ends at this cell
        st = 0;
        stopped = true;
      }
    }
  }
  decode();  // the words still in the ring
  if (nops > cap && status == 0) status = -8;  // MSA_ERR_CAPACITY
  if (pend) vm_wait_all();  // no load left in flight when the wave ends
  if (lane == 0) {
    info[0] = nops;
    info[1] = i + 1;
    info[2] = j + 1;
    info[3] = status;
    info[4] = n_switch;
    info[5] = n_sync;
#ifdef MSA_TB_STATS
    info[3] = n_outer;
    info[5] = n_win;
    info[7] = t_win;
#endif
    info[6] = (long long)__builtin_amdgcn_s_memtime() - t_begin;  // s_memtime ticks, whole walk
#ifndef MSA_TB_STATS
    info[7] = t_wait;
#endif
  }
}

}  // namespace msa
