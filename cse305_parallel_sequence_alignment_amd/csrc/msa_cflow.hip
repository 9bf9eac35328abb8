// msa_cflow.hip -- score-only Smith-Waterman batches of packed pair couples (config C4: 1024 pairs of
// 4k x 4k, sharded over GPUs: one rank holds 128 pairs at 8 GPUs) as flag-synchronised stripe chains.
// Replaces, for this configuration, the reference's pair-level fan-out (testing.cpp:112-158,
// :269-280: one std::thread per pair, each a row sweep -- subproblem_alignment.cpp:329-332).
//
// stripe_kernel's batch mode runs a couple's 63 stripes in lock-step phases of 16 steps (one
// s_barrier per phase, 8 waves cycling over the couple's stripes).  Measured (stamps, 128 pairs):
// a phase takes ~1.0 us -- ~0.46 us issuing the 16 steps, the rest the barrier and the LDS round
// trip after it -- and a stripe starts ~5.3 phases after the one above it.  This kernel runs the
// flow kernels' pass-1 protocol instead (msa_flow.hip): no barrier, a producer's lane 63 writes
// each 16-column block of its bottom row to an LDS ring and bumps a phase counter, the consumer
// reads counter and block half a phase ahead; items of W stripes chain through {epoch, value}
// granules (the last link's bottom row, copied by the io-out wave).  Per DP step a compute wave
// issues for BOTH pairs of its couple (int16 halves):
//     up = DPP wave_shr:1 (lane r-1's G; lane 0: the row above),  s = v_perm (two profile bytes)
//     G  = max(max(G_diag + s, G_left), up)         G = H + g(i+j)   (v_pk_add_u16, 2 v_pk_max_i16)
//     pb = max(pb, G + (-g k))                      the phase's best of G - g k (2 packed ops)
// and once per phase best = max(best, pb - g(i+j) at the phase's step 0): no scalar arithmetic per
// step.  Items are claimed in ITEM-MAJOR order (every couple's first W stripes, then every couple's
// second, ...), so the fronts of all chains run at once and an item only ever waits on an earlier
// ticket (no deadlock whatever the residency); several workgroups share a CU (the chain waves of a
// small share leave most issue slots idle).
#pragma once

namespace msa {

#ifndef CF_W
#define CF_W 4    // compute waves (stripes) per item
#endif
#ifndef CF_WPE
#define CF_WPE 4  // waves per SIMD the register budget is sized for (128 VGPRs): three workgroups of W + 1 waves per CU
#endif

// Packed profile of one row (pair couple halves separately): score + 2g for codes 0..6, code 7 (the
// virtual column outside [1, n]) 2g: H = 0 left of column 1 (G = g(i+j) exactly) and never above a
// real cell right of n -- as stripe_kernel's MSA_ALG_SWLP.
__device__ __forceinline__ void cf_profile(int match, int mismatch, int g, unsigned ac, unsigned& plo, unsigned& phi) {
  const int sm = match + 2 * g, sx = mismatch + 2 * g;
  const unsigned bx = (unsigned)(sx & 0xff) * 0x01010101u;
  unsigned lo = bx, hi = bx;
  const unsigned bm = (unsigned)(sm & 0xff);
  if (ac < 4) lo = (lo & ~(0xffu << (8 * ac))) | (bm << (8 * ac));
  else hi = (hi & ~(0xffu << (8 * (ac - 4)))) | (bm << (8 * (ac - 4)));
  hi = (hi & 0x00ffffffu) | ((unsigned)((2 * g) & 0xff) << 24);
  plo = lo;
  phi = hi;
}

// Diagnostic build (-DMSA_STAMPS): couples 0..3 record, per item (group < 16) and compute wave,
// stamps[((cpl * 16 + grp) * 16 + w) * 4096 * 4 + slot]: 0 s_memrealtime at the stripe's start (its
// phase-0 inputs landed), 1 at its end, 2 phases that waited on the producer, 3 s_memtime ticks spent
// waiting on the producer; [+4] ticks waiting on the consumer, [+5] the item's claim time (io-in)
#ifdef MSA_STAMPS
#define CF_STAMP(w_, slot_, v_)                                                                  \
  do {                                                                                           \
    if (a.stamps && lane == 0 && cpl < 4 && grp < 16)                                            \
      a.stamps[(((size_t)(cpl * 16 + grp) * 16 + (w_)) * 4096) * 4 + (slot_)] = (v_);            \
  } while (0)
#else
#define CF_STAMP(w_, slot_, v_) do {} while (0)
#endif

template <int W>
__global__ __launch_bounds__((W + 1) * 64) __attribute__((amdgpu_waves_per_eu(CF_WPE, 8))) void cflow_kernel(KArgs a) {
  constexpr int NCP = FL_NCOPY;
  constexpr int PKNEG = (int)0x80008000u;  // -32768 in both halves: "-inf" of a packed value
  extern __shared__ __attribute__((aligned(16))) int smem[];
  const msa_kparams& kp = a.kp;
  const int lane = threadIdx.x & 63;
  const int w = uni(threadIdx.x >> 6);
  // flags: [0] item; prog[l] 32+l (l = 0: io-in's published blocks, l = c+1: compute wave c's
  // finished phases); [64+W] io-out's taken blocks of the last link; dummy sink 96..127
  int* flags = smem;
  int* rings = smem + FL_FLAGS;                                         // [W+1 links][256]
  uint8_t* codes = reinterpret_cast<uint8_t*>(rings + (W + 1) * 256);  // [NCP][cstr] whole rows
  const int L8 = kp.lds_code_bytes;
  const int cstr = L8 + 16;
  const int g = kp.gap_ext;
  const unsigned ep = kp.epoch;
  const int ncpl = (kp.n_pairs + 1) / 2;  // couples (an odd count repeats its last pair in the high halves)
  // io-in: the code segment whose whole rows the LDS copies hold (C4's couples share one column
  // sequence: a workgroup loads it once, not per item -- ~2.5 us of an item's start)
  long long res_cod = -1;
  int res_Yr = 0;  // bytes [0, res_Yr) of every copy's code row of segment res_cod are in LDS

  for (;;) {
    if (threadIdx.x == 0) flags[0] = atomicAdd(a.ticket, 1);
    if (threadIdx.x >= 16 && threadIdx.x < 128) flags[threadIdx.x] = 0;
    __syncthreads();
    const int item = uni(flags[0]);
    if (item >= kp.n_items) break;
    // item-major: item = group * ncpl + couple; the item above is item - ncpl (same couple)
    const int grp = item / ncpl;
    const int cpl = item - grp * ncpl;
    const msa_pair_desc pd = a.pairs[2 * cpl];
    const msa_pair_desc pd1 = a.pairs[min(2 * cpl + 1, kp.n_pairs - 1)];
    const int m = pd.m, n = pd.n;
    const int S = (m + 63) / 64;
    const int k0 = grp * W;
    if (k0 >= S) {  // a shorter couple than the launch's longest: nothing here, nobody waits on it
      __syncthreads();
      continue;
    }
    unsigned long long* const g_out = a.gbuf + (size_t)item * a.gbuf_stride;
    const unsigned long long* const g_in = a.gbuf + (size_t)(grp > 0 ? item - ncpl : 0) * a.gbuf_stride;

    if (w == W) {
      // =================== io wave ===================
      // in: codes + the row above stripe k0 (row 0, or item - ncpl's granules) -> link 0's ring
      // out: the last link's blocks -> granules for item + ncpl.  One wave does both (a workgroup is
      // W + 1 waves: three fit a CU at 128 VGPRs), issuing a round's granule polls, then copying the
      // out blocks while the polls fly.
      int* ring = rings;
      int* pub = flags + 32;
      const int* cons = flags + 33;  // compute wave 0's finished phases = blocks it no longer needs
      const int cs_c = fl_cs(k0);
      const int Pc = fl_P(k0, m, n);
      const int Bmax = (k0 == 0) ? Pc - 1 : min(Pc - 1, fl_bmax(k0, m, n));
      const int kc = k0 + W;  // the next item's first stripe (consumer of the last link)
      const int bmx = (kc < S) ? fl_bmax(kc, m, n) : -1;
      const int cs_o = fl_cs(kc);
      const uint8_t* gcod = a.cod + pd.cod_off;
      // bytes [0, Yr) of every copy's code row are in LDS: what the previous item of this workgroup
      // loaded when it had the same column segment (carried, not assumed whole: an item loads only the
      // prefix its blocks need)
      int Yr = (pd.cod_off == res_cod) ? res_Yr : 0;
      res_cod = pd.cod_off;
      auto load_codes = [&](int Y1) __attribute__((always_inline)) {
        Y1 = min(Y1, L8);
        if (Y1 <= Yr) return;
        const int tot = NCP * ((Y1 - Yr) / 16);  // 16-byte chunks over all copies
        for (int c0 = 0; c0 < tot; c0 += 4 * 64) {  // 4 loads in flight per lane
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
            if (c < tot) *(lds_int4*)(codes + x * cstr + y) = fl_v4i{v[r].x, v[r].y, v[r].z, v[r].w};
          }
        }
        Yr = uni(max(Yr, Y1));
      };
      CF_STAMP(w, 5, __builtin_amdgcn_s_memrealtime());
      int b = 0, bl = 0;
      load_codes(1024);
      int consv = 0;
      unsigned spins = 0;
      while (b <= Bmax || bl <= bmx) {
        bool prog = false;
        // ---- in: poll the next round's granules (up to 16 blocks; lane l, load r -> block b + 4r + l/16)
        unsigned long long gv[4];
        const bool in_act = b <= Bmax;
        if (in_act) {
          if (Yr < L8 && Yr < 16 * b + 768) load_codes(Yr + 1024);
          if (k0 > 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int col = cs_c + 16 * b + 64 * r + lane;
              gv[r] = gload(g_in + min(max(col + MSA_GOFF, 0), a.gbuf_stride - 1));
            }
          }
        }
        // ---- out: up to 4 blocks of the last link (while the polls fly)
        if (bl <= bmx) {
          const int avail = min(uni(lds_vload(flags + 32 + W)) - fl_dq(kc), bmx + 1);
          FL_CBAR();
          if (avail > bl) {
            const int nbo = min(4, avail - bl);
            const int j = lane >> 4, c = lane & 15;
            const int blk = bl + min(j, nbo - 1);  // (lanes past nbo repeat the last block: no exec branch)
            const int v = *(const lds_int*)(rings + W * 256 + (blk & (FL_RINGB - 1)) * 16 + c);
            const int col = cs_o + 16 * blk + c;
            if (col + MSA_GOFF >= 0 && col + MSA_GOFF < a.gbuf_stride)
              gstore(g_out + col + MSA_GOFF, ((unsigned long long)ep << 32) | (unsigned)v);
            bl += nbo;
            FL_CBAR();
            if (lane == 0) lds_vstore(flags + 64 + W, bl);
            prog = true;
          }
        }
        // ---- in: publish the landed prefix of the round
        if (in_act) {
          int val[4];
          int nb = 0;
          if (k0 == 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r) val[r] = pk2(g * (cs_c + 16 * b + 64 * r + lane));  // row 0: H = 0
            nb = min(16, Bmax - b + 1);
          } else {
            bool run = true;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              val[r] = (int)(unsigned)gv[r];
              const int blk = b + 4 * r + (lane >> 4);
              const unsigned long long bal = __ballot((blk > Bmax) || ((unsigned)(gv[r] >> 32) == ep));
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
          // codes for the blocks' phases must be in LDS before they are published
          if (Yr < L8 && Yr < 16 * (b + nb) + 192) {
            load_codes(16 * (b + nb) + 1024);
            if (Yr < L8) nb = min(nb, (Yr - 192) / 16 - b);
          }
          if (nb > 0) {
            // (every lane stores: blocks past b + nb go to the sink, so no exec-masked branch sits in
            // the wait loop)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int blk = b + 4 * r + (lane >> 4);
              int* dst = (blk < b + nb) ? ring + (blk & (FL_RINGB - 1)) * 16 : flags + 96;
              *L(dst + (lane & 15)) = val[r];
            }
            FL_CBAR();
            if (lane == 0) lds_vstore(pub, b + nb);
            b += nb;
            prog = true;
          }
        }
        if (!prog) {
          // (granule polls pace themselves: the sleep only when nothing was polled this round)
          if (!in_act || k0 == 0 || consv + FL_RINGB <= b) __builtin_amdgcn_s_sleep(FL_IOSLEEP);
          if (++spins > FL_SPIN_MAX) break;
        }
      }
      // (after the loop: a wave-uniform wait loop -- tests/test_host.py::test_wait_loops_are_wave_uniform)
      if ((b <= Bmax || bl <= bmx) && lane == 0) atomicExch(a.err, 20);
      res_Yr = Yr;
    } else if (k0 + w < S) {
      // =================== compute wave: stripe k of the couple ===================
      const int k = k0 + w;
      const int cs = fl_cs(k);
      const int P = fl_P(k, m, n);
      const int row_i = 64 * k + lane + 1;
      const unsigned ac = (row_i <= m) ? (a.A[pd.a_off + row_i - 1] & 7u) : 0u;
      const unsigned ac2 = (row_i <= m) ? (a.A[pd1.a_off + row_i - 1] & 7u) : 0u;
      const bool has_out = (k < S - 1);
      const int Bin = (k == 0) ? P - 1 : min(P - 1, fl_bmax(k, m, n));
      const int dq_in = (w == 0) ? 0 : fl_dq(k);  // producer's counter counts phases (io-in: blocks)
      const int dq = has_out ? fl_dq(k + 1) : 0;  // phase q writes out block q - dq
      const unsigned a_ring_in = lds_addr(rings + w * 256);
      const unsigned a_prog_in = lds_addr(flags + 32 + w);
      const unsigned a_ring_out = lds_addr(rings + (w + 1) * 256);
      const unsigned a_prog_me = lds_addr(flags + 32 + w + 1);
      // out-ring consumer: the next compute wave, or io-out for the last link
      const unsigned a_cons = lds_addr(w + 1 < W ? flags + 32 + w + 2 : flags + 64 + W);
      const unsigned a_dummy = lds_addr(flags + 96 + 8 * (w & 1));  // sink for a phase with nothing to hand off
      unsigned plo, phi, plo2, phi2;
      cf_profile(kp.match, kp.mismatch, g, ac, plo, phi);
      cf_profile(kp.match, kp.mismatch, g, ac2, plo2, phi2);
      unsigned a_cring, y_code;
      {
        const int c0 = cs - lane + FL_OFF;
        const int x = c0 & (NCP - 1);
        a_cring = lds_addr(reinterpret_cast<int*>(codes + x * cstr));
        y_code = (unsigned)(c0 - x);
      }
      // H = G - g(i+j), i+j = 64k + 1 + cs + t for every lane of step t: per step the phase's best of
      // G - g kx (gk: SGPR constants), per phase minus g(i+j) at its step 0
      const int negct0 = -g * (64 * k + 1 + cs);
      int gk[16];  // pk2(-g k); only k = 1, 2, 4, 8 are used (the tree's level offsets)
#pragma unroll
      for (int kx = 0; kx < 16; ++kx) {
        gk[kx] = pk2(-g * kx);
        if (kx == 1 || kx == 2 || kx == 4 || kx == 8) asm("" : "+s"(gk[kx]));
      }
      // left neighbour and diagonal at step 0: virtual cells, H = 0 (G = g(i+j))
      int X = pk2(g * (64 * k + cs));
      int U = pk2(g * (64 * k + cs - 1));
      int best = 0;
      int pubv = 0, consv = 0;
      unsigned spins = 0;
      bool stuck = false;
      fl_v4i INa[4], INb[4];
      fl_v4u CWa, CWb;
      const unsigned long long m63 = 1ull << 63;
      auto issue_reads = [&](int q, fl_v4i (&IN)[4], fl_v4u& CW, int& pubn) __attribute__((always_inline)) {
        const unsigned ra = a_ring_in + (unsigned)((q & (FL_RINGB - 1)) * 64);
        pubn = ds_read_b32(a_prog_in);
        IN[0] = ds_read_b128<0>(ra);
        IN[1] = ds_read_b128<16>(ra);
        IN[2] = ds_read_b128<32>(ra);
        IN[3] = ds_read_b128<48>(ra);
        CW = ds_read2_b64(a_cring + y_code + 16u * (unsigned)q);
      };
      auto reread_in = [&](int q, fl_v4i (&IN)[4]) __attribute__((always_inline)) {
        ds_reread_b128x4(a_ring_in + (unsigned)((q & (FL_RINGB - 1)) * 64), IN);
      };
#ifdef MSA_STAMPS
      unsigned long long tw_in = 0, tw_cons = 0;
      int nslow = 0;
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
        stuck = stuck || val < need;  // (reported after the stripe: no divergent store in a wait loop)
#ifdef MSA_STAMPS
        tw_in += __builtin_amdgcn_s_memtime() - t0;
#endif
      };
      auto refresh_cons = [&](int need) __attribute__((always_inline)) {
#ifdef MSA_STAMPS
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#endif
        while (consv < need) {
          int c1 = ds_read_b32(a_cons);
          lgkm_wait<0>(c1);
          consv = uni(c1);
          if (consv < need) {
            __builtin_amdgcn_s_sleep(0);
            if (++spins > FL_SPIN_MAX) break;
          }
        }
        stuck = stuck || consv < need;
#ifdef MSA_STAMPS
        tw_cons += __builtin_amdgcn_s_memtime() - t0;
#endif
      };
      auto mask_in = [&](int q, fl_v4i (&IN)[4]) __attribute__((always_inline)) {
        if (q > Bin) {  // past the producer's last column (all > n)
#pragma unroll
          for (int u = 0; u < 4; ++u) IN[u] = fl_v4i{PKNEG, PKNEG, PKNEG, PKNEG};
        }
      };
      wait_flag(a_prog_in, pubv, min(1, Bin + 1) + dq_in);
      {
        int pub0;
        issue_reads(0, INa, CWa, pub0);
        lgkm_wait_v<0>(INa, CWa);
        lgkm_wait<0>(pub0);
        mask_in(0, INa);
      }
      CF_STAMP(w, 0, __builtin_amdgcn_s_memrealtime());
#ifdef MSA_STAMPS
      tw_in = 0;
#endif
      auto run_phase = [&](const int q, fl_v4i (&IN)[4], fl_v4u& CW, fl_v4i (&INn)[4], fl_v4u& CWn, auto MASK_)
          __attribute__((always_inline)) {
        constexpr bool MASK = decltype(MASK_)::value;  // phase q+1 may lie past the producer's last block
        const int need = MASK ? min(q + 1, Bin + 1) : q + 1;
        if (__builtin_expect(pubv - dq_in < need, 0)) {
#ifdef MSA_STAMPS
          ++nslow;
#endif
          wait_flag(a_prog_in, pubv, need + dq_in);
          reread_in(q, IN);
          if constexpr (MASK) mask_in(q, IN);
        }
        int xo[16];
        int pubn = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const unsigned s4 = __builtin_amdgcn_perm(phi, plo, CW[u]);
          const unsigned s4b = __builtin_amdgcn_perm(phi2, plo2, CW[u]);
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) {
            const int kx = 4 * u + kk;
            if (kx == FL_PF) issue_reads(q + 1, INn, CWn, pubn);  // prefetch phase q+1 (6 DS ops)
            // both pairs' score + 2g as int16: {s4 byte kk, 0, s4b byte kk, 0}
            const int s = (int)__builtin_amdgcn_perm(s4b, s4, 0x0c000c00u | ((4u + kk) << 16) | (unsigned)kk);
            // diagonal and left first (no wait on this step's DPP), then the cell above.  The DPP goes
            // through the intrinsic, not inline asm: gfx950 needs 2 wait states between the VALU write
            // of X and the DPP's read, and only the compiler's hazard recognizer pads (or schedules)
            // for them -- round 5's asm DPP read X one instruction after the write at 47 sites
            // (tests/test_host.py::test_dpp_reads_have_their_wait_states).  `old` = the ring value, so
            // lane 0 takes the row above and the DPP writes in place (no copy: 113 VGPRs as before)
            const int dl = pk_max(pk_add(U, s), X);
            const int up = dpp_shr1(IN[u][kk], X);
            X = pk_max(dl, up);
            U = up;
            xo[kx] = X;
          }
        }
        // the phase's best of both pairs' H: max over k of G_k - g k as a tree (four levels of
        // independent ops, no serial chain), minus g(i+j) at step 0
        {
          int r8[8], r4[4], r2[2];
#pragma unroll
          for (int j = 0; j < 8; ++j) r8[j] = pk_max(xo[2 * j], pk_add(xo[2 * j + 1], gk[1]));
#pragma unroll
          for (int j = 0; j < 4; ++j) r4[j] = pk_max(r8[2 * j], pk_add(r8[2 * j + 1], gk[2]));
#pragma unroll
          for (int j = 0; j < 2; ++j) r2[j] = pk_max(r4[2 * j], pk_add(r4[2 * j + 1], gk[4]));
          const int r1 = pk_max(r2[0], pk_add(r2[1], gk[8]));
          best = pk_max(best, pk_add(r1, pk2(negct0 - 16 * g * q)));
        }
        lgkm_wait<5>(pubn);  // the counter read (oldest of the six) has landed
        pubv = uni(pubn);
        // hand-off: lane 63's 16 values of this phase = block q - dq of the out ring
        const int bq = q - dq;
        const bool wr = has_out && bq >= 0;
        if (__builtin_expect(wr && consv < bq - (FL_RINGB - 1), 0)) refresh_cons(bq - (FL_RINGB - 1));
        const unsigned wa = wr ? a_ring_out + (unsigned)((bq & (FL_RINGB - 1)) * 64) : a_dummy;
        ds_handoff_tid(m63, wa - 252u, xo, a_prog_me, q + 1);
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
      if (stuck && lane == 0) atomicExch(a.err, 22);
      CF_STAMP(w, 1, __builtin_amdgcn_s_memrealtime());
#ifdef MSA_STAMPS
      CF_STAMP(w, 2, (unsigned long long)nslow);
      CF_STAMP(w, 3, tw_in);
      CF_STAMP(w, 4, tw_cons);
#endif
      // ---- stripe finalize: each half separately (pair 2c: low halves, 2c+1: high) ----
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const int bv = half ? (best >> 16) : (int)(short)(best & 0xffff);
        int bb = (row_i <= m) ? bv : INT32_MIN;
        int bi = row_i;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
          const int ob = __shfl_xor(bb, off);
          const int oi = __shfl_xor(bi, off);
          if (ob > bb || (ob == bb && oi < bi)) { bb = ob; bi = oi; }
        }
        if (lane == 0) {
          msa_stripe_meta* md = a.meta + (half ? pd1.stripe0 : pd.stripe0) + k;
          md->best = bb;
          md->best_i = bi;
          md->best_j = -1;
          md->cs = cs;
          md->phases = P;
        }
      }
    }
    __syncthreads();
  }
}

}  // namespace msa
