// msa_band.hip -- one banded pair (config C3: ~100k x 100k, band 512, int32 H written): the
// reference's Gotoh recurrence restricted to |i - j| <= band (MSA_ALG_NWA, msa_kernels.hip;
// subproblem_alignment.cpp:396-398 per cell) as flag-synchronised stripe chains.
//
// A workgroup = 4 compute waves (one 64-row stripe each, one per SIMD) + 1 io wave and runs one
// ITEM: 4 consecutive stripes.  Stripe k's lane r holds row 64k+r+1 and at step t column
// cs_k + t - r, with stripe_kernel's banded geometry (stripe_geom: cs_k = the band's first column
// rounded so that cs_k = k (mod 16); a stripe sweeps ~(2 band + 64) / 16 phases of 16 steps), so
// the stripe_kernel cell layout, meta and checksum hold unchanged.  One producer phase is one
// consumer block of 16 columns (producer phase q -> block q - dq_k, dq_k = 4 - (cs_{k-1} + 1 -
// cs_k) / 16: 7 or 8 for a band, the 64-column shift between stripes).
//   * inside an item: lane 63 hands its phase's 16 (Z, F~) values to the next wave's LDS ring
//     and bumps its counter (msa_flow.hip's affine hand-off); no s_barrier anywhere;
//   * between items: the io wave stages the row above the item's first stripe (row 0, a guessed
//     row, or the previous item's {epoch, value} granules) and stores the item's last row as
//     granules for the next item (and, chunked, as checkpoint rows);
//   * column codes: the item's column span in 4 byte-shifted LDS copies (two ds_read2_b32 per
//     lane per phase).
// Values are shifted by g(i+j) (g = gap extension, h = gap open - extension), which takes the
// extension out of the recurrence:
//     F~(i,j) = max(Z(i-1,j), F~(i-1,j)),  E~(i,j) = max(Z(i,j-1), E~(i,j-1)),
//     H~(i,j) = max(Z(i-1,j-1) + f + 2g + h, E~, F~),  Z = H~ - h,   H = H~ - g(i+j)
// (T3 = F, T2 = E; f = 1 on a match, else 0).  Band edges as stripe_kernel's band_fix: a lane
// runs the bare recurrence on every step, also outside its row's band; those values reach an
// in-band cell only through two cells, fixed up in the head / tail phases: at column jlo - 1 the
// state becomes the left border (column 0 for rows <= band, else -inf), at column jhi + 1 Z and
// F~ become -inf (the up value of the row below's last in-band cell and of the next stripe).
// Launch modes: exact (kp.single == 1): items = the pair's stripes in groups of 4, each item
// waiting on the previous one's granules; chunked (kp.single == 2, rank convergence as in
// msa_kernels.hip): chunk c outputs stripes [c C, (c+1) C) and starts chunk_warm stripes earlier
// from a guessed row; its items (kp.groups slots) chain through granules, its warm-up stripes
// write no cells, and the io wave saves the warm-up's last row and the chunk's last row into the
// checkpoint buffer for chunk_check_kernel / chunk_add_kernel.
#pragma once

namespace msa {

#define BK_W 4                 // compute waves per workgroup (one stripe each)
#define BK_NCOPY 4             // LDS code copies (4-byte aligned 16-code reads)
#define BK_LINKS (BK_W + 1)    // rings: 0 io -> wave 0, w+1: wave w -> w+1, BK_W: last stripe -> io

__host__ __device__ inline void bk_geom(int k, int m, int n, int band, int& cs, int& P) {
  StripeGeom g;
  stripe_geom(k, m, n, band, g, 16);
  cs = g.cs;
  P = g.P;
}
// link kc-1 -> kc: producer phase q writes consumer block q - bk_dq(kc); its last block bk_bmax(kc)
__host__ __device__ inline int bk_dq(int kc, int m, int n, int band) {
  int cp, Pp, cc, Pc;
  bk_geom(kc - 1, m, n, band, cp, Pp);
  bk_geom(kc, m, n, band, cc, Pc);
  return 4 - (cp + 1 - cc) / 16;  // (the difference is a multiple of 16)
}
__host__ __device__ inline int bk_bmax(int kc, int m, int n, int band) {
  int cp, Pp;
  bk_geom(kc - 1, m, n, band, cp, Pp);
  return Pp - 1 - bk_dq(kc, m, n, band);
}
// bytes per LDS code copy for an item (its 4 stripes' columns, one phase of prefetch past the last)
__host__ inline int bk_code_bytes(int m, int n, int band) {
  // lane r of stripe k reads bytes cs_k - r + FL_OFF - colbase + 16 q + [0, 16) (colbase = the item's
  // first cs rounded down to 16), q <= P_k (the prefetch one phase past the last)
  const int S = (m + 63) / 64;
  int mx = 0;
  for (int k0 = 0; k0 < S; k0 += BK_W) {
    int c0, P0;
    bk_geom(k0, m, n, band, c0, P0);
    for (int k = k0; k < std::min(S, k0 + BK_W); ++k) {
      int ck, Pk;
      bk_geom(k, m, n, band, ck, Pk);
      mx = std::max(mx, ck - (c0 & ~15) + FL_OFF + 16 * Pk + 16);
    }
  }
  return (mx + 16 + 15) & ~15;
}
__host__ __device__ inline size_t bk_lds_bytes(int code_bytes) {
  return (size_t)(FL_FLAGS + BK_LINKS * 512) * 4 + (size_t)BK_NCOPY * code_bytes;
}

__global__ __launch_bounds__((BK_W + 1) * 64) void band_kernel(KArgs a) {
  extern __shared__ __attribute__((aligned(16))) int smem[];
  const msa_kparams& kp = a.kp;
  const int lane = threadIdx.x & 63;
  const int w = uni(threadIdx.x >> 6);
  constexpr int W = BK_W;
  // the exact launch queued behind a chunked run: nothing to do when every chunk converged
  if (a.skip && uni(*(volatile const int*)a.skip)) return;
  // flags: [0] item; [32] io's published blocks (ring 0); [33 + w] compute wave w's finished
  // phases; [64] io's stored output blocks (ring W's consumer); 96.. sink
  int* flags = smem;
  int* rings = smem + FL_FLAGS;  // [BK_LINKS][Z 256 | F~ 256]
  uint8_t* codes = reinterpret_cast<uint8_t*>(rings + BK_LINKS * 512);  // [BK_NCOPY][L8]
  const int L8 = kp.lds_code_bytes;
  const msa_pair_desc pd = a.pairs[0];
  const int m = pd.m, n = pd.n;
  const int S = (m + 63) / 64;
  const int band = kp.band, g = kp.gap_ext, hh = kp.h;
  const unsigned ep = kp.epoch;
  const bool chunked = kp.single == 2;
  const int C = chunked ? kp.chunk_c : S;
  const int Wm = chunked ? kp.chunk_warm : 0;
  const int IPC = kp.groups;  // item slots per chunk
  const int nch = (S + C - 1) / C;
  const int seg = ((n + 2 * MSA_CPAD) + 63) & ~63;  // bytes of the staged code copies of this pair

  for (;;) {
    if (threadIdx.x == 0) flags[0] = atomicAdd(a.ticket, 1);
    if (threadIdx.x >= 16 && threadIdx.x < 128) flags[threadIdx.x] = 0;
    __syncthreads();
    const int item = uni(flags[0]);
    if (item >= kp.n_items) break;
    // chunked: tickets go item-major (every chunk's item 0, then every chunk's item 1, ...): the
    // resident workgroups run the front of every chunk's chain at once, and an item only waits on a
    // smaller ticket (its chunk's previous item)
    const int c = chunked ? item % nch : item / IPC, j = chunked ? item / nch : item - c * IPC;
    const int ks0 = c * C, ke = min(S, ks0 + C);
    int kb = ks0 - Wm;
    if (kb < 0 || kb * 64 <= band + 64) kb = 0;  // a warm-up reaching the border starts at row 0, exactly
    const int k0 = kb + W * j;
    const int ns = min(W, ke - k0);
    if (ns <= 0) {  // an empty slot (a chunk near the start has a shorter warm-up)
      __syncthreads();
      continue;
    }
    const bool guessed = (j == 0 && kb > 0);  // the item starts from a guessed row (chunked)
    int cs0, P0;
    bk_geom(k0, m, n, band, cs0, P0);
    const int colbase = cs0 & ~15;
    {
      // the item's column codes -> LDS: copy x byte y = column colbase + y + x - FL_OFF
      // (= staged copy x, byte colbase + y + 160)
      const uint8_t* gcod = a.cod + pd.cod_off;
      const int per = L8 / 16;
      for (int t = threadIdx.x; t < BK_NCOPY * per; t += (W + 1) * 64) {
        const int x = t / per, y = 16 * (t - x * per);
        const int b = colbase + y + MSA_CPAD - 1 - FL_OFF;
        if (b >= 0 && b + 16 <= seg) {
          const int4 v = *reinterpret_cast<const int4*>(gcod + (size_t)x * a.cod_copy + b);
          *(lds_int4*)(codes + x * L8 + y) = fl_v4i{v.x, v.y, v.z, v.w};
        }
      }
    }
    __syncthreads();

    if (w == W) {
      // =================== io: row above the item in, its last row out ===================
      const int Bmax = (k0 == 0 || guessed) ? P0 - 1 : min(P0 - 1, bk_bmax(k0, m, n, band));
      // granule slots are chunk-major (slot c IPC + j), whatever the ticket order
      const int slot = c * IPC + j;
      const unsigned long long* g_in = a.gbuf + (size_t)(slot > 0 ? slot - 1 : 0) * 2 * a.gbuf_stride;
      const int r0 = 64 * k0;  // the row above the item
      const int kl = k0 + ns - 1;
      const bool gnext = k0 + W < ke;  // another item of this chunk follows
      const int ckslot = !chunked ? -1 : (kl == ks0 - 1 ? 2 * c : ((kl == ke - 1 && c < nch - 1) ? 2 * c + 1 : -1));
      const bool oout = gnext || ckslot >= 0;  // (then the item is full: its last wave is W - 1)
      const int obmax = oout ? bk_bmax(kl + 1, m, n, band) : -1;
      const int odq = oout ? bk_dq(kl + 1, m, n, band) : 0;
      int csn = 0, Pn = 0;
      if (oout) bk_geom(kl + 1, m, n, band, csn, Pn);
      const int ro = 64 * (kl + 1);  // the row the item hands on
      unsigned long long* g_out = a.gbuf + (size_t)slot * 2 * a.gbuf_stride;
      int b = 0, ob = 0, consv = 0;
      unsigned spins = 0;
      // (the loop's condition, progress counters and idle test are explicitly wave-uniform: with the
      // phase code's per-kind instantiations the compiler turned this loop's back-edge exec-masked --
      // tests/test_host.py::test_wait_loops_are_wave_uniform)
      while (uni((b <= Bmax || ob <= obmax) ? 1 : 0)) {
        bool any = false;
        if (b <= Bmax) {
          int val[4], valf[4];
          int nb = 0;
          if (k0 == 0 || guessed) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int col = cs0 + 16 * b + 64 * r + lane;
              // row 0: H(0,0) = 0, H(0,c) = -h - g c for 1 <= c <= band; the guessed row r0 > 0:
              // H = -h - g |c - r0| inside the band (the border's tent moved to the diagonal); F = -inf
              // (every lane computes both tents and selects: no lane-conditional block in the io
              // loop, whose latch the compiler otherwise closes with an exec-mask branch)
              const int d = col > r0 ? col - r0 : r0 - col;
              int t0 = -hh - g * col, t1 = -hh - g * d;
              asm("" : "+v"(t0), "+v"(t1));
              const int hv = (k0 == 0) ? ((col == 0) ? 0 : ((col >= 1 && col <= band) ? t0 : MSA_NEG))
                                       : ((d <= band) ? t1 : MSA_NEG);
              int zv = hv + g * (r0 + col) - hh;  // Z = H~ - h
              asm("" : "+v"(zv));
              val[r] = (hv == MSA_NEG) ? MSA_NEG : zv;
              valf[r] = MSA_NEG;
            }
            nb = min(16, Bmax - b + 1);
          } else {
            unsigned long long gv[4], gf[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int ci = min(16 * b + 64 * r + lane, a.gbuf_stride - 1);
              gv[r] = gload(g_in + ci);
              gf[r] = gload(g_in + a.gbuf_stride + ci);
            }
            bool run = true;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              val[r] = (int)(unsigned)gv[r];
              valf[r] = (int)(unsigned)gf[r];
              const int blk = b + 4 * r + (lane >> 4);
              const bool ok = (blk > Bmax) || ((unsigned)(gv[r] >> 32) == ep && (unsigned)(gf[r] >> 32) == ep);
              const unsigned long long bal = __ballot(ok);
#pragma unroll
              for (int jj = 0; jj < 4; ++jj) {
                run = run && (((bal >> (16 * jj)) & 0xffffull) == 0xffffull);
                if (run) nb = 4 * r + jj + 1;
              }
            }
            nb = uni(min(nb, Bmax - b + 1));
          }
          // ring slots: block x is free once wave 0 has finished phase x - 16
          if (consv < b + nb - FL_RINGB) consv = uni(lds_vload(flags + 33));
          nb = min(nb, consv + FL_RINGB - b);
          if (nb > 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int blk = b + 4 * r + (lane >> 4);
              if (blk < b + nb) {
                *L(rings + (blk & (FL_RINGB - 1)) * 16 + (lane & 15)) = val[r];
                *L(rings + 256 + (blk & (FL_RINGB - 1)) * 16 + (lane & 15)) = valf[r];
              }
            }
            FL_CBAR();
            if (lane == 0) lds_vstore(flags + 32, b + nb);
            b = uni(b + nb);
            any = true;
          }
        }
        if (ob <= obmax) {
          // the last wave's finished phases: block q - odq of ring W is complete
          const int pv = uni(lds_vload(flags + 33 + ns - 1));
          FL_CBAR();
          const int avail = min(pv - odq, obmax + 1);
          if (avail > ob) {
            const int nb = min(4, avail - ob);
            const int jb = lane >> 4, cc = lane & 15;
            if (jb < nb) {
              const int blk = ob + jb;
              const int v = *(const lds_int*)(rings + W * 512 + (blk & (FL_RINGB - 1)) * 16 + cc);
              const int vf = *(const lds_int*)(rings + W * 512 + 256 + (blk & (FL_RINGB - 1)) * 16 + cc);
              if (gnext) {
                gstore(g_out + 16 * blk + cc, ((unsigned long long)ep << 32) | (unsigned)v);
                gstore(g_out + a.gbuf_stride + 16 * blk + cc, ((unsigned long long)ep << 32) | (unsigned)vf);
              }
              if (ckslot >= 0) {  // checkpoint row: unshifted (H, F) over the band row
                const int col = csn + 16 * blk + cc;
                const int e = col - (ro - band);
                if (e >= 0 && e <= 2 * band && col >= 1 && col <= n) {
                  const int sh = g * (ro + col);
                  a.ck[(size_t)(2 * ckslot) * a.ckw + e] = v + hh - sh;
                  a.ck[(size_t)(2 * ckslot + 1) * a.ckw + e] = vf - sh;
                }
              }
            }
            ob = uni(ob + nb);
            FL_CBAR();
            if (lane == 0) lds_vstore(flags + 64, ob);
            any = true;
          }
        }
        if (!uni(any ? 1 : 0)) {
          __builtin_amdgcn_s_sleep(FL_IOSLEEP);
          if (++spins > FL_SPIN_MAX) break;
        }
      }
      // (reported after the loop: a divergent store inside it would make the wait loop's control flow
      // exec-mask based -- tests/test_host.py::test_wait_loops_are_wave_uniform)
      if (spins > FL_SPIN_MAX && lane == 0) atomicExch(a.err, 30);
    } else if (w < ns) {
      // =================== compute wave: stripe k ===================
      const int k = k0 + w;
      StripeGeom sg;
      stripe_geom(k, m, n, band, sg, 16);
      const int cs = uni(sg.cs), P = uni(sg.P);
      const int row_i = 64 * k + lane + 1;
      const unsigned ac = (row_i <= m) ? (a.A[pd.a_off + row_i - 1] & 7u) : 0u;
      const int tmin = jlo_of(row_i, band) - cs + lane;
      const int tmax = (row_i <= m) ? jhi_of(row_i, n, band) - cs + lane : -1;
      const int ZLB = (row_i <= band) ? -2 * hh : MSA_NEG;  // left border: column 0 (rows <= band), else -inf
      // phases [qlo, qhi) have every lane inside its band at every step: column jlo - 1 falls in a
      // phase < qlo, column jhi + 1 in a phase >= qhi
      const int qlo = (uni(sg.mask_lo) + 15) / 16;
      const int qhi = (uni(sg.mask_hi) + 1) / 16;
      const bool fin_stripe = (k == S - 1);
      const int Bin = (w == 0) ? ((k0 == 0 || guessed) ? P - 1 : min(P - 1, bk_bmax(k, m, n, band)))
                               : min(P - 1, bk_bmax(k, m, n, band));
      const int dq_in = (w == 0) ? 0 : bk_dq(k, m, n, band);
      const unsigned a_prog_in = lds_addr(w == 0 ? flags + 32 : flags + 33 + w - 1);
      const unsigned a_ring_in = lds_addr(rings + w * 512);
      const bool last = (w == ns - 1);
      const bool gnext = k0 + W < ke;
      const int ckslot = !chunked ? -1 : ((k == ks0 - 1) ? 2 * c : ((k == ke - 1 && c < nch - 1) ? 2 * c + 1 : -1));
      const bool has_out = !last || gnext || (last && ckslot >= 0);
      const int dq = has_out ? bk_dq(k + 1, m, n, band) : 0;
      const unsigned a_ring_out = lds_addr(rings + (last ? W : w + 1) * 512);
      const unsigned a_cons = lds_addr(last ? flags + 64 : flags + 33 + w + 1);
      int* const prog_me = flags + 33 + w;
      const unsigned a_prog_me = lds_addr(prog_me);
      const bool outp = (k >= ks0) && (a.outH != nullptr);
      int32_t* const orow = a.outH + pd.out_off + (size_t)k * pd.pmax * MSA_K * 64 + 4 * lane;
      // chunked, chunk >= 1, int16 chunk cells (msa_plan_create): H relative to the guessed row, 2 B per
      // cell, widened by chunk_add_kernel
      const bool o16 = chunked && c >= 1 && a.outH16 != nullptr;
      // (MSA_H16_PAIRED: a lane's cells of u-blocks 2h and 2h+1 side by side, one 16-B store per two
      // u-blocks; chunk_add_kernel undoes the pairing)
      int16_t* const orow16 = a.outH16 + (size_t)(k - C) * pd.pmax * MSA_K * 64 + (MSA_H16_PAIRED ? 8 : 4) * lane;
      unsigned plo, phi;
      {
        const int sm = 1 + 2 * g + hh, sx = 2 * g + hh;  // f + 2g + h, f = 1 on a match
        const unsigned bx = (unsigned)(sx & 0xff) * 0x01010101u;
        unsigned lo = bx, hi = bx;
        const unsigned bm = (unsigned)(sm & 0xff);
        if (ac < 4) lo = (lo & ~(0xffu << (8 * ac))) | (bm << (8 * ac));
        else hi = (hi & ~(0xffu << (8 * (ac - 4)))) | (bm << (8 * (ac - 4)));
        plo = lo;
        phi = hi;
      }
      unsigned a_code;
      {
        const int c0 = cs - lane + FL_OFF - colbase;  // >= 29
        const int x = c0 & (BK_NCOPY - 1);
        a_code = lds_addr(codes + x * L8 + (c0 - x));
      }
      // H = H~ - g(i+j) = Z + h - g(i+j); i + j = 64k + 1 + cs + t at every lane of step t
      const int ct0 = hh - g * (64 * k + 1 + cs);
      int Z = MSA_NEG, E = MSA_NEG, F = MSA_NEG, U = MSA_NEG;
      int fin0 = 0, fin1 = 0, fin2 = 0;
      int pubv = 0, consv = 0;
      unsigned spins = 0;
      fl_v4i ZA[4], FA[4], ZB[4], FB[4];
      fl_v2u CAl, CAh, CBl, CBh;
      const unsigned long long m63 = 1ull << 63;
      auto issue_reads = [&](int q, fl_v4i (&Zi)[4], fl_v4i (&Fi)[4], fl_v2u& Cl, fl_v2u& Ch, int& pubn)
          __attribute__((always_inline)) {
        const unsigned ra = a_ring_in + (unsigned)((q & (FL_RINGB - 1)) * 64);
        pubn = ds_read_b32(a_prog_in);
        Zi[0] = ds_read_b128<0>(ra);
        Zi[1] = ds_read_b128<16>(ra);
        Zi[2] = ds_read_b128<32>(ra);
        Zi[3] = ds_read_b128<48>(ra);
        Fi[0] = ds_read_b128<1024>(ra);
        Fi[1] = ds_read_b128<1040>(ra);
        Fi[2] = ds_read_b128<1056>(ra);
        Fi[3] = ds_read_b128<1072>(ra);
        ds_read_codes16(a_code + 16u * (unsigned)q, Cl, Ch);
      };
      auto wait_flag = [&](int need) __attribute__((always_inline)) {
        while (pubv < need) {
          int v = ds_read_b32(a_prog_in);
          lgkm_wait<0>(v);
          pubv = uni(v);
          if (pubv < need) {
            __builtin_amdgcn_s_sleep(0);
            if (++spins > FL_SPIN_MAX) break;
          }
        }
        if (pubv < need && lane == 0) atomicExch(a.err, 31);
      };
      // the stripe's start: its producer may be a whole item behind -- poll gently (a waiting wave
      // shares its SIMD with another workgroup's chain wave)
      {
        const int need0 = Bin < 0 ? 0 : min(1, Bin + 1) + dq_in;
        while (pubv < need0) {
          int v = ds_read_b32(a_prog_in);
          lgkm_wait<0>(v);
          pubv = uni(v);
          if (pubv < need0) {
            __builtin_amdgcn_s_sleep(4);
            if (++spins > FL_SPIN_MAX) break;
          }
        }
      }
      auto refresh_cons = [&](int need) __attribute__((always_inline)) {
        while (consv < need) {
          int c1 = ds_read_b32(a_cons);
          lgkm_wait<0>(c1);
          consv = uni(c1);
          if (consv < need) {
            __builtin_amdgcn_s_sleep(0);
            if (++spins > FL_SPIN_MAX) break;
          }
        }
        if (consv < need && lane == 0) atomicExch(a.err, 32);
      };
      auto mask_in = [&](int q, fl_v4i (&Zi)[4], fl_v4i (&Fi)[4]) __attribute__((always_inline)) {
        if (q > Bin) {  // past the producer's last column: -inf
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            Zi[u] = fl_v4i{MSA_NEG, MSA_NEG, MSA_NEG, MSA_NEG};
            Fi[u] = fl_v4i{MSA_NEG, MSA_NEG, MSA_NEG, MSA_NEG};
          }
        }
      };
      // (Bin < 0: the producer hands on no in-band column -- every input is -inf, nothing to wait for)
      wait_flag(Bin < 0 ? 0 : min(1, Bin + 1) + dq_in);
      {
        int pub0;
        issue_reads(0, ZA, FA, CAl, CAh, pub0);
        lgkm_wait_aff<0>(ZA, FA, CAl, CAh);
        lgkm_wait<0>(pub0);
        mask_in(0, ZA, FA);
      }
      // MODE bit 0: column jlo - 1 may fall in the phase; bit 1: column jhi + 1 (and the final cell)
      auto run_phase = [&](const int q, fl_v4i (&Zi)[4], fl_v4i (&Fi)[4], fl_v2u& Cl, fl_v2u& Ch, fl_v4i (&Zn)[4],
                           fl_v4i (&Fn)[4], fl_v2u& Cln, fl_v2u& Chn, auto MODE_, auto OUT_) __attribute__((always_inline)) {
        constexpr int MODE = decltype(MODE_)::value;
        constexpr int OUT = decltype(OUT_)::value;  // 0: no cells (warm-up), 1: int32 cells, 2: int16 chunk cells
        const int need = Bin < 0 ? 0 : min(q + 1, Bin + 1) + dq_in;
        if (pubv < need) {
          wait_flag(need);
          const unsigned ra = a_ring_in + (unsigned)((q & (FL_RINGB - 1)) * 64);
          ds_reread_b128x4(ra, Zi);
          ds_reread_b128x4(ra + 1024u, Fi);
          mask_in(q, Zi, Fi);
        }
        int xz[16], xf[16], ho[16];
        fl_v2u h16lo = {0u, 0u};
        int pubn = 0;
        const int ctq = ct0 - 16 * g * q;
        const unsigned cw[4] = {Cl.x, Cl.y, Ch.x, Ch.y};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const unsigned s4 = __builtin_amdgcn_perm(phi, plo, cw[u]);
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) {
            const int kx = 4 * u + kk;
            if (kx == FL_PF) issue_reads(q + 1, Zn, Fn, Cln, Chn, pubn);
            const int sc = ((int)(s4 << (24 - 8 * kk))) >> 24;
            const int zu = dpp_shr1(Zi[u][kk], Z);
            const int fu = dpp_shr1(Fi[u][kk], F);
            int fn = imax(zu, fu);
            int en = imax(Z, E);
            int h = imax3(U + sc, en, fn);
            asm("" : "+v"(h));
            int zn = h - hh;
            if constexpr ((MODE & 1) != 0) {
              const bool fl = (16 * q + kx == tmin - 1);  // the left neighbour of the row's first cell
              zn = fl ? ZLB : zn;
              en = fl ? MSA_NEG : en;
            }
            if constexpr ((MODE & 2) != 0) {
              const int t = 16 * q + kx;
              if (fin_stripe) {  // the final cell (m, n), unshifted
                const bool fe = (t == tmax && row_i == m);
                const int sh = g * (m + n);
                fin0 = fe ? h - sh : fin0;
                fin1 = fe ? en - sh : fin1;
                fin2 = fe ? fn - sh : fin2;
              }
              const bool fr = (t == tmax + 1);
              zn = fr ? MSA_NEG : zn;
              fn = fr ? MSA_NEG : fn;
            }
            U = zu;
            Z = zn;
            E = en;
            F = fn;
            xz[kx] = zn;
            xf[kx] = fn;
            ho[kx] = zn + (ctq - g * kx);
          }
#ifndef BK_NOSTORE
          if constexpr (OUT != 0) {
            if constexpr (OUT == 2) {
              const fl_v2u hv = {__builtin_amdgcn_perm((unsigned)ho[4 * u + 1], (unsigned)ho[4 * u], 0x05040100u),
                                 __builtin_amdgcn_perm((unsigned)ho[4 * u + 3], (unsigned)ho[4 * u + 2], 0x05040100u)};
              if constexpr (MSA_H16_PAIRED) {
                if (u & 1) {
                  const fl_v4u hp = {h16lo.x, h16lo.y, hv.x, hv.y};
                  __builtin_nontemporal_store(hp, reinterpret_cast<fl_v4u*>(orow16 + (size_t)(2 * q + (u >> 1)) * 512));
                } else {
                  h16lo = hv;
                }
              } else {
                __builtin_nontemporal_store(hv, reinterpret_cast<fl_v2u*>(orow16 + (size_t)(4 * q + u) * 256));
              }
            } else {
              const msa_v4i hv = {ho[4 * u], ho[4 * u + 1], ho[4 * u + 2], ho[4 * u + 3]};
              __builtin_nontemporal_store(hv, reinterpret_cast<msa_v4i*>(orow + (size_t)(4 * q + u) * 256));
            }
          }
#endif
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
        mask_in(q + 1, Zn, Fn);
      };
      // phase q reads buffer A when q is even, B when odd (and prefetches into the other).  Every range
      // but the last starts and ends on an even phase (the boundaries below are rounded towards the more
      // general edge mode), so a range is whole A/B pairs: at every range boundary buffer A is the
      // current one and B is dead -- an odd-phase prologue / epilogue would keep both buffers live across
      // the boundaries and make the compiler copy every DPP input of the B phases (32 v_mov per phase)
      auto run_range = [&](int lo, int hi, auto M_, auto O_) __attribute__((always_inline)) {
        for (int q = lo; q + 1 < hi; q += 2) {
          run_phase(q, ZA, FA, CAl, CAh, ZB, FB, CBl, CBh, M_, O_);
          run_phase(q + 1, ZB, FB, CBl, CBh, ZA, FA, CAl, CAh, M_, O_);
        }
      };
      using M0_ = std::integral_constant<int, 0>;
      using M1_ = std::integral_constant<int, 1>;
      using M2_ = std::integral_constant<int, 2>;
      using M3_ = std::integral_constant<int, 3>;
      // head [0, qa): left edges only; [qa, qb): both (a band too narrow for a clean middle);
      // middle [qb, qc): none; tail [qc, P): right edges and the final cell
      const int qa0 = max(0, min(min(qlo, qhi), P));
      const int qb0 = max(qa0, min(qlo, P));
      const int qc0 = max(qb0, min(qhi, P));
      // even boundaries within the even part Pe of [0, P), each rounded so that a phase moves only to a
      // more general mode (both edges ⊇ left edges, none; right edges ⊇ none); an odd last phase runs
      // with both edges
      const int Pe = P & ~1;
      const int qa = min(qa0 & ~1, Pe);
      const int qb = min((qb0 + 1) & ~1, Pe);
      const int qc = min(max(qb, qc0 & ~1), Pe);
      // the cell stores' kind is the stripe's (uniform): one instantiation per kind, no branch per u-block
      auto run_all = [&](auto O_) __attribute__((always_inline)) {
        run_range(0, qa, M1_{}, O_);
        run_range(qa, qb, M3_{}, O_);
        run_range(qb, qc, M0_{}, O_);
        run_range(qc, Pe, M2_{}, O_);
        if (P & 1) run_phase(P - 1, ZA, FA, CAl, CAh, ZB, FB, CBl, CBh, M3_{}, O_);
      };
      if (!outp) run_all(std::integral_constant<int, 0>{});
      else if (o16) run_all(std::integral_constant<int, 2>{});
      else run_all(std::integral_constant<int, 1>{});
      lgkm_drain();
      if (k >= ks0 && lane == 0) {
        msa_stripe_meta* md = a.meta + pd.stripe0 + k;
        md->cs = cs;
        md->phases = P;
      }
      if (fin_stripe && row_i == m) {
        msa_stripe_meta* md = a.meta + pd.stripe0 + k;
        md->fin[0] = fin0;
        md->fin[1] = fin1;
        md->fin[2] = fin2;
        md->has_fin = 1;
      }
    }
    __syncthreads();
  }
}

}  // namespace msa
