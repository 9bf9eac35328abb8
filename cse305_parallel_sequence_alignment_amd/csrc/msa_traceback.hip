// msa_traceback.hip -- on-device Smith-Waterman traceback (config C5).
//
// The fill (stripe_kernel, MSA_ALG_SWA, MSA_OUT_DIR) leaves one direction byte
// per cell in the skewed stripe layout: cell (64s + r + 1, cs_s + t - r) at
// byte (s*pmax + t/16)*1024 + r*16 + t%16 of the pair's block -- a 16-step x
// 64-row block is 1 KiB, one 16-byte row segment per lane.  Bits 0-1: where H
// came from (0 = local start, 1 = diagonal, 2 = E / horizontal gap, 3 = F /
// vertical gap); bit 2: E here opened from H(i, j-1); bit 3: F here opened from
// H(i-1, j).  The walk is the tie order of oracle orc_sw (first maximum).
//
// One wave walks the path from the pair's end cell (read from the reduction's
// PairResult on the same stream, no host round trip).  Its state is uniform
// (SGPRs); the block under the walk sits in four VGPRs per lane and a step
// reads its byte with v_readlane from lane r -- no LDS, no per-step memory
// access.  A diagonal step keeps t (r-1, j-1), a gap step lowers t by one, so
// a near-diagonal path stays inside one block for up to 64 steps.  While
// walking, the wave prefetches the block it will need next (the stripe above,
// at the column the path will leave through, or the block to the left) into a
// second VGPR set, so most block switches find their bytes already loaded.
// Ops are packed four per dword in an SGPR, parked in one lane of a VGPR (a
// lane-select) and stored 256 at a time with one vector store (no scalar-cache
// writes).
// Output: ops from the end cell back to the start ('M' diagonal, 'D' a gap
// consuming B, 'I' a gap consuming A), info = {n_ops, beg_i, beg_j, status}.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace msa {

__device__ __forceinline__ unsigned dir_byte(const uint4& v, int r, int q) {
  // byte q (0..15) of lane r's 16-byte row segment
  const int w = q >> 2;
  const unsigned x = (w == 0) ? __builtin_amdgcn_readlane(v.x, r)
                   : (w == 1) ? __builtin_amdgcn_readlane(v.y, r)
                   : (w == 2) ? __builtin_amdgcn_readlane(v.z, r)
                              : __builtin_amdgcn_readlane(v.w, r);
  return (x >> ((q & 3) * 8)) & 0xffu;
}

__global__ __launch_bounds__(64) void sw_traceback_kernel(const uint8_t* __restrict__ dir,
                                                          const msa_pair_desc* __restrict__ pairs,
                                                          const msa_stripe_meta* __restrict__ meta,
                                                          const PairResult* __restrict__ res, int pair,
                                                          uint8_t* __restrict__ ops, long long cap,
                                                          long long* __restrict__ info) {
  const int lane = threadIdx.x;
  const msa_pair_desc pd = pairs[pair];
  const PairResult r0 = res[pair];
  const uint8_t* base = dir + pd.out_off;
  const long long pmax = pd.pmax;
  long long i = r0.end_i, j = r0.end_j;
  long long nops = 0;
  int st = 0;  // 0: in H, 1: in E (horizontal gap), 2: in F (vertical gap)
  int status = 0;
  uint4 cur = make_uint4(0, 0, 0, 0), nxt = make_uint4(0, 0, 0, 0);
  long long cur_blk = -1, nxt_blk = -1;
  long long s_cached = -1;
  int cs = 0, cs_up = 0;
  unsigned word = 0;                     // four ops, byte k = op 4q + k
  unsigned parked = 0;                   // this lane's dword of the 256-op buffer
  // store the parked dwords of the 256-op group starting at g0, up to op `upto`
  auto flush = [&](long long g0, long long upto) {
    const long long o = g0 + 4ll * lane;
    if (o >= upto) return;
    if (o + 4 <= cap) {
      *(unsigned*)(ops + o) = parked;
    } else {
      for (int k = 0; k < 4 && o + k < cap; ++k) ops[o + k] = (uint8_t)(parked >> (8 * k));
    }
  };
  auto emit = [&](unsigned op) {
    word |= op << (8 * (nops & 3));
    ++nops;
    if ((nops & 3) == 0) {
      if (lane == (int)(((nops - 4) >> 2) & 63)) parked = word;
      word = 0;
      if ((nops & 255) == 0) flush(nops - 256, nops);
    }
  };
  if (r0.score > 0) {
    while (i > 0 && j > 0) {
      const long long s = (i - 1) >> 6;
      const int r = (int)((i - 1) & 63);
      if (s != s_cached) {
        cs = meta[pd.stripe0 + s].cs;
        cs_up = s > 0 ? meta[pd.stripe0 + s - 1].cs : 0;
        s_cached = s;
      }
      const long long t = j - cs + r;
      const long long blk = s * pmax + (t >> 4);
      if (blk != cur_blk) {
        if (blk == nxt_blk) {
          cur = nxt;
          cur_blk = nxt_blk;
          nxt_blk = -1;
        } else {
          cur = *(const uint4*)(base + blk * 1024 + lane * 16);
          cur_blk = blk;
        }
      }
      // prefetch the block the walk will need next: near the top rows, the stripe above
      // at the column a diagonal path leaves through; near the block's left edge, the
      // block to the left
      long long want = -1;
      if (r < 12 && s > 0) {
        const long long tu = (j - r) - cs_up + 63;
        if (tu >= 0) want = (s - 1) * pmax + (tu >> 4);
      } else if ((t & 15) < 3 && (t >> 4) > 0) {
        want = blk - 1;
      }
      if (want >= 0 && want != nxt_blk && want != cur_blk) {
        nxt = *(const uint4*)(base + want * 1024 + lane * 16);
        nxt_blk = want;
      }
      const unsigned d = dir_byte(cur, r, (int)(t & 15));
      if (st == 0) {
        const unsigned hs = d & 3u;
        if (hs == 0) break;  // local start
        if (hs == 1) {
          emit('M');
          --i;
          --j;
        } else {
          st = (hs == 2) ? 1 : 2;
        }
      } else if (st == 1) {
        emit('D');
        st = (d & 4u) ? 0 : 1;
        --j;
      } else {
        emit('I');
        st = (d & 8u) ? 0 : 2;
        --i;
      }
      if (nops > cap) {
        status = -8;  // MSA_ERR_CAPACITY
        break;
      }
    }
  }
  // flush the partial word and the parked dwords of the last (partial) 256-op group
  if ((nops & 3) && lane == (int)((nops >> 2) & 63)) parked = word;
  if (nops & 255) flush(nops & ~255ll, nops);
  if (lane == 0) {
    info[0] = nops;
    info[1] = i + 1;
    info[2] = j + 1;
    info[3] = status;
  }
}

}  // namespace msa
