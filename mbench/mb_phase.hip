// Microbenchmark: one wave running the flow kernel's pass-1 phase loop (16 DP
// steps per phase) with its pieces switched on one by one.  Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int dpp_shr1(int old, int src) { return __builtin_amdgcn_update_dpp(old, src, 0x138, 0xf, 0xf, false); }
__device__ __forceinline__ int imax3(int a, int b, int c) { return max(max(a, b), c); }
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)(p);
}
template <int OFF>
__device__ __forceinline__ v4i rd128(unsigned a) {
  v4i v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(a), "i"(OFF) : "memory");
  return v;
}
__device__ __forceinline__ v4u rd2b64(unsigned a) {
  v4u v;
  asm volatile("ds_read2_b64 %0, %1 offset1:1" : "=v"(v) : "v"(a) : "memory");
  return v;
}
__device__ __forceinline__ int rd32(unsigned a) {
  int v;
  asm volatile("ds_read_b32 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}
template <int N>
__device__ __forceinline__ void waitv(v4i (&in)[4], v4u& cw, int& p) {
  asm volatile("s_waitcnt lgkmcnt(%6)" : "+v"(in[0]), "+v"(in[1]), "+v"(in[2]), "+v"(in[3]), "+v"(cw), "+v"(p) : "i"(N) : "memory");
}
__device__ __forceinline__ void handoff(unsigned long long m63, unsigned ra, v4i x0, v4i x1, v4i x2, v4i x3, unsigned pa,
                                        int pv) {
  unsigned long long sv;
  asm volatile(
      "s_mov_b64 %[sv], exec\n\ts_mov_b64 exec, %[m]\n\t"
      "ds_write_b128 %[ra], %[x0]\n\tds_write_b128 %[ra], %[x1] offset:16\n\t"
      "ds_write_b128 %[ra], %[x2] offset:32\n\tds_write_b128 %[ra], %[x3] offset:48\n\t"
      "ds_write_b32 %[pa], %[pv]\n\t"
      "s_mov_b64 exec, %[sv]\n\ts_nop 4"
      : [sv] "=&s"(sv)
      : [m] "s"(m63), [ra] "v"(ra), [x0] "v"(x0), [x1] "v"(x1), [x2] "v"(x2), [x3] "v"(x3), [pa] "v"(pa), [pv] "v"(pv)
      : "memory");
}
// lane-63 hand-off via 16 ds_write_addtid_b32 (M0 = slot - 252) + counter
__device__ __forceinline__ void handoff_tid(unsigned long long m63, unsigned m0v, const int (&x)[16], unsigned pa, int pv) {
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
// shift-register hand-off: lanes 48..63 hold the phase's 16 values; one ds_write_b32 + counter
__device__ __forceinline__ void handoff_shreg(unsigned long long m16, unsigned ra, int v, unsigned pa, int pv) {
  unsigned long long sv;
  asm volatile(
      "s_mov_b64 %[sv], exec\n\ts_mov_b64 exec, %[m]\n\t"
      "ds_write_b32 %[ra], %[v]\n\t"
      "ds_write_b32 %[pa], %[pv]\n\t"
      "s_mov_b64 exec, %[sv]\n\ts_nop 4"
      : [sv] "=&s"(sv)
      : [m] "s"(m16), [ra] "v"(ra), [v] "v"(v), [pa] "v"(pa), [pv] "v"(pv)
      : "memory");
}
__device__ __forceinline__ int dpp_shl1(int old, int src) { return __builtin_amdgcn_update_dpp(old, src, 0x130, 0xf, 0xf, false); }
// F bits: 64 hand-off via addtid, 128 hand-off via DPP shift register
// F bits: 1 prefetch reads + waits, 2 hand-off, 4 SDWA score (else a plain add), 8 perm per 4 steps,
//         16 s_nop 4 removed from hand-off (timing only), 32 no asm opaque on h
template <int F>
__global__ void kphase(int* out, unsigned long long* cyc, int nph) {
  extern __shared__ __attribute__((aligned(16))) int sm[];
  const int lane = threadIdx.x;
  for (int i = lane; i < 16384; i += 64) sm[i] = i & 7;
  __syncthreads();
  const unsigned a_ring = lds_addr(sm), a_pub = lds_addr(sm + 4096), a_code = lds_addr(sm + 1024) + 8 * (lane & 7);
  const unsigned a_out = lds_addr(sm + 2048);
  unsigned plo = 0x01000000u * (lane & 3) + 0x00020001u, phi = 0x00010203u;
  int X = lane, U = lane - 1;
  v4i INa[4], INb[4];
  v4u CWa, CWb;
  int pa = 0, pb = 0;
  INa[0] = rd128<0>(a_ring); INa[1] = rd128<16>(a_ring); INa[2] = rd128<32>(a_ring); INa[3] = rd128<48>(a_ring);
  CWa = rd2b64(a_code);
  pa = rd32(a_pub);
  waitv<0>(INa, CWa, pa);
  const unsigned long long m63 = 1ull << 63;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  auto phase = [&](int q, v4i (&IN)[4], v4u& CW, v4i (&INn)[4], v4u& CWn, int& pn) __attribute__((always_inline)) {
    int xo[16];
    int shreg = 0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const unsigned s4 = (F & 8) ? __builtin_amdgcn_perm(phi, plo, CW[u]) : CW[u];
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int kx = 4 * u + kk;
        if (kx == 8) {
          if constexpr (F & 1) {
            const unsigned ra = a_ring + (unsigned)((q & 15) * 64);
            pn = rd32(a_pub);
            INn[0] = rd128<0>(ra); INn[1] = rd128<16>(ra); INn[2] = rd128<32>(ra); INn[3] = rd128<48>(ra);
            CWn = rd2b64(a_code + 16 * (q & 63));
          }
        }
        const int s = (F & 4) ? (((int)(s4 << (24 - 8 * kk))) >> 24) : (int)(s4 & 3) + kk;
        const int in = IN[kx >> 2][kx & 3];
        const int up = dpp_shr1(in, X);
        int h = imax3(U + s, up, X);
        if constexpr (!(F & 32)) asm("" : "+v"(h));
        U = up;
        X = h;
        xo[kx] = X;
        if constexpr (F & 128) shreg = dpp_shl1(X, shreg);
      }
    }
    if constexpr (F & 1) waitv<0>(INn, CWn, pn);
    else {
#pragma unroll
      for (int u = 0; u < 4; ++u) INn[u] = IN[u];
      CWn = CW;
    }
    if constexpr (F & 2)
      handoff(m63, a_out + (unsigned)((q & 15) * 64), v4i{xo[0], xo[1], xo[2], xo[3]}, v4i{xo[4], xo[5], xo[6], xo[7]},
              v4i{xo[8], xo[9], xo[10], xo[11]}, v4i{xo[12], xo[13], xo[14], xo[15]}, a_pub + 64, q);
    if constexpr (F & 64) handoff_tid(m63, a_out + (unsigned)((q & 15) * 64) - 252, xo, a_pub + 64, q);
    if constexpr (F & 128) {
      const unsigned ra = a_out + (unsigned)((q & 15) * 64) + 4 * (unsigned)(lane - 48);
      handoff_shreg(0xffff000000000000ull, ra, shreg, a_pub + 64, q);
    }
  };
  for (int q = 0; q < nph; q += 2) {
    phase(q, INa, CWa, INb, CWb, pb);
    phase(q + 1, INb, CWb, INa, CWa, pa);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) cyc[0] = t1 - t0;
  if (X == 0x7fffffff) out[lane] = pa + pb;
}

template <int F>
void run(const char* name, int* d_out, unsigned long long* d_cyc) {
  const int nph = 2000;
  hipFuncSetAttribute((const void*)kphase<F>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
  for (int it = 0; it < 2; ++it) {
    hipLaunchKernelGGL(kphase<F>, dim3(1), dim3(64), 65536, 0, d_out, d_cyc, nph);
    hipDeviceSynchronize();
  }
  unsigned long long c;
  hipMemcpy(&c, d_cyc, 8, hipMemcpyDeviceToHost);
  printf("%-48s %.1f cyc/step\n", name, (double)c / (nph * 16));
}

int main() {
  int* d_out; unsigned long long* d_cyc;
  hipMalloc(&d_out, 64 * 4);
  hipMalloc(&d_cyc, 64);
  run<0>("chain: dpp + plain add + max3", d_out, d_cyc);
  run<32>("  (no opaque asm on h)", d_out, d_cyc);
  run<4>("chain: dpp + sdwa add + max3", d_out, d_cyc);
  run<4 | 8>("  + perm per 4 steps", d_out, d_cyc);
  run<4 | 8 | 1>("  + prefetch reads/wait", d_out, d_cyc);
  run<4 | 8 | 2>("  + hand-off (no prefetch)", d_out, d_cyc);
  run<4 | 8 | 1 | 2>("  + prefetch + hand-off (pass 1 loop)", d_out, d_cyc);
  run<4 | 8 | 64>("  + hand-off addtid x16 (no prefetch)", d_out, d_cyc);
  run<4 | 8 | 128>("  + hand-off shift register (no prefetch)", d_out, d_cyc);
  run<4 | 8 | 1 | 64>("  + prefetch + hand-off addtid", d_out, d_cyc);
  run<4 | 8 | 1 | 128>("  + prefetch + hand-off shift register", d_out, d_cyc);
  return 0;
}
