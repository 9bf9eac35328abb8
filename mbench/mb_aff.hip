// mb_aff.hip -- cycles per DP step of the affine SW recurrence (shifted space, affine flow
// kernel pass 1) for lone waves, by formulation.  Diagnostic only.
//   0: R=1 as in flow_kernel<..., AFF>: 2 DPP movs, add, max e, max f, max floor, max3, sub
//   1: R=1 with fused DPP VOP2 ops (f = max(dpp(F), dpp(Z)) as one DPP max + one DPP mov)
//   2: R=2 rows per lane: row 1 takes Z/F~ from lane r-1's row 2 (2 DPPs), row 2 from row 1
//   3: R=1 without the floor (cost of the floor term)
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ int dpp_shr1(int old, int src) { return __builtin_amdgcn_update_dpp(old, src, 0x138, 0xf, 0xf, false); }
__device__ __forceinline__ int imax(int a, int b) { return a > b ? a : b; }
__device__ __forceinline__ int imax3(int a, int b, int c) { return imax(imax(a, b), c); }

template <int V>
__global__ void kaff(int* out, unsigned long long* cyc, int nphase, int g, int oe, int active) {
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  if (w >= active) return;
  unsigned plo = 0x01000000u * lane + 0x00020001u, phi = 0x00010203u;
  int Zl = lane, U = lane - 1, E = -100, Fo = -100;
  int Zl2 = lane + 1, E2 = -100, Fo2 = -100;
  int acc = 0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int q = 0; q < nphase; ++q) {
    int INZ[16], INF[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) { INZ[k] = q + k; INF[k] = q - k; asm("" : "+v"(INZ[k]), "+v"(INF[k])); }
    const int flq = g * 16 * q;
    unsigned cw[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) { cw[u] = (unsigned)(q * 0x01010101u + u + lane); asm("" : "+v"(cw[u])); }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const unsigned s4 = __builtin_amdgcn_perm(phi, plo, cw[u]);
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int kx = 4 * u + kk;
        const int sc = ((int)(s4 << (24 - 8 * kk))) >> 24;
        const int flr = flq + g * kx;
        if constexpr (V == 0 || V == 3) {
          const int upZ = dpp_shr1(INZ[kx], Zl);
          const int upF = dpp_shr1(INF[kx], Fo);
          const int e = imax(E, Zl);
          const int f = imax(upF, upZ);
          const int d = V == 3 ? U + sc : imax(U + sc, flr);
          int h = imax3(d, e, f);
          asm("" : "+v"(h));
          U = upZ; E = e; Fo = f; Zl = h - oe;
        } else if constexpr (V == 1) {
          // lane r-1 publishes P = max(F~, Z) (its contribution to the row below): one DPP mov
          const int upZ = dpp_shr1(INZ[kx], Zl);
          const int f = dpp_shr1(INF[kx], Fo);  // Fo holds P
          const int e = imax(E, Zl);
          const int d = imax(U + sc, flr);
          int h = imax3(d, e, f);
          asm("" : "+v"(h));
          U = upZ; E = e; Zl = h - oe; Fo = imax(f, Zl);
        } else {
          const int sb = sc ^ 1;
          const int upZ = dpp_shr1(INZ[kx], Zl2);
          const int upF = dpp_shr1(INF[kx], Fo2);
          const int e1 = imax(E, Zl);
          const int f1 = imax(upF, upZ);
          const int d1 = imax(U + sc, flr);
          int h1 = imax3(d1, e1, f1);
          asm("" : "+v"(h1));
          const int zprev = Zl;
          U = upZ; E = e1; Zl = h1 - oe;
          const int e2 = imax(E2, Zl2);
          const int f2 = imax(f1, Zl);
          const int d2 = imax(zprev + sb, flr + g);
          int h2 = imax3(d2, e2, f2);
          asm("" : "+v"(h2));
          E2 = e2; Fo2 = f2; Zl2 = h2 - oe;
        }
      }
    }
    acc ^= Zl + Zl2;
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) cyc[blockIdx.x * 16 + w] = t1 - t0;
  if (acc == 0x7fffffff) out[lane] = acc + E + Fo + E2 + Fo2 + U;
}

template <int V>
void run(const char* name, int waves, unsigned long long* d_cyc, int* d_out) {
  const int nphase = 2000;
  hipLaunchKernelGGL(kaff<V>, dim3(1), dim3(64 * waves), 0, 0, d_out, d_cyc, nphase, 1, 2, waves);
  hipDeviceSynchronize();
  hipLaunchKernelGGL(kaff<V>, dim3(1), dim3(64 * waves), 0, 0, d_out, d_cyc, nphase, 1, 2, waves);
  unsigned long long c[16];
  hipMemcpy(c, d_cyc, sizeof(c), hipMemcpyDeviceToHost);
  std::printf("%-28s waves %d: %7.2f ticks/step (wave 0)\n", name, waves, (double)c[0] / (nphase * 16));
}

int main() {
  unsigned long long* d_cyc;
  int* d_out;
  hipMalloc(&d_cyc, 16 * 8);
  hipMalloc(&d_out, 4096);
  for (int waves : {1, 4}) {
    run<0>("R1 (flow AFF)", waves, d_cyc, d_out);
    run<1>("R1 P=max(F,Z) one DPP", waves, d_cyc, d_out);
    run<2>("R2 two rows per lane", waves, d_cyc, d_out);
    run<3>("R1 no floor", waves, d_cyc, d_out);
  }
  return 0;
}
