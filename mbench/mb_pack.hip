// mb_pack.hip -- cycles per DP step of the C2 pass-1 recurrence for one wave, unpacked vs
// packed int16 (two stripes per lane, lagged 64 columns, so stripe s+1's
// lane 0 takes stripe s's lane 63 through a DPP rotate).  Diagnostic only.
//   0: R=2 int32 (flow_kernel pass 1): DPP, per row an SDWA byte add + v_max3       2 cells
//   1: R=2 packed, two stripes: DPP rotate + v_perm lane-0 fix-up, per row v_pk_add_u16 +
//      2 v_pk_max_i16 (no v_pk_max3_i16 on gfx950), score = per-step v_perm of two packed
//      profile lookups                                                               4 cells
//   2: R=1 packed, two stripes (the same without the second row)                     2 cells
#include <hip/hip_runtime.h>
#include <cstdio>

typedef short s2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ int dpp_shr1(int old, int src) { return __builtin_amdgcn_update_dpp(old, src, 0x138, 0xf, 0xf, false); }
__device__ __forceinline__ int dpp_ror1(int src) { return __builtin_amdgcn_update_dpp(src, src, 0x13C, 0xf, 0xf, false); }
__device__ __forceinline__ int imax3(int a, int b, int c) { return max(max(a, b), c); }
__device__ __forceinline__ int pk_add(int a, int b) {
  s2 x = __builtin_bit_cast(s2, a), y = __builtin_bit_cast(s2, b);
  return __builtin_bit_cast(int, (s2)(x + y));
}
__device__ __forceinline__ int pk_max(int a, int b) {
  s2 x = __builtin_bit_cast(s2, a), y = __builtin_bit_cast(s2, b);
  return __builtin_bit_cast(int, __builtin_elementwise_max(x, y));
}

template <int V>
__global__ void kstep(int* out, unsigned long long* cyc, int nphase) {
  const int lane = threadIdx.x;
  unsigned plo = 0x01000000u * lane + 0x00020001u, phi = 0x00010203u;
  unsigned plo2 = plo ^ 0x01010101u, phi2 = phi ^ 0x02020202u;
  int X = lane, U = lane - 1, X2 = lane + 1;
  // lane 0's fix-up selector: low half from the ring input, high half from lane 63's low half
  // (v_perm: selector bytes 0-3 pick the second operand's bytes, 4-7 the first's)
  const unsigned sel = lane == 0 ? 0x01000504u : 0x03020100u;
  int acc = 0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int q = 0; q < nphase; ++q) {
    int IN[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) { IN[k] = q * 3 + k; asm("" : "+v"(IN[k])); }
    unsigned cw[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) { cw[u] = (unsigned)(q * 0x01010101u + u + lane); asm("" : "+v"(cw[u])); }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const unsigned s4 = __builtin_amdgcn_perm(phi, plo, cw[u]);
      const unsigned s4b = __builtin_amdgcn_perm(phi2, plo2, cw[u]);
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int kx = 4 * u + kk;
        if constexpr (V == 0) {
          const int s = ((int)(s4 << (24 - 8 * kk))) >> 24;
          const int sb = ((int)(s4b << (24 - 8 * kk))) >> 24;
          const int up = dpp_shr1(IN[kx], X2);
          int h1 = imax3(U + s, up, X);
          asm("" : "+v"(h1));
          U = up;
          const int xp = X;
          X = h1;
          int h2 = imax3(xp + sb, X, X2);
          asm("" : "+v"(h2));
          X2 = h2;
        } else {
          // both stripes' scores as int16 pairs: bytes kk of the two lookups, sign-extended
          const unsigned sp = __builtin_amdgcn_perm(s4b, s4, 0x0c000c00u | ((4u + kk) << 16) | kk);
          const int sx = (int)sp;  // (C2's profile bytes s + 2g are >= 0: no sign extension)
          const int rot = dpp_ror1(V == 1 ? X2 : X);
          const int up = (int)__builtin_amdgcn_perm((unsigned)IN[kx], (unsigned)rot, sel);
          int h1 = pk_max(pk_max(pk_add(U, sx), up), X);
          asm("" : "+v"(h1));
          U = up;
          const int xp = X;
          X = h1;
          if constexpr (V == 1) {
            int h2 = pk_max(pk_max(pk_add(xp, sx), X), X2);
            asm("" : "+v"(h2));
            X2 = h2;
          }
        }
      }
    }
    acc ^= X + X2;
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) cyc[0] = t1 - t0;
  if (acc == 0x7fffffff) out[lane] = acc + U;
}

template <int V>
void run(const char* name, int cells, unsigned long long* d_cyc, int* d_out) {
  const int nphase = 4000;
  for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(kstep<V>, dim3(1), dim3(64), 0, 0, d_out, d_cyc, nphase);
  hipDeviceSynchronize();
  unsigned long long c;
  hipMemcpy(&c, d_cyc, 8, hipMemcpyDeviceToHost);
  const double t = (double)c / (nphase * 16);
  std::printf("%-34s %6.2f ticks/step, %d cells/lane/step: %6.2f ticks/cell\n", name, t, cells, t / cells);
}

int main() {
  unsigned long long* d_cyc;
  int* d_out;
  hipMalloc(&d_cyc, 8);
  hipMalloc(&d_out, 4096);
  run<0>("R=2 int32 (flow pass 1)", 2, d_cyc, d_out);
  run<1>("R=2 packed int16, two stripes", 4, d_cyc, d_out);
  run<2>("R=1 packed int16, two stripes", 2, d_cyc, d_out);
  return 0;
}
