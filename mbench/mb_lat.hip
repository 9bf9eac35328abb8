// Microbenchmark: dependent-chain latency of the ops on the DP step chain (one wave). Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CTRL>
__device__ __forceinline__ int dpp(int old, int src) { return __builtin_amdgcn_update_dpp(old, src, CTRL, 0xf, 0xf, false); }
__device__ __forceinline__ int imax3(int a, int b, int c) { return max(max(a, b), c); }

template <int V>
__global__ void klat(int* out, unsigned long long* cyc, int n) {
  const int lane = threadIdx.x;
  int X = lane, Y = lane * 3, A = lane ^ 5, B = lane + 7;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      if constexpr (V == 0) { X = imax3(X, A + k, B); asm("" : "+v"(X)); }                       // max3 chain
      if constexpr (V == 1) { X = dpp<0x138>(A, X); asm("" : "+v"(X)); }                          // wave_shr:1 chain
      if constexpr (V == 2) { X = dpp<0x111>(A, X); asm("" : "+v"(X)); }                          // row_shr:1 chain
      if constexpr (V == 3) { int up = dpp<0x138>(A, X); X = imax3(Y + k, up, X); Y = up; asm("" : "+v"(X)); }  // core wave_shr
      if constexpr (V == 4) { int up = dpp<0x111>(A, X); X = imax3(Y + k, up, X); Y = up; asm("" : "+v"(X)); }  // core row_shr
      if constexpr (V == 5) { int up = X + A; X = imax3(Y + k, up, X); Y = up; asm("" : "+v"(X)); }  // add + max3
      if constexpr (V == 6) { X = X + k; asm("" : "+v"(X)); }                                       // add chain
      if constexpr (V == 7) {  // row_shr on chain + row_bcast15 off chain (skewed row groups)
        int b = dpp<0x142>(A + k, Y);  // bcast15 of X(t-2) (kept in Y)
        int up = dpp<0x111>(b, X);
        Y = X;
        X = imax3(B + k, up, X);
        asm("" : "+v"(X));
      }
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) cyc[0] = t1 - t0;
  if (X == 0x7fffffff) out[lane] = X + Y;
}

template <int V>
void run(const char* name, int* d_out, unsigned long long* d_cyc) {
  const int n = 4000;
  hipLaunchKernelGGL(klat<V>, dim3(1), dim3(64), 0, 0, d_out, d_cyc, n);
  hipDeviceSynchronize();
  hipLaunchKernelGGL(klat<V>, dim3(1), dim3(64), 0, 0, d_out, d_cyc, n);
  hipDeviceSynchronize();
  unsigned long long c;
  hipMemcpy(&c, d_cyc, 8, hipMemcpyDeviceToHost);
  printf("%-40s %.2f cyc/step\n", name, (double)c / (n * 16));
}

int main() {
  int* d_out; unsigned long long* d_cyc;
  hipMalloc(&d_out, 64 * 4);
  hipMalloc(&d_cyc, 64);
  run<0>("max3 chain", d_out, d_cyc);
  run<6>("add chain", d_out, d_cyc);
  run<1>("dpp wave_shr:1 chain", d_out, d_cyc);
  run<2>("dpp row_shr:1 chain", d_out, d_cyc);
  run<3>("step: wave_shr + max3", d_out, d_cyc);
  run<4>("step: row_shr + max3", d_out, d_cyc);
  run<5>("step: add + max3", d_out, d_cyc);
  run<7>("step: row_shr + max3, bcast15 off-chain", d_out, d_cyc);
  return 0;
}
