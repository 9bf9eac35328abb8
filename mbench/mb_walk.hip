// mb_walk.hip -- one-wave scalar-loop cost probe (traceback walk design): how many
// clock ticks one iteration of a dependent scalar chain takes for a lone wave,
// with and without an LDS byte read + readfirstlane per iteration.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void walk_salu(int n, long long* out) {
  unsigned x = 1, y = 7;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int k = 0; k < n; ++k) {
    x = __builtin_amdgcn_readfirstlane(x * 1664525u + 1013904223u);
    y ^= x >> 7;
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = y; }
}

__global__ void walk_lds(int n, long long* out) {
  __shared__ unsigned char buf[4096];
  for (int k = threadIdx.x; k < 4096; k += 64) buf[k] = (unsigned char)(k * 37);
  __syncthreads();
  unsigned a = 5, acc = 0;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int k = 0; k < n; ++k) {
    const unsigned d = __builtin_amdgcn_readfirstlane((unsigned)buf[a & 4095]);
    acc += d;
    a = a * 33u + d + 1u;
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = acc; }
}

int main() {
  long long* d;
  long long h[2];
  hipMalloc(&d, 16);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int n = 200000;
  for (int v = 0; v < 2; ++v) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0);
      if (v == 0) hipLaunchKernelGGL(walk_salu, dim3(1), dim3(64), 0, 0, n, d);
      else hipLaunchKernelGGL(walk_lds, dim3(1), dim3(64), 0, 0, n, d);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
      printf("%s: %.3f ms, %lld ticks, %.1f ticks/iter, %.2f ns/iter\n", v ? "lds" : "salu", ms, h[0],
             (double)h[0] / n, ms * 1e6 / n);
    }
  }
  return 0;
}
