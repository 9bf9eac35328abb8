// Microbenchmark: per-CU store throughput by waves/CU and cache policy; ds_write cost in the step loop.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef int v4i __attribute__((ext_vector_type(4)));

template <int POL>
__device__ __forceinline__ void st(v4i* p, v4i v) {
  if constexpr (POL == 0) *p = v;
  if constexpr (POL == 1) __builtin_nontemporal_store(v, p);
  if constexpr (POL == 2) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" :: "v"(p), "v"(v) : "memory");
  if constexpr (POL == 3) asm volatile("global_store_dwordx4 %0, %1, off sc1" :: "v"(p), "v"(v) : "memory");
}

// each wave stores `nq` KiB (1 KiB per instruction) to its own region
template <int POL>
__global__ void kst(v4i* out, unsigned long long* cyc, int nq) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v4i* base = out + ((size_t)(blockIdx.x * 16 + w) * nq) * 64 + lane;
  v4i v = {lane, w, 3, 4};
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < nq; i += 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u) { st<POL>(base + (size_t)(i + u) * 64, v); v.x += 1; }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) cyc[blockIdx.x * 16 + w] = t1 - t0;
}

template <int POL>
void run(const char* name, int blocks, int waves, v4i* d_out, unsigned long long* d_cyc) {
  const int nq = 4096;  // KiB per wave  (blocks*waves*4 MiB <= buffer)
  hipLaunchKernelGGL(kst<POL>, dim3(blocks), dim3(64 * waves), 0, 0, d_out, d_cyc, nq);
  hipDeviceSynchronize();
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(kst<POL>, dim3(blocks), dim3(64 * waves), 0, 0, d_out, d_cyc, nq);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> c(blocks * 16);
  hipMemcpy(c.data(), d_cyc, c.size() * 8, hipMemcpyDeviceToHost);
  unsigned long long mx = 0;
  for (int b = 0; b < blocks; ++b) for (int w = 0; w < waves; ++w) mx = std::max(mx, c[b * 16 + w]);
  const double bytes_cu = (double)waves * nq * 1024;
  printf("%-10s blocks %3d waves %2d: %.1f B/clk per CU (memtime), total %.1f GB/s wall\n", name, blocks, waves,
         bytes_cu / mx, (double)blocks * bytes_cu / (ms * 1e6));
}

int main() {
  v4i* d_out; unsigned long long* d_cyc;
  const size_t bytes = (size_t)32 * 16 * 4096 * 1024;  // 32 blocks x 16 waves x 4 MiB = 2 GiB
  if (hipMalloc(&d_out, bytes) != hipSuccess) { printf("alloc failed\n"); return 1; }
  hipMalloc(&d_cyc, 256 * 16 * 8);
  for (int wv : {1, 4, 8, 16}) {
    run<0>("plain", 1, wv, d_out, d_cyc);
    run<1>("nt", 1, wv, d_out, d_cyc);
    run<2>("sc0 sc1", 1, wv, d_out, d_cyc);
    run<3>("sc1", 1, wv, d_out, d_cyc);
  }
  run<1>("nt", 32, 4, d_out, d_cyc);
  run<1>("nt", 32, 16, d_out, d_cyc);
  run<0>("plain", 32, 16, d_out, d_cyc);
  return 0;
}
