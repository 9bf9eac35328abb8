// mb_gissue.hip -- issue cost and latency of a 16 KiB group load for the device walk (one wave):
//   A: 16 x global_load_lds_dwordx4 (LDS-DMA, the walk's glds16x16), ticks to issue, ticks to land
//   B: 16 x global_load_dwordx4 into VGPRs, the same
//   C: A issued while 48 earlier LDS-DMA loads are in flight (the walk's steady state)
// s_memtime ticks; groups 4 MiB apart (cold in L2 each time).  Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ void glds16x16(const unsigned char* g, unsigned lds_dst) {
  const unsigned char* g1 = g + 4096;
  const unsigned char* g2 = g + 8192;
  const unsigned char* g3 = g + 12288;
  unsigned keep;
#define L4(v)                                                                                  \
  "global_load_lds_dwordx4 " v ", off\n\tglobal_load_lds_dwordx4 " v ", off offset:1024\n\t"   \
  "global_load_lds_dwordx4 " v ", off offset:2048\n\tglobal_load_lds_dwordx4 " v ", off offset:3072\n\t"
#define M0 "s_add_u32 m0, m0, 0x1000\n\ts_nop 0\n\t"
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %5\n\ts_nop 0\n\t" L4("%1") M0 L4("%2") M0 L4("%3") M0 L4("%4")
               "s_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(g), "v"(g1), "v"(g2), "v"(g3), "s"(lds_dst)
               : "memory");
#undef L4
#undef M0
}

template <int V>
__global__ void k(const unsigned char* g, long long* out, int reps) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[4 * 16384];
  typedef __attribute__((address_space(3))) unsigned char l8;
  const unsigned base = (unsigned)(uintptr_t)(l8*)&lds[0];
  const int lane = threadIdx.x;
  long long ti = 0, tl = 0;
  int acc = 0;
  for (int r = 0; r < reps; ++r) {
    const unsigned char* p = g + (size_t)r * (4u << 20) + lane * 16;
    if (V == 2) {  // three earlier groups in flight
      glds16x16(p + (1u << 20), base + 16384);
      glds16x16(p + (2u << 20), base + 32768);
      glds16x16(p + (3u << 20), base + 49152);
    }
    const long long t0 = __builtin_amdgcn_s_memtime();
    if (V == 1) {
      typedef int v4i __attribute__((ext_vector_type(4)));
      v4i v[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) v[q] = __builtin_nontemporal_load(reinterpret_cast<const v4i*>(p + 1024 * q));
      const long long t1 = __builtin_amdgcn_s_memtime();
#pragma unroll
      for (int q = 0; q < 16; ++q) acc += v[q].x ^ v[q].w;
      const long long t2 = __builtin_amdgcn_s_memtime();
      ti += t1 - t0;
      tl += t2 - t0;
    } else {
      glds16x16(p, base);
      const long long t1 = __builtin_amdgcn_s_memtime();
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const long long t2 = __builtin_amdgcn_s_memtime();
      ti += t1 - t0;
      tl += t2 - t0;
    }
  }
  if (lane == 0) {
    out[0] = ti / reps;
    out[1] = tl / reps;
    out[2] = acc + lds[lane];
  }
}

int main() {
  unsigned char* g;
  long long* o;
  const int reps = 32;
  hipMalloc(&g, (size_t)(reps + 4) * (4u << 20));
  hipMemset(g, 1, (size_t)(reps + 4) * (4u << 20));
  hipMalloc(&o, 64);
  const char* nm[] = {"A LDS-DMA group", "B VGPR loads", "C LDS-DMA behind 48"};
  for (int v = 0; v < 3; ++v) {
    for (int rep = 0; rep < 2; ++rep) {
      if (v == 0) hipLaunchKernelGGL(k<0>, dim3(1), dim3(64), 0, 0, g, o, reps);
      if (v == 1) hipLaunchKernelGGL(k<1>, dim3(1), dim3(64), 0, 0, g, o, reps);
      if (v == 2) hipLaunchKernelGGL(k<2>, dim3(1), dim3(64), 0, 0, g, o, reps);
      hipDeviceSynchronize();
    }
    long long h[3];
    hipMemcpy(h, o, 24, hipMemcpyDeviceToHost);
    std::printf("%-22s issue %6lld ticks, landed %6lld ticks\n", nm[v], h[0], h[1]);
  }
  return 0;
}
