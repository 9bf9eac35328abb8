// mb_dma.hip -- single-CU streaming rate of 32 KiB groups from HBM (the walk loader's access pattern:
// one 32 KiB contiguous group per stripe, consecutive groups a stripe apart = MBs), by
//   LDS-DMA (global_load_lds_dwordx4, W waves sharing each group's 32 loads, D groups in flight), or
//   plain global_load_dwordx4 into VGPRs (W waves, one group at a time per wave).
// Prints s_memtime ticks per group, cold (first pass over the buffer) and warm (second pass).
//   hipcc --offload-arch=gfx950 -O3 -o mb_dma mb_dma.hip && ./mb_dma
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <int W, int D>
__global__ __launch_bounds__(256) void k_dma(const unsigned char* g, long long stride, int ngroups, long long* out) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[4 * 32768];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  constexpr int PER = 32 / W;  // loads per wave per group
  const unsigned base = (unsigned)(uintptr_t)&lds[0];
  __syncthreads();
  const long long t0 = (long long)__builtin_amdgcn_s_memtime();
  for (int gi = 0; gi < ngroups; ++gi) {
    const unsigned char* p = g + gi * stride + lane * 16;
    const unsigned dst0 = base + 32768u * (unsigned)(gi & 3);
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int ld = wave * PER + q;  // 1 KiB load index in the group
      unsigned keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(p + 1024 * ld), "s"(dst0 + 1024u * ld) : "memory");
    }
    if constexpr (D == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if constexpr (D == 2) {
      if constexpr (PER == 32) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
      else if constexpr (PER == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      else if constexpr (PER == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      if constexpr (PER == 16) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
      else if constexpr (PER == 8) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(48)" ::: "memory");
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) out[0] = (long long)__builtin_amdgcn_s_memtime() - t0;
}

template <int W>
__global__ __launch_bounds__(256) void k_vgpr(const uint4* g, long long stride16, int ngroups, long long* out,
                                               unsigned* sink) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr int PER = 32 / W;
  unsigned acc = 0;
  __syncthreads();
  const long long t0 = (long long)__builtin_amdgcn_s_memtime();
  for (int gi = 0; gi < ngroups; ++gi) {
    uint4 v[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) v[q] = g[gi * stride16 + (wave * PER + q) * 64 + lane];
#pragma unroll
    for (int q = 0; q < PER; ++q) acc ^= v[q].x ^ v[q].w;
  }
  __syncthreads();
  if (threadIdx.x == 0) out[0] = (long long)__builtin_amdgcn_s_memtime() - t0;
  if (acc == 0x12345678u) sink[threadIdx.x] = acc;
}

// where does wave 1's LDS-DMA land: M0 + 16 x lane, or M0 + 16 x (thread id in the workgroup)?
__global__ void k_tid(const unsigned* g, unsigned* out) {
  __shared__ __attribute__((aligned(16))) unsigned lds[1024];
  for (int x = threadIdx.x; x < 1024; x += 128) lds[x] = 0xdeadbeefu;
  __syncthreads();
  if (threadIdx.x >= 64) {
    const unsigned char* p = reinterpret_cast<const unsigned char*>(g) + (threadIdx.x & 63) * 16;
    const unsigned dst = (unsigned)(uintptr_t)&lds[0];
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0\n\ts_waitcnt vmcnt(0)"
                 : "=&s"(keep) : "v"(p), "s"(dst) : "memory");
  }
  __syncthreads();
  if (threadIdx.x == 0) { out[0] = lds[0]; out[1] = lds[256]; out[2] = lds[4]; out[3] = lds[260]; }
}

// does an LDS read of the issuing wave wait behind its own LDS-DMA (lgkmcnt, or the LDS queue)?
__global__ void k_lgkm(const unsigned char* g, long long* out) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[65536];
  __shared__ int flag;
  if (threadIdx.x == 0) flag = 7;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const unsigned dst0 = (unsigned)(uintptr_t)&lds[0];
  const unsigned char* p = g + lane * 16;
  const long long t0 = (long long)__builtin_amdgcn_s_memtime();
#pragma unroll
  for (int ld = 0; ld < 32; ++ld) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(p + 1024 * ld), "s"(dst0 + 1024u * ld) : "memory");
  }
  const long long t1 = (long long)__builtin_amdgcn_s_memtime();
  const int f = __hip_atomic_load(&flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);  // ds_read + lgkmcnt wait
  asm volatile("s_waitcnt lgkmcnt(0)" : : "v"(f) : "memory");
  const long long t2 = (long long)__builtin_amdgcn_s_memtime();
  __hip_atomic_store(&flag, f + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);  // ds_write + lgkmcnt wait
  asm volatile("s_waitcnt lgkmcnt(0)" : : : "memory");
  const long long t2b = (long long)__builtin_amdgcn_s_memtime();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const long long t3 = (long long)__builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = t2 - t1; out[2] = t3 - t2b; out[3] = t2b - t2; }
}

int main(int argc, char** argv) {
  if (argc > 1) {
    // mb_dma <stride MiB> <groups> <backwards 0/1>: one W=1 D=2 pass over a big buffer (TLB reach)
    const long long st = atoll(argv[1]) << 20;
    const int ng = atoi(argv[2]);
    const int back = argc > 3 ? atoi(argv[3]) : 0;
    unsigned char* gb;
    long long* ob;
    if (hipMalloc(&gb, (size_t)st * ng + 65536) != hipSuccess) { std::printf("alloc failed\n"); return 1; }
    hipMalloc(&ob, 8);
    hipMemset(gb, 1, (size_t)st * ng + 65536);
    hipDeviceSynchronize();
    const unsigned char* p0 = back ? gb + (size_t)st * (ng - 1) : gb;
    const long long sst = back ? -st : st;
    for (int pass = 0; pass < 2; ++pass) {
      hipLaunchKernelGGL((k_dma<1, 2>), 1, 64, 0, 0, p0 + pass * 32768, sst, ng, ob);
      hipDeviceSynchronize();
      long long t;
      hipMemcpy(&t, ob, 8, hipMemcpyDeviceToHost);
      std::printf("stride %lld MiB, %d groups, %s, pass %d: %.0f ticks/group\n", st >> 20, ng, back ? "backwards" : "forwards",
                  pass, (double)t / ng);
    }
    return 0;
  }
  {
    unsigned h[256], *gg, *oo, r[4];
    for (int x = 0; x < 256; ++x) h[x] = 0x1000 + x;
    hipMalloc(&gg, 1024); hipMalloc(&oo, 16);
    hipMemcpy(gg, h, 1024, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_tid, dim3(1), dim3(128), 0, 0, gg, oo);
    hipMemcpy(r, oo, 16, hipMemcpyDeviceToHost);
    std::printf("wave-1 DMA: lds[0]=%x lds[256]=%x lds[4]=%x lds[260]=%x (lds[0]=1000: lane-relative; lds[256]=1000: thread-id relative)\n",
                r[0], r[1], r[2], r[3]);
  }
  const long long stride = 12LL << 20;  // 12 MiB between consecutive groups (a 97k-column stripe)
  const int ngroups = 200;
  const size_t bytes = (size_t)stride * ngroups + 65536;
  unsigned char* g;
  long long* o;
  unsigned* sink;
  hipMalloc(&g, bytes);
  hipMalloc(&o, 8);
  hipMalloc(&sink, 1024);
  hipMemset(g, 1, bytes);
  auto run = [&](const char* name, auto launch) {
    long long t[2];
    for (int pass = 0; pass < 2; ++pass) {
      // evict: touch a 1 GiB buffer in between (the first pass reads cold data)
      launch();
      hipDeviceSynchronize();
      hipMemcpy(&t[pass], o, 8, hipMemcpyDeviceToHost);
    }
    std::printf("%-28s cold %7.0f ticks/group (%5.1f B/tick)  warm %7.0f ticks/group\n", name, (double)t[0] / ngroups,
                32768.0 * ngroups / t[0], (double)t[1] / ngroups);
  };
  {
    long long* o4;
    hipMalloc(&o4, 32);
    long long r[4];
    for (int rep = 0; rep < 3; ++rep) {
      hipLaunchKernelGGL(k_lgkm, dim3(1), dim3(64), 0, 0, g + (size_t)(rep + 100) * stride, o4);
      hipMemcpy(r, o4, 32, hipMemcpyDeviceToHost);
      std::printf("lgkm: issue 32 DMA %lld ticks, then an LDS read %lld ticks, then vmcnt(0) %lld ticks (an LDS write before it: %lld ticks)\n",
                  r[0], r[1], r[2], r[3]);
    }
  }
  // a fresh region per variant so that the first pass is cold
  long long off = 0;
  auto next = [&]() { off += 65536; return g + off; };
  const unsigned char* p;
  p = next(); run("dma W=1 D=1", [&] { hipLaunchKernelGGL((k_dma<1, 1>), 1, 64, 0, 0, p, stride, ngroups, o); });
  p = next(); run("dma W=1 D=2", [&] { hipLaunchKernelGGL((k_dma<1, 2>), 1, 64, 0, 0, p, stride, ngroups, o); });
  p = next(); run("dma W=2 D=1", [&] { hipLaunchKernelGGL((k_dma<2, 1>), 1, 128, 0, 0, p, stride, ngroups, o); });
  p = next(); run("dma W=2 D=3", [&] { hipLaunchKernelGGL((k_dma<2, 3>), 1, 128, 0, 0, p, stride, ngroups, o); });
  p = next(); run("dma W=4 D=1", [&] { hipLaunchKernelGGL((k_dma<4, 1>), 1, 256, 0, 0, p, stride, ngroups, o); });
  p = next(); run("dma W=4 D=3", [&] { hipLaunchKernelGGL((k_dma<4, 3>), 1, 256, 0, 0, p, stride, ngroups, o); });
  p = next(); run("vgpr W=1", [&] { hipLaunchKernelGGL((k_vgpr<1>), 1, 64, 0, 0, (const uint4*)p, stride / 16, ngroups, o, sink); });
  p = next(); run("vgpr W=4", [&] { hipLaunchKernelGGL((k_vgpr<4>), 1, 256, 0, 0, (const uint4*)p, stride / 16, ngroups, o, sink); });
  return 0;
}
