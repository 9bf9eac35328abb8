// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE for the flow kernels' own access patterns (the
// guide calibrates 16-B-per-lane streaming reads and stores only): each kernel moves exactly 64 MiB.
//   st_nt16   : 16 B per lane non-temporal stores, 1 KiB per wave instruction (pass 2's plane stores)
//   st_nt16x2 : the same, two 1 KiB stores per 2 KiB block (pass 2 R = 2: row-1 then row-2 segment)
//   st_g8     : 8 B per lane agent-scope (sc1) stores, 512 B per instruction (BR / SNAP / granules)
//   ld_g8     : 8 B per lane agent-scope loads, 512 B per instruction (pass 2 reading BR / SNAP)
//   ld_16     : 16 B per lane plain loads, 1 KiB per instruction (the guide's calibrated read)
//   hipcc --offload-arch=gfx950 -O3 -o mbench/mb_wcal mbench/mb_wcal.hip
//   rocprofv3 --pmc WRITE_SIZE -- ./mbench/mb_wcal ; rocprofv3 --pmc FETCH_SIZE -- ./mbench/mb_wcal
#include <hip/hip_runtime.h>
#include <cstdio>
typedef unsigned v4u __attribute__((ext_vector_type(4)));

constexpr size_t kBytes = 64ull << 20;

__global__ void st_nt16(v4u* out) {
  // one wave per 64 KiB: 64 instructions of 1 KiB
  const int lane = threadIdx.x & 63;
  const size_t wave = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  v4u* p = out + wave * 4096 + lane;
  v4u v = {(unsigned)lane, 1u, 2u, 3u};
  for (int i = 0; i < 64; ++i) { __builtin_nontemporal_store(v, p + (size_t)i * 64); v.x += 1; }
}
__global__ void st_nt16x2(v4u* out) {
  const int lane = threadIdx.x & 63;
  const size_t wave = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  v4u* p = out + wave * 4096 + lane;
  v4u v = {(unsigned)lane, 1u, 2u, 3u};
  for (int q = 0; q < 32; ++q) {
    __builtin_nontemporal_store(v, p + (size_t)q * 128);
    v.y += 1;
    __builtin_nontemporal_store(v, p + (size_t)q * 128 + 64);
    v.x += 1;
  }
}
// the R = 2 pattern paced like pass 2 (one 2 KiB phase per ~1,000 cycles), 16 KiB blocks claimed from a
// counter in stripe-interleaved order over a buffer larger than the Infinity Cache
__global__ void st_paced(v4u* out, int* ticket, int nblk, int nseg) {
  const int lane = threadIdx.x & 63;
  for (;;) {
    int t = 0;
    if (lane == 0) t = atomicAdd(ticket, 1);
    t = __builtin_amdgcn_readlane(t, 0);
    if (t >= nblk) break;
    const int s = t % (nblk / nseg), seg = t / (nblk / nseg);  // block (stripe s, segment seg)
    v4u* p = out + ((size_t)s * nseg + seg) * 1024 + lane;    // 16 KiB per block
    v4u v = {(unsigned)lane, (unsigned)t, 2u, 3u};
    for (int q = 0; q < 8; ++q) {
      __builtin_amdgcn_s_sleep(15);
      __builtin_nontemporal_store(v, p + (size_t)q * 128);
      v.y += 1;
      __builtin_nontemporal_store(v, p + (size_t)q * 128 + 64);
      v.x += 1;
    }
  }
}
__global__ void st_g8(unsigned long long* out) {
  const int lane = threadIdx.x & 63;
  const size_t wave = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  unsigned long long* p = out + wave * 8192 + lane;
  for (int i = 0; i < 128; ++i)
    __hip_atomic_store(p + (size_t)i * 64, (unsigned long long)(i + lane), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__global__ void ld_g8(const unsigned long long* in, unsigned long long* sink) {
  const int lane = threadIdx.x & 63;
  const size_t wave = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  const unsigned long long* p = in + wave * 8192 + lane;
  unsigned long long acc = 0;
  for (int i = 0; i < 128; ++i) acc += __hip_atomic_load(p + (size_t)i * 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (acc == 0x123456789ull) sink[0] = acc;  // (never: keeps the loads)
}
__global__ void ld_16(const v4u* in, unsigned* sink) {
  const int lane = threadIdx.x & 63;
  const size_t wave = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  const v4u* p = in + wave * 4096 + lane;
  unsigned acc = 0;
  for (int i = 0; i < 64; ++i) { const v4u v = p[(size_t)i * 64]; acc += v.x ^ v.y ^ v.z ^ v.w; }
  if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
  void *a, *b, *sink;
  // two buffers well past the 256 MiB Infinity Cache between uses (the reads come from HBM)
  if (hipMalloc(&a, kBytes) != hipSuccess || hipMalloc(&b, 512ull << 20) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) {
    printf("alloc failed\n");
    return 1;
  }
  const int waves = (int)(kBytes / 65536), wpb = 4;  // 1024 waves of 64 KiB, 4 per block
  for (int r = 0; r < 2; ++r) {
    hipLaunchKernelGGL(st_nt16, dim3(waves / wpb), dim3(64 * wpb), 0, 0, (v4u*)a);
    hipLaunchKernelGGL(st_nt16x2, dim3(waves / wpb), dim3(64 * wpb), 0, 0, (v4u*)a);
    hipLaunchKernelGGL(st_g8, dim3(waves / wpb), dim3(64 * wpb), 0, 0, (unsigned long long*)a);
    (void)hipMemsetAsync(b, 1, 512ull << 20, 0);  // evicts the 64 MiB from the Infinity Cache
    hipLaunchKernelGGL(ld_g8, dim3(waves / wpb), dim3(64 * wpb), 0, 0, (const unsigned long long*)a,
                       (unsigned long long*)sink);
    (void)hipMemsetAsync(b, 2, 512ull << 20, 0);
    hipLaunchKernelGGL(ld_16, dim3(waves / wpb), dim3(64 * wpb), 0, 0, (const v4u*)a, (unsigned*)sink);
  }
  // 400 MiB (C5's plane) as 25,600 blocks of 16 KiB, 160 stripes x 160 segments
  int* tk;
  if (hipMalloc(&tk, 8) != hipSuccess) return 1;
  for (int r = 0; r < 2; ++r) {
    (void)hipMemsetAsync(tk, 0, 8, 0);
    hipLaunchKernelGGL(st_paced, dim3(1024), dim3(256), 0, 0, (v4u*)b, tk, 25600, 160);
  }
  if (hipDeviceSynchronize() != hipSuccess) { printf("failed\n"); return 1; }
  printf("ok: each kernel moves %zu bytes\n", kBytes);
  return 0;
}
