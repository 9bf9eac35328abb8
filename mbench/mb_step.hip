// Microbenchmark: cycles per DP step of the SW-linear recurrence for ONE wave
// (variants of the per-step instruction mix).  Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__device__ __forceinline__ int dpp_shr1(int old, int src) { return __builtin_amdgcn_update_dpp(old, src, 0x138, 0xf, 0xf, false); }
__device__ __forceinline__ int imax3(int a, int b, int c) { return max(max(a, b), c); }

__device__ __forceinline__ int* smem_ptr() { extern __shared__ int sm[]; return sm; }
template <int V>
__global__ void kstep(const unsigned* codes, int* out, unsigned long long* cyc, int nsteps, int nwaves_active) {
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  if (w >= nwaves_active) return;
  unsigned plo = 0x01000000u * lane + 0x00020001u, phi = 0x00010203u;
  int X = lane, U = lane - 1, best = 0;
  int negct = -5;
  int gk[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) { gk[k] = -k; asm("" : "+v"(gk[k])); }
  int4 acc = make_int4(0, 0, 0, 0);
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  int hold[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) hold[k] = 0;
  for (int q = 0; q < nsteps / 16; ++q) {
    int hv[16];
    unsigned cw[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) cw[u] = codes[(q * 4 + u) & 1023] + lane;  // scalar-ish load; hoisted by L1
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const unsigned s4 = __builtin_amdgcn_perm(phi, plo, cw[u]);
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int kx = 4 * u + kk;
        const int s = ((int)(s4 << (24 - 8 * kk))) >> 24;
        const int up = dpp_shr1(q + kx, X);
        int h = imax3(U + s, up, X);
        asm("" : "+v"(h));
        U = up;
        X = h;
        if constexpr (V >= 1) hv[kx] = h + negct + gk[kx]; else hv[kx] = h;
      }
      if constexpr (V == 5) {
        typedef int v4l __attribute__((ext_vector_type(4)));
        typedef __attribute__((address_space(3))) v4l lds_v4;
        lds_v4* dstl = (lds_v4*)(smem_ptr()) + (((q & 3) * 4 + u) * 64 + lane) + w * 1024;
        *dstl = v4l{hv[4 * u], hv[4 * u + 1], hv[4 * u + 2], hv[4 * u + 3]};
      } else if constexpr (V >= 3) {
        typedef int v4i __attribute__((ext_vector_type(4)));
        v4i* dst = reinterpret_cast<v4i*>(out) + ((size_t)(blockIdx.x * 16 + w) * 4096 + (q & 1023) * 4 + u) * 64 + lane;
        __builtin_nontemporal_store(v4i{hv[4 * u], hv[4 * u + 1], hv[4 * u + 2], hv[4 * u + 3]}, dst);
      }
    }
    if constexpr (V == 4) {
      // last use of the previous phase's store data: registers stay untouched for a phase
#pragma unroll
      for (int k = 0; k < 16; ++k) asm volatile("" :: "v"(hold[k]));
#pragma unroll
      for (int k = 0; k < 16; ++k) hold[k] = hv[k];
    }
    if constexpr (V >= 2) {
#pragma unroll
      for (int kx = 0; kx < 16; kx += 2) best = imax3(best, hv[kx], hv[kx + 1]);
    } else {
      acc.x ^= hv[15];
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) cyc[blockIdx.x * 16 + w] = t1 - t0;
  if (X == 0x7fffffff) out[lane] = best + acc.x;
}

template <int V>
void run(const char* name, int nblocks, int waves, int active, unsigned* d_codes, int* d_out, unsigned long long* d_cyc) {
  const int nsteps = 16 * 2000;
  hipFuncSetAttribute((const void*)kstep<V>, hipFuncAttributeMaxDynamicSharedMemorySize, 16 * 16384);
  hipLaunchKernelGGL(kstep<V>, dim3(nblocks), dim3(64 * waves), waves * 16384, 0, d_codes, d_out, d_cyc, nsteps, active);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(kstep<V>, dim3(nblocks), dim3(64 * waves), waves * 16384, 0, d_codes, d_out, d_cyc, nsteps, active);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> c(nblocks * 16);
  hipMemcpy(c.data(), d_cyc, c.size() * 8, hipMemcpyDeviceToHost);
  double avg = 0; int cnt = 0;
  for (int b = 0; b < nblocks; ++b) for (int w = 0; w < active; ++w) { avg += c[b * 16 + w]; ++cnt; }
  avg /= cnt;
  printf("%-28s blocks %4d waves/blk %2d active %2d : %.1f cyc/step (memtime)  %.1f ns/step wall\n", name, nblocks, waves,
         active, avg / nsteps, ms * 1e6 / nsteps);
}

int main() {
  unsigned* d_codes; int* d_out; unsigned long long* d_cyc;
  const size_t out_bytes = (size_t)4 * 16 * 4096 * 64 * 16;  // blocks<=4, waves<=16, 4096 quads, 64 lanes, 16 B
  hipMalloc(&d_codes, 4096 * 4); hipMemset(d_codes, 1, 4096 * 4);
  hipMalloc(&d_out, out_bytes);
  hipMalloc(&d_cyc, 256 * 16 * 8);
  for (int wa : {1, 4, 8}) {
    run<2>("+H +best", 1, wa, wa, d_codes, d_out, d_cyc);
    run<3>("+global store", 1, wa, wa, d_codes, d_out, d_cyc);
    run<5>("+ds_write_b128 instead", 1, wa, wa, d_codes, d_out, d_cyc);
  }
  return 0;
}
