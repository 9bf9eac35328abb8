// mb_walk2.hip -- latency of one dependent step of a lone wave's walk, by mechanism:
//   0 readlane:  idx = readlane(w, idx) & 63                        (VALU -> SGPR -> lane select)
//   1 readlane + the walk's step ops (64-bit shift, and, bfe, add)
//   2 movrels:   idx = s[base + idx] & 15  (s_movrels_b32 over 16 SGPRs, pure SALU)
//   3 salu4:     four dependent SALU ops
//   4 lds:       idx = readfirstlane(lds[idx]) & 63  (ds_read_b32 + readfirstlane)
//   5 sload:     idx = s_load_dword(tab + 4 idx) & 63 (scalar cache hit)
//   6 bpermute:  v = ds_bpermute(v * 4, w): a VGPR chain through the LDS crossbar
//   7 readlane pair: two independent chains interleaved (does a second walk overlap?)
// Prints ticks per step (s_memtime) and ns per step.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int V>
__global__ void chain(int n, const unsigned* __restrict__ tab, long long* out) {
  __shared__ unsigned lds[64];
  const int lane = threadIdx.x;
  const unsigned w = (unsigned)((lane * 37 + 11) & 63) | (1u << 31) | ((unsigned)(lane & 7) << 8);
  lds[lane] = w & 63u;
  __syncthreads();
  unsigned idx = 3, idx2 = 5, sh = 0, acc = 0;
  unsigned vv = (unsigned)lane;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int k = 0; k < n; ++k) {
    if constexpr (V == 0) {
      idx = (unsigned)__builtin_amdgcn_readlane((int)w, (int)idx) & 63u;
    } else if constexpr (V == 1) {
      const unsigned long long w64 = (13ull << 32) | (unsigned)__builtin_amdgcn_readlane((int)w, (int)idx);
      const unsigned f = (unsigned)(w64 >> sh);
      const unsigned dl = f & 63u;
      sh = (f >> 8) & 3u;
      idx = (idx + dl) & 63u;
      acc |= dl << (k & 31);
    } else if constexpr (V == 2) {
      unsigned r;
      asm volatile(
          "s_mov_b32 m0, %1\n\t"
          "s_movrels_b32 %0, s80\n\t"
          : "=s"(r)
          : "s"(idx)
          : "m0");
      idx = r & 15u;
    } else if constexpr (V == 3) {
      idx = ((idx * 5u + 1u) ^ (idx >> 3)) & 63u;
      idx = (idx + 7u) & 63u;
    } else if constexpr (V == 4) {
      typedef __attribute__((address_space(3))) unsigned lds_u32;
      const unsigned v = *(volatile lds_u32*)(lds_u32*)&lds[idx];
      idx = __builtin_amdgcn_readfirstlane(v) & 63u;
    } else if constexpr (V == 5) {
      idx = tab[idx];
      idx = __builtin_amdgcn_readfirstlane(idx) & 63u;
    } else if constexpr (V == 6) {
      vv = (unsigned)__builtin_amdgcn_ds_bpermute((int)(vv * 4u), (int)w) & 63u;
    } else {
      idx = (unsigned)__builtin_amdgcn_readlane((int)w, (int)idx) & 63u;
      idx2 = (unsigned)__builtin_amdgcn_readlane((int)w, (int)idx2) & 63u;
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned v0 = __builtin_amdgcn_readfirstlane(vv);
  if (lane == 0) { out[0] = t1 - t0; out[1] = idx + idx2 + acc + sh + v0; }
}

// sets s80..s95 to a 16-entry table, then runs variant 2
__global__ void chain_movrels(int n, const unsigned* tab, long long* out) {
  asm volatile(
      "s_mov_b32 s80, 5\n\ts_mov_b32 s81, 9\n\ts_mov_b32 s82, 14\n\ts_mov_b32 s83, 1\n\t"
      "s_mov_b32 s84, 7\n\ts_mov_b32 s85, 3\n\ts_mov_b32 s86, 12\n\ts_mov_b32 s87, 0\n\t"
      "s_mov_b32 s88, 11\n\ts_mov_b32 s89, 2\n\ts_mov_b32 s90, 15\n\ts_mov_b32 s91, 6\n\t"
      "s_mov_b32 s92, 4\n\ts_mov_b32 s93, 8\n\ts_mov_b32 s94, 13\n\ts_mov_b32 s95, 10" ::
          : "s80", "s81", "s82", "s83", "s84", "s85", "s86", "s87", "s88", "s89", "s90", "s91", "s92", "s93",
            "s94", "s95");
  unsigned idx = 3;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int k = 0; k < n; ++k) {
    unsigned r;
    asm volatile("s_mov_b32 m0, %1\n\ts_movrels_b32 %0, s80" : "=s"(r) : "s"(idx) : "m0", "s80", "s81", "s82", "s83",
                 "s84", "s85", "s86", "s87", "s88", "s89", "s90", "s91", "s92", "s93", "s94", "s95");
    idx = r & 15u;
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = idx; }
}

int main() {
  long long* d;
  unsigned* tab;
  long long h[3];
  hipMalloc(&d, 24);
  hipMalloc(&tab, 256);
  unsigned ht[64];
  for (int i = 0; i < 64; ++i) ht[i] = (unsigned)((i * 37 + 11) & 63);
  hipMemcpy(tab, ht, 256, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int n = 100000;
  const char* names[] = {"readlane", "readlane+step", "movrels", "salu4", "lds+rfl", "sload", "bpermute", "readlane x2"};
  for (int v = 0; v < 8; ++v) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0);
      switch (v) {
        case 0: hipLaunchKernelGGL(chain<0>, dim3(1), dim3(64), 0, 0, n, tab, d); break;
        case 1: hipLaunchKernelGGL(chain<1>, dim3(1), dim3(64), 0, 0, n, tab, d); break;
        case 2: hipLaunchKernelGGL(chain_movrels, dim3(1), dim3(64), 0, 0, n, tab, d); break;
        case 3: hipLaunchKernelGGL(chain<3>, dim3(1), dim3(64), 0, 0, n, tab, d); break;
        case 4: hipLaunchKernelGGL(chain<4>, dim3(1), dim3(64), 0, 0, n, tab, d); break;
        case 5: hipLaunchKernelGGL(chain<5>, dim3(1), dim3(64), 0, 0, n, tab, d); break;
        case 6: hipLaunchKernelGGL(chain<6>, dim3(1), dim3(64), 0, 0, n, tab, d); break;
        default: hipLaunchKernelGGL(chain<7>, dim3(1), dim3(64), 0, 0, n, tab, d); break;
      }
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
      if (rep == 1)
        std::printf("%-16s %8.2f ticks/step  %7.2f ns/step\n", names[v], (double)h[0] / n, ms * 1e6 / n);
    }
  }
  return 0;
}
