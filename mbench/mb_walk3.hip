// mb_walk3.hip -- (1) does v_readlane_b32 use only the low 6 bits of its lane select (wave64)?
// (2) ticks per step of the walk's step formulations (a lone wave, 7-step windows unrolled):
//   A: current: f = {13, readlane(w, idx)} >> sh; dl = f & 15; sh = bfe(f, 4, 5); idx += dl; rec |= dl << 4k
//   B: absolute lanes: f = readlane(w, f) >> sh; sh = (f >> 3) & 24; (lane select = f, low 6 bits)
//   C: as B with an explicit & 63 on the lane select
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void lanesel(int* out, int base) {
  const int v = 1000 + (int)threadIdx.x;
  // base is a runtime value: lane selects base + 5 + 64k
  for (int k = 0; k < 4; ++k) {
    const int sel = __builtin_amdgcn_readfirstlane(base + 5 + 64 * k);
    const int r = __builtin_amdgcn_readlane(v, sel);
    if (threadIdx.x == 0) out[k] = r;
  }
}

template <int V>
__global__ void steps(int nwin, unsigned long long* out) {
  const int lane = threadIdx.x;
  const int a = lane >> 3, b = lane & 7;
  // a word whose field s (8 bits at 8s) moves diagonally and keeps the state (lanes stay < 64 within 7 steps)
  unsigned wB = 0, wA = 0;
  for (int s = 0; s < 3; ++s) wB |= (unsigned)((lane + 9) | (s << 6)) << (8 * s);
  wB |= (unsigned)(lane | (3 << 6)) << 24;
  for (int s = 0; s < 3; ++s) wA |= ((lane < 55 ? 9u : 0u) | ((unsigned)(9 * s) << 4)) << (9 * s);
  wA |= 1u << 31;
  (void)a; (void)b;
  unsigned long long rec = 0;
  unsigned sh = 0;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int wdx = 0; wdx < nwin; ++wdx) {
    unsigned r0 = 0, r1 = 0;
    if constexpr (V == 0) {
      int idx = 0;
      unsigned wcode = 0;
#pragma unroll
      for (int kk = 0; kk < 7; ++kk) {
        const unsigned long long w64 = (13ull << 32) | (unsigned)__builtin_amdgcn_readlane((int)wA, idx);
        const unsigned f = (unsigned)(w64 >> sh);
        const unsigned dl = f & 15u;
        sh = (f >> 4) & 31u;
        idx += (int)dl;
        wcode |= dl << (4 * kk);
      }
      r0 = wcode;
      r1 = (unsigned)idx;
    } else {
      unsigned f = 0;
      unsigned fs[7];
#pragma unroll
      for (int kk = 0; kk < 7; ++kk) {
        const unsigned sel = V == 2 ? (f & 63u) : f;
        f = (unsigned)__builtin_amdgcn_readlane((int)wB, (int)sel) >> sh;
        sh = (f >> 3) & 24u;
        fs[kk] = f;
      }
      r0 = (fs[0] & 0xffffu) | (fs[1] << 16) | ((fs[2] & 255u) << 8);
      r1 = (fs[3] & 0xffffu) | (fs[4] << 16) | ((fs[5] & 255u) << 8) | (fs[6] << 24);
    }
    rec += r0 ^ (r1 << 7);
    sh &= 8u;
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) { out[0] = t1 - t0; out[1] = rec; }
}

int main() {
  int* d;
  unsigned long long* o;
  hipMalloc(&d, 64);
  hipMalloc(&o, 64);
  hipLaunchKernelGGL(lanesel, dim3(1), dim3(64), 0, 0, d, 0);
  int h[4];
  hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
  std::printf("readlane(v, 5 + 64k) = %d %d %d %d (lane 5 holds 1005)\n", h[0], h[1], h[2], h[3]);
  const int nwin = 20000;
  const char* nm[] = {"A current step", "B absolute lanes", "C absolute & 63"};
  for (int v = 0; v < 3; ++v) {
    for (int rep = 0; rep < 2; ++rep) {
      if (v == 0) hipLaunchKernelGGL(steps<0>, dim3(1), dim3(64), 0, 0, nwin, o);
      else if (v == 1) hipLaunchKernelGGL(steps<1>, dim3(1), dim3(64), 0, 0, nwin, o);
      else hipLaunchKernelGGL(steps<2>, dim3(1), dim3(64), 0, 0, nwin, o);
      hipDeviceSynchronize();
    }
    unsigned long long r[2];
    hipMemcpy(r, o, 16, hipMemcpyDeviceToHost);
    std::printf("%-20s %7.2f ticks/step\n", nm[v], (double)r[0] / (7.0 * nwin));
  }
  return 0;
}
