// mb_glds.hip -- where does global_load_lds_dwordx4 with an instruction offset land in LDS?
// Loads global bytes [1024, 2048) (value = byte index / 16) with M0 = 0 and offset:1024, then
// prints the LDS dword at 0 and at 1024.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(const unsigned* g, unsigned* out) {
  __shared__ unsigned lds[1024];
  for (int x = threadIdx.x; x < 1024; x += 64) lds[x] = 0xdeadbeefu;
  __syncthreads();
  typedef __attribute__((address_space(3))) unsigned char l8;
  const unsigned dst = (unsigned)(uintptr_t)(l8*)&lds[0];
  const unsigned char* p = reinterpret_cast<const unsigned char*>(g) + threadIdx.x * 16;
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off offset:1024\n\ts_mov_b32 m0, %0\n\ts_waitcnt vmcnt(0)"
               : "=&s"(keep) : "v"(p), "s"(dst) : "memory");
  __syncthreads();
  if (threadIdx.x == 0) { out[0] = lds[0]; out[1] = lds[256]; out[2] = lds[4]; out[3] = lds[260]; }
}
int main() {
  unsigned h[1024], *g, *o, r[4];
  for (int x = 0; x < 1024; ++x) h[x] = x;
  hipMalloc(&g, 4096); hipMalloc(&o, 16);
  hipMemcpy(g, h, 4096, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, g, o);
  hipMemcpy(r, o, 16, hipMemcpyDeviceToHost);
  std::printf("lds[0]=%x lds[256]=%x lds[4]=%x lds[260]=%x (global dword 256 = 0x100: offset applied to LDS too if lds[256]=100)\n", r[0], r[1], r[2], r[3]);
  return 0;
}
