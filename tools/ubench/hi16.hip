// Diagnostics: what 16-bit VOP2 ops (v_max_u16, v_add_u16) leave in bits 16-31 of the
// destination on gfx950: zeroed, preserved, or the source's.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
__global__ void k(uint32_t* out) {
  uint32_t d0, d1, d2;
  const uint32_t a = 0x12340005u, b = 0x56780007u;
  asm volatile("v_mov_b32 %0, 0xdead0000\n\tv_max_u16 %0, %1, %2" : "=&v"(d0) : "v"(a), "v"(b));
  asm volatile("v_mov_b32 %0, 0xdead0000\n\tv_add_u16 %0, %1, %2" : "=&v"(d1) : "v"(a), "v"(b));
  asm volatile("v_mov_b32 %0, 0xdead0000\n\tv_max_i16 %0, %1, %2" : "=&v"(d2) : "v"(a), "v"(b));
  if (threadIdx.x == 0) {
    out[0] = d0;
    out[1] = d1;
    out[2] = d2;
  }
}
int main() {
  uint32_t* o;
  (void)hipMalloc(&o, 16);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, o);
  uint32_t h[3];
  (void)hipMemcpy(h, o, 12, hipMemcpyDeviceToHost);
  printf("v_max_u16 -> %08x\nv_add_u16 -> %08x\nv_max_i16 -> %08x\n", h[0], h[1], h[2]);
  return 0;
}
