// Diagnostics: where the dispatcher places the blocks of a k_fill-shaped grid
// (768 blocks x 256 threads, at most 3 blocks per CU by LDS): per wave its
// block, XCC, SE, CU and SIMD (HW_ID / XCC_ID registers).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

__global__ __launch_bounds__(256) void k_probe(unsigned* out, unsigned long long spin) {
  extern __shared__ unsigned lds[];
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_ID
  const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);  // XCC_ID
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  unsigned x = threadIdx.x;
  while (__builtin_amdgcn_s_memtime() - t0 < spin) x = x * 1664525u + 1013904223u;
  lds[threadIdx.x] = x;
  if ((threadIdx.x & 63) == 0) {
    const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
    out[w * 4 + 0] = blockIdx.x;
    out[w * 4 + 1] = hw;
    out[w * 4 + 2] = xcc;
    out[w * 4 + 3] = lds[(threadIdx.x + 1) & 255];
  }
}

int main(int argc, char** argv) {
  const int nb = argc > 1 ? atoi(argv[1]) : 768;
  const size_t ldsb = argc > 2 ? (size_t)atoi(argv[2]) : 50 * 1024;
  unsigned* d;
  hipMalloc(&d, (size_t)nb * 16 * 4);
  hipLaunchKernelGGL(k_probe, dim3(nb), dim3(256), ldsb, 0, d, 2000000ull);
  hipDeviceSynchronize();
  unsigned* h = (unsigned*)malloc((size_t)nb * 16 * 4);
  hipMemcpy(h, d, (size_t)nb * 16 * 4, hipMemcpyDeviceToHost);
  printf("wave block xcc se sh cu simd waveid\n");
  for (int w = 0; w < nb * 4; w++) {
    const unsigned hw = h[w * 4 + 1];
    printf("%d %u %u %u %u %u %u %u\n", w, h[w * 4], h[w * 4 + 2] & 15, (hw >> 13) & 7, (hw >> 12) & 1,
           (hw >> 8) & 15, (hw >> 4) & 3, hw & 15);
  }
  return 0;
}
