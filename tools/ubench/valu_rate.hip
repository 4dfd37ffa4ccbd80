// VALU issue-rate microbenchmark (diagnostics): wave64 instructions per
// SIMD-cycle for int32 add/max/alignbit, fp32 fma and packed int16 ops.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define N_ITERS 4096
#define CHAINS 8

template <int OP>
__global__ __launch_bounds__(256) void k(uint32_t* out, uint32_t seed) {
  uint32_t v[CHAINS];
  float f[CHAINS];
  for (int i = 0; i < CHAINS; i++) {
    v[i] = seed * (threadIdx.x + i + 1);
    f[i] = (float)v[i] * 1e-9f;
  }
  for (int it = 0; it < N_ITERS; it++) {
#pragma unroll
    for (int i = 0; i < CHAINS; i++) {
      if (OP == 0) v[i] = v[i] + (seed ^ (uint32_t)i);                          // v_add_u32
      if (OP == 1) v[i] = (uint32_t)max((int)v[i], (int)(seed + i)) + 1u;        // v_max + v_add
      if (OP == 2) v[i] = __builtin_amdgcn_alignbit(v[i], v[(i + 1) % CHAINS], 31);  // alignbit
      if (OP == 3) f[i] = __builtin_fmaf(f[i], 1.0000001f, 1e-7f);                // v_fma_f32
      if (OP == 4) {                                                            // v_pk_add_u16
        typedef short s2 __attribute__((ext_vector_type(2)));
        s2 a = __builtin_bit_cast(s2, v[i]);
        s2 b = {(short)seed, (short)i};
        v[i] = __builtin_bit_cast(uint32_t, (s2)(a + b));
      }
    }
  }
  uint32_t acc = 0;
  for (int i = 0; i < CHAINS; i++) acc ^= v[i] ^ __builtin_bit_cast(uint32_t, f[i]);
  if (acc == 0x12345678u) out[threadIdx.x] = acc;
}

int main() {
  uint32_t* out;
  hipMalloc(&out, 1024 * 4);
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int blocks = p.multiProcessorCount * 8;  // 8 waves per SIMD
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const char* names[] = {"v_add_u32", "v_max_i32+v_add_u32", "v_alignbit_b32", "v_fma_f32", "v_pk_add_u16"};
  for (int op = 0; op < 5; op++) {
    for (int rep = 0; rep < 2; rep++) {
      hipEventRecord(a);
      switch (op) {
        case 0: hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, 3u); break;
        case 1: hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, 3u); break;
        case 2: hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, out, 3u); break;
        case 3: hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(256), 0, 0, out, 3u); break;
        case 4: hipLaunchKernelGGL(k<4>, dim3(blocks), dim3(256), 0, 0, out, 3u); break;
      }
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      const double ops_per_chain = (op == 1) ? 2.0 : 1.0;
      const double waveinst = (double)blocks * 4 * N_ITERS * CHAINS * ops_per_chain;
      const double simd_cycles = ms * 1e-3 * 2.4e9 * p.multiProcessorCount * 4;
      if (rep == 1)
        printf("%-22s %.3f ms  %.2f cycles per wave-instruction per SIMD (at 2.4 GHz)\n", names[op], ms,
               simd_cycles / waveinst);
    }
  }
  return 0;
}
