// VALU issue-rate microbenchmark, third set of forms (float max, DPP, 64-bit shifts) (diagnostics): cycles per wave64
// instruction per SIMD at 8 waves/SIMD, for the instruction forms the DP
// kernels use.  Each form runs as 8 independent dependency chains written in
// inline asm (nothing can be folded).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define N_ITERS 2048
#define CHAINS 8

#define BODY(INS)                                                          \
  for (int it = 0; it < N_ITERS; it++) {                                   \
    _Pragma("unroll") for (int i = 0; i < CHAINS; i++) {                   \
      asm volatile(INS : "+v"(v[i]) : "v"(w[i]));                          \
    }                                                                      \
  }

template <int OP>
__global__ __launch_bounds__(256) void k(uint32_t* out, uint32_t seed) {
  uint32_t v[CHAINS], w[CHAINS];
  for (int i = 0; i < CHAINS; i++) {
    v[i] = 0x40000000u + seed * (threadIdx.x + i + 1);
    w[i] = 0x40000000u + (seed ^ (threadIdx.x * 7 + i));
  }
  if (OP == 0) BODY("v_add_u32 %0, %0, %1")
  if (OP == 1) BODY("v_max_i32 %0, %0, %1")
  if (OP == 2) BODY("v_max_f32 %0, %0, %1")
  if (OP == 3) BODY("v_add_f32 %0, %0, %1")
  if (OP == 4) BODY("v_sub_f32 %0, %0, %1")
  if (OP == 5) BODY("v_max3_f32 %0, %0, %1, %1")
  if (OP == 6) BODY("v_max3_i32 %0, %0, %1, %1")
  if (OP == 7) BODY("v_alignbit_b32 %0, %0, %1, 31")
  if (OP == 8) BODY("v_mov_b32_dpp %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1")
  if (OP == 9) BODY("v_cndmask_b32_e64 %0, %0, %1, s[0:1]")
  if (OP == 10) BODY("v_bfe_u32 %0, %1, %0, 4")
  if (OP == 11) BODY("v_min_f32 %0, %0, %1")
  if (OP == 12) BODY("v_sub_u32 %0, %0, %1")
  if (OP == 13) BODY("v_add3_u32 %0, %0, %1, %1")
  if (OP == 14) BODY("v_max_i16 %0, %0, %1")
  if (OP == 15) BODY("v_pk_max_i16 %0, %0, %1")
  if (OP == 16) BODY("v_pk_add_u16 %0, %0, %1")
  if (OP == 17) BODY("v_lshrrev_b32 %0, 31, %1")
  if (OP == 18) BODY("v_max_u16 %0, %0, %1")
  if (OP == 19) BODY("v_mul_f32 %0, %0, %1")
  uint32_t acc = 0;
  for (int i = 0; i < CHAINS; i++) acc ^= v[i];
  if (acc == 0x12345678u) out[threadIdx.x] = acc;
}
template <int OP>
static float run(int blocks, uint32_t* out) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, out, 3u);
  (void)hipEventRecord(a);
  hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, out, 3u);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms;
}

int main() {
  uint32_t* out;
  (void)hipMalloc(&out, 1024 * 4);
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  const int blocks = p.multiProcessorCount * 8;
  { float ms = run<0>(blocks, out); printf("%-22s %.3f ms  %.2f cycles per wave64 instruction per SIMD\n", "v_add_u32", ms, ms * 1e-3 * 2.4e9 * p.multiProcessorCount * 4 / ((double)blocks * 4 * N_ITERS * CHAINS)); }
  { float ms = run<1>(blocks, out); printf("%-22s %.3f ms  %.2f cycles per wave64 instruction per SIMD\n", "v_max_i32", ms, ms * 1e-3 * 2.4e9 * p.multiProcessorCount * 4 / ((double)blocks * 4 * N_ITERS * CHAINS)); }
  { float ms = run<2>(blocks, out); printf("%-22s %.3f ms  %.2f cycles per wave64 instruction per SIMD\n", "v_max_f32", ms, ms * 1e-3 * 2.4e9 * p.multiProcessorCount * 4 / ((double)blocks * 4 * N_ITERS * CHAINS)); }
  { float ms = run<3>(blocks, out); printf("%-22s %.3f ms  %.2f cycles per wave64 instruction per SIMD\n", "v_add_f32", ms, ms * 1e-3 * 2.4e9 * p.multiProcessorCount * 4 / ((double)blocks * 4 * N_ITERS * CHAINS)); }
  { float ms = run<4>(blocks, out); printf("%-22s %.3f ms  %.2f cycles per wave64 instruction per SIMD\n", "v_sub_f32", ms, ms * 1e-3 * 2.4e9 * p.multiProcessorCount * 4 / ((double)blocks * 4 * N_ITERS * CHAINS)); }
  { float ms = run<5>(blocks, out); printf("%-22s %.3f ms  %.2f cycles per wave64 instruction per SIMD\n", "v_max3_f32", ms, ms * 1e-3 * 2.4e9 * p.multiProcessorCount * 4 / ((double)blocks * 4 * N_ITERS * CHAINS)); }
  { float ms = run<6>(blocks, out); printf("%-22s %.3f ms  %.2f cycles per wave64 instruction per SIMD\n", "v_max3_i32", ms, ms * 1e-3 * 2.4e9 * p.multiProcessorCount * 4 / ((double)blocks * 4 * N_ITERS * CHAINS)); }
  { float ms = run<7>(blocks, out); printf("%-22s %.3f ms  %.2f cycles per wave64 instruction per SIMD\n", "v_alignbit_b32", ms, ms * 1e-3 * 2.4e9 * p.multiProcessorCount * 4 / ((double)blocks * 4 * N_ITERS * CHAINS)); }
  { float ms = run<8>(blocks, out); printf("%-22s %.3f ms  %.2f cycles per wave64 instruction per SIMD\n", "v_mov_b32_dpp", ms, ms * 1e-3 * 2.4e9 * p.multiProcessorCount * 4 / ((double)blocks * 4 * N_ITERS * CHAINS)); }
  { float ms = run<9>(blocks, out); printf("%-22s %.3f ms  %.2f cycles per wave64 instruction per SIMD\n", "v_cndmask_e64 s", ms, ms * 1e-3 * 2.4e9 * p.multiProcessorCount * 4 / ((double)blocks * 4 * N_ITERS * CHAINS)); }
  { float ms = run<10>(blocks, out); printf("%-22s %.3f ms  %.2f cycles per wave64 instruction per SIMD\n", "v_bfe_u32 vshift", ms, ms * 1e-3 * 2.4e9 * p.multiProcessorCount * 4 / ((double)blocks * 4 * N_ITERS * CHAINS)); }
  { float ms = run<11>(blocks, out); printf("%-22s %.3f ms  %.2f cycles per wave64 instruction per SIMD\n", "v_min_f32", ms, ms * 1e-3 * 2.4e9 * p.multiProcessorCount * 4 / ((double)blocks * 4 * N_ITERS * CHAINS)); }
  { float ms = run<12>(blocks, out); printf("%-22s %.3f ms  %.2f cycles per wave64 instruction per SIMD\n", "v_sub_u32", ms, ms * 1e-3 * 2.4e9 * p.multiProcessorCount * 4 / ((double)blocks * 4 * N_ITERS * CHAINS)); }
  { float ms = run<13>(blocks, out); printf("%-22s %.3f ms  %.2f cycles per wave64 instruction per SIMD\n", "v_add3_u32", ms, ms * 1e-3 * 2.4e9 * p.multiProcessorCount * 4 / ((double)blocks * 4 * N_ITERS * CHAINS)); }
  { float ms = run<14>(blocks, out); printf("%-22s %.3f ms  %.2f cycles per wave64 instruction per SIMD\n", "v_max_i16", ms, ms * 1e-3 * 2.4e9 * p.multiProcessorCount * 4 / ((double)blocks * 4 * N_ITERS * CHAINS)); }
  { float ms = run<15>(blocks, out); printf("%-22s %.3f ms  %.2f cycles per wave64 instruction per SIMD\n", "v_pk_max_i16", ms, ms * 1e-3 * 2.4e9 * p.multiProcessorCount * 4 / ((double)blocks * 4 * N_ITERS * CHAINS)); }
  { float ms = run<16>(blocks, out); printf("%-22s %.3f ms  %.2f cycles per wave64 instruction per SIMD\n", "v_pk_add_u16", ms, ms * 1e-3 * 2.4e9 * p.multiProcessorCount * 4 / ((double)blocks * 4 * N_ITERS * CHAINS)); }
  { float ms = run<17>(blocks, out); printf("%-22s %.3f ms  %.2f cycles per wave64 instruction per SIMD\n", "v_lshrrev_b32 c31", ms, ms * 1e-3 * 2.4e9 * p.multiProcessorCount * 4 / ((double)blocks * 4 * N_ITERS * CHAINS)); }
  { float ms = run<18>(blocks, out); printf("%-22s %.3f ms  %.2f cycles per wave64 instruction per SIMD\n", "v_max_u16", ms, ms * 1e-3 * 2.4e9 * p.multiProcessorCount * 4 / ((double)blocks * 4 * N_ITERS * CHAINS)); }
  { float ms = run<19>(blocks, out); printf("%-22s %.3f ms  %.2f cycles per wave64 instruction per SIMD\n", "v_mul_f32", ms, ms * 1e-3 * 2.4e9 * p.multiProcessorCount * 4 / ((double)blocks * 4 * N_ITERS * CHAINS)); }
  return 0;
}
