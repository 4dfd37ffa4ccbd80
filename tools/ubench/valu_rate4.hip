// VALU issue-rate microbenchmark, fourth set (diagnostics): carry-chain bit
// pushes (v_sub_co_u32 / v_cmp into vcc + v_addc_co_u32) against alignbit,
// and the e32 / e64 forms of the ops the band fills use.  Cycles per wave64
// instruction (or per listed pair) per SIMD at 8 (or argv[1]) waves/SIMD, 8 independent
// chains per wave, as valu_rate3.hip.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define N_ITERS 2048
#define CHAINS 8

#define BODY(INS)                                                          \
  for (int it = 0; it < N_ITERS; it++) {                                   \
    _Pragma("unroll") for (int i = 0; i < CHAINS; i++) {                   \
      asm volatile(INS : "+v"(v[i]) : "v"(w[i]) : "vcc");                  \
    }                                                                      \
  }
// two-instruction forms with a scratch VGPR
#define BODY2(INS)                                                         \
  for (int it = 0; it < N_ITERS; it++) {                                   \
    _Pragma("unroll") for (int i = 0; i < CHAINS; i++) {                   \
      uint32_t tmp;                                                        \
      asm volatile(INS : "+v"(v[i]), "=&v"(tmp) : "v"(w[i]) : "vcc");     \
    }                                                                      \
  }

template <int OP>
__global__ __launch_bounds__(256) void k(uint32_t* out, uint32_t seed) {
  uint32_t v[CHAINS], w[CHAINS];
  for (int i = 0; i < CHAINS; i++) {
    v[i] = 0x4000u + seed * (threadIdx.x + i + 1);
    w[i] = 0x4000u + (seed ^ (threadIdx.x * 7 + i));
  }
  if (OP == 0) BODY("v_add_u32 %0, %0, %1")
  if (OP == 1) BODY("v_sub_co_u32 %0, vcc, %0, %1")
  if (OP == 2) BODY("v_addc_co_u32 %0, vcc, %0, %0, vcc")
  if (OP == 3) BODY("v_cmp_gt_u32 vcc, %0, %1\n v_addc_co_u32 %0, vcc, %0, %0, vcc")
  if (OP == 4) BODY2("v_sub_co_u32 %1, vcc, %0, %2\n v_addc_co_u32 %0, vcc, %0, %0, vcc")
  if (OP == 5) BODY2("v_sub_u32 %1, %0, %2\n v_alignbit_b32 %0, %0, %1, 31")
  if (OP == 6) BODY("v_max_u32 %0, %0, %1")
  if (OP == 7) BODY("v_max_i32_e64 %0, %0, %1")
  if (OP == 8) BODY("v_and_b32 %0, %0, %1")
  if (OP == 9) BODY("v_or_b32 %0, %0, %1")
  if (OP == 10) BODY("v_lshlrev_b32 %0, 1, %0")
  if (OP == 11) BODY("v_cndmask_b32 %0, %0, %1, vcc")
  if (OP == 12) BODY("v_lshl_add_u32 %0, %0, 1, %1")
  if (OP == 13) BODY("v_add_u16 %0, %0, %1")
  if (OP == 14) BODY("v_sub_u16 %0, %0, %1")
  if (OP == 15) BODY("v_lshrrev_b32 %0, %1, %0")
  if (OP == 16) BODY("v_max_u16 %0, %0, %1")
  if (OP == 17) BODY("v_max_i32 %0, %0, %1")
  if (OP == 18) BODY("v_min_u32 %0, %0, %1")
  if (OP == 19) BODY("v_mov_b32 %0, %1")
  if (OP == 20) BODY("v_xor_b32 %0, %0, %1")
  if (OP == 21) BODY("v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0")
  if (OP == 22) BODY("v_mad_u32_u24 %0, %0, %1, %0")
  if (OP == 23) BODY("v_mul_u32_u24 %0, %0, %1")
  uint32_t acc = 0;
  for (int i = 0; i < CHAINS; i++) acc ^= v[i];
  if (acc == 0x12345678u) out[threadIdx.x] = acc;
}
template <int OP>
static void run(int blocks, uint32_t* out, const char* name, int ninst, int ncu) {
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
  printf("%-34s %.3f ms  %.2f cycles per wave64 form per SIMD (%d inst)\n", name, ms,
         ms * 1e-3 * 2.4e9 * ncu * 4 / ((double)blocks * 4 * N_ITERS * CHAINS), ninst);
}

int main(int argc, char** argv) {
  uint32_t* out;
  (void)hipMalloc(&out, 1024 * 4);
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  const int wps = argc > 1 ? atoi(argv[1]) : 8;  // waves per SIMD
  const int n = p.multiProcessorCount, blocks = n * wps;
  printf("%d waves per SIMD\n", wps);
  run<0>(blocks, out, "v_add_u32", 1, n);
  run<1>(blocks, out, "v_sub_co_u32 e32 (vcc)", 1, n);
  run<2>(blocks, out, "v_addc_co_u32 e32 (vcc)", 1, n);
  run<3>(blocks, out, "v_cmp_gt_u32 e32 + v_addc_co_u32", 2, n);
  run<4>(blocks, out, "v_sub_co_u32 + v_addc_co_u32", 2, n);
  run<5>(blocks, out, "v_sub_u32 + v_alignbit_b32", 2, n);
  run<6>(blocks, out, "v_max_u32", 1, n);
  run<7>(blocks, out, "v_max_i32_e64", 1, n);
  run<8>(blocks, out, "v_and_b32", 1, n);
  run<9>(blocks, out, "v_or_b32", 1, n);
  run<10>(blocks, out, "v_lshlrev_b32 c1", 1, n);
  run<11>(blocks, out, "v_cndmask_b32 e32 (vcc)", 1, n);
  run<12>(blocks, out, "v_lshl_add_u32", 1, n);
  run<13>(blocks, out, "v_add_u16", 1, n);
  run<14>(blocks, out, "v_sub_u16", 1, n);
  run<15>(blocks, out, "v_lshrrev_b32 v", 1, n);
  run<16>(blocks, out, "v_max_u16", 1, n);
  run<17>(blocks, out, "v_max_i32", 1, n);
  run<18>(blocks, out, "v_min_u32", 1, n);
  run<19>(blocks, out, "v_mov_b32", 1, n);
  run<20>(blocks, out, "v_xor_b32", 1, n);
  run<21>(blocks, out, "v_add_u32_sdwa byte0", 1, n);
  run<22>(blocks, out, "v_mad_u32_u24", 1, n);
  run<23>(blocks, out, "v_mul_u32_u24", 1, n);
  return 0;
}
