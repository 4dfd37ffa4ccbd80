// VALU issue-rate microbenchmark (diagnostics): cycles per wave64
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
    v[i] = seed * (threadIdx.x + i + 1);
    w[i] = seed ^ (threadIdx.x * 7 + i);
  }
  if (OP == 0) BODY("v_add_u32 %0, %0, %1")
  if (OP == 1) BODY("v_max_i32 %0, %0, %1")
  if (OP == 2) BODY("v_alignbit_b32 %0, %0, %1, 31")
  if (OP == 3) BODY("v_add3_u32 %0, %0, %1, %1")
  if (OP == 4) BODY("v_max_f32 %0, %0, %1")
  if (OP == 5) BODY("v_add_f32 %0, %0, %1")
  if (OP == 6) BODY("v_sub_f32 %0, %0, %1")
  if (OP == 7) BODY("v_pk_max_i16 %0, %0, %1")
  if (OP == 8) BODY("v_pk_add_i16 %0, %0, %1 clamp")
  if (OP == 9) BODY("v_pk_sub_i16 %0, %0, %1 clamp")
  if (OP == 10) BODY("v_and_or_b32 %0, %0, %1, %1")
  if (OP == 11) BODY("v_mov_b32 %0, %1")
  if (OP == 12) BODY("v_bfe_i32 %0, %0, %1, 4")
  if (OP == 13) BODY("v_pk_max_f16 %0, %0, %1")
  if (OP == 14) BODY("v_cvt_f32_i32 %0, %1")
  if (OP == 15) BODY("v_max3_f32 %0, %0, %1, %1")

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
  const int blocks = p.multiProcessorCount * 8;  // 8 waves per SIMD
  const char* names[] = {"v_add_u32", "v_max_i32", "v_alignbit_b32", "v_add3_u32", "v_max_f32",
                         "v_add_f32", "v_sub_f32", "v_pk_max_i16", "v_pk_add_i16 clamp",
                         "v_pk_sub_i16 clamp", "v_and_or_b32", "v_mov_b32", "v_bfe_i32",
                         "v_pk_max_f16", "v_cvt_f32_i32", "v_max3_f32"};
  float ms[16];
  ms[0] = run<0>(blocks, out);
  ms[1] = run<1>(blocks, out);
  ms[2] = run<2>(blocks, out);
  ms[3] = run<3>(blocks, out);
  ms[4] = run<4>(blocks, out);
  ms[5] = run<5>(blocks, out);
  ms[6] = run<6>(blocks, out);
  ms[7] = run<7>(blocks, out);
  ms[8] = run<8>(blocks, out);
  ms[9] = run<9>(blocks, out);
  ms[10] = run<10>(blocks, out);
  ms[11] = run<11>(blocks, out);
  ms[12] = run<12>(blocks, out);
  ms[13] = run<13>(blocks, out);
  ms[14] = run<14>(blocks, out);
  ms[15] = run<15>(blocks, out);

  const double waveinst = (double)blocks * 4 * N_ITERS * CHAINS;
  for (int op = 0; op < 16; op++) {
    const double simd_cycles = ms[op] * 1e-3 * 2.4e9 * p.multiProcessorCount * 4;
    printf("%-20s %7.3f ms  %.2f cycles per wave64 instruction per SIMD (2.4 GHz)\n", names[op],
           ms[op], simd_cycles / waveinst);
  }
  return 0;
}
