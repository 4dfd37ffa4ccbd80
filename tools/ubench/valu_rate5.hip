// VALU issue-rate microbenchmark, fifth set (diagnostics): cycles per wave64
// instruction per SIMD at 1, 2, 3, 4 and 8 waves per SIMD, for the forms a
// v_perm_b32 direction-bit assembly would use (16-bit subs into one half,
// v_perm_b32, v_and_or_b32) beside the current ones (v_sub_u32, v_alignbit_b32,
// v_max_u16) and the 64-bit shift of the match-bit tracking.  CHAINS
// independent dependency chains per wave (8: issue-bound; 1: latency-bound).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define N_ITERS 1024

template <int OP, int CHAINS>
__global__ __launch_bounds__(256) void k(uint32_t* out, uint32_t seed) {
  uint32_t v[CHAINS], w[CHAINS];
  uint64_t q[CHAINS];
  const uint32_t sel = 0x0B0A0908u;
  for (int i = 0; i < CHAINS; i++) {
    v[i] = 0x40000000u + seed * (threadIdx.x + i + 1);
    w[i] = 0x00004000u + (seed ^ (threadIdx.x * 7 + i));
    q[i] = ((uint64_t)v[i] << 32) | w[i];
  }
  for (int it = 0; it < N_ITERS; it++) {
#pragma unroll
    for (int i = 0; i < CHAINS; i++) {
      if (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(v[i]) : "v"(w[i]));
      if (OP == 1) asm volatile("v_max_u16 %0, %0, %1" : "+v"(v[i]) : "v"(w[i]));
      if (OP == 2) asm volatile("v_sub_u16 %0, %0, %1" : "+v"(v[i]) : "v"(w[i]));
      if (OP == 3)
        asm volatile("v_sub_u16_sdwa %0, %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0"
                     : "+v"(v[i]) : "v"(w[i]));
      if (OP == 4) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(v[i]) : "v"(w[i]), "s"(sel));
      if (OP == 5) asm volatile("v_and_or_b32 %0, %1, %0, %0" : "+v"(v[i]) : "v"(w[i]));
      if (OP == 6) asm volatile("v_alignbit_b32 %0, %0, %1, 31" : "+v"(v[i]) : "v"(w[i]));
      if (OP == 7) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(v[i]) : "v"(w[i]));
      if (OP == 8) asm volatile("v_lshrrev_b64 %0, 1, %0" : "+v"(q[i]));
      if (OP == 9) asm volatile("v_lshl_or_b32 %0, %0, 1, %1" : "+v"(v[i]) : "v"(w[i]));
      if (OP == 10) asm volatile("v_bfe_u32 %0, %1, %0, 4" : "+v"(v[i]) : "v"(w[i]));
      if (OP == 11) asm volatile("v_mov_b32_dpp %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"
                                 : "+v"(v[i]) : "v"(w[i]));
      if (OP == 12) asm volatile("v_pk_max_u16 %0, %0, %1" : "+v"(v[i]) : "v"(w[i]));
      if (OP == 13) asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(v[i]) : "v"(w[i]));
      if (OP == 14) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(v[i]) : "v"(w[i]));
      if (OP == 15) asm volatile("v_pk_sub_u16 %0, %0, %1" : "+v"(v[i]) : "v"(w[i]));
      if (OP == 16)  // three simple 32-bit-encoded ops per chain step (counted as 3 instructions)
        asm volatile("v_max_u16 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_sub_u16 %0, %0, %1" : "+v"(v[i]) : "v"(w[i]));
      if (OP == 17)  // their packed forms
        asm volatile("v_pk_max_u16 %0, %0, %1\n v_pk_add_u16 %0, %0, %1\n v_pk_sub_u16 %0, %0, %1" : "+v"(v[i]) : "v"(w[i]));
    }
  }
  uint32_t acc = 0;
  for (int i = 0; i < CHAINS; i++) acc ^= v[i] ^ (uint32_t)q[i];
  if (acc == 0x12345678u) out[threadIdx.x] = acc;
}
static const char* NAMES[] = {"v_add_u32", "v_max_u16", "v_sub_u16", "v_sub_u16_sdwa(hi,pres)", "v_perm_b32",
                              "v_and_or_b32", "v_alignbit_b32", "v_sub_u32", "v_lshrrev_b64", "v_lshl_or_b32",
                              "v_bfe_u32", "v_mov_b32_dpp", "v_pk_max_u16", "v_cndmask_b32_e32",
                              "v_pk_add_u16", "v_pk_sub_u16", "max/add/sub (per op)", "pk max/add/sub (per op)"};
template <int OP, int CHAINS>
static double cyc(int cus, int wps, uint32_t* out) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const int blocks = cus * wps;  // 256 threads = one wave on each of the CU's 4 SIMDs
  hipLaunchKernelGGL((k<OP, CHAINS>), dim3(blocks), dim3(256), 0, 0, out, 3u);
  (void)hipEventRecord(a);
  hipLaunchKernelGGL((k<OP, CHAINS>), dim3(blocks), dim3(256), 0, 0, out, 3u);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  // SIMD cycles / (wave-instructions per SIMD)
  return ms * 1e-3 * 2.4e9 / ((double)wps * N_ITERS * CHAINS * (OP >= 16 ? 3 : 1));
}
template <int OP>
static void row(int cus, uint32_t* out) {
  printf("%-24s", NAMES[OP]);
  const int W[5] = {1, 2, 3, 4, 8};
  for (int i = 0; i < 5; i++) printf(" %6.2f", cyc<OP, 8>(cus, W[i], out));
  printf("   | 1 chain:");
  for (int i = 0; i < 5; i++) printf(" %6.2f", cyc<OP, 1>(cus, W[i], out));
  printf("\n");
}
int main() {
  uint32_t* out;
  (void)hipMalloc(&out, 1024 * 4);
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  printf("cycles per wave64 instruction per SIMD (2.4 GHz), 8 chains at 1/2/3/4/8 waves per SIMD | 1 chain\n");
  row<0>(cus, out); row<1>(cus, out); row<2>(cus, out); row<3>(cus, out); row<4>(cus, out);
  row<5>(cus, out); row<6>(cus, out); row<7>(cus, out); row<8>(cus, out); row<9>(cus, out);
  row<10>(cus, out); row<11>(cus, out); row<12>(cus, out); row<13>(cus, out);
  row<14>(cus, out); row<15>(cus, out); row<16>(cus, out); row<17>(cus, out);
  return 0;
}
