// gsnapdp_gather.hip -- op-stream compaction for the multi-GPU gather.
//
// A batch's op streams live at capacity offsets (op_offsets[i], L1 + L2 + 2
// words per window) because a window's traceback length is only known after
// the fill.  What leaves the GPU -- the RCCL gather of result records and op
// streams to the root rank -- is the compact form: window i's nops words,
// windows in batch order, so the root rebuilds every offset from the nops
// column of the results alone (exclusive prefix sum).  Two launches: per-block
// op counts, then each block's base (sum of the preceding blocks' counts), an
// in-block scan and the copy.  Deterministic layout, no atomics.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gsnapdp.h"
#include "gsnapdp_ctx.h"

namespace {

constexpr int CT = 1024;  // windows per block (one per thread)

__device__ inline int op_count(const gsnapdp_result* __restrict__ res, const int64_t* __restrict__ off,
                               int i) {
  const int64_t cap = off[i + 1] - off[i];
  int c = res[i].nops;
  if (c < 0) c = 0;
  if ((int64_t)c > cap) c = (int)cap;  // status 2 (op overflow): only `cap` ops were written
  return c;
}

__device__ inline int64_t block_sum(int64_t x, int64_t* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
  if (ln == 0) red[wv] = x;
  __syncthreads();
  int64_t t = 0;
#pragma unroll
  for (int k = 0; k < CT / 64; k++) t += red[k];
  __syncthreads();
  return t;
}

__global__ __launch_bounds__(CT) void k_compact_count(const gsnapdp_result* __restrict__ res, int n,
                                                      const int64_t* __restrict__ off,
                                                      int64_t* __restrict__ bsum) {
  __shared__ int64_t red[CT / 64];
  const int i = blockIdx.x * CT + threadIdx.x;
  const int64_t c = i < n ? op_count(res, off, i) : 0;
  const int64_t t = block_sum(c, red);
  if (threadIdx.x == 0) bsum[blockIdx.x] = t;
}

__global__ __launch_bounds__(CT) void k_compact_write(const gsnapdp_result* __restrict__ res, int n,
                                                      const uint32_t* __restrict__ ops,
                                                      const int64_t* __restrict__ off,
                                                      const int64_t* __restrict__ bsum,
                                                      uint32_t* __restrict__ out, int64_t out_cap,
                                                      int64_t* __restrict__ header) {
  __shared__ int64_t red[CT / 64];
  __shared__ int64_t wsum[CT / 64];
  int64_t pre = 0;
  for (int b = threadIdx.x; b < (int)blockIdx.x; b += CT) pre += bsum[b];
  const int64_t base = block_sum(pre, red);
  const int i = blockIdx.x * CT + threadIdx.x;
  const int c = i < n ? op_count(res, off, i) : 0;
  // inclusive wave scan, then the waves' totals
  const int ln = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int64_t x = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t y = __shfl_up(x, o);
    if (ln >= o) x += y;
  }
  if (ln == 63) wsum[wv] = x;
  __syncthreads();
  int64_t wbase = 0;
  for (int k = 0; k < wv; k++) wbase += wsum[k];
  const int64_t o0 = base + wbase + x - c;  // exclusive prefix of window i
  if (i < n && o0 + c <= out_cap) {
    const uint32_t* src = ops + off[i];
    for (int k = 0; k < c; k++) out[o0 + k] = src[k];
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == CT - 1) {
    header[0] = o0 + c;
    header[1] = (o0 + c) > out_cap ? 1 : 0;
  }
}

}  // namespace

extern "C" int gsnapdp_compact_ops_device(gsnapdp_ctx* ctx, const gsnapdp_result* d_results, int n,
                                          const uint32_t* d_ops, const int64_t* d_op_offsets,
                                          uint32_t* d_out, int64_t out_cap, int64_t* d_header,
                                          void* stream_v) {
  if (!ctx || n < 0 || out_cap < 0) return -1;
  hipStream_t st = stream_v ? (hipStream_t)stream_v : ctx->stream;
  std::lock_guard<std::mutex> lock(ctx->mu);
  HIPCHK(hipSetDevice(ctx->device));
  if (n == 0) {
    HIPCHK(hipMemsetAsync(d_header, 0, 2 * sizeof(int64_t), st));
    return 0;
  }
  const int nb = (n + CT - 1) / CT;
  if (nb > ctx->csum_cap) {
    (void)hipFree(ctx->d_csum);
    ctx->d_csum = nullptr;
    const int cap = nb + nb / 4 + 64;
    HIPCHK(hipMalloc(&ctx->d_csum, (size_t)cap * sizeof(int64_t)));
    ctx->csum_cap = cap;
  }
  hipLaunchKernelGGL(k_compact_count, dim3(nb), dim3(CT), 0, st, d_results, n, d_op_offsets,
                     ctx->d_csum);
  hipLaunchKernelGGL(k_compact_write, dim3(nb), dim3(CT), 0, st, d_results, n, d_ops, d_op_offsets,
                     ctx->d_csum, d_out, out_cap, d_header);
  HIPCHK(hipGetLastError());
  return 0;
}
