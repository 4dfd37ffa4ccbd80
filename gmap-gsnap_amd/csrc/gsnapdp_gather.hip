// gsnapdp_gather.hip -- op-stream compaction for the multi-GPU gather.
//
// A batch's op streams live at capacity offsets (op_offsets[i], L1 + L2 + 2
// words per window) because a window's traceback length is only known after
// the fill.  What leaves the GPU -- the RCCL gather of result records and op
// streams to the root rank -- is the compact form: window i's nops words,
// windows in batch order, so the root rebuilds every offset from the nops
// column of the results alone (exclusive prefix sum).  One launch: each block
// counts its windows' ops, publishes the count, and finds its base by a
// decoupled look-back over the preceding blocks' status words (blocks are
// dispatched in index order, so a block only waits on blocks already
// running); then an in-block scan and the copy.  Deterministic layout.
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

// status word of a block: epoch (24 bits) | flag (2 bits) | value (38 bits)
constexpr int ST_VBITS = 38;
constexpr uint64_t ST_VMASK = (1ull << ST_VBITS) - 1;
constexpr uint64_t ST_AGG = 1ull << ST_VBITS, ST_INCL = 2ull << ST_VBITS;
constexpr int ST_EPOCH_SHIFT = ST_VBITS + 2;

__device__ inline int64_t wave_sum64(int64_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  return x;
}

// The ops of the blocks before block b: wave 0 reads 64 predecessors' status
// words at a time, nearest first, and sums them up to the nearest inclusive
// total; an unpublished word stops the window there and is read again.
__device__ inline int64_t look_back(const uint64_t* status, int b, uint64_t epoch, int ln) {
  int64_t acc = 0;
  int p = b - 1;
  while (p >= 0) {
    const int q = p - ln;
    const uint64_t v = q >= 0 ? __hip_atomic_load(status + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                              : ((epoch << ST_EPOCH_SHIFT) | ST_INCL);  // before block 0: total 0
    const bool ok = (v >> ST_EPOCH_SHIFT) == epoch && (v & (ST_AGG | ST_INCL)) != 0;
    const uint64_t incl = __ballot(ok && (v & ST_INCL) != 0), bad = __ballot(!ok);
    const int fi = incl ? __builtin_ctzll(incl) : 64, fb = bad ? __builtin_ctzll(bad) : 64;
    const int lim = fi < fb ? fi + 1 : fb;  // lanes consumed: up to the inclusive one, or the first gap
    acc += wave_sum64(ln < lim ? (int64_t)(v & ST_VMASK) : 0);
    if (fi < fb) break;
    p -= lim;
    if (lim == 0) __builtin_amdgcn_s_sleep(1);
  }
  return acc;
}

__global__ __launch_bounds__(CT) void k_compact(const gsnapdp_result* __restrict__ res, int n,
                                                const uint32_t* __restrict__ ops,
                                                const int64_t* __restrict__ off,
                                                uint64_t* __restrict__ status, uint64_t epoch,
                                                uint32_t* __restrict__ out, int64_t out_cap,
                                                int64_t* __restrict__ header) {
  __shared__ int64_t wsum[CT / 64];
  __shared__ int64_t sbase;
  const int b = (int)blockIdx.x;
  const int i = b * CT + threadIdx.x;
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
  if (wv == 0) {
    int64_t t = 0;
#pragma unroll
    for (int k = 0; k < CT / 64; k++) t += wsum[k];
    const uint64_t tag = epoch << ST_EPOCH_SHIFT;
    if (ln == 0) __hip_atomic_store(status + b, tag | (b == 0 ? ST_INCL : ST_AGG) | (uint64_t)t,
                                    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int64_t base = b == 0 ? 0 : look_back(status, b, epoch, ln);
    if (ln == 0) {
      if (b > 0)
        __hip_atomic_store(status + b, tag | ST_INCL | (uint64_t)(base + t), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      sbase = base;
    }
  }
  __syncthreads();
  int64_t wbase = 0;
  for (int k = 0; k < wv; k++) wbase += wsum[k];
  const int64_t o0 = sbase + wbase + x - c;  // exclusive prefix of window i
  if (i < n && o0 + c <= out_cap) {
    const uint32_t* src = ops + off[i];
    for (int k = 0; k < c; k++) out[o0 + k] = src[k];
  }
  if (b == (int)gridDim.x - 1 && threadIdx.x == CT - 1) {
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
    ctx->compact_epoch = 0;
  }
  // The status words are the context's, so two compactions must not overlap on
  // the GPU (one call's epoch would hide the words the other's look-back waits
  // for, and it would spin forever): each launch waits for the previous one,
  // whatever stream either was issued on.
  if (!ctx->compact_done) HIPCHK(hipEventCreateWithFlags(&ctx->compact_done, hipEventDisableTiming));
  else HIPCHK(hipStreamWaitEvent(st, ctx->compact_done, 0));
  // a fresh epoch per call, so no status word of an earlier call matches;
  // the words are cleared once per 2^24 calls (and on allocation)
  ctx->compact_epoch = (ctx->compact_epoch + 1) & 0xFFFFFFu;
  if (ctx->compact_epoch == 0) ctx->compact_epoch = 1;
  if (ctx->compact_epoch == 1)
    HIPCHK(hipMemsetAsync(ctx->d_csum, 0, (size_t)ctx->csum_cap * sizeof(int64_t), st));
  hipLaunchKernelGGL(k_compact, dim3(nb), dim3(CT), 0, st, d_results, n, d_ops, d_op_offsets,
                     (uint64_t*)ctx->d_csum, (uint64_t)ctx->compact_epoch, d_out, out_cap, d_header);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(ctx->compact_done, st));
  return 0;
}

int gsnapdp__gather_lds_check(size_t max_lds) { return gsnapdp__lds_fits((const void*)&k_compact, 0, max_lds, "k_compact"); }
