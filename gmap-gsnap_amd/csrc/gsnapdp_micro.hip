// gsnapdp_micro.hip -- Dynprog_microexon_int (reference src/dynprog.c:7128-7432,
// non-PMAP, use_genomicseg_p false) on gfx950, batched: one wave per call.
//
// Per call the wave
//   1. finds the left / right boundaries (the second query/genome mismatch
//      from either end, :7241-7290) with ballots over 64 positions at a time;
//   2. enumerates the (cL, cR) pairs with the intron dinucleotides (GT..AG, or
//      CT..AC antisense) in the reference's loop order (:7292-7320);
//   3. for each pair finds every exact hit of the middle query segment in the
//      intron (BoyerMoore_nt, boyer-moore.c:384: the good-suffix / bad-character
//      shifts only skip positions that cannot match, so the hit set is the set
//      of exact matches), lane-parallel over text positions, from the intron
//      staged once in LDS as 2-bit classes;
//   4. scores every hit whose flanks carry the intron dinucleotides with the
//      MaxEnt site probabilities (:7338-7378) and keeps the best by the f64 sum
//      prob2 + prob3 under the reference's strict `>` in its visiting order
//      (pairs in loop order, hits of a pair from the largest offset down: the
//      Intlist pushes them as they are found);
//   5. records the last hit examined, which the reference passes to
//      make_microexon_pairs_double instead of the best one (:7412-7413).
// The host rebuilds the pairs (gsnapdp_micro_expand, gsnapdp_host.cpp).
//
// The minimum microexon length (:7226-7238) is a ceil of libm pow/log of the
// intron span; so that it matches the reference's libm bit for bit, the host
// tabulates, per quality bin, the spans at which it steps (micro_thresholds)
// and the kernel only compares the span against them.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <mutex>

#include "gsnapdp_ctx.h"
#include "gsnapdp_device.h"
#include "gsnapdp_internal.h"

using namespace gsnapdp;

namespace {

constexpr int MIN_MICROEXON_LENGTH = 3;   // dynprog.c:133
constexpr int MAX_MICROEXON_LENGTH = 12;  // dynprog.c:137 (non-PMAP)
constexpr int GTAG_FWD = 0x20, GTAG_REV = 0x04, NONINTRON = 0x00;  // intron.h
constexpr int TEXT_CAP = 8192;  // LDS bytes of staged intron per wave
constexpr int NTHR = MAX_MICROEXON_LENGTH + 2 - MIN_MICROEXON_LENGTH;  // thresholds for 4..13

struct Thresholds {
  // span >= t[b][v - 4] <=> min_microexon_length (before the MIN clamp) >= v, v = 4..13
  int t[3][NTHR - 1];
};

// min_microexon_length after the MIN clamp; > MAX means "no search" (:7230-7238)
__device__ inline int min_length(const Thresholds& T, int bin, int span) {
  int v = MIN_MICROEXON_LENGTH;
  for (int k = 0; k < NTHR - 1; k++) v += span >= T.t[bin][k] ? 1 : 0;
  return v;
}

// get_genomic_nt of boyer-moore.c:361-380 (no '*' rules) as a class 0..4
__device__ inline int raw_class(const uint32_t* __restrict__ blocks, uint64_t nwords, const Lane& L,
                                int gpos) {
  const uint32_t pos = L.watson ? (L.base + (uint32_t)gpos)
                                : (L.base + (uint32_t)(L.glen - 1) - (uint32_t)gpos);
  const uint64_t ptr = (uint64_t)(pos >> 5) * 3u;
  if (ptr + 2 >= nwords) return 4;
  const uint32_t bit = pos & 31u;
  if ((blocks[ptr + 2] >> bit) & 1u) return 4;
  const uint32_t word = bit < 16 ? blocks[ptr + 1] : blocks[ptr];
  const int code = (int)((word >> ((bit & 15u) * 2u)) & 3u);
  return L.watson ? code : 3 - code;
}

// `sequenceuc1[i] != c` of :7249 / :7276 with c a get_genomic_nt class
__device__ inline bool nt_class_eq(unsigned char u, int g) {
  return u == (unsigned char)("ACGTN*"[g]);
}

__device__ inline int nt_class(unsigned char c) {
  return c == 'A' ? 0 : c == 'C' ? 1 : c == 'G' ? 2 : c == 'T' ? 3 : 4;
}

// lane index of the k-th (0-based) set bit of m, or 64
__device__ inline int nth_bit(uint64_t m, int k) {
  for (int i = 0; i < k && m; i++) m &= m - 1;
  return m ? __ffsll((unsigned long long)m) - 1 : 64;
}

__global__ __launch_bounds__(256) void k_micro(const gsnapdp_micro_window* __restrict__ Wn, int n,
                                               const char* __restrict__ q, const char* __restrict__ qu,
                                               const uint32_t* __restrict__ blocks, uint64_t nwords,
                                               const double* __restrict__ tables, Thresholds T,
                                               gsnapdp_micro_result* __restrict__ res) {
  __shared__ uint8_t text_lds[4][TEXT_CAP];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint8_t* text = text_lds[wv];
  const int gw = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const int nw = (int)((gridDim.x * blockDim.x) >> 6);
  for (int wi = gw; wi < n; wi += nw) {
    const gsnapdp_micro_window w = Wn[wi];
    gsnapdp_micro_result R;
    memset(&R, 0, sizeof(R));
    R.dynprogindex = w.dynprogindex;
    const int L1 = w.length1, span = w.revoffset2R - w.offset2L;
    const int cdir = w.cdna_direction;
    R.microintrontype = cdir > 0 ? GTAG_FWD : cdir < 0 ? GTAG_REV : NONINTRON;
    if (cdir == 0 || span <= 0 || tables == nullptr) {  // the reference aborts (:7203, :7223)
      R.status = ST_UNSUPPORTED;
      if (lane == 0) res[wi] = R;
      continue;
    }
    const double dr = (double)w.defect_rate;
    const int bin = dr < 0.003 ? 0 : (dr < 0.014 ? 1 : 2);
    const int minlen = min_length(T, bin, span);
    if (minlen > MAX_MICROEXON_LENGTH || L1 <= 0) {
      R.microintrontype = NONINTRON;
      if (lane == 0) res[wi] = R;
      continue;
    }
    // get_genomic_nt of dynprog.c (the '*' rules) through a Lane view
    gsnapdp_window lw;
    memset(&lw, 0, sizeof(lw));
    lw.chroffset = w.chroffset;
    lw.chrhigh = w.chrhigh;
    lw.chrpos = w.chrpos;
    lw.genomiclength = w.genomiclength;
    lw.watsonp = w.watsonp;
    lw.length1 = 1;
    lw.length2 = 1;
    const Lane L = make_lane(lw);
    auto gnt = [&](int p) { return gclass(blocks, nwords, L, p); };
    const int i1 = cdir > 0 ? 2 : 1, i2 = 3, i3 = 0, i4 = cdir > 0 ? 2 : 1;  // GT..AG / CT..AC
    const char* u1 = qu + w.qpos;
    // ---- boundaries: the second mismatch from each end (:7241-7290)
    int leftbound = L1 - 2, rightbound = L1 - 1;
    {
      int seen = 0;
      for (int b = 0; b < L1 - 1 && seen < 2; b += 64) {
        const int p = b + lane;
        const bool mm = p < L1 - 1 && nt_class_eq((unsigned char)u1[p], gnt(w.offset2L + p)) == 0;
        const uint64_t m = __ballot(mm);
        const int need = 2 - seen;
        const int at = nth_bit(m, need - 1);
        if (at < 64) {
          leftbound = min(leftbound, b + at);
          seen = 2;
        } else {
          seen += __popcll(m);
        }
      }
      seen = 0;
      for (int b = 0; b < L1 && seen < 2; b += 64) {
        const int k = b + lane;
        const bool mm = k < L1 && nt_class_eq((unsigned char)u1[L1 - 1 - k], gnt(w.revoffset2R - k)) == 0;
        const uint64_t m = __ballot(mm);
        const int at = nth_bit(m, 2 - seen - 1);
        if (at < 64) {
          rightbound = min(rightbound, b + at);
          seen = 2;
        } else {
          seen += __popcll(m);
        }
      }
    }
    // ---- stage the intron text [offset2L, revoffset2R] as raw classes
    const int tlo = w.offset2L, tlen = span + 1;
    const bool staged = tlen <= TEXT_CAP;
    if (staged) {
      for (int p = lane; p < tlen; p += 64) text[p] = (uint8_t)raw_class(blocks, nwords, L, tlo + p);
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    auto tch = [&](int p) -> int {
      return staged ? (int)text[p - tlo] : raw_class(blocks, nwords, L, p);
    };
    // ---- pairs, hits, probabilities
    double bestprob = 0.0, bp2 = 0.0, bp3 = 0.0;
    int bestcL = -1, bestcR = -1, bestmid = 0, candidate = 0;
    for (int cb = 1; cb <= leftbound; cb += 64) {
      const int cLl = cb + lane;
      const bool gt = cLl <= leftbound && gnt(w.offset2L + cLl) == i1 && gnt(w.offset2L + cLl + 1) == i2;
      uint64_t gm = __ballot(gt);
      while (gm) {
        const int cL = cb + __ffsll((unsigned long long)gm) - 1;
        gm &= gm - 1;
        const int mincR = max(1, L1 - MAX_MICROEXON_LENGTH - cL);
        const int maxcR = min(rightbound, L1 - minlen - cL);
        for (int cR = mincR; cR <= maxcR; cR++) {
          if (!(gnt(w.revoffset2R - cR - 1) == i3 && gnt(w.revoffset2R - cR) == i4)) continue;
          const int mid = L1 - cL - cR;
          const int textleft = w.offset2L + cL + MICROINTRON_LENGTH;
          const int textright = w.revoffset2R - cR - MICROINTRON_LENGTH;
          const int textlen = textright - textleft;
          // query_okay (boyer-moore.c:313): A C G T only; the middle as classes
          uint32_t qcode = 0;
          bool ok = true;
          for (int k = 0; k < mid; k++) {
            const int c = nt_class((unsigned char)u1[cL + k]);
            ok = ok && c < 4;
            qcode |= (uint32_t)(c & 3) << (2 * k);
          }
          if (!ok) continue;
          const int nj = textlen - mid + 1;  // j in [0, textlen - mid]
          int lastmin = 1 << 30;              // smallest hit j of this pair
          double pbest = -1.0, pp2 = 0.0, pp3 = 0.0;
          int pj = -1;                        // this lane's chosen j (largest among its ties)
          for (int j0 = 0; j0 < nj; j0 += 64) {
            const int j = j0 + lane;
            bool hit = j < nj;
            for (int k = 0; k < mid && hit; k++) {
              const int c = tch(textleft + j + k);
              hit = c == (int)((qcode >> (2 * k)) & 3u);
            }
            if (!hit) continue;
            lastmin = min(lastmin, j);
            const int cand = textleft + j;
            if (gnt(cand - 2) == i3 && gnt(cand - 1) == i4 && gnt(cand + mid) == i1 &&
                gnt(cand + mid + 1) == i2) {
              // :7338-7378, use_genomicseg_p false
              int m2, m3;
              uint32_t sp2, sp3;
              if (w.watsonp) {
                sp2 = w.chrpos + (uint32_t)(cand - 1) + 1u;
                sp3 = w.chrpos + (uint32_t)cand + (uint32_t)mid;
                m2 = cdir > 0 ? GSNAPDP_ACCEPTOR : GSNAPDP_ANTIDONOR;
                m3 = cdir > 0 ? GSNAPDP_DONOR : GSNAPDP_ANTIACCEPTOR;
              } else {
                sp2 = w.chrpos + (w.genomiclength - 1u) - (uint32_t)(cand - 1);
                sp3 = w.chrpos + (w.genomiclength - 1u) - (uint32_t)(cand + mid) + 1u;
                m2 = cdir > 0 ? GSNAPDP_ANTIACCEPTOR : GSNAPDP_DONOR;
                m3 = cdir > 0 ? GSNAPDP_ANTIDONOR : GSNAPDP_ACCEPTOR;
              }
              const double p2 = maxent_prob(m2, w.chroffset + sp2, w.chroffset, blocks, nwords, tables);
              const double p3 = maxent_prob(m3, w.chroffset + sp3, w.chroffset, blocks, nwords, tables);
              const double sum = __dadd_rn(p2, p3);
              // visiting order within a pair is j descending: a later (larger) j
              // of this lane wins ties
              if (sum >= pbest) {
                pbest = sum;
                pp2 = p2;
                pp3 = p3;
                pj = j;
              }
            }
          }
          // the pair's last-examined hit (the smallest j), if any
          int lm = lastmin;
#pragma unroll
          for (int o = 32; o > 0; o >>= 1) lm = min(lm, __shfl_xor(lm, o));
          if (lm < (1 << 30)) candidate = textleft + lm;
          // ordered argmax over lanes: largest sum, then largest j
          double bs = pj >= 0 ? pbest : -1.0;
          int bj = pj;
#pragma unroll
          for (int o = 32; o > 0; o >>= 1) {
            const double os = __shfl_xor(bs, o);
            const int oj = __shfl_xor(bj, o);
            if (os > bs || (os == bs && oj > bj)) {
              bs = os;
              bj = oj;
            }
          }
          if (bj >= 0 && bs > bestprob) {  // `prob2 + prob3 > bestprob` (:7380)
            const int src = __ffsll((unsigned long long)__ballot(pj == bj && pj >= 0)) - 1;
            bp2 = __shfl(pp2, src);
            bp3 = __shfl(pp3, src);
            bestprob = bs;
            bestcL = cL;
            bestcR = cR;
            bestmid = mid;
          }
        }
      }
    }
    if (bestcL < 0 || bestcR < 0) {
      R.microintrontype = NONINTRON;
      R.bestprob2 = 0.0;
      R.bestprob3 = 0.0;
    } else {
      R.found = 1;
      R.bestprob2 = bp2;
      R.bestprob3 = bp3;
      R.bestcL = bestcL;
      R.bestcR = bestcR;
      R.middlelength = bestmid;
      R.offset2M = candidate;
      R.dynprogindex = step_dpi(w.dynprogindex);
    }
    if (lane == 0) res[wi] = R;
  }
}

}  // namespace

// Spans at which min_microexon_length steps, per quality bin, computed with
// the host libm exactly as dynprog.c:7226-7229 computes it.
static int host_min_len(double pvalue, int span) {
  int m = (int)ceil(-log(1.0 - pow(1.0 - pvalue, 1.0 / (double)span)) / log(4));
  return m - 8;
}

static const Thresholds& micro_thresholds() {
  static Thresholds T;
  static std::once_flag once;
  std::call_once(once, [] {
    const double pv[3] = {0.01, 0.001, 0.0001};  // MICROEXON_PVALUE_HIGHQ/MEDQ/LOWQ (:128-130)
    for (int b = 0; b < 3; b++) {
      for (int v = MIN_MICROEXON_LENGTH + 1; v <= MAX_MICROEXON_LENGTH + 1; v++) {
        // smallest span >= 1 with host_min_len >= v (nondecreasing in span)
        int lo = 1, hi = 0x7fffffff;
        if (host_min_len(pv[b], hi) < v) {
          T.t[b][v - 4] = 0x7fffffff;
          continue;
        }
        while (lo < hi) {
          const int m = lo + (hi - lo) / 2;
          if (host_min_len(pv[b], m) >= v) hi = m;
          else lo = m + 1;
        }
        T.t[b][v - 4] = lo;
      }
    }
  });
  return T;
}

extern "C" int gsnapdp_micro_run_device(gsnapdp_ctx* ctx, const gsnapdp_micro_window* d_windows,
                                        int n, const char* d_query, const char* d_query_uc,
                                        gsnapdp_micro_result* d_results, void* stream_v) {
  if (!ctx) return -1;
  if (n <= 0) return 0;
  hipStream_t st = stream_v ? (hipStream_t)stream_v : ctx->stream;
  std::lock_guard<std::mutex> lock(ctx->mu);
  HIPCHK(hipSetDevice(ctx->device));
  const Thresholds& T = micro_thresholds();
  const int blocks = std::min((n + 3) / 4, ctx->num_cus * 8);
  hipLaunchKernelGGL(k_micro, dim3(blocks), dim3(256), 0, st, d_windows, n, d_query, d_query_uc,
                     ctx->d_blocks, (uint64_t)ctx->nwords, ctx->d_tables, T, d_results);
  HIPCHK(hipGetLastError());
  return 0;
}

extern "C" int gsnapdp_micro_run_host(gsnapdp_ctx* ctx, const gsnapdp_micro_window* windows, int n,
                                      const char* query, const char* query_uc, size_t query_bytes,
                                      gsnapdp_micro_result* results) {
  if (!ctx) return -1;
  if (n <= 0) return 0;
  // one host round trip at a time: the staging buffer is the context's
  std::lock_guard<std::mutex> host_lock(ctx->host_mu);
  HIPCHK(hipSetDevice(ctx->device));
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t szw = al((size_t)n * sizeof(gsnapdp_micro_window));
  const size_t szq = al(query_bytes + 4);
  const size_t szr = al((size_t)n * sizeof(gsnapdp_micro_result));
  const size_t total = szw + 2 * szq + szr;
  {
    std::lock_guard<std::mutex> lock(ctx->mu);
    if (total > ctx->ggap_stage_cap) {
      (void)hipFree(ctx->d_ggap_stage);
      ctx->d_ggap_stage = nullptr;
      HIPCHK(hipMalloc(&ctx->d_ggap_stage, total));
      ctx->ggap_stage_cap = total;
    }
  }
  char* b = (char*)ctx->d_ggap_stage;
  gsnapdp_micro_window* dw = (gsnapdp_micro_window*)b;
  char* dq = b + szw;
  char* du = dq + szq;
  gsnapdp_micro_result* dr = (gsnapdp_micro_result*)(du + szq);
  hipStream_t st = ctx->stream;
  HIPCHK(hipMemcpyAsync(dw, windows, (size_t)n * sizeof(gsnapdp_micro_window), hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(dq, query, query_bytes, hipMemcpyHostToDevice, st));
  // a caller that passes one buffer for both (query already upper case) pays one copy
  if (query_uc == query) du = dq;
  else HIPCHK(hipMemcpyAsync(du, query_uc, query_bytes, hipMemcpyHostToDevice, st));
  if (gsnapdp_micro_run_device(ctx, dw, n, dq, du, dr, st)) return -1;
  HIPCHK(hipMemcpyAsync(results, dr, (size_t)n * sizeof(gsnapdp_micro_result), hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  return 0;
}

int gsnapdp__micro_lds_check(size_t max_lds) { return gsnapdp__lds_fits((const void*)&k_micro, 0, max_lds, "k_micro"); }
