// gsnapdp_kernels.hip -- MI355X (gfx950) kernels for GMAP/GSNAP's stage-3
// gap-filling DP (reference src/dynprog.c, 2012-07-03).
//
// Design (DESIGN.md has the long form):
//   * one LANE per DP window (inter-window parallelism; 64 windows per wave);
//   * the window's band lives in registers as WMAX "slots", one per diagonal
//     d = r - c + rband, bottom-aligned so slot WMAX-1 is the lowest diagonal
//     and the sentinel below it (dynprog.c:1508-1513) is a compile-time NEG;
//   * column-major sweep (the reference's own order, dynprog.c:1491-1563):
//     per column every slot does gap1 (from slot+1), gap2 (chained from slot-1)
//     and nogap (same slot) with the sequential tie rule;
//   * waves are made uniform in (band, tie rule, endpoint mode) by an on-device
//     counting sort (k_plan / k_scan / k_scatter), so band edges are scalar;
//   * 4-bit direction nibbles stream to HBM scratch; each lane then walks its
//     own traceback and emits a compact op stream (include/gsnapdp.h).
//   End gaps and windows too wide (W > 48) or too long (L2 > 640) for
//   registers run on the row-lane kernel k_rows (gsnapdp_ggap.hip).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>
#include <utility>

#include "gsnapdp_device.h"
#include "gsnapdp_internal.h"

using namespace gsnapdp;

namespace {

// ------------------------------------------------------------------ k_plan
// Early returns, QUERYEND_NOGAPS windows (no fill at all) and bucketing.
__global__ void k_plan(const gsnapdp_window* __restrict__ W, int n, const char* __restrict__ q,
                       const char* __restrict__ qu, const uint32_t* __restrict__ blocks,
                       uint64_t nwords, const uint32_t* __restrict__ prof,
                       gsnapdp_result* __restrict__ res, uint32_t* __restrict__ ops,
                       const int64_t* __restrict__ op_off, int* __restrict__ keys,
                       int* __restrict__ hist, int* __restrict__ big_list,
                       int* __restrict__ big_count, int list_cap) {
  __shared__ int lh[NKEYS];  // block-local histogram: one global atomic per key per block
  __shared__ int lbig[RW_NCLS], lbase[RW_NCLS];  // block-local row-lane list appends
  for (int k = threadIdx.x; k < NKEYS; k += blockDim.x) lh[k] = 0;
  if (threadIdx.x < RW_NCLS) lbig[threadIdx.x] = 0;
  __syncthreads();
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  int key = -1, big = -1;  // k_fill bucket key, or row-lane class
  if (i < n) {
    const gsnapdp_window w = W[i];
    const Lane L = make_lane(w);
    if (L.d.status != ST_OK) {
      gsnapdp_result R = {};
      R.finalscore = L.d.early_score;
      R.status = L.d.status;
      R.length1 = L.d.L1;
      R.length2 = L.d.L2;
      R.reserved = L.d.early_dpi_step ? step_dpi(w.dynprogindex) : w.dynprogindex;
      res[i] = R;
    } else if (L.d.mode == 3) {  // traceback_nogaps (dynprog.c:2815-2872) from (min,min)
      Tally t = {0, 0, 0, 0};
      OpWriter ow = {ops + op_off[i], (int)(op_off[i + 1] - op_off[i]), 0, 0};
      const int m = min(L.d.L1, L.d.L2);
      const uint32_t* ptab = prof + L.d.mt * 128;
      for (int r = m, c = m; r > 0 && c > 0; r--, c--) {
        const int g = gclass(blocks, nwords, L, L.g0 + L.gstep * (c - 1));
        if (g != 5) {
          const int qi = L.qbase + L.qstep * (r - 1);
          const unsigned char c1 = qchar(q, qi);
          const unsigned char u1 = (unsigned char)qu[qi];
          if (u1 == (unsigned char)("ACGTN"[g]) || ((ptab[c1] >> (24 + g)) & 1u)) t.nmatches++;
          else t.nmismatches++;
        }
        ow.run++;
      }
      ow.flush();
      write_result(&res[i], w, L, 0, m, m, t, ow);
    } else if (L.d.mode == 0 && L.d.W <= FAST_WMAX && L.d.L2 <= FAST_L2MAX) {
      key = (L.d.W * (FAST_WMAX + 1) + L.d.lband) * 2 + L.d.jl;
    } else {
      big = rows_class(L.d.L1, L.d.L2, L.d.W);
      if (big < 0) {  // beyond the row-lane scratch: fail loudly
        gsnapdp_result R = {};
        R.finalscore = 0;
        R.status = ST_UNSUPPORTED;
        R.length1 = L.d.L1;
        R.length2 = L.d.L2;
        R.reserved = w.dynprogindex;
        res[i] = R;
      }
    }
    keys[i] = key;
  }
  if (key >= 0) atomicAdd(&lh[key], 1);
  const int lslot = big >= 0 ? atomicAdd(&lbig[big], 1) : 0;
  __syncthreads();
  // one global append per non-empty row-lane class per block (list order is free:
  // k_rows writes each window's own result slot)
  if (threadIdx.x < RW_NCLS)
    lbase[threadIdx.x] = lbig[threadIdx.x] > 0 ? atomicAdd(big_count + threadIdx.x, lbig[threadIdx.x]) : 0;
  for (int k = threadIdx.x; k < NKEYS; k += blockDim.x)
    if (lh[k] > 0) atomicAdd(&hist[k], lh[k]);
  __syncthreads();
  if (big >= 0) big_list[(size_t)big * list_cap + lbase[big] + lslot] = i;
}

// Exclusive scan of bucket sizes, each padded to whole waves of its class
// (64 / CLASS_LPW windows).  cursor[k] = first perm entry of bucket k;
// class_start[c] = first perm entry of class c (a multiple of its wave size,
// since wave sizes shrink as W grows and are powers of two).
__device__ inline int padded_bucket(int k, int h) {
  const int ng = 64 / CLASS_LPW[class_of_w(k / KEYS_PER_W)];
  return (h + ng - 1) / ng * ng;
}

// Also writes -1 into every bucket's padding entries of perm, so perm needs
// no clearing.
// (also zeroes the histogram for the next batch: the context clears it once at
// allocation, so no per-batch memset is needed)
__global__ void k_scan(int* __restrict__ hist, int* __restrict__ cursor,
                       int* __restrict__ class_start, int* __restrict__ perm) {
  __shared__ int part[1024];
  const int tid = threadIdx.x;
  const int per = (NKEYS + 1023) / 1024;
  const int lo = tid * per, hi = min(NKEYS, lo + per);
  int s = 0;
  for (int k = lo; k < hi; k++) s += padded_bucket(k, hist[k]);
  part[tid] = s;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {  // Hillis-Steele inclusive scan
    int v = tid >= off ? part[tid - off] : 0;
    __syncthreads();
    part[tid] += v;
    __syncthreads();
  }
  int run = part[tid] - s;
  for (int k = lo; k < hi; k++) {
    const int h = hist[k], p = padded_bucket(k, h);
    cursor[k] = run;
    for (int e = run + h; e < run + p; e++) perm[e] = -1;
    run += p;
    hist[k] = 0;
  }
  __syncthreads();
  if (tid == 0) {
    // class c covers W in (CLASS_W[c-1], CLASS_W[c]]; keys are W-major
    int wlo = 0;
    for (int c = 0; c < NCLASS; c++) {
      const int kfirst = (wlo + 1) * KEYS_PER_W;
      class_start[c] = kfirst < NKEYS ? cursor[kfirst] : part[1023];
      wlo = CLASS_W[c];
    }
    class_start[NCLASS] = part[1023];
  }
}

// Block-local ranks (LDS atomics), one global reservation per key per block.
__global__ void k_scatter(const int* __restrict__ keys, int n, int* __restrict__ cursor,
                          int* __restrict__ perm) {
  __shared__ int lh[NKEYS];
  for (int k = threadIdx.x; k < NKEYS; k += blockDim.x) lh[k] = 0;
  __syncthreads();
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int key = i < n ? keys[i] : -1;
  const int rank = key >= 0 ? atomicAdd(&lh[key], 1) : 0;
  __syncthreads();
  for (int k = threadIdx.x; k < NKEYS; k += blockDim.x)
    if (lh[k] > 0) lh[k] = atomicAdd(&cursor[k], lh[k]);  // the block's base in bucket k
  __syncthreads();
  if (key >= 0) perm[lh[key] + rank] = i;
}

// ------------------------------------------------------------------ k_fill
// Per-lane column genome stream: class of column c for the window, branch
// free.  pos(c) = P0 + PS*c in reference uint32 arithmetic (get_genomic_nt).
struct ColStream {
  uint32_t P0;
  int PS;        // +1 / -1
  int cvlo, cvhi;  // columns whose genomicpos is inside [0, genomiclength)
  int xorc;      // 0 watson, 3 crick (complement of the 2-bit code)
  __device__ inline void init(const Lane& L) {
    const int gstep = L.gstep;
    if (L.watson) {
      P0 = L.base + (uint32_t)(L.g0 - gstep);
      PS = gstep;
    } else {
      P0 = L.base + (uint32_t)(L.glen - 1) - (uint32_t)(L.g0 - gstep);
      PS = -gstep;
    }
    if (gstep > 0) {
      cvlo = 1 - L.g0;
      cvhi = L.glen - L.g0;
    } else {
      cvlo = L.g0 + 2 - L.glen;
      cvhi = L.g0 + 1;
    }
    if (L.allstar) {
      cvlo = 1 << 30;
      cvhi = -(1 << 30);
    }
    xorc = L.watson ? 0 : 3;
  }
  __device__ inline int cls(const uint32_t* __restrict__ blocks, uint64_t nwords, int c) const {
    const uint32_t pos = P0 + (uint32_t)(PS * c);
    const uint64_t ptr = (uint64_t)(pos >> 5) * 3u;
    const bool inr = c >= cvlo && c <= cvhi;
    const bool ing = ptr + 2 < nwords;
    const uint64_t p = (inr && ing) ? ptr : 0;
    const uint32_t bit = pos & 31u;
    const uint32_t fl = blocks[p + 2];
    const uint32_t word = blocks[p + (bit < 16 ? 1 : 0)];
    const int code = (int)((word >> ((bit & 15u) * 2u)) & 3u) ^ xorc;
    const bool isn = !ing || ((fl >> bit) & 1u);
    return !inr ? 5 : (isn ? 4 : code);
  }
};

// ------------------------------------------------------------------ k_fill
// Register-band fill, endpoint and traceback for one wave of 64/LPW single-gap
// windows sharing (lband, rband, jl) (Dynprog_single_gap, dynprog.c:4471-4575).
//
// Band layout.  A window's band is bottom-aligned in WMAX = S*LPW diagonal
// slots: global slot gs holds diagonal gs - stop (stop = WMAX - W), i.e. row
// r = c - rband + gs - stop of column c.  Lane j of the window's lane group
// owns slots j*S .. j*S+S-1 in registers.  The group runs a skewed wavefront:
// at step t lane j computes column t - j, so the gap2 chain (top to bottom of
// a column, dynprog.c:1532-1542) arrives from lane j-1's previous step and the
// gap1 input of the lowest slot (dynprog.c:1519-1529) from lane j+1's slot 0
// of this step; both move by DPP row shifts.
//
// Offset scores.  Registers hold X(r,c) - (r+c)*ext for X in {H, E, F}.  This
// is an exact change of variables of the recurrences of dynprog.c:1519-1561:
// gap1 and gap2 lose their "+ extend", the nogap step gains a constant
// -2*ext, and every comparison is between two values of the same cell, so
// each tie decision is the reference's.  The endpoint score is converted back.
//
// Slots above the band (gs < stop) run the same code with a -2^29 bias on
// their nogap score, and rows <= 0 need no special case: the only edge from
// them into the band is the top slot's gap2 input, which then holds a
// NEG-like value exactly where the reference reads its NEG_INFINITY sentinel
// (dynprog.c:1501-1506), and row 0's gap1 chain reproduces the open + c*ext
// initialisation (dynprog.c:1464-1475).  NEG-like values never compete with
// reachable ones ("Band edges").
//
// Per cell the fill streams 4 direction bits (the sign bits of differences,
// pushed with alignbit into four bit planes v1 | h1 | dF | dE of S bits each;
// a jump-late fill stores their complements) and a match bit (consistent_array or uppercase
// equality, dynprog.c:2650-2656) to per-wave scratch.  The traceback is then
// a backward column sweep over that scratch: every lane reloads the words it
// wrote (coalesced, prefetched two columns ahead) and the group's traceback
// lane walks the reference's traceback (dynprog.c:2611-2712) one column per
// step, so no step waits on a dependent global load.
#ifndef GSNAPDP_FILL_WAVES
#define GSNAPDP_FILL_WAVES 4  // k_fill waves per SIMD (register budget 512 / waves)
#endif
constexpr int FILL_SC_BIAS = 6;  // -2 * SINGLE_EXTEND (dynprog.c:222)
#ifndef GSNAPDP_TB_AHEAD
#define GSNAPDP_TB_AHEAD 1
#endif
constexpr int TB_AHEAD = GSNAPDP_TB_AHEAD;  // traceback prefetch distance, in 4-column groups

// k_fill's LDS profile word: each signed 4-bit pairdistance nibble s becomes
// the unsigned nibble s + 6 (s in -5..3, so 1..9); match bits unchanged.
__device__ inline uint32_t fill_profile_word(uint32_t w) {
  uint32_t o = w & 0xFF000000u;
#pragma unroll
  for (int g = 0; g < 6; g++) {
    const int n = (int)((w >> (4 * g)) & 0xFu);
    const int sn = n >= 8 ? n - 16 : n;
    o |= (uint32_t)((sn + FILL_SC_BIAS) & 0xF) << (4 * g);
  }
  return o;
}
constexpr int UTAB = 4 * 128;  // LDS profile: 4 x 128 pairdistance words, then 256 uppercase words
constexpr int MLUT = UTAB + 256;  // then 32 uint64: the 5 match bits of a profile word spread to bit 7 of bytes 0..4
constexpr int SPROF_WORDS = MLUT + 64;
__host__ __device__ constexpr uint64_t spread_match(uint32_t m5) {
  uint64_t x = 0;
  for (int k = 0; k < 5; k++)
    if ((m5 >> k) & 1u) x |= (uint64_t)1 << (8 * k + 7);
  return x;
}

// f(integral_constant<int, U>) for U in the sequence, in order
template <int... U, class F>
__device__ inline void unroll_seq(std::integer_sequence<int, U...>, F&& f) {
  (f(std::integral_constant<int, U>()), ...);
}
// k_fill's cell values.  By default they are 16-bit: value + FV_BIAS, NEG-like
// values from FV_NEG up, all zero-extended in 32-bit registers, so the maxima
// are v_max_u16 (twice the issue rate of v_max_i32 on gfx950; 16-bit VOP2
// results zero bits 16-31) while sums and differences stay 32-bit adds.
// In-band reachable values lie in [2*open + 1, 9 * steps] (offset
// coordinates, open >= -12 for the single gaps k_fill serves), NEG-like ones
// in [FV_NEG + open, FV_NEG + 9 * steps]; with at most 688 steps both ranges
// stay apart and inside 0..65535 (static_assert below).
#ifndef GSNAPDP_FILL32
using FV = uint32_t;
constexpr uint32_t FV_NEG = 1024u;
constexpr uint32_t FV_BIAS = 16384u;
__device__ inline FV fv_max(FV a, FV b) {
  FV d;
  asm("v_max_u16 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
  return d;
}
static_assert(FV_NEG >= 12 && FV_NEG + 9u * 688u < FV_BIAS - 2u * 12u &&
                  FV_BIAS + 9u * 688u < 65536u && FAST_L2MAX + 48 <= 688,
              "16-bit k_fill value ranges");
#else
using FV = int;
constexpr int FV_NEG = NEG;
constexpr int FV_BIAS = 0;
__device__ inline FV fv_max(FV a, FV b) { return max(a, b); }
#endif
__device__ inline uint32_t push_sign(uint32_t acc, int d) {
  return __builtin_amdgcn_alignbit(acc, (uint32_t)d, 31u);  // (acc << 1) | (d < 0)
}
// the same register of lane-1 / lane+1 (rows of 16 lanes; groups never straddle rows)
__device__ inline int from_lane_above(int v) {
  return __builtin_amdgcn_mov_dpp(v, 0x111, 0xF, 0xF, true);  // row_shr:1
}
__device__ inline int from_lane_below(int v) {
  return __builtin_amdgcn_mov_dpp(v, 0x101, 0xF, 0xF, true);  // row_shl:1
}

// Per-wave LDS rings of k_fill (sizes per band class): for each window of the
// wave, the profile words of the rows its lanes' bottom slots will need and the
// genome classes of the columns they will need, staged RING_K columns at a time.
constexpr int RING_K = 16;
constexpr int pow2ceil(int x) {
  int p = 1;
  while (p < x) p <<= 1;
  return p;
}
template <int S, int LPW>
struct Rings {
  static constexpr int NG = 64 / LPW;
  static constexpr int SPAN = (LPW - 1) * (S - 1);  // rows between the group's bottom slots
  static constexpr int RR = pow2ceil(RING_K + SPAN);
  static constexpr int CR = pow2ceil(RING_K + LPW - 1);
  static constexpr int WORDS = NG * RR + (NG * CR + 3) / 4;
};
constexpr int RING_WORDS_MAX = 1280;  // max Rings<S,LPW>::WORDS over the classes (checked below)

template <int S, int LPW, int LOW, int JL>
__device__ void fill_group(const gsnapdp_window* __restrict__ Wn, int wi, bool active, int lane,
                           uint32_t* __restrict__ D, uint8_t* __restrict__ M,
                           const char* __restrict__ q, const char* __restrict__ qu,
                           const uint32_t* __restrict__ blocks, uint64_t nwords,
                           const uint32_t* sprof, uint32_t* ring,
                           gsnapdp_result* __restrict__ res, uint32_t* __restrict__ ops,
                           const int64_t* __restrict__ op_off) {
  static_assert(S >= 2 && S <= 8 && LPW <= 16 && 64 % LPW == 0, "class shape");
  using RG = Rings<S, LPW>;
  static_assert(RG::WORDS <= RING_WORDS_MAX, "LDS ring budget");
  constexpr int WMAX = S * LPW;
  constexpr int NG = 64 / LPW;
  constexpr int NAB = (WMAX - LOW) < S ? (WMAX - LOW) : S;  // local slots that may lie above the band
  const int j = lane % LPW;
  const int gbase = lane - j;
  const int g = lane / LPW;
  int lband, rband, open, ext, L1, L2, stop, maxL2, mtoff, cvlo, cvhi, qbase, qstep, xorc, gps;
  uint32_t gp0;  // genome position of column c: gp0 + gps*c
  {
    const Lane L = make_lane(Wn[wi]);
    lband = __builtin_amdgcn_readfirstlane(L.d.lband);  // wave-uniform (bucket key)
    rband = __builtin_amdgcn_readfirstlane(L.d.rband);
    open = __builtin_amdgcn_readfirstlane(L.d.open);
    ext = __builtin_amdgcn_readfirstlane(L.d.ext);
    L1 = active ? L.d.L1 : 0;
    L2 = active ? L.d.L2 : 0;
    stop = WMAX - (lband + rband + 1);
    mtoff = L.d.mt * 128;
    ColStream cs;
    cs.init(L);
    cvlo = cs.cvlo;
    cvhi = cs.cvhi;
    gp0 = cs.P0;
    gps = cs.PS;
    xorc = cs.xorc;
    qbase = L.qbase;
    qstep = L.qstep;
  }
  maxL2 = __builtin_amdgcn_readfirstlane(wave_max(L2));
  // the nogap step's constant -2*extend (= +6: k_fill serves single gaps, extend -3)
  // is folded into the LDS profile nibbles (FILL_SC_BIAS); the nogap value of a
  // slot above the band (only lane 0 has them) is held at NEG
  const int row0 = j * S - stop - rband;  // row of local slot 0 at column 0

  // profile word of row r; rows outside 1..L1 get a neutral word (their cells
  // never feed a reachable in-band cell)
  auto row_word = [&](int r) -> uint32_t {
    uint32_t qb = 0u, ub = 255u;
    if (r >= 1 && r <= L1) {
      const int qi = qbase + qstep * (r - 1);
      qb = (unsigned char)q[qi] & 127u;
      ub = (unsigned char)qu[qi];
    }
    return sprof[mtoff + qb] | sprof[UTAB + ub];
  };
  const uint64_t gmax = nwords >= 3 ? (nwords - 3) / 3 : 0;  // last whole genome block

  FV H[S], E[S], F[S];
  uint32_t P[S];
  // Match bits of the lane's S rows against each genome class: byte k of MB
  // holds, in bits 0..S-1, whether slot s's query row matches class k
  // (consistent_array or uppercase equality, dynprog.c:2650-2656).  The rows
  // move up one slot per column, so MB shifts right by one and the entering
  // row's bits come in at bit S-1 of each byte (from the LDS lookup table).
  const uint64_t* mlut = (const uint64_t*)(sprof + MLUT);
  constexpr uint64_t MB_KEEP = 0x0101010101ull * ((1u << (S - 1)) - 1u);
  auto row_spread = [&](uint32_t pw) -> uint64_t { return mlut[(pw >> 24) & 31u] >> (8 - S); };
  uint64_t MB = 0;
  // column 0 (dynprog.c:1460-1488) in offset coordinates
#pragma unroll
  for (int s = 0; s < S; s++) {
    const int r = row0 + s;
    H[s] = (r == 0) ? FV_BIAS : FV_NEG;
    E[s] = FV_NEG;
    F[s] = (r >= 1) ? FV_BIAS + open : FV_NEG;  // open + r*ext - r*ext
    P[s] = row_word(r);
    MB = ((MB >> 1) & MB_KEEP) | row_spread(P[s]);
  }
  // Rings: lane j of a window stages the rows / columns congruent to j mod
  // LPW.  Lane j's bottom slot holds row t + j*(S-1) + rbase at step t, its
  // column is t - j.  Before step 1: rows [1+rbase, K+rbase+SPAN], columns
  // [1, K]; after step t = nK: rows (t+rbase+SPAN, t+K+rbase+SPAN], columns
  // (t, t+K].  Same-wave LDS writes are visible to later reads in order.
  uint32_t* rr = ring + g * RG::RR;
  uint8_t* cr = (uint8_t*)(ring + NG * RG::RR) + g * RG::CR;
  const int rbase = S - 1 - stop - rband;
  auto stage = [&](auto nrows_tag, int rlo, int clo) {
    constexpr int NR = decltype(nrows_tag)::value;
    constexpr int ER = (NR + LPW - 1) / LPW, EC = (RING_K + LPW - 1) / LPW;
    // all loads first (clamped addresses, no branches), then the words
    uint32_t qb[ER], ub[ER], gw[EC], gf[EC];
#pragma unroll
    for (int e = 0; e < ER; e++) {
      const int r = rlo + e * LPW + j;
      const int rc = (r >= 1 && r <= L1) ? r : 1;
      const int qi = qbase + qstep * (rc - 1);
      qb[e] = (unsigned char)q[qi];
      ub[e] = (unsigned char)qu[qi];
    }
#pragma unroll
    for (int e = 0; e < EC; e++) {
      const int c = clo + e * LPW + j;
      const uint32_t pos = gp0 + (uint32_t)(gps * c);
      const uint64_t b = (uint64_t)(pos >> 5);
      const uint64_t ptr = (b <= gmax ? b : gmax) * 3u;
      gw[e] = blocks[ptr + ((pos & 31u) < 16 ? 1 : 0)];
      gf[e] = blocks[ptr + 2];
    }
#pragma unroll
    for (int e = 0; e < ER; e++) {
      const int r = rlo + e * LPW + j;
      const bool ok = r >= 1 && r <= L1;
      const uint32_t w = sprof[mtoff + (ok ? (qb[e] & 127u) : 0u)] | sprof[UTAB + (ok ? ub[e] : 255u)];
      if (e * LPW + j < NR) rr[r & (RG::RR - 1)] = w;
    }
#pragma unroll
    for (int e = 0; e < EC; e++) {
      const int c = clo + e * LPW + j;
      const uint32_t pos = gp0 + (uint32_t)(gps * c);
      const uint32_t bit = pos & 31u;
      const bool ing = (uint64_t)(pos >> 5) <= gmax;  // outside the genome: N
      const int code = (int)((gw[e] >> ((bit & 15u) * 2u)) & 3u) ^ xorc;
      const bool inr = c >= cvlo && c <= cvhi;
      const int k = !inr ? 5 : ((!ing || ((gf[e] >> bit) & 1u)) ? 4 : code);
      if (e * LPW + j < RING_K) cr[c & (RG::CR - 1)] = (uint8_t)k;
    }
    __builtin_amdgcn_s_waitcnt(0);  // nothing of the staging stays in flight into the column loop
  };
  stage(std::integral_constant<int, RING_K + RG::SPAN>(), 1 + rbase, 1);
  uint32_t pnext = rr[(1 + j * (S - 1) + rbase) & (RG::RR - 1)];
  int gnext = cr[(1 - j) & (RG::CR - 1)];
  FV fin = FV_NEG;
  const int se = stop + L1 - L2 + rband;  // global slot of the endpoint (L1,L2)
  const int je = se / S, sle = se - je * S;
  // scratch layout: column c's words are D[c*64 + (j*NG + g)], one 256-byte
  // row per column (coalesced stores); the match bytes likewise in M.  Lane
  // (j, g) stores column c = t - j at the wave-uniform row t-(LPW-1) plus a
  // non-negative lane offset.
  const int lane_off = (LPW - 1 - j) * 64 + j * NG + g;

  // One skewed step.  MASKED steps (the first and last LPW-1) leave lanes
  // whose column is outside 1..maxL2 untouched.
  // ROT < 0: the row words shift down one slot per step (P[s] = P[s+1]).
  // ROT = u >= 0 (full steps unrolled S at a time): the words stay put and
  // slot s reads P[(s + u + 1) % S], the entering row overwriting P[u], so
  // after S steps the layout is back where it started.
  auto step = [&](auto masked, auto rot, int t) {
    constexpr bool MASKED = decltype(masked)::value;
    constexpr int ROT = decltype(rot)::value;
    static_assert(!MASKED || ROT < 0, "rotating steps are full steps");
    auto pslot = [&](int s) -> uint32_t { return ROT < 0 ? P[s] : P[(s + ROT + 1) % S]; };
    const int c = t - j;
    // a window stops at its own last column, so its registers end on column L2
    const bool act = !MASKED || (c >= 1 && c <= L2);
    FV hp = FV_NEG, fp = FV_NEG;  // new (nogap, gap2) just above local slot 0
    if (LPW > 1) {
      const FV h = (FV)from_lane_above((int)H[S - 1]), f = (FV)from_lane_above((int)F[S - 1]);
      if (j != 0) {
        hp = h;
        fp = f;
      }
    }
    // four bit planes (v1, h1, dF, dE), each a short independent chain
    uint32_t av = 0u, ah = 0u, af = 0u, ae = 0u, gsh = 0u;
    auto cell = [&](int s, FV Hr, FV Er) {
      const FV Hd = H[s], Ed = E[s], Fd = F[s];
      const uint32_t pw = pslot(s);
      const FV a = Hr + open;
      const FV b = hp + open;
      const FV m1 = fv_max(Hd, Ed);
      const FV sc = (FV)__builtin_amdgcn_ubfe(pw, gsh, 4);  // pairdistance - 2*extend
      const bool above = (s < NAB) && (j * S + s < stop);  // loop-invariant lane mask
      const FV hn = above ? FV_NEG : fv_max(m1, Fd) + sc;
      const int dv = JL ? (int)(Fd - m1) : (int)(m1 - Fd);  // v1: nogap from gap2
      const int dh = JL ? (int)(Ed - Hd) : (int)(Hd - Ed);  // h1: nogap from gap1
      const int df = JL ? (int)(fp - b) : (int)(b - fp);    // dF: gap2 extends
      const int de = JL ? (int)(Er - a) : (int)(a - Er);    // dE: gap1 extends
      av = push_sign(av, dv);  // (the first push shifts in zeros: one op, not a compare)
      ah = push_sign(ah, dh);
      af = push_sign(af, df);
      ae = push_sign(ae, de);
      E[s] = fv_max(a, Er);
      const FV f = fv_max(b, fp);
      F[s] = f;
      H[s] = hn;
      hp = hn;
      fp = f;
    };
    uint32_t macc = 0u;  // this column's match bits, bit s = slot s
    if (act) {
      if constexpr (ROT < 0) {
#pragma unroll
        for (int s = 0; s < S - 1; s++) P[s] = P[s + 1];
        P[S - 1] = pnext;
      } else {
        P[ROT] = pnext;
      }
      MB = ((MB >> 1) & MB_KEEP) | row_spread(pnext);
      gsh = 4u * (uint32_t)gnext;
      macc = (uint32_t)(MB >> (8u * (uint32_t)gnext));
      cell(0, H[1], E[1]);
    }
    FV hb = FV_NEG, eb = FV_NEG;  // old (nogap, gap1) just below the lowest local slot
    if (LPW > 1) {
      const FV h = (FV)from_lane_below((int)H[0]), e = (FV)from_lane_below((int)E[0]);
      if (j != LPW - 1) {
        hb = h;
        eb = e;
      }
    }
    if (act) {
#pragma unroll
      for (int s = 1; s < S - 1; s++) cell(s, H[s + 1], E[s + 1]);
      cell(S - 1, hb, eb);
      const uint32_t acc = (((((av << S) | ah) << S) | af) << S) | ae;
#ifndef EXP_NOSTORE
      D[(ptrdiff_t)(t - (LPW - 1)) * 64 + lane_off] = acc;
#ifndef EXP_NOMATCH
      M[(ptrdiff_t)(t - (LPW - 1)) * 64 + lane_off] = (uint8_t)macc;
#endif
#else
      if (acc == 0x12345678u && macc == 77u) D[0] = 1u;
#endif
    }
    // next column's inputs from the rings (every lane, every step)
    if (t % RING_K == 0) stage(std::integral_constant<int, RING_K>(), t + 1 + rbase + RG::SPAN, t + 1);
    pnext = rr[(t + 1 + j * (S - 1) + rbase) & (RG::RR - 1)];
    gnext = cr[(t + 1 - j) & (RG::CR - 1)];
  };
  using Masked = std::integral_constant<bool, true>;
  using Full = std::integral_constant<bool, false>;
  using Shift = std::integral_constant<int, -1>;
  // full-rate steps while every lane's column is inside 1..its own L2
  const int minL2 = __builtin_amdgcn_readfirstlane(-wave_max(active ? -L2 : -maxL2));
  int t = 1;
  for (; t < LPW && t < maxL2 + LPW; t++) step(Masked(), Shift(), t);
#ifndef EXP_NOROT
  for (; t + S - 1 <= minL2; t += S)
    unroll_seq(std::make_integer_sequence<int, S>(),
               [&](auto u) { step(Full(), u, t + decltype(u)::value); });
#endif
  for (; t <= minL2; t++) step(Full(), Shift(), t);
  for (; t < maxL2 + LPW; t++) step(Masked(), Shift(), t);
  // endpoint (L1,L2): the lanes stopped on column L2 (dynprog.c:4545)
#pragma unroll
  for (int s = 0; s < S; s++)
    if (j == je && s == sle) fin = H[s];
  fin = __shfl(fin, gbase + je);
  const int finalscore = (int)(fin - FV_BIAS) + (L1 + L2) * ext;
#ifdef EXP_NOTRACE
  if (active && j == 0) res[wi].finalscore = finalscore;
  return;
#endif
  if (!active || j != 0) return;

  // ---- traceback (dynprog.c:2611-2712) on the group's lane 0, as a backward
  // sweep in which every lane visits the same column at the same time (a
  // window waits until the sweep reaches its own L2).  The path's current
  // diagonal (slot, owning lane, bit position) stays in registers, so a
  // diagonal step costs a few ALU ops; the direction and match words of that
  // lane arrive four columns per group, one group ahead.  VERT / HORIZ runs
  // take the general path; a gap that moves the path to another lane's slots
  // costs one dependent load.
  const gsnapdp_window w = Wn[wi];
  const Lane L = make_lane(w);
  enum { T_WAIT = 0, T_DIAG = 1, T_VERT = 2, T_HORIZ = 3, T_DONE = 4 };
  int st = T_WAIT;
  int r = L1, dist = 0;
  int jj = 0, pb = 0;  // DIAG: lane holding the path's diagonal, bit of its slot in each plane
  Tally tal = {0, 0, 0, 0};
  OpWriter ow = {ops + op_off[wi], (int)(op_off[wi + 1] - op_off[wi]), 0, 0};
  const uint32_t jlbit = JL ? 1u : 0u;
  const int wband = lband + rband;
  const uint32_t* Dg = D + g;
  const uint8_t* Mg = M + g;
  auto set_diag = [&](int rr, int cc) {
    const int sg = stop + rr - cc + rband;
    const int sgc = sg < 0 ? 0 : (sg >= WMAX ? WMAX - 1 : sg);  // out of band: DONE next
    jj = sgc / S;
    pb = S - 1 - (sgc - jj * S);
  };
  auto ldw = [&](int cc, int jw) -> uint32_t { return Dg[(size_t)cc * 64 + jw * NG]; };
  auto ldm = [&](int cc, int jw) -> uint32_t { return Mg[(size_t)cc * 64 + jw * NG]; };
  struct Grp {
    uint32_t w[4], m[4];
    int jw;
  };
  auto fetch_group = [&](Grp& x, int G, int jw) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int cc = 4 * G + k;
      x.w[k] = ldw(cc, jw);
      x.m[k] = ldm(cc, jw);
    }
    x.jw = jw;
  };
  auto column = [&](int c, uint32_t wk, uint32_t mk, int jw) {
    auto inb = [&](int rr) {
      const int d = rr - c + rband;
      return rr >= 1 && c >= 1 && d >= 0 && d <= wband;
    };
    auto plane_bit = [&](int rr, int plane) -> uint32_t {  // planes dE | dF | h1 | v1 from bit 0
      const int sg = stop + rr - c + rband;
      const int jr = sg / S, sl = sg - jr * S;
      const uint32_t x = (jr == jw) ? wk : ldw(c, jr);
      return ((x >> (plane * S + S - 1 - sl)) & 1u) ^ jlbit;
    };
    if (st == T_WAIT && c == L2) {
      st = T_DIAG;
      set_diag(r, c);
    }
    if (st == T_VERT) {  // gap2 chain in this column (add_queryskip, dynprog.c:2372)
      while (c == 0 ? (r >= 2 && r <= lband && r <= L1) : (inb(r) && plane_bit(r, 1))) {
        dist++;
        r--;
      }
      r--;
      ow.flush();
      ow.put(GSNAPDP_OP(GSNAPDP_OP_VSKIP, dist));
      tal.nopens++;
      tal.nindels += dist;
      st = T_DIAG;
      set_diag(r, c);
    }
    if (st == T_HORIZ) {  // gap1 chain, one column per step (add_genomeskip, dynprog.c:2416)
      const bool more = (r == 0) ? (c >= 2 && c <= rband && c <= L2) : (inb(r) && plane_bit(r, 0));
      if (more) {
        dist++;
      } else {
        // skipped columns c .. c+dist-1; the path lands in column c-1
        bool dashes = true;
        if (dist >= MICROINTRON_LENGTH) {
          const int cl = c, cr = c + dist - 1;
          const int gl = L.g0 + L.gstep * (cl - 1), gr = L.g0 + L.gstep * (cr - 1);
          const int lo = L.d.rev ? gr : gl, hi = L.d.rev ? gl : gr;
          const int l1 = gclass(blocks, nwords, L, lo), l2 = gclass(blocks, nwords, L, lo + 1);
          const int r2 = gclass(blocks, nwords, L, hi - 1), r1 = gclass(blocks, nwords, L, hi);
          dashes = intron_type_codes(l1, l2, r2, r1, L.cdna_direction) == 0;
        }
        ow.flush();
        ow.put(GSNAPDP_OP(dashes ? GSNAPDP_OP_HDASH : GSNAPDP_OP_HGAP, dist));
        if (dashes) {
          tal.nopens++;
          tal.nindels += dist;
        }
        st = T_DIAG;
        set_diag(r, c - 1);
      }
    } else if (st == T_DIAG) {
      if (!inb(r)) {
        st = T_DONE;
      } else {
        const uint32_t x = ((jj == jw) ? wk : ldw(c, jj)) >> pb;
        if (c >= cvlo && c <= cvhi) {  // not a '*' column (dynprog.c:2644)
          const uint32_t mb = (((jj == jw) ? mk : ldm(c, jj)) >> (S - 1 - pb)) & 1u;
          tal.nmatches += (int)mb;
          tal.nmismatches += 1 - (int)mb;
        }
        ow.run++;
        if (((x >> (3 * S)) & 1u) ^ jlbit) {  // v1: VERT
          st = T_VERT;
          dist = 1;
        } else if (((x >> (2 * S)) & 1u) ^ jlbit) {  // h1: HORIZ
          st = T_HORIZ;
          dist = 1;
        }
        r--;
      }
    }
  };
  // wave-uniform sweep from the wave's longest window down to column -1
  int G = maxL2 >> 2;
  set_diag(L1, L2);
  // pre[0] is the group being visited, pre[1..TB_AHEAD] the next ones,
  // loaded TB_AHEAD groups ahead of their visit (global scratch latency)
  Grp pre[TB_AHEAD + 1];
#pragma unroll
  for (int i = 0; i <= TB_AHEAD; i++) fetch_group(pre[i], G - i >= 0 ? G - i : 0, jj);
  Grp& ga = pre[0];
  const uint32_t invall = JL ? 0xFFFFFFFFu : 0u;
  // one iteration per 4-column group G; its columns are visited one by one
  // only when some lane of the wave cannot take the group in one bulk step
  for (; G >= 0; G--) {
    const int chi = min(4 * G + 3, maxL2);  // the first group may be partial
    bool fast4 = false;
    if (chi == 4 * G + 3) {
      // Four diagonal steps at once: the path stays on its diagonal through
      // columns c .. c-3 (no v1/h1 there), inside the band and the query, and
      // the four columns are all inside or all outside the window's genome.
      const int c = chi;
      const int dd = (S - 1 - pb) + jj * S - stop;  // the diagonal's offset in the band
      fast4 = st == T_DIAG && jj == ga.jw && r >= 4 && c >= 4 && dd >= 0 && dd <= wband;
      if (fast4) {
        const uint32_t x0 = (ga.w[0] ^ invall) >> pb, x1 = (ga.w[1] ^ invall) >> pb;
        const uint32_t x2 = (ga.w[2] ^ invall) >> pb, x3 = (ga.w[3] ^ invall) >> pb;
        const bool inside = c - 3 >= cvlo && c <= cvhi;
        const bool outside = c < cvlo || c - 3 > cvhi;
        const uint32_t vh = (1u << (2 * S)) | (1u << (3 * S));  // h1 and v1 of this slot
        fast4 = ((x0 | x1 | x2 | x3) & vh) == 0u && (inside || outside);
        if (fast4) {
          if (inside) {
            const int mb = S - 1 - pb;  // match bit of the diagonal's slot
            const int mcount = (int)(((ga.m[0] >> mb) & 1u) + ((ga.m[1] >> mb) & 1u) +
                                     ((ga.m[2] >> mb) & 1u) + ((ga.m[3] >> mb) & 1u));
            tal.nmatches += mcount;
            tal.nmismatches += 4 - mcount;
          }
          ow.run += 4;
          r -= 4;
        }
      }
    }
    // lanes with nothing to do in this group: bulk-stepped, done, or still
    // waiting for their own L2
    const bool idle = fast4 || st == T_DONE || (st == T_WAIT && L2 < 4 * G);
    if (__builtin_amdgcn_ballot_w64(!idle) != 0) {
      for (int c = chi; c >= 4 * G; c--) {
        const int k = c & 3;
        if (!fast4 && st != T_DONE && (st != T_WAIT || c == L2)) {
          const uint32_t wk = k == 0 ? ga.w[0] : k == 1 ? ga.w[1] : k == 2 ? ga.w[2] : ga.w[3];
          const uint32_t mk = k == 0 ? ga.m[0] : k == 1 ? ga.m[1] : k == 2 ? ga.m[2] : ga.m[3];
          column(c, wk, mk, ga.jw);
        }
      }
    }
    // leaving group G
    if (__builtin_amdgcn_ballot_w64(st != T_DONE) == 0) break;
#pragma unroll
    for (int i = 0; i < TB_AHEAD; i++) {
      pre[i] = pre[i + 1];
      // a gap moved the path to another lane: reload the groups already in flight
      if (G - 1 - i >= 0 && pre[i].jw != jj) fetch_group(pre[i], G - 1 - i, jj);
    }
    if (G - 1 - TB_AHEAD >= 0) fetch_group(pre[TB_AHEAD], G - 1 - TB_AHEAD, jj);  // predicted unchanged
  }
  if (st != T_DONE && st != T_WAIT) column(-1, 0u, 0u, -1);
  ow.flush();
  write_result(res + wi, w, L, finalscore, L1, L2, tal, ow);
}

// This wave's wave-tasks of class (S, LPW, LOW): task t covers the 64/LPW
// windows perm[t*NG ..]; the wave runs t = t0, t0 + stride, ... < t1.  Not
// inlined, so each class gets its own register allocation (inlining the
// classes into the kernel spills across them); called once per wave and
// class rather than once per task, so the call's callee-saved VGPR saves and
// restores (48 VGPRs to scratch, ~24 KB per call) are paid per wave, not per
// task.  The pointers carry their address spaces (global / LDS) so that the
// body still compiles to global_* and ds_* accesses rather than flat ones.
#define AS_GLOBAL __attribute__((address_space(1)))
#define AS_LDS __attribute__((address_space(3)))
template <int S, int LPW, int LOW>
__device__ __noinline__ void fill_tasks(int t0, int t1, int stride, const AS_GLOBAL gsnapdp_window* Wn1,
                                        const AS_GLOBAL int* perm1, const AS_GLOBAL char* q1,
                                        const AS_GLOBAL char* qu1, const AS_GLOBAL uint32_t* blocks1,
                                        uint64_t nwords, const AS_LDS uint32_t* sprof3,
                                        AS_LDS uint32_t* ring3,
                                        AS_GLOBAL uint32_t* D1, AS_GLOBAL gsnapdp_result* res1,
                                        AS_GLOBAL uint32_t* ops1, const AS_GLOBAL int64_t* op_off1) {
  const gsnapdp_window* __restrict__ Wn = (const gsnapdp_window*)Wn1;
  const int* __restrict__ perm = (const int*)perm1;
  const char* __restrict__ q = (const char*)q1;
  const char* __restrict__ qu = (const char*)qu1;
  const uint32_t* __restrict__ blocks = (const uint32_t*)blocks1;
  const uint32_t* sprof = (const uint32_t*)sprof3;
  uint32_t* ring = (uint32_t*)ring3;
  uint32_t* __restrict__ D = (uint32_t*)D1;
  gsnapdp_result* __restrict__ res = (gsnapdp_result*)res1;
  uint32_t* __restrict__ ops = (uint32_t*)ops1;
  const int64_t* __restrict__ op_off = (const int64_t*)op_off1;
  constexpr int NG = 64 / LPW;
  const int lane = threadIdx.x & 63;
  uint8_t* M = (uint8_t*)(D + (size_t)(FAST_L2MAX + 4) * 64);
  const int g = lane / LPW;
  for (int t = t0; t < t1; t += stride) {
    const int wi0 = perm[(size_t)t * NG + g];
    const int w0 = __builtin_amdgcn_readfirstlane(perm[(size_t)t * NG]);  // group 0: a real window
    const bool active = wi0 >= 0;
    const int wi = active ? wi0 : w0;  // idle groups shadow group 0 (reads only)
    const int jl = __builtin_amdgcn_readfirstlane((int)Wn[w0].jump_late_p);
    if (jl)
      fill_group<S, LPW, LOW, 1>(Wn, wi, active, lane, D, M, q, qu, blocks, nwords, sprof, ring,
                                 res, ops, op_off);
    else
      fill_group<S, LPW, LOW, 0>(Wn, wi, active, lane, D, M, q, qu, blocks, nwords, sprof, ring,
                                 res, ops, op_off);
  }
}

// All register-band classes in one persistent launch: the wave-tasks of the
// classes form one index space (class by class), so one class's tail overlaps
// the next class's work and empty classes cost nothing.  Register budget:
// 128 VGPRs (4 waves per SIMD); the few spills this forces sit in the task
// call's prologue/epilogue and loop preheaders, not in the column loops.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(GSNAPDP_FILL_WAVES, 8))) void k_fill(
    const gsnapdp_window* __restrict__ Wn, const int* __restrict__ perm,
    const int* __restrict__ class_start, const char* __restrict__ q, const char* __restrict__ qu,
    const uint32_t* __restrict__ blocks, uint64_t nwords, const uint32_t* __restrict__ prof,
    uint32_t* __restrict__ dirpool, size_t wave_stride, gsnapdp_result* __restrict__ res,
    uint32_t* __restrict__ ops, const int64_t* __restrict__ op_off) {
  __shared__ alignas(8) uint32_t sprof[SPROF_WORDS];
  __shared__ uint32_t rings[4][RING_WORDS_MAX];  // one per wave of the block
  for (int i = threadIdx.x; i < MLUT; i += blockDim.x)
    sprof[i] = i < UTAB ? fill_profile_word(prof[i]) : (i - UTAB < 128 ? prof[i] : 0u);
  for (int i = threadIdx.x; i < 32; i += blockDim.x) {
    const uint64_t x = spread_match((uint32_t)i);
    sprof[MLUT + 2 * i] = (uint32_t)x;
    sprof[MLUT + 2 * i + 1] = (uint32_t)(x >> 32);
  }
  __syncthreads();
  uint32_t* ring = rings[threadIdx.x >> 6];
  const int gw = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nw = (gridDim.x * blockDim.x) >> 6;
  uint32_t* D = dirpool + (size_t)gw * wave_stride;
  int tfirst[NCLASS + 1];  // first task index of each class, then the total
  tfirst[0] = 0;
#pragma unroll
  for (int c = 0; c < NCLASS; c++)
    tfirst[c + 1] = tfirst[c] + (class_start[c + 1] - class_start[c]) / (64 / CLASS_LPW[c]);
  // the wave takes global task indices tau = gw, gw + nw, ...; those of class c
  // are its tasks t = base_c + (tau - tfirst[c]), visited class by class
  static_assert(NCLASS <= 8, "k_fill dispatches at most 8 classes");
#define FILL_CLASS(C)                                                                            \
  if constexpr (C < NCLASS) {                                                                    \
    const int lo = tfirst[C], hi = tfirst[C + 1];                                                \
    const int tau0 = gw >= lo ? gw : gw + (lo - gw + nw - 1) / nw * nw;                          \
    if (tau0 < hi) {                                                                             \
      const int base = class_start[C] / (64 / CLASS_LPW[C]) - lo;                                \
      fill_tasks<CLASS_S[C % NCLASS], CLASS_LPW[C % NCLASS], class_low(C % NCLASS)>(             \
          base + tau0, base + hi, nw, (const AS_GLOBAL gsnapdp_window*)Wn,                        \
          (const AS_GLOBAL int*)perm, (const AS_GLOBAL char*)q, (const AS_GLOBAL char*)qu,        \
          (const AS_GLOBAL uint32_t*)blocks, nwords, (const AS_LDS uint32_t*)sprof,               \
          (AS_LDS uint32_t*)ring, (AS_GLOBAL uint32_t*)D, (AS_GLOBAL gsnapdp_result*)res,         \
          (AS_GLOBAL uint32_t*)ops, (const AS_GLOBAL int64_t*)op_off);                            \
    }                                                                                            \
  }
  FILL_CLASS(0) FILL_CLASS(1) FILL_CLASS(2) FILL_CLASS(3)
  FILL_CLASS(4) FILL_CLASS(5) FILL_CLASS(6) FILL_CLASS(7)
#undef FILL_CLASS
}

// --------------------------------------------------------------- k_maxent
__global__ void k_maxent(const uint8_t* __restrict__ model, const uint32_t* __restrict__ pos,
                         const uint32_t* __restrict__ chroff, double* __restrict__ out, int n,
                         const uint32_t* __restrict__ blocks, uint64_t nwords,
                         const double* __restrict__ T) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = maxent_prob(model[i], pos[i], chroff[i], blocks, nwords, T);
}

}  // namespace

// ======================================================================
// Host side: context and the C-ABI of include/gsnapdp.h
// ======================================================================
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <string>
#include <vector>

#include "gsnapdp_ctx.h"

static thread_local std::string g_err;
void gsnapdp__set_err(const std::string& s) { g_err = s; }

// per-wave k_fill scratch: direction words (u32) then match bytes, one
// 64-lane row per column 0 .. FAST_L2MAX + 3 (the traceback reads whole
// 4-column groups)
static const size_t FILL_COLS = (size_t)FAST_L2MAX + 4;
static const size_t WAVE_STRIDE_DW = FILL_COLS * 64 + FILL_COLS * 16;

extern "C" const char* gsnapdp_last_error(void) { return g_err.c_str(); }

extern "C" gsnapdp_ctx* gsnapdp_create(int device, const uint32_t* blocks, size_t nwords,
                                        int mode) {
  gsnapdp_ctx* ctx = new gsnapdp_ctx();
  ctx->device = device;
  ctx->h_blocks = blocks;
  ctx->nwords = nwords;
  ctx->mode = mode;
  auto fail = [&](const char* what, hipError_t e) -> gsnapdp_ctx* {
    gsnapdp__set_err(std::string(what) + ": " + hipGetErrorString(e));
    delete ctx;
    return nullptr;
  };
  hipError_t e;
  if ((e = hipSetDevice(device)) != hipSuccess) return fail("hipSetDevice", e);
  hipDeviceProp_t prop;
  if ((e = hipGetDeviceProperties(&prop, device)) != hipSuccess) return fail("props", e);
  ctx->arch = prop.gcnArchName;
  if (ctx->arch.find("gfx950") == std::string::npos) {
    gsnapdp__set_err("gsnapdp is built for gfx950 only; device is " + ctx->arch);
    delete ctx;
    return nullptr;
  }
  ctx->fill_waves = prop.multiProcessorCount * 4 * GSNAPDP_FILL_WAVES;  // k_fill's occupancy
  ctx->num_cus = prop.multiProcessorCount;
  if ((e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking)) != hipSuccess)
    return fail("stream", e);
  if ((e = hipMalloc(&ctx->d_blocks, (nwords + 8) * 4)) != hipSuccess) return fail("malloc blocks", e);
  if ((e = hipMemset(ctx->d_blocks, 0xFF, (nwords + 8) * 4)) != hipSuccess) return fail("memset", e);
  if ((e = hipMemcpy(ctx->d_blocks, blocks, nwords * 4, hipMemcpyHostToDevice)) != hipSuccess)
    return fail("copy blocks", e);
  build_profile_table(mode, ctx->h_prof);
  if ((e = hipMalloc(&ctx->d_prof, sizeof(ctx->h_prof))) != hipSuccess) return fail("malloc prof", e);
  if ((e = hipMemcpy(ctx->d_prof, ctx->h_prof, sizeof(ctx->h_prof), hipMemcpyHostToDevice)) !=
      hipSuccess)
    return fail("copy prof", e);
  const size_t small = (size_t)2 * NKEYS + NCLASS + 1 + 1 + 64;
  if ((e = hipMalloc(&ctx->d_small, small * 4)) != hipSuccess) return fail("malloc small", e);
  if ((e = hipMemset(ctx->d_small, 0, small * 4)) != hipSuccess) return fail("memset small", e);

  ctx->dirpool_waves = (size_t)ctx->fill_waves;
  if ((e = hipMalloc(&ctx->d_dirpool, ctx->dirpool_waves * WAVE_STRIDE_DW * 4)) != hipSuccess)
    return fail("malloc dirpool", e);
  return ctx;
}

extern "C" void gsnapdp_destroy(gsnapdp_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  (void)hipFree(ctx->d_blocks);
  (void)hipFree(ctx->d_prof);
  (void)hipFree(ctx->d_tables);
  (void)hipFree(ctx->d_keys);
  (void)hipFree(ctx->d_perm);
  (void)hipFree(ctx->d_big_list);
  (void)hipFree(ctx->d_small);
  (void)hipFree(ctx->d_dirpool);
  (void)hipFree(ctx->d_bigpool);
  (void)hipFree(ctx->d_largepool);
  (void)hipFree(ctx->d_ggap_lists);
  (void)hipFree(ctx->d_ggap_counts);
  (void)hipFree(ctx->d_ggap_pool);
  (void)hipFree(ctx->d_ggap_stage);
  (void)hipFree(ctx->d_sj_lists);
  (void)hipFree(ctx->d_sj_win);
  (void)hipFree(ctx->d_stage);
  (void)hipFree(ctx->d_csum);
  if (ctx->h_small) (void)hipHostFree(ctx->h_small);
  if (ctx->h_in) (void)hipHostFree(ctx->h_in);
  if (ctx->h_mx) (void)hipHostFree(ctx->h_mx);
  (void)hipFree(ctx->d_mx_stage);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

extern "C" const char* gsnapdp_device_arch(gsnapdp_ctx* ctx) { return ctx ? ctx->arch.c_str() : ""; }

extern "C" int gsnapdp_sync(gsnapdp_ctx* ctx) {
  HIPCHK(hipStreamSynchronize(ctx->stream));
  return 0;
}

extern "C" size_t gsnapdp_scratch_bytes(gsnapdp_ctx* ctx, int n, int max_length1, int max_length2) {
  (void)max_length1;
  (void)max_length2;
  const size_t waves = (size_t)n / 64 + NKEYS;
  return (size_t)n * 8 + waves * 64 * 4 + (ctx ? ctx->dirpool_waves : 0) * WAVE_STRIDE_DW * 4 +
         (size_t)RW_BIG_WAVES * RW_BIG_WORDS * 4 +
         (size_t)(ctx ? ctx->num_cus : 256) * RW_LARGE_WAVES_PER_CU * RW_LARGE_WORDS * 4;
}

static int ensure_capacity(gsnapdp_ctx* ctx, int n) {
  if (n <= ctx->cap_n) return 0;
  int cap = n + n / 4 + 1024;
  (void)hipFree(ctx->d_keys);
  (void)hipFree(ctx->d_perm);
  (void)hipFree(ctx->d_big_list);
  HIPCHK(hipMalloc(&ctx->d_keys, (size_t)cap * 4));
  HIPCHK(hipMalloc(&ctx->d_big_list, (size_t)RW_NCLS * cap * 4));
  // perm: every bucket padded to a whole wave
  ctx->perm_cap = ((size_t)cap + (size_t)NKEYS * 64 + 63) & ~(size_t)63;
  HIPCHK(hipMalloc(&ctx->d_perm, ctx->perm_cap * 4));
  ctx->cap_n = cap;
  return 0;
}

extern "C" int gsnapdp_run_device(gsnapdp_ctx* ctx, const gsnapdp_window* d_windows, int n,
                                  const char* d_query, const char* d_query_uc,
                                  gsnapdp_result* d_results, uint32_t* d_ops,
                                  const int64_t* d_op_offsets, void* stream_v) {
  if (!ctx) return -1;
  if (n <= 0) return 0;
  hipStream_t st = stream_v ? (hipStream_t)stream_v : ctx->stream;
  std::lock_guard<std::mutex> lock(ctx->mu);
  HIPCHK(hipSetDevice(ctx->device));
  if (ensure_capacity(ctx, n)) return -1;
  int* hist = ctx->d_small;
  int* cursor = hist + NKEYS;
  int* class_start = cursor + NKEYS;
  int* big_count = class_start + NCLASS + 1;  // RW_NCLS row-lane class counts
  HIPCHK(hipMemsetAsync(big_count, 0, 4 * RW_NCLS, st));
  if (gsnapdp__rows_pools(ctx)) return -1;
  const int tb = 1024, nb = (n + tb - 1) / tb;
  auto mark = [&](int stage, int end) { gsnapdp__mark(ctx, st, stage, end); };
  mark(0, 0);
  hipLaunchKernelGGL(k_plan, dim3(nb), dim3(tb), 0, st, d_windows, n, d_query, d_query_uc,
                     ctx->d_blocks, (uint64_t)ctx->nwords, ctx->d_prof, d_results, d_ops,
                     d_op_offsets, ctx->d_keys, hist, ctx->d_big_list, big_count,
                     ctx->cap_n);
  mark(0, 1);
  mark(1, 0);
  hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, st, hist, cursor, class_start, ctx->d_perm);
  hipLaunchKernelGGL(k_scatter, dim3(nb), dim3(tb), 0, st, ctx->d_keys, n, cursor, ctx->d_perm);
  mark(1, 1);
  const int blocks = (int)(ctx->dirpool_waves / 4);
  const uint64_t nw = (uint64_t)ctx->nwords;
  // (k_fill keeps every CU busy, so k_rows runs after it on the same stream: a
  // side stream measured slower)
  mark(2, 0);
  hipLaunchKernelGGL(k_fill, dim3(blocks), dim3(256), 0, st, d_windows, ctx->d_perm, class_start,
                     d_query, d_query_uc, ctx->d_blocks, nw, ctx->d_prof, ctx->d_dirpool,
                     WAVE_STRIDE_DW, d_results, d_ops, d_op_offsets);
  mark(2, 1);
  mark(3, 0);
  if (gsnapdp__rows_launch(ctx, st, d_windows, ctx->d_big_list, big_count, ctx->cap_n, d_query,
                           d_query_uc, d_results, d_ops, d_op_offsets))
    return -1;
  mark(3, 1);
  HIPCHK(hipGetLastError());
  return 0;
}

extern "C" int gsnapdp_run_host(gsnapdp_ctx* ctx, const gsnapdp_window* windows, int n,
                                const char* query, const char* query_uc, size_t query_bytes,
                                gsnapdp_result* results, uint32_t* ops,
                                const int64_t* op_offsets) {
  if (!ctx) return -1;
  if (n <= 0) return 0;
  HIPCHK(hipSetDevice(ctx->device));
  // one host round trip at a time per context (the staging buffers are shared)
  std::lock_guard<std::mutex> host_lock(ctx->host_mu);
  const size_t nops = (size_t)op_offsets[n];
  const size_t szw = (size_t)n * sizeof(gsnapdp_window);
  const size_t szq = (query_bytes + 255) & ~(size_t)255;
  const size_t szr = (size_t)n * sizeof(gsnapdp_result);
  const size_t szo = (nops + 1) * 4;
  const size_t szoff = (size_t)(n + 1) * 8;
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const bool alias = query_uc == query;  // one buffer for both (query already upper case): one copy
  // inputs first (windows, query, query_uc, op offsets), then the outputs
  const size_t in_bytes = al(szw) + (alias ? 1 : 2) * al(szq) + al(szoff);
  const size_t total = in_bytes + al(szr) + 2 * al(szo) + 256;
  // a small batch (the per-call drop-in's) is one packed H2D copy, the kernels,
  // and its results and uncompacted ops back in the same synchronisation
  const bool small = in_bytes <= ((size_t)1 << 20) && szo <= ((size_t)1 << 20);
  {
    std::lock_guard<std::mutex> lock(ctx->mu);
    if (total > ctx->stage_cap) {
      (void)hipFree(ctx->d_stage);
      ctx->d_stage = nullptr;
      HIPCHK(hipMalloc(&ctx->d_stage, total));
      ctx->stage_cap = total;
    }
    if (!ctx->h_small) HIPCHK(hipHostMalloc(&ctx->h_small, 256));
    if (small && in_bytes > ctx->h_in_cap) {
      if (ctx->h_in) (void)hipHostFree(ctx->h_in);
      ctx->h_in = nullptr;
      HIPCHK(hipHostMalloc(&ctx->h_in, (size_t)1 << 20));
      ctx->h_in_cap = (size_t)1 << 20;
    }
  }
  char* base = (char*)ctx->d_stage;
  const size_t o_q = al(szw), o_u = o_q + al(szq), o_off = o_u + (alias ? 0 : al(szq));
  gsnapdp_window* dw = (gsnapdp_window*)base;
  char* dq = base + o_q;
  char* du = alias ? dq : base + o_u;
  int64_t* doff = (int64_t*)(base + o_off);
  gsnapdp_result* dr = (gsnapdp_result*)(base + in_bytes);
  uint32_t* dops = (uint32_t*)((char*)dr + al(szr));
  uint32_t* dcomp = (uint32_t*)((char*)dops + al(szo));
  int64_t* dhdr = (int64_t*)((char*)dcomp + al(szo));
  hipStream_t st = ctx->stream;
  if (small) {
    char* h = (char*)ctx->h_in;
    memcpy(h, windows, szw);
    memcpy(h + o_q, query, query_bytes);
    if (!alias) memcpy(h + o_u, query_uc, query_bytes);
    memcpy(h + o_off, op_offsets, szoff);
    HIPCHK(hipMemcpyAsync(base, h, o_off + szoff, hipMemcpyHostToDevice, st));
    if (gsnapdp_run_device(ctx, dw, n, dq, du, dr, dops, doff, st)) return -1;
    HIPCHK(hipMemcpyAsync(results, dr, szr, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(ops, dops, nops * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));  // the pinned staging is reused by the next call
    return 0;
  }
  HIPCHK(hipMemcpyAsync(dw, windows, szw, hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(dq, query, query_bytes, hipMemcpyHostToDevice, st));
  if (!alias) HIPCHK(hipMemcpyAsync(du, query_uc, query_bytes, hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(doff, op_offsets, szoff, hipMemcpyHostToDevice, st));
  if (gsnapdp_run_device(ctx, dw, n, dq, du, dr, dops, doff, st)) return -1;
  // only the ops each window wrote come back: compacted on the device, then
  // scattered to op_offsets on the host (the capacity layout is ~100x larger)
  if (gsnapdp_compact_ops_device(ctx, dr, n, dops, doff, dcomp, (int64_t)nops, dhdr, st)) return -1;
  HIPCHK(hipMemcpyAsync(results, dr, szr, hipMemcpyDeviceToHost, st));
  int64_t* hdr = (int64_t*)ctx->h_small;
  HIPCHK(hipMemcpyAsync(hdr, dhdr, 2 * sizeof(int64_t), hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  const int64_t got = hdr[0];
  if (got < 0 || (size_t)got > nops) {
    gsnapdp__set_err("gsnapdp_run_host: compacted op count out of range");
    return -1;
  }
  if (got == 0) return 0;
  std::vector<uint32_t>& comp = ctx->h_comp;
  comp.resize((size_t)got);
  HIPCHK(hipMemcpyAsync(comp.data(), dcomp, (size_t)got * 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  size_t k = 0;
  for (int i = 0; i < n; i++) {
    int64_t c = results[i].nops < 0 ? 0 : results[i].nops;
    const int64_t cap = op_offsets[i + 1] - op_offsets[i];
    if (c > cap) c = cap;
    if (c) memcpy(ops + op_offsets[i], comp.data() + k, (size_t)c * 4);
    k += (size_t)c;
  }
  return 0;
}

extern "C" void* gsnapdp_host_alloc(size_t bytes) {
  void* p = nullptr;
  if (hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) {
    gsnapdp__set_err("hipHostMalloc failed");
    return nullptr;
  }
  return p;
}

extern "C" void gsnapdp_host_free(void* p) {
  if (p) (void)hipHostFree(p);
}

// stage timing: events on the launch stream around each kernel
void gsnapdp__mark(gsnapdp_ctx* ctx, hipStream_t st, int stage, int end) {
  if (!ctx->prof_on) return;
  hipEvent_t& e = ctx->ev[2 * stage + end];
  if (!e) (void)hipEventCreate(&e);
  (void)hipEventRecord(e, st);
  ctx->ev_used[stage] = 1;
}

static const char* const kStageNames[] = {"k_plan", "k_scan+k_scatter", "k_fill", "k_rows",
                                          "k_ggap_plan", "k_ggap"};
static const int kNStages = (int)(sizeof(kStageNames) / sizeof(kStageNames[0]));

extern "C" const char* gsnapdp_stage_name(int stage) {
  return (stage >= 0 && stage < kNStages) ? kStageNames[stage] : "";
}

extern "C" int gsnapdp_profile(gsnapdp_ctx* ctx, int enable) {
  if (!ctx) return -1;
  ctx->prof_on = enable ? 1 : 0;
  return kNStages;
}

extern "C" int gsnapdp_profile_read(gsnapdp_ctx* ctx, double* ms, int nstages) {
  if (!ctx) return -1;
  HIPCHK(hipSetDevice(ctx->device));
  for (int i = 0; i < kNStages && i < nstages; i++) {
    if (!ctx->ev_used[i]) continue;
    HIPCHK(hipEventSynchronize(ctx->ev[2 * i + 1]));
    float t = 0.f;
    HIPCHK(hipEventElapsedTime(&t, ctx->ev[2 * i], ctx->ev[2 * i + 1]));
    ms[i] += (double)t;
    ctx->ev_used[i] = 0;  // each read reports the stages recorded since the last one
  }
  return kNStages;
}

extern "C" int gsnapdp_load_maxent_tables(gsnapdp_ctx* ctx, const double* tables, size_t nd) {
  if (!ctx) return -1;
  if (nd != (size_t)12 * 16384 + 4 * 16) {
    gsnapdp__set_err("maxent tables: expected 196672 doubles");
    return -1;
  }
  HIPCHK(hipSetDevice(ctx->device));
  if (!ctx->d_tables) HIPCHK(hipMalloc(&ctx->d_tables, nd * 8));
  HIPCHK(hipMemcpy(ctx->d_tables, tables, nd * 8, hipMemcpyHostToDevice));
  ctx->ntables = nd;
  return 0;
}

extern "C" int gsnapdp_maxent_device(gsnapdp_ctx* ctx, const uint8_t* d_model,
                                     const uint32_t* d_pos, const uint32_t* d_chroff,
                                     double* d_out, int n, void* stream_v) {
  if (!ctx || !ctx->d_tables) {
    gsnapdp__set_err("maxent tables not loaded");
    return -1;
  }
  if (n <= 0) return 0;
  hipStream_t st = stream_v ? (hipStream_t)stream_v : ctx->stream;
  hipLaunchKernelGGL(k_maxent, dim3((n + 255) / 256), dim3(256), 0, st, d_model, d_pos, d_chroff,
                     d_out, n, ctx->d_blocks, (uint64_t)ctx->nwords, ctx->d_tables);
  HIPCHK(hipGetLastError());
  return 0;
}

extern "C" int gsnapdp_maxent_host(gsnapdp_ctx* ctx, const uint8_t* model, const uint32_t* pos,
                                   const uint32_t* chroff, double* out, int n) {
  if (!ctx) return -1;
  if (n <= 0) return 0;
  HIPCHK(hipSetDevice(ctx->device));
  // persistent device staging and one packed page-locked H2D copy:
  // positions | chromosome offsets | models, then the probabilities
  const size_t o_c = (size_t)n * 4, o_m = 2 * o_c, o_out = (o_m + n + 7) & ~(size_t)7;
  const size_t total = o_out + (size_t)n * 8;
  std::lock_guard<std::mutex> host_lock(ctx->host_mu);
  {
    std::lock_guard<std::mutex> lock(ctx->mu);
    if (total > ctx->mx_cap) {
      (void)hipFree(ctx->d_mx_stage);
      ctx->d_mx_stage = nullptr;
      const size_t cap = total + total / 2 + 4096;
      HIPCHK(hipMalloc(&ctx->d_mx_stage, cap));
      ctx->mx_cap = cap;
    }
    if (total > ctx->h_mx_cap) {
      if (ctx->h_mx) (void)hipHostFree(ctx->h_mx);
      ctx->h_mx = nullptr;
      const size_t cap = total + total / 2 + 4096;
      HIPCHK(hipHostMalloc(&ctx->h_mx, cap));
      ctx->h_mx_cap = cap;
    }
  }
  char* h = (char*)ctx->h_mx;
  char* d = ctx->d_mx_stage;
  memcpy(h, pos, (size_t)n * 4);
  memcpy(h + o_c, chroff, (size_t)n * 4);
  memcpy(h + o_m, model, (size_t)n);
  hipStream_t st = ctx->stream;
  HIPCHK(hipMemcpyAsync(d, h, o_m + n, hipMemcpyHostToDevice, st));
  int rc = gsnapdp_maxent_device(ctx, (const uint8_t*)(d + o_m), (const uint32_t*)d,
                                 (const uint32_t*)(d + o_c), (double*)(d + o_out), n, st);
  if (rc == 0) {
    HIPCHK(hipMemcpyAsync(h + o_out, d + o_out, (size_t)n * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    memcpy(out, h + o_out, (size_t)n * 8);
  }
  return rc;
}

// exposed for gsnapdp_host.cpp (expansion needs the host genome and tables)
extern "C" const uint32_t* gsnapdp__host_blocks(gsnapdp_ctx* ctx) { return ctx->h_blocks; }
extern "C" size_t gsnapdp__host_nwords(gsnapdp_ctx* ctx) { return ctx->nwords; }
extern "C" const uint32_t* gsnapdp__host_prof(gsnapdp_ctx* ctx) { return ctx->h_prof; }
