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
//     counting sort (k_plan, whose last block scans, / k_scatter), so band edges are scalar;
//   * 4-bit direction nibbles stream to HBM scratch; each lane then walks its
//     own traceback and emits a compact op stream (include/gsnapdp.h).
//   End gaps in find_best_endpoint mode run here too (the END fills); the
//   other end gaps and windows too wide (W > 48) or too long (L2 > 640) for
//   registers run on the row-lane kernel k_rows (gsnapdp_ggap.hip).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>
#include <utility>

#include "gsnapdp_band.h"
#include "gsnapdp_device.h"
#include "gsnapdp_internal.h"

using namespace gsnapdp;

namespace {

// End gaps that k_fill scans (its END fills, below): 1 find_best_endpoint
// (the rank of a band cell must fit END_RANK_BITS), 2 the last row's scan of
// find_best_endpoint_to_queryend_indels; 0 not on the register band.
constexpr int END_RANK_BITS = 14;
// k_fill's match bits: 1 (default) -- the fill tracks a match byte per
// lane-column in the scratch beside the direction words and the traceback
// reads it; 0 -- the fill keeps no match bits, its tracebacks count diagonal
// steps only and k_count splits them afterwards from the op streams.  Both are
// bit-exact (all GPU tests); 0 makes k_fill 7.7 % faster on C3 (3.50 -> 3.23 ms)
// but k_count costs 0.62 ms per 1M windows (latency-bound: a chain of five
// dependent loads per window), so 1 stays the product (k_fill).
#ifndef GSNAPDP_FILL_MATCH
#define GSNAPDP_FILL_MATCH 1
#endif
constexpr bool FILL_MATCH = GSNAPDP_FILL_MATCH != 0;
constexpr int END_RANK_MAX = (1 << END_RANK_BITS) - 1;
__device__ inline int end_kind(const Derived& d) {
#ifdef GSNAPDP_FILL32
  return 0;  // (the END fills need the 16-bit values)
#endif
  if (d.W > FAST_WMAX || d.L2 > FAST_L2MAX) return 0;
  if (d.mode == 1) return d.eb <= FAST_WMAX && 2 * d.eb * d.L1 + d.L2 + d.eb <= END_RANK_MAX ? 1 : 0;
  return d.mode == 2 ? 2 : 0;
}

// Exclusive scan of bucket sizes, each padded to whole waves of its class
// (64 / CLASS_LPW windows).  cursor[k] = first perm entry of bucket k;
// class_start[c] = first perm entry of class c (a multiple of its wave size,
// since wave sizes shrink as W grows and are powers of two).
// The wave size (64 / CLASS_LPW) of key k's class, branch-free: W from the
// key's triangle index t = k / (2 NEND) (W (W - 1) / 2 <= t < W (W + 1) / 2).
__device__ inline int key_wave(int k) {
  const int t = k / (2 * NEND);
  int W = (int)((1.0f + __builtin_sqrtf((float)(8 * t + 1))) * 0.5f);
  W += key_tri(W + 1) <= t ? 1 : 0;
  W -= key_tri(W) > t ? 1 : 0;
  int c = 0;
#pragma unroll
  for (int j = 0; j < NCLASS - 1; j++) c += W > CLASS_W[j] ? 1 : 0;
  int lpw = CLASS_LPW[0];
#pragma unroll
  for (int j = 1; j < NCLASS; j++) lpw = c == j ? CLASS_LPW[j] : lpw;
  return 64 >> __builtin_ctz(lpw);
}

// Run by the last k_plan block to finish (1024 threads; stage: its NKEYS-word
// LDS histogram, free by then).  Also writes -1 into every bucket's padding
// entries of perm, so perm needs no clearing, and zeroes the global histogram
// for the next batch (the context clears it once at allocation).  Keys are
// read and written coalesced (key tid + 1024 i); the scan runs over each
// thread's contiguous PER keys in LDS.
constexpr int SCAN_PAD_SHIFT = 26;  // stage word: count | padding << 26
__device__ void scan_buckets(int* __restrict__ hist, int* __restrict__ cursor,
                             int* __restrict__ class_start, int* __restrict__ perm, int* stage) {
  __shared__ int wtot[16];  // the 16 waves' totals
  constexpr int PER = (NKEYS + 1023) / 1024;
  const int tid = threadIdx.x;
  {
    // the other blocks' histogram atomics, read (and cleared) by atomics where
    // they were performed, all of this thread's in flight at once
    int v[PER];
#pragma unroll
    for (int i = 0; i < PER; i++) v[i] = tid + i * 1024 < NKEYS ? atomicExch(hist + tid + i * 1024, 0) : 0;
#pragma unroll
    for (int i = 0; i < PER; i++) {
      const int k = tid + i * 1024;
      if (k < NKEYS) {
        const int ng = key_wave(k);
        stage[k] = v[i] | ((((v[i] + ng - 1) & -ng) - v[i]) << SCAN_PAD_SHIFT);
      }
    }
  }
  __syncthreads();
  // exclusive scan of the padded sizes: this thread's PER keys, then the
  // wave by shuffles, then the waves' totals
  const int lo = tid * PER;
  int s = 0;
#pragma unroll
  for (int i = 0; i < PER; i++) {
    if (lo + i < NKEYS) {
      const int x = stage[lo + i];
      s += (x & ((1 << SCAN_PAD_SHIFT) - 1)) + (int)((unsigned)x >> SCAN_PAD_SHIFT);
    }
  }
  const int ln = tid & 63, wv = tid >> 6;
  int x = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o);
    if (ln >= o) x += y;
  }
  if (ln == 63) wtot[wv] = x;
  __syncthreads();
  int run = x - s, total = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    run += k < wv ? wtot[k] : 0;
    total += wtot[k];
  }
  // this thread's own entries become cursors; its buckets' padding entries
  // of perm (at most 63 each, after the bucket's count) get -1
#pragma unroll
  for (int i = 0; i < PER; i++) {
    if (lo + i < NKEYS) {
      const int w = stage[lo + i];
      const int h = w & ((1 << SCAN_PAD_SHIFT) - 1), pad = (int)((unsigned)w >> SCAN_PAD_SHIFT);
      stage[lo + i] = run;
      for (int e = run + h; e < run + h + pad; e++) perm[e] = -1;
      run += h + pad;
    }
  }
  __syncthreads();
  for (int k = tid; k < NKEYS; k += 1024) cursor[k] = stage[k];  // coalesced
  if (tid < NCLASS) {
    // class c covers W in (CLASS_W[c-1], CLASS_W[c]] and keys are W-major
    const int k = first_key_of_w(class_low(tid));
    class_start[tid] = k < NKEYS ? stage[k] : total;
  }
  if (tid == 0) class_start[NCLASS] = total;
}

// ------------------------------------------------------------------ k_plan
// Early returns, QUERYEND_NOGAPS windows (no fill at all) and bucketing.
__global__ void k_plan(const gsnapdp_window* __restrict__ W, int n, const char* __restrict__ q,
                       const char* __restrict__ qu, const uint32_t* __restrict__ blocks,
                       uint64_t nwords, const uint32_t* __restrict__ prof,
                       gsnapdp_result* __restrict__ res, uint32_t* __restrict__ ops,
                       const int64_t* __restrict__ op_off, int* __restrict__ keys,
                       int* __restrict__ hist, int* __restrict__ big_list,
                       int* __restrict__ big_count, int list_cap, int ends_on_band,
                       int* __restrict__ cursor, int* __restrict__ class_start,
                       int* __restrict__ perm, int* __restrict__ ticket) {
  __shared__ int lh[NKEYS];  // block-local histogram: one global atomic per key per block
  __shared__ int lbig[RW_NCLS], lbase[RW_NCLS];  // block-local row-lane list appends
  __shared__ int lend;                             // block-local END task kinds (bits 1, 2)
  __shared__ int last;                             // this block finished last
  for (int k = threadIdx.x; k < NKEYS; k += blockDim.x) lh[k] = 0;
  if (threadIdx.x < RW_NCLS) lbig[threadIdx.x] = 0;
  if (threadIdx.x == 0) lend = 0;
  __syncthreads();
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  int key = -1, big = -1;  // k_fill bucket key, or row-lane class
  if (i < n && W[i].kind != KIND_SKIP) {
    const gsnapdp_window w = W[i];
    const Lane L = make_lane(w);
    int ek = 0;
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
      key = fill_key(L.d.W, L.d.lband, L.d.jl, 0);
    } else if (ends_on_band && (ek = end_kind(L.d)) != 0) {
      key = fill_key(L.d.W, L.d.lband, L.d.jl, ek);
      atomicOr(&lend, 1 << ek);  // k_fill: this batch has END tasks of kind ek
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
  }
  if (i < n) keys[i] = key;
  if (key >= 0) atomicAdd(&lh[key], 1);
  const int lslot = big >= 0 ? atomicAdd(&lbig[big], 1) : 0;
  __syncthreads();
  // one global append per non-empty row-lane class per block (list order is free:
  // k_rows writes each window's own result slot)
  if (threadIdx.x < RW_NCLS)
    lbase[threadIdx.x] = lbig[threadIdx.x] > 0 ? atomicAdd(big_count + threadIdx.x, lbig[threadIdx.x]) : 0;
  if (threadIdx.x == 0 && lend != 0) atomicOr(big_count + RW_NCLS, lend);
  // returning atomics, their results consumed below: each thread holds the
  // values its histogram atomics returned before the block takes its ticket
  int seen = 0;
  for (int k = threadIdx.x; k < NKEYS; k += blockDim.x)
    if (lh[k] > 0) seen |= __hip_atomic_fetch_add(&hist[k], lh[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (seen < 0) lend = -1;  // counts are never negative: keeps the returned values live
  __syncthreads();
  if (big >= 0) big_list[(size_t)big * list_cap + lbase[big] + lslot] = i;
  // The last block to finish scans the histogram (no separate k_scan launch).
  // Ordering, and the hardware property it rests on (measured, not an
  // architectural guarantee: MI355X_MICROARCH.md's inter-workgroup hand-off
  // table, the "last adder told by its returned value" row): the histogram
  // words and the ticket are only ever accessed by agent-scope atomics, which
  // gfx950 performs at the memory side, past the non-coherent per-XCD L2s, so
  // every atomic on a word reads the latest value in its modification order.  A block takes its ticket only
  // after every thread has the RESULTS of its histogram atomics back (returned
  // value = performed there); the ticket's own atomic order then puts every
  // block's histogram adds before the last block's atomicExch reads in
  // scan_buckets.  No release/acquire pair is used because an agent-scope
  // release on gfx950 writes back the XCD's L2 (buffer_wbl2): 0.28 ms per 1M
  // batch when tried.  tests/test_gpu_parity.py::test_gpu_bucket_scan_stress
  // checks the buckets over many batches of varying size.
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0)
    last = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
           (int)gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  scan_buckets(hist, cursor, class_start, perm, lh);
  if (threadIdx.x == 0) *ticket = 0;  // for the next batch
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
// per-wave k_fill scratch: TB_BATCH regions of direction words (u32) then match
// bytes, one 64-lane row per column 0 .. FAST_L2MAX + 3 (the traceback reads
// whole 4-column groups)
#ifndef GSNAPDP_TB_BATCH
#define GSNAPDP_TB_BATCH 8  // regions per wave; a class sweeps min(LPW, this) tasks at once (64 lanes)
#endif
constexpr int TB_BATCH = GSNAPDP_TB_BATCH;
// GSNAPDP_PERMBITS: the direction bits by v_perm_b32 (one byte per plane) instead
// of four alignbit pushes per cell
#ifndef GSNAPDP_PERMBITS
#define GSNAPDP_PERMBITS 1
#endif
constexpr int FILL_PL = GSNAPDP_PERMBITS ? 8 : 0;  // the plane stride (0: S)
// GSNAPDP_DPP_MIN: the lane shifts as v_min_u16_dpp against a per-lane cap
// instead of a DPP move and a select
#ifndef GSNAPDP_DPP_MIN
#define GSNAPDP_DPP_MIN 1
#endif
// GSNAPDP_BUFSTAGE: the ring staging's loads as buffer loads with 32-bit offsets
#ifndef GSNAPDP_BUFSTAGE
#define GSNAPDP_BUFSTAGE 1
#endif
// GSNAPDP_ANDOR: each cell's direction bits joined by one v_and_or_b32
#ifndef GSNAPDP_ANDOR
#define GSNAPDP_ANDOR 1
#endif
// GSNAPDP_GOPEN: each cell's H + open computed once (G) and read twice, as the
// gap2 opening of the slot below (this step) and the gap1 opening of the slot
// above (next step), instead of two adds per cell
#ifndef GSNAPDP_GOPEN
#define GSNAPDP_GOPEN 1
#endif
constexpr bool GOPEN = GSNAPDP_GOPEN != 0;
[[maybe_unused]] constexpr uint32_t PERM_SIGNS = 0x0B0A0908u;  // result bytes 0..3 = signs of bytes 1, 3, 5, 7
constexpr size_t FILL_COLS_DEV = (size_t)FAST_L2MAX + 4;
constexpr size_t FILL_REGION_DW = FILL_COLS_DEV * 64 + FILL_COLS_DEV * 16;

// End gaps in find_best_endpoint mode (QUERYEND_GAP / BEST_LOCAL, dynprog.c:
// 2235-2290) on the register band (END = 1).  Three changes to the fill:
//  * rows below L1 are capped to a NEG-like value: their profile word carries
//    FV_NEG_END in bits 16..31 where a live row's has bit 31 set, and the
//    nogap value is min'ed with that half (they never feed a live row);
//  * the ENDQ nibbles are signed (END_SC_BIAS) and NEG-like values start at
//    FV_NEG_END (gsnapdp_band.h);
//  * every cell of the unwidened band |c - r| <= extraband offers
//    key = score * 2^14 + (row-major rank or its complement) to a per-lane
//    maximum, so that one max per cell reproduces the reference's scan order:
//    the first best cell for '>', the last for the jump-late '>='.  The rank
//    of (r, c) is 2*eb*r + c + eb (the band's cells in row-major order); the
//    start (0, 0) with 0 has rank eb, below every cell's.
// END = 2: find_best_endpoint_to_queryend_indels (:2293-2355) scans the last
// row only.  Row L1's profile word alone has bit 31 set (no cap: rows below L1
// cannot reach row L1), a cell offers min(H, that bit spread over 16 bits) --
// its nogap value in row L1, 0 elsewhere -- to the column's maximum, and the
// column's key is that value * 2^14 + (column or its complement).
// Segment windows (seg != nullptr; Dynprog_end5/3_splicejunction,
// use_genomicseg_p, :1535 / :1690): column c's genome is the caller's segment
// byte seg[spos + gstep * (c - 1)] instead of the packed genome.
struct FillOut {
  int score, br, bc;  // finalscore and the traceback's start cell
};

// (always inlined into fill_tasks: an outlined call costs a callee-saved
// register spill per task and its own register allocation)
template <int S, int LPW, int LOW, int JL, int END>
__device__ __forceinline__ FillOut fill_group(const gsnapdp_window* __restrict__ Wn, int wi, bool active, int lane,
                              uint32_t* __restrict__ D, uint8_t* __restrict__ M,
                              const char* __restrict__ q, const char* __restrict__ qu,
                              const uint32_t* __restrict__ blocks, uint64_t nwords,
                              const uint32_t* sprof, uint32_t* ring,
                              const gsnapdp_sj_window* __restrict__ sjw) {
  static_assert(S >= 2 && S <= 8 && LPW <= 16 && 64 % LPW == 0, "class shape");
  using RG = Rings<S, LPW>;
  static_assert(RG::WORDS <= RING_WORDS_MAX, "LDS ring budget");
  constexpr int WMAX = S * LPW;
  constexpr int NG = 64 / LPW;
  constexpr int NAB = (WMAX - LOW) < S ? (WMAX - LOW) : S;  // local slots that may lie above the band
  constexpr FV NEGV = END ? (FV)FV_NEG_END : (FV)FV_NEG;
  constexpr uint32_t LIVE = END == 1 ? 0x80000000u : 0u;  // END 1: a live row's cap (bits 16..31) is >= 2^15
  constexpr uint32_t DEAD = (uint32_t)NEGV << 16;          // END 1: a row below L1
  constexpr uint32_t LAST = 0x80000000u;                   // END 2: row L1
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
    if (sjw) {  // a segment: every column 1..L2 is inside it
      cvlo = 1;
      cvhi = L2;
      gp0 = sjw[wi].spos - L.gstep;  // segment byte of column c: gp0 + gps*c
      gps = L.gstep;
    }
    qbase = L.qbase;
    qstep = L.qstep;
  }
  // wave-uniform (a kernel argument; made so for the compiler, which sees a
  // non-inlined function argument in VGPRs and would branch per lane)
  const bool segw = __builtin_amdgcn_readfirstlane(sjw != nullptr ? 1 : 0) != 0;
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
    if (END == 1 && r > L1) return DEAD;
    return sprof[mtoff + qb] | sprof[UTAB + ub] | LIVE | (END == 2 && r == L1 ? LAST : 0u);
  };
  const uint64_t gmax = nwords >= 3 ? (nwords - 3) / 3 : 0;  // last whole genome block

  FV H[S], E[S], F[S];
  // GOPEN: G[s] = H[s] + open (the gap openings from slot s); otherwise unused
  [[maybe_unused]] FV G[S];
  uint32_t P[S];
  // Match bits of the lane's S rows against each genome class: byte k of MB
  // holds, in bits 0..S-1, whether slot s's query row matches class k
  // (consistent_array or uppercase equality, dynprog.c:2650-2656).  The rows
  // move up one slot per column, so MB shifts right by one and the entering
  // row's bits come in at bit S-1 of each byte (from the LDS lookup table).
  const uint64_t* mlut = (const uint64_t*)(sprof + MLUT);
  constexpr uint64_t MB_KEEP = 0x0101010101ull * ((1u << (S - 1)) - 1u);
#ifdef EXP_NOMLUT  // timing experiment only: no LDS lookup (wrong match bits)
  auto row_spread = [&](uint32_t pw) -> uint64_t { return ((uint64_t)(pw & 0x1F000000u) << 8) >> (8 - S); };
#else
  auto row_spread = [&](uint32_t pw) -> uint64_t { return mlut[(pw >> 24) & 31u] >> (8 - S); };
#endif
  uint64_t MB = 0;
  // column 0 (dynprog.c:1460-1488) in offset coordinates
#pragma unroll
  for (int s = 0; s < S; s++) {
    const int r = row0 + s;
    H[s] = (r == 0) ? FV_BIAS : NEGV;
    E[s] = NEGV;
    F[s] = (r >= 1) ? FV_BIAS + open : NEGV;  // open + r*ext - r*ext
    P[s] = row_word(r);
    if constexpr (GOPEN) G[s] = H[s] + open;
    if constexpr (FILL_MATCH) MB = ((MB >> 1) & MB_KEEP) | row_spread(P[s]);
  }
  // Rings: lane j of a window stages the rows / columns congruent to j mod
  // LPW.  Lane j's bottom slot holds row t + j*(S-1) + rbase at step t, its
  // column is t - j.  Before step 1: rows [1+rbase, K+rbase+SPAN], columns
  // [1, K]; after step t = nK: rows (t+rbase+SPAN, t+K+rbase+SPAN], columns
  // (t, t+K].  Same-wave LDS writes are visible to later reads in order.
  uint32_t* rr = ring + g * RG::RR;
  uint8_t* cr = (uint8_t*)(ring + NG * RG::RR) + g * RG::CR;
  const int rbase = S - 1 - stop - rband;
#if GSNAPDP_BUFSTAGE
  // the staging's buffer resources (raw, byte offsets < 2^31; the genome's
  // ends at its last word, so a block past it reads as 0)
  // (the pointers arrive as arguments of a non-inlined function, in VGPRs: made
  // wave-uniform first, so the resources live in SGPRs and no load needs a
  // waterfall loop)
  auto uniform = [](const void* p) -> void* {
    const uint64_t a = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    return (void*)(((uint64_t)hi << 32) | lo);
  };
  const int nbytes = __builtin_amdgcn_readfirstlane((int)(nwords * 4 < 0x7FFFFFFFull ? nwords * 4 : 0x7FFFFFFFull));
  const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc(uniform(q), 0, 0x7FFFFFFF, 0x00020000);
  const __amdgpu_buffer_rsrc_t rqu = __builtin_amdgcn_make_buffer_rsrc(uniform(qu), 0, 0x7FFFFFFF, 0x00020000);
  const __amdgpu_buffer_rsrc_t rgb = __builtin_amdgcn_make_buffer_rsrc(uniform(blocks), 0, nbytes, 0x00020000);
  const int L1c = L1 > 0 ? L1 : 1, L2c = L2 > 0 ? L2 : 1, qb1 = qbase - qstep;
  // the direction / match scratch of this task, based LPW - 1 rows (of 64 lanes)
  // early: a step's row offset t * 256 (t * 64) is then non-negative
  const __amdgpu_buffer_rsrc_t rD = __builtin_amdgcn_make_buffer_rsrc(
      uniform((const void*)((const char*)D - (LPW - 1) * 256)), 0, 0x7FFFFFFF, 0x00020000);
  const __amdgpu_buffer_rsrc_t rM = __builtin_amdgcn_make_buffer_rsrc(
      uniform((const void*)((const char*)M - (LPW - 1) * 64)), 0, 0x7FFFFFFF, 0x00020000);
  const uint32_t gmax32 = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(gmax < 0xFFFFFFFFull ? gmax : 0xFFFFFFFFull));
#endif
  auto stage = [&](auto nrows_tag, int rlo, int clo) {
    constexpr int NR = decltype(nrows_tag)::value;
    constexpr int ER = (NR + LPW - 1) / LPW, EC = (RING_K + LPW - 1) / LPW;
    // all loads first (clamped addresses, no branches), then the words
    uint32_t qb[ER], ub[ER], gw[EC], gf[EC];
#if GSNAPDP_BUFSTAGE
    // buffer loads with 32-bit offsets (buffer resources rq / rqu / rgb below):
    // a clamp and a 24-bit multiply-add per row, no 64-bit address arithmetic
#pragma unroll
    for (int e = 0; e < ER; e++) {
      const int r = rlo + e * LPW + j;
      const int qi = __mul24(qstep, min(max(r, 1), L1c)) + qb1;
      qb[e] = __builtin_amdgcn_raw_buffer_load_b8(rq, qi, 0, 0);
      ub[e] = __builtin_amdgcn_raw_buffer_load_b8(rqu, qi, 0, 0);
    }
#pragma unroll
    for (int e = 0; e < EC; e++) {
      const int c = clo + e * LPW + j;
      if (segw) {  // the segment byte of column c (clamped into 1..L2; a shadow group's L2 is 0)
        const int cc = min(max(c, 1), L2c);
        gw[e] = __builtin_amdgcn_raw_buffer_load_b8(rq, (int)gp0 + __mul24(gps, cc), 0, 0);
        gf[e] = 0u;
      } else {
        // block b of position pos at byte 12 b (a block past the genome reads 0: the
        // resource ends at the genome's last word; such columns are N anyway)
        const uint32_t pos = gp0 + (uint32_t)__mul24(gps, c);
        const uint32_t b = pos >> 5;
        const uint32_t ob = (b << 3) + (b << 2);
        gw[e] = __builtin_amdgcn_raw_buffer_load_b32(rgb, (int)(ob + ((pos & 16u) ? 0u : 4u)), 0, 0);
        gf[e] = __builtin_amdgcn_raw_buffer_load_b32(rgb, (int)(ob + 8u), 0, 0);
      }
    }
#else
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
      if (segw) {  // the segment byte of column c (clamped into 1..L2; a shadow group's L2 is 0)
        const int cc = max(1, min(c, L2));
        gw[e] = (unsigned char)q[gp0 + (uint32_t)(gps * cc)];
        gf[e] = 0u;
      } else {
        const uint32_t pos = gp0 + (uint32_t)(gps * c);
        const uint64_t b = (uint64_t)(pos >> 5);
        const uint64_t ptr = (b <= gmax ? b : gmax) * 3u;
        gw[e] = blocks[ptr + ((pos & 31u) < 16 ? 1 : 0)];
        gf[e] = blocks[ptr + 2];
      }
    }
#endif
#pragma unroll
    for (int e = 0; e < ER; e++) {
      const int r = rlo + e * LPW + j;
      const bool ok = r >= 1 && r <= L1;
      uint32_t w = sprof[mtoff + (ok ? (qb[e] & 127u) : 0u)] | sprof[UTAB + (ok ? ub[e] : 255u)] | LIVE;
      if (END == 1 && r > L1) w = DEAD;
      if (END == 2 && r == L1) w |= LAST;
      if (e * LPW + j < NR) rr[r & (RG::RR - 1)] = w;
    }
#pragma unroll
    for (int e = 0; e < EC; e++) {
      const int c = clo + e * LPW + j;
#if GSNAPDP_BUFSTAGE
      const uint32_t pos = gp0 + (uint32_t)__mul24(gps, c);
      const bool ing = (pos >> 5) <= gmax32;  // outside the genome: N
#else
      const uint32_t pos = gp0 + (uint32_t)(gps * c);
      const bool ing = (uint64_t)(pos >> 5) <= gmax;  // outside the genome: N
#endif
      const uint32_t bit = pos & 31u;
      const int code = (int)((gw[e] >> ((bit & 15u) * 2u)) & 3u) ^ xorc;
      const bool inr = c >= cvlo && c <= cvhi;
      int k = !inr ? 5 : ((!ing || ((gf[e] >> bit) & 1u)) ? 4 : code);
      if (segw) k = inr ? seg_class((unsigned char)gw[e]) : 5;
      if (e * LPW + j < RING_K) cr[c & (RG::CR - 1)] = (uint8_t)k;
    }
    __builtin_amdgcn_s_waitcnt(0);  // nothing of the staging stays in flight into the column loop
  };
  stage(std::integral_constant<int, RING_K + RG::SPAN>(), 1 + rbase, 1);
  uint32_t pnext = rr[(1 + j * (S - 1) + rbase) & (RG::RR - 1)];
  int gnext = cr[(1 - j) & (RG::CR - 1)];
  FV fin = NEGV;
  const int se = stop + L1 - L2 + rband;  // global slot of the endpoint (L1,L2)
  const int je = se / S, sle = se - je * S;
  // END: the scan key of slot s is (H << 14) + Qs[s] + R(c); Qs[s] holds the
  // slot's diagonal d = c - r (or kills a slot outside |d| <= eb), R(c) the
  // column's share, kept in Rc and stepped by dR with the lane's column.
  int ebw = 0, Rc = 0, dR = 0, Bt = 0;
  int Qs[S];
  if constexpr (END == 2) {  // the last row's scan: R(c) = the column's share of the key
    auto Rof = [&](int c) {
      return ((L1 + c) * ext - (int)FV_BIAS) * (1 << END_RANK_BITS) + (JL ? c : END_RANK_MAX - c);
    };
    Rc = Rof(1 - j);
    dR = Rof(2 - j) - Rc;
    Bt = -(1 << 30);  // below every cell's key: the start (L1, 0) with NEG_INFINITY (:2302)
  }
  if constexpr (END == 1) {
    ebw = min(lband, rband);  // wave-uniform: derive() widens one side only
    const int kq = -ext * (1 << END_RANK_BITS) + (JL ? -2 * ebw : 2 * ebw);
#pragma unroll
    for (int s = 0; s < S; s++) {
      const int d = rband + stop - j * S - s;
      Qs[s] = (d >= -ebw && d <= ebw) ? d * kq : -(1 << 30);
    }
    auto Rof = [&](int c) {
      return (2 * c * ext - (int)FV_BIAS) * (1 << END_RANK_BITS) +
             (JL ? (2 * ebw + 1) * c + ebw : END_RANK_MAX - (2 * ebw + 1) * c - ebw);
    };
    Rc = Rof(1 - j);  // the lane's column at step 1
    dR = Rof(2 - j) - Rc;
    Bt = JL ? ebw : END_RANK_MAX - ebw;  // find_best_endpoint's start: (0, 0) with 0 (:2243)
  }
  // scratch layout: column c's words are D[c*64 + (j*NG + g)], one 256-byte
  // row per column (coalesced stores); the match bytes likewise in M.  Lane
  // (j, g) stores column c = t - j at the wave-uniform row t-(LPW-1) plus a
  // non-negative lane offset.
  const int lane_off = (LPW - 1 - j) * 64 + j * NG + g;
  // the lane shifts' caps: NEGV on the group's first (above) / last (below) lane
  [[maybe_unused]] const FV capA = j == 0 ? NEGV : (FV)0xFFFFu, capB = j == LPW - 1 ? NEGV : (FV)0xFFFFu;
  // their loop-carried results (the first lane of each 16-lane row never writes
  // its above pair, the last never its below pair: they stay NEGV)
  [[maybe_unused]] FV hpA = NEGV, fpA = NEGV, hbB = NEGV, ebB = NEGV;

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
    // new (nogap, gap2) just above local slot 0 (GOPEN: nogap + open)
    FV hp = NEGV, fp = NEGV;
#if GSNAPDP_DPP_MIN
    // lane j = 0 takes min(the lane above's value, NEGV): a NEG-like value (every
    // value of the fill is >= the NEG-like floor, so the min is either NEGV or a
    // NEG-like value itself; DESIGN.md "Band edges"), in one v_min_u16_dpp each
    if (LPW > 1) {
      // (GOPEN: G instead of H; min(G, NEGV) is NEG-like exactly when
      // min(H, NEGV) + open is, so the cap stays NEGV)
      min2_from_lane_above(hpA, fpA, GOPEN ? G[S - 1] : H[S - 1], F[S - 1], capA);
      hp = hpA;
      fp = fpA;
    }
#else
    if (LPW > 1) {
      const FV h = (FV)from_lane_above((int)(GOPEN ? G[S - 1] : H[S - 1])), f = (FV)from_lane_above((int)F[S - 1]);
      if (j != 0) {
        hp = h;
        fp = f;
      }
    }
#endif
    // four bit planes (v1, h1, dF, dE), each a short independent chain
    [[maybe_unused]] uint32_t av = 0u, ah = 0u, af = 0u, ae = 0u;
    uint32_t gsh = 0u;
    [[maybe_unused]] uint32_t bits = 0u;  // GSNAPDP_PERMBITS: the four planes, one byte each
    int bstep = END == 2 ? 0 : -(1 << 30);  // END: this column's best scan key (END 2: value), less R(c)
    auto cell = [&](int s, FV Hr, FV Er) {  // (GOPEN: Hr is the slot below's G)
      const FV Hd = H[s], Ed = E[s], Fd = F[s];
      const uint32_t pw = pslot(s);
      const FV a = GOPEN ? Hr : Hr + open;
      const FV b = GOPEN ? hp : hp + open;
      const FV m1 = fv_max(Hd, Ed);
      // pairdistance - 2*extend
      const FV sc = END ? (FV)__builtin_amdgcn_sbfe((int)pw, (int)gsh, 4) : (FV)__builtin_amdgcn_ubfe(pw, gsh, 4);
      const bool above = (s < NAB) && (j * S + s < stop);  // loop-invariant lane mask
      FV hn = fv_max(m1, Fd) + sc;
      if constexpr (END == 1) hn = fv_cap_hi(hn, pw);  // rows below L1
      hn = above ? NEGV : hn;
      if constexpr (END == 1) bstep = max(bstep, (int)(hn << END_RANK_BITS) + Qs[s]);
      if constexpr (END == 2) bstep = (int)fv_max((FV)bstep, fv_min(hn, (uint32_t)((int)pw >> 31)));  // row L1 only
      const int dv = JL ? (int)(Fd - m1) : (int)(m1 - Fd);  // v1: nogap from gap2
      const int dh = JL ? (int)(Ed - Hd) : (int)(Hd - Ed);  // h1: nogap from gap1
      const int df = JL ? (int)(fp - b) : (int)(b - fp);    // dF: gap2 extends
      const int de = JL ? (int)(Er - a) : (int)(a - Er);    // dE: gap1 extends
#if GSNAPDP_PERMBITS
      // the cell's four signs in one dword: (dh, dv) and (de, df) as the low and
      // high halves of two 16-bit difference pairs (|difference| < 2^15, so bit
      // 15 of each half is its sign), v_perm_b32 selectors 8-11 spread the four
      // sign bits over the four bytes (plane p in byte p), and one and-or keeps
      // bit S-1-s of each byte: the layout the four pushes built, at byte stride
      {
        uint32_t p01, p23, sg;
        asm("v_sub_u16 %0, %1, %2" : "=v"(p01) : "v"(JL ? Ed : Hd), "v"(JL ? Hd : Ed));
        asm("v_sub_u16_sdwa %0, %1, %2 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0"
            : "+v"(p01)
            : "v"(JL ? Fd : m1), "v"(JL ? m1 : Fd));
        asm("v_sub_u16 %0, %1, %2" : "=v"(p23) : "v"(JL ? Er : a), "v"(JL ? a : Er));
        asm("v_sub_u16_sdwa %0, %1, %2 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0"
            : "+v"(p23)
            : "v"(JL ? fp : b), "v"(JL ? b : fp));
        asm("v_perm_b32 %0, %1, %2, %3" : "=v"(sg) : "v"(p01), "v"(p23), "s"(PERM_SIGNS));
#if GSNAPDP_ANDOR
        // one v_and_or_b32 per cell (the compiler's and + or3 tree issues twice as many)
        if (s == 0) {
          bits = sg & (0x01010101u << (S - 1));
        } else {
          asm("v_and_or_b32 %0, %1, %2, %0" : "+v"(bits) : "v"(sg), "s"(0x01010101u << (S - 1 - s)));
        }
#else
        bits = s == 0 ? (sg & (0x01010101u << (S - 1))) : ((sg & (0x01010101u << (S - 1 - s))) | bits);
#endif
      }
      (void)dv, (void)dh, (void)df, (void)de;
#elif defined(EXP_NODIFF)  // timing experiments only (wrong direction bits)
      (void)dv, (void)dh, (void)df, (void)de;
#elif defined(EXP_ADDPUSH)
      av += (uint32_t)dv, ah += (uint32_t)dh, af += (uint32_t)df, ae += (uint32_t)de;
#else
      av = push_sign(av, dv);  // (the first push shifts in zeros: one op, not a compare)
      ah = push_sign(ah, dh);
      af = push_sign(af, df);
      ae = push_sign(ae, de);
#endif
      E[s] = fv_max(a, Er);
      const FV f = fv_max(b, fp);
      F[s] = f;
      H[s] = hn;
      if constexpr (GOPEN) {
        G[s] = hn + open;
        hp = G[s];
      } else {
        hp = hn;
      }
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
      gsh = 4u * (uint32_t)gnext;
      if constexpr (FILL_MATCH) {
        MB = ((MB >> 1) & MB_KEEP) | row_spread(pnext);
        macc = (uint32_t)(MB >> (8u * (uint32_t)gnext));
      }
      cell(0, GOPEN ? G[1] : H[1], E[1]);
    }
    FV hb = NEGV, eb = NEGV;  // old (nogap, gap1) just below the lowest local slot
#if GSNAPDP_DPP_MIN
    if (LPW > 1) {
      min2_from_lane_below(hbB, ebB, GOPEN ? G[0] : H[0], E[0], capB);
      hb = hbB;
      eb = ebB;
    }
#else
    if (LPW > 1) {
      const FV h = (FV)from_lane_below((int)(GOPEN ? G[0] : H[0])), e = (FV)from_lane_below((int)E[0]);
      if (j != LPW - 1) {
        hb = h;
        eb = e;
      }
    }
#endif
    if (act) {
#pragma unroll
      for (int s = 1; s < S - 1; s++) cell(s, GOPEN ? G[s + 1] : H[s + 1], E[s + 1]);
      cell(S - 1, hb, eb);
      if constexpr (END == 1) Bt = max(Bt, bstep + Rc);
      if constexpr (END == 2) Bt = max(Bt, (bstep << END_RANK_BITS) + Rc);
#if GSNAPDP_PERMBITS
      const uint32_t acc = bits;
#else
      const uint32_t acc = (((((av << S) | ah) << S) | af) << S) | ae;
#endif
#ifndef EXP_NOSTORE
#if GSNAPDP_BUFSTAGE
      // buffer stores: the lane's constant offset in a VGPR, the step's row in an
      // SGPR (t * 256 / t * 64 from resources based LPW - 1 rows below D / M),
      // so a step's two stores need no address arithmetic
      __builtin_amdgcn_raw_buffer_store_b32(acc, rD, lane_off * 4, t * 256, 0);
#ifndef EXP_NOMATCH
      if constexpr (FILL_MATCH) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)macc, rM, lane_off, t * 64, 0);
#endif
#else
      D[(ptrdiff_t)(t - (LPW - 1)) * 64 + lane_off] = acc;
#ifndef EXP_NOMATCH
      if constexpr (FILL_MATCH) M[(ptrdiff_t)(t - (LPW - 1)) * 64 + lane_off] = (uint8_t)macc;
#endif
#endif
#else
      if (acc == 0x12345678u && macc == 77u) D[0] = 1u;
#endif
    }
    if constexpr (END) Rc += dR;
    // next column's inputs from the rings (every lane, every step)
    if (t % RING_K == 0) stage(std::integral_constant<int, RING_K>(), t + 1 + rbase + RG::SPAN, t + 1);
#ifdef EXP_NORINGREAD  // timing experiment only: no per-step LDS reads (wrong inputs)
    pnext = pnext * 3u + (uint32_t)t;
    gnext = (gnext + 1) & 3;
#else
    pnext = rr[(t + 1 + j * (S - 1) + rbase) & (RG::RR - 1)];
    gnext = cr[(t + 1 - j) & (RG::CR - 1)];
#endif
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
  if constexpr (END == 2) {
#pragma unroll
    for (int o = LPW / 2; o > 0; o >>= 1) Bt = max(Bt, __shfl_xor(Bt, o));
    const int post = Bt & END_RANK_MAX;
    return FillOut{Bt >> END_RANK_BITS, L1, JL ? post : END_RANK_MAX - post};
  }
  if constexpr (END == 1) {
    // the group's best key: score, then rank (row-major order)
#pragma unroll
    for (int o = LPW / 2; o > 0; o >>= 1) Bt = max(Bt, __shfl_xor(Bt, o));
    const int post = Bt & END_RANK_MAX;
    const int rank = JL ? post : END_RANK_MAX - post;
    const int br = rank / (2 * ebw + 1);
    return FillOut{Bt >> END_RANK_BITS, br, br + rank - br * (2 * ebw + 1) - ebw};
  }
  // endpoint (L1,L2): the lanes stopped on column L2 (dynprog.c:4545)
#pragma unroll
  for (int s = 0; s < S; s++)
    if (j == je && s == sle) fin = H[s];
  fin = __shfl(fin, gbase + je);
  return FillOut{(int)(fin - FV_BIAS) + (L1 + L2) * ext, L1, L2};
}

// The tracebacks of up to TB_BATCH wave-tasks of one class in ONE backward
// sweep, one window per lane: lane k * NG + g traces group g of the batch's
// task k (direction scratch region k).  A task's own sweep would run on lane 0
// of each group only (NG of the 64 lanes); this sweep keeps up to
// TB_BATCH * NG lanes busy.  wi < 0: no window on this lane.
// The pointers carry the global address space (as fill_tasks' do), so that the
// sweep's loads compile to global_load and the compiler can wait on the group
// being visited (vmcnt) while the next group's prefetch stays in flight; with
// generic pointers they were flat loads, each use a full vmcnt(0) lgkmcnt(0) drain.
template <int S, int LPW>
__device__ void trace_batch(int lane, int wi, FillOut fo, int jl,
                            const AS_GLOBAL gsnapdp_window* Wn1, const AS_GLOBAL uint32_t* D1,
                            const AS_GLOBAL uint32_t* blocks1, uint64_t nwords,
                            AS_GLOBAL gsnapdp_result* res1, AS_GLOBAL uint32_t* ops1,
                            const AS_GLOBAL int64_t* op_off1, const AS_GLOBAL gsnapdp_sj_window* sjw1,
                            const AS_GLOBAL char* q1) {
  const gsnapdp_window* __restrict__ Wn = wave_uniform((const gsnapdp_window*)Wn1);
  const uint32_t* __restrict__ D = wave_uniform((const uint32_t*)D1);
  const uint32_t* __restrict__ blocks = wave_uniform((const uint32_t*)blocks1);
  gsnapdp_result* __restrict__ res = wave_uniform((gsnapdp_result*)res1);
  uint32_t* __restrict__ ops = wave_uniform((uint32_t*)ops1);
  const int64_t* __restrict__ op_off = wave_uniform((const int64_t*)op_off1);
  const gsnapdp_sj_window* __restrict__ sjw = wave_uniform((const gsnapdp_sj_window*)sjw1);
  const char* __restrict__ q = wave_uniform((const char*)q1);
  constexpr int NG = 64 / LPW;
  constexpr int WMAX = S * LPW;
  const int k = lane / NG, g = lane % NG;
  const bool tr = wi >= 0;
  const gsnapdp_window w = Wn[tr ? wi : 0];
  const Lane L = make_lane(w);
  const int maxC = __builtin_amdgcn_readfirstlane(wave_max(tr ? fo.bc : 0));
#ifdef EXP_NOTRACE
  if (tr) res[wi].finalscore = fo.score;
  return;
#endif
  if (!tr) return;
  const uint32_t* Dk = D + (size_t)k * FILL_REGION_DW;
  const uint8_t* Mk = (const uint8_t*)(Dk + FILL_COLS_DEV * 64);
  ColStream cs;
  cs.init(L);
  Tally tal = {0, 0, 0, 0, 0};
  OpWriter ow = {ops + op_off[wi], (int)(op_off[wi + 1] - op_off[wi]), 0, 0};
  // a segment window's genome classes (the long-gap intron test) come from its segment
  const SegCls sc = {sjw ? (const unsigned char*)q + sjw[wi].spos : nullptr, L.g0};
  band_traceback<S, LPW, FILL_MATCH, FILL_PL ? FILL_PL : S>(Dk, Mk, g, fo.br, fo.bc, maxC, L.d.lband, L.d.rband, WMAX - L.d.W,
                         sjw ? 1 : cs.cvlo, sjw ? L.d.L2 : cs.cvhi, jl, L, blocks, nwords, tal, ow, sc);
  // Dynprog_end5/3_splicejunction score the alignment from its counts (:5541 / :6045)
  // (without the fill's match bits k_count does both once it has the counts)
  const int score = sjw && FILL_MATCH
                        ? tal.nmatches * 3 - 5 * tal.nmismatches + tal.nopens * L.d.open + tal.nindels * L.d.ext
                        : fo.score;
  write_result(res + wi, w, L, score, fo.br, fo.bc, tal, ow, FILL_MATCH);
}

// This wave's wave-tasks of class (S, LPW, LOW), in batches of B (<= TB_BATCH)
// tasks whose tracebacks share one sweep: task t covers the 64/LPW
// windows perm[t*NG ..]; the wave runs t = t0, t0 + stride, ... < t1.  Not
// inlined, so each class gets its own register allocation (inlining the
// classes into the kernel spills across them); called once per wave and
// class rather than once per task, so the call's callee-saved VGPR saves and
// restores (48 VGPRs to scratch, ~24 KB per call) are paid per wave, not per
// task.  The pointers carry their address spaces (global / LDS) so that the
// body still compiles to global_* and ds_* accesses rather than flat ones.
template <int S, int LPW, int LOW, int END>
__device__ __noinline__ void fill_tasks(int t0, int t1, int stride, const AS_GLOBAL gsnapdp_window* Wn1,
                                        const AS_GLOBAL int* perm1, const AS_GLOBAL char* q1,
                                        const AS_GLOBAL char* qu1, const AS_GLOBAL uint32_t* blocks1,
                                        uint64_t nwords, const AS_LDS uint32_t* sprof3,
                                        AS_LDS uint32_t* ring3,
                                        AS_GLOBAL uint32_t* D1, AS_GLOBAL gsnapdp_result* res1,
                                        AS_GLOBAL uint32_t* ops1, const AS_GLOBAL int64_t* op_off1,
                                        const AS_GLOBAL gsnapdp_sj_window* sjw1, int lag) {
  const gsnapdp_window* __restrict__ Wn = wave_uniform((const gsnapdp_window*)Wn1);
  const int* __restrict__ perm = wave_uniform((const int*)perm1);
  const char* __restrict__ q = wave_uniform((const char*)q1);
  const char* __restrict__ qu = wave_uniform((const char*)qu1);
  const uint32_t* __restrict__ blocks = wave_uniform((const uint32_t*)blocks1);
  const uint32_t* sprof = (const uint32_t*)sprof3;
  uint32_t* ring = (uint32_t*)ring3;
  uint32_t* __restrict__ D = wave_uniform((uint32_t*)D1);
  const gsnapdp_sj_window* __restrict__ sjw = wave_uniform((const gsnapdp_sj_window*)sjw1);
  constexpr int NG = 64 / LPW;
  constexpr int B = LPW < TB_BATCH ? LPW : TB_BATCH;  // tasks per traceback sweep
  const int lane = threadIdx.x & 63;
  const int g = lane / LPW;
  // the class's single-gap and end-gap tasks (bucket keys end in the END kind)
  // run in one call per kind, END = 0, 1, 2, each over the tasks of its kind only
  auto kind_of = [&](int t) {
    const int m = derive(Wn[perm[(size_t)t * NG]]).mode;
    return __builtin_amdgcn_readfirstlane(m == 1 || m == 2 ? m : 0);
  };
  int t = t0;
  while (t < t1 && kind_of(t) != END) t += stride;
  // lag > 0: the wave's first batch is lag tasks short, so that the waves
  // sharing a SIMD reach their (latency-bound) traceback sweeps at different
  // times instead of together
  int bsz = lag > 0 ? (B - lag > 1 ? B - lag : 1) : B;
  while (t < t1) {
    // this lane's window in the batch's sweep: group (lane % NG) of task lane / NG
    int my_wi = -1, my_jl = 0;
    FillOut my = {0, 0, 0};
    const int bk = bsz;
    bsz = B;
    for (int k = 0; k < bk && t < t1; k++) {
      uint32_t* Dk = D + (size_t)k * FILL_REGION_DW;
      uint8_t* Mk = (uint8_t*)(Dk + FILL_COLS_DEV * 64);
      const int wi0 = perm[(size_t)t * NG + g];
      const int w0 = __builtin_amdgcn_readfirstlane(perm[(size_t)t * NG]);  // group 0: a real window
      const bool active = wi0 >= 0;
      const int wi = active ? wi0 : w0;  // idle groups shadow group 0 (reads only)
      // the bucket's tie rule (an end5 gap's fill is reversed with !jump_late_p)
      const int jl = __builtin_amdgcn_readfirstlane(derive(Wn[w0]).jl);
#ifdef TB_PROF
      const uint64_t t0 = __builtin_amdgcn_s_memtime();
#endif
      const FillOut fo =
          jl ? fill_group<S, LPW, LOW, 1, END>(Wn, wi, active, lane, Dk, Mk, q, qu, blocks, nwords, sprof, ring, sjw)
             : fill_group<S, LPW, LOW, 0, END>(Wn, wi, active, lane, Dk, Mk, q, qu, blocks, nwords, sprof, ring, sjw);
#ifdef TB_PROF
      TB_COUNT(4, __builtin_amdgcn_s_memtime() - t0);
#endif
      const int src = (lane % NG) * LPW;  // lane 0 of group lane % NG
      const int v_wi = __shfl(wi0, src);
      const FillOut v = {__shfl(fo.score, src), __shfl(fo.br, src), __shfl(fo.bc, src)};
      if (lane / NG == k) {
        my_wi = v_wi;
        my = v;
        my_jl = jl;
      }
      do t += stride;
      while (t < t1 && kind_of(t) != END);
    }
#ifdef TB_PROF
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
#endif
    trace_batch<S, LPW>(lane, my_wi, my, my_jl, Wn1, D1, blocks1, nwords, res1, ops1, op_off1, sjw1, q1);
#ifdef TB_PROF
    TB_COUNT(5, __builtin_amdgcn_s_memtime() - t1);
#endif
  }
}

// All register-band classes in one persistent launch: the wave-tasks of the
// classes form one index space (class by class), so one class's tail overlaps
// the next class's work and empty classes cost nothing.  Register budget:
// 512 / GSNAPDP_FILL_WAVES VGPRs (168 at 3 waves per SIMD); any spills sit in the task
// call's prologue/epilogue and loop preheaders, not in the column loops.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(GSNAPDP_FILL_WAVES, 8))) void k_fill(
    const gsnapdp_window* __restrict__ Wn, const int* __restrict__ perm,
    const int* __restrict__ class_start, const char* __restrict__ q, const char* __restrict__ qu,
    const uint32_t* __restrict__ blocks, uint64_t nwords, const uint32_t* __restrict__ prof,
    uint32_t* __restrict__ dirpool, size_t wave_stride, gsnapdp_result* __restrict__ res,
    uint32_t* __restrict__ ops, const int64_t* __restrict__ op_off, const int* __restrict__ end_flag,
    const gsnapdp_sj_window* __restrict__ sjw, int min_tasks, int stagger, int split_mode, int split_w) {
  __shared__ alignas(8) uint32_t sprof[SPROF_WORDS];
  __shared__ uint32_t rings[4][RING_WORDS_MAX];  // one per wave of the block
#ifdef TB_PROF
  const uint64_t kt0 = __builtin_amdgcn_s_memtime();
#endif
  for (int i = threadIdx.x; i < MLUT; i += blockDim.x)
    sprof[i] = i < UTAB ? fill_profile_word(prof[i], i >= MT_ENDQ * 128 ? END_SC_BIAS : FILL_SC_BIAS)
                        : (i - UTAB < 128 ? prof[i] : 0u);
  for (int i = threadIdx.x; i < 32; i += blockDim.x) {
    const uint64_t x = spread_match((uint32_t)i);
    sprof[MLUT + 2 * i] = (uint32_t)x;
    sprof[MLUT + 2 * i + 1] = (uint32_t)(x >> 32);
  }
  __syncthreads();
  uint32_t* ring = rings[threadIdx.x >> 6];
  uint32_t* D = dirpool + (size_t)((blockIdx.x * blockDim.x + threadIdx.x) >> 6) * wave_stride;
  // the kinds of task in the batch (bit e: END = e; k_plan sets bits 1, 2; a
  // segment batch has end gaps only): each kind's bodies are called only when present
  const int ends = (sjw ? 0 : 1) | *end_flag;
  const int lag = (int)(blockIdx.x % GSNAPDP_FILL_WAVES) * stagger;  // fill_tasks: the first batch's shortfall
  int tfirst[NCLASS + 1];  // first task index of each class, then the total
  tfirst[0] = 0;
#pragma unroll
  for (int c = 0; c < NCLASS; c++)
    tfirst[c + 1] = tfirst[c] + (class_start[c + 1] - class_start[c]) / (64 / CLASS_LPW[c]);
  // Small batches: a wave's traceback sweep serves up to TB_BATCH tasks and
  // costs about the same with one task as with four, so a batch with fewer
  // than min_tasks tasks per wave runs on kw < GSNAPDP_FILL_WAVES waves per
  // SIMD.  The grid is GSNAPDP_FILL_WAVES blocks per CU; block b is active when
  // b % GSNAPDP_FILL_WAVES < kw, which leaves every CU kw of its blocks
  // whether the dispatcher places blocks across the CUs first or per CU.
  int kw = GSNAPDP_FILL_WAVES;
  if (min_tasks > 0) {
    const int simds = (int)((gridDim.x * blockDim.x) >> 6) / GSNAPDP_FILL_WAVES;
    kw = (tfirst[NCLASS] + min_tasks * simds - 1) / (min_tasks * simds);
    kw = kw < 1 ? 1 : (kw > GSNAPDP_FILL_WAVES ? GSNAPDP_FILL_WAVES : kw);
  }
  if ((int)(blockIdx.x % GSNAPDP_FILL_WAVES) >= kw) return;  // (no block barrier follows)
  const int gw = ((((int)blockIdx.x / GSNAPDP_FILL_WAVES) * kw + (int)blockIdx.x % GSNAPDP_FILL_WAVES) *
                      (int)blockDim.x + (int)threadIdx.x) >> 6;
  const int nw = ((int)gridDim.x / GSNAPDP_FILL_WAVES * kw * (int)blockDim.x) >> 6;
  // Large batches (more than TB_BATCH tasks per wave): the wave takes global
  // task indices tau = gw, gw + nw, ...; those of class c are its tasks
  // t = first_c + (tau - tfirst[c]), visited class by class, so every wave gets
  // the same mix of classes.  Small batches: the waves are split among the
  // classes in proportion to their task counts weighted by a task's rough cost
  // (S + split_w: S cell updates and the per-column work of a step) and a wave
  // strides over its own class only, so it runs one traceback sweep instead of
  // one per class (at 125k reads two sweeps for three tasks; the split measured
  // 3 % faster there, and 6-9 % slower at 1M with either weight, so large
  // batches keep the mix; GSNAPDP_FILL_SPLIT / _W override for experiments).
  // A class too small for a wave of its own is spread one task per wave.
  const bool split = split_mode < 0 ? tfirst[NCLASS] <= TB_BATCH * nw : split_mode != 0;
  int64_t wcum[NCLASS + 1];
  wcum[0] = 0;
#pragma unroll
  for (int c = 0; c < NCLASS; c++) wcum[c + 1] = wcum[c] + (int64_t)(tfirst[c + 1] - tfirst[c]) * (CLASS_S[c] + split_w);
  static_assert(NCLASS <= 8, "k_fill dispatches at most 8 classes");
#define FILL_BODY(C, E)                                                                          \
  fill_tasks<CLASS_S[C % NCLASS], CLASS_LPW[C % NCLASS], class_low(C % NCLASS), E>(               \
      t0, t1, stride, (const AS_GLOBAL gsnapdp_window*)Wn, (const AS_GLOBAL int*)perm,             \
      (const AS_GLOBAL char*)q, (const AS_GLOBAL char*)qu, (const AS_GLOBAL uint32_t*)blocks,      \
      nwords, (const AS_LDS uint32_t*)sprof, (AS_LDS uint32_t*)ring, (AS_GLOBAL uint32_t*)D,       \
      (AS_GLOBAL gsnapdp_result*)res, (AS_GLOBAL uint32_t*)ops, (const AS_GLOBAL int64_t*)op_off,  \
      (const AS_GLOBAL gsnapdp_sj_window*)sjw, lag);
#define FILL_CLASS(C)                                                                            \
  if constexpr (C < NCLASS) {                                                                    \
    const int lo = tfirst[C], hi = tfirst[C + 1];                                                \
    const int cb = class_start[C] / (64 / CLASS_LPW[C]); /* the class's first task */            \
    int t0 = -1, t1 = 0, stride = nw;                                                            \
    if (!split) {                                                                                \
      const int tau0 = gw >= lo ? gw : gw + (lo - gw + nw - 1) / nw * nw;                        \
      if (tau0 < hi) {                                                                           \
        t0 = cb + tau0 - lo;                                                                     \
        t1 = cb + hi - lo;                                                                       \
      }                                                                                          \
    } else if (hi > lo) {                                                                        \
      const int w0 = (int)(((int64_t)nw * wcum[C] + wcum[NCLASS] - 1) / wcum[NCLASS]);            \
      const int w1 = (int)(((int64_t)nw * wcum[C + 1] + wcum[NCLASS] - 1) / wcum[NCLASS]);        \
      if (w1 > w0) {                                                                             \
        if (gw >= w0 && gw < w1) {                                                               \
          t0 = cb + gw - w0;                                                                     \
          t1 = cb + hi - lo;                                                                     \
          stride = w1 - w0;                                                                      \
        }                                                                                        \
      } else if (gw < hi - lo) {                                                                 \
        t0 = cb + gw;                                                                            \
        t1 = cb + hi - lo;                                                                       \
      }                                                                                          \
    }                                                                                            \
    if (t0 >= 0 && t0 < t1) {                                                                    \
      if (ends & 1) FILL_BODY(C, 0)                                                              \
      if (ends & 2) FILL_BODY(C, 1)                                                              \
      if (ends & 4) FILL_BODY(C, 2)                                                              \
    }                                                                                            \
  }
  FILL_CLASS(0) FILL_CLASS(1) FILL_CLASS(2) FILL_CLASS(3)
  FILL_CLASS(4) FILL_CLASS(5) FILL_CLASS(6) FILL_CLASS(7)
#undef FILL_BODY
#undef FILL_CLASS
#ifdef TB_PROF
  TB_COUNT(6, __builtin_amdgcn_s_memtime() - kt0);  // the wave's whole time
  TB_COUNT(7, 1);
#endif
}

// --------------------------------------------------------------- k_count
// The match / mismatch split of k_fill's tracebacks (k_fill counts every
// diagonal step inside the window's genome in nmismatches, FILL_MATCH = 0).
// One lane per window replays the op stream from the traceback's start cell
// as the host expansion does (gsnapdp_host.cpp replay: DIAG r--, c--; HDASH /
// HGAP c -= n; VSKIP r -= n) and tests each diagonal cell as dynprog.c:2644-2656
// does: '*' columns are skipped, a match is uppercase equality or
// consistent_array.  Then the post-rules of write_result that need the split
// (the end-gap zeroing, dynprog.c:5259-5262 / 5715-5718) and the
// splice-junction ends' score from the counts (:5541 / :6045).
constexpr int COUNT_LANES = 16;                        // k_count: lanes per window
constexpr int COUNT_ROWS = FAST_L2MAX + FAST_WMAX + 16;  // > any k_fill window's length1 (<= L2 + lband)
constexpr int COUNT_COLS = FAST_L2MAX + 16;
__global__ __launch_bounds__(256) void k_count(const gsnapdp_window* __restrict__ Wn, const int* __restrict__ perm,
                                               const int* __restrict__ class_start, const char* __restrict__ q,
                                               const char* __restrict__ qu, const uint32_t* __restrict__ blocks,
                                               uint64_t nwords, const uint32_t* __restrict__ prof,
                                               gsnapdp_result* __restrict__ res, const uint32_t* __restrict__ ops,
                                               const int64_t* __restrict__ op_off,
                                               const gsnapdp_sj_window* __restrict__ sjw) {
  // match bits (bit g: class g of A C G T N) of consistent_array per matrix
  // type and query character, then of uppercase equality per query_uc byte
  __shared__ uint8_t mbits[5 * 128];
  // per window of the block: each row's match bits against the five classes,
  // and each column's genome class
  __shared__ uint8_t mrow[256 / COUNT_LANES][COUNT_ROWS];
  __shared__ uint8_t gcol[256 / COUNT_LANES][COUNT_COLS];
  for (int x = threadIdx.x; x < 5 * 128; x += blockDim.x) mbits[x] = (uint8_t)((prof[x] >> 24) & 31u);
  __syncthreads();
  const int u0 = threadIdx.x % COUNT_LANES;
  const int slot = threadIdx.x / COUNT_LANES;
  const int i = (blockIdx.x * blockDim.x + threadIdx.x) / COUNT_LANES;
  if (i >= class_start[NCLASS]) return;
  const int wi = perm[i];
  if (wi < 0) return;  // (the whole lane group leaves together; no block barrier below)
  gsnapdp_result R = res[wi];
  if (R.status == ST_OPS_OVERFLOW || R.status == ST_INTERNAL) return;
  const gsnapdp_window w = Wn[wi];
  const Lane L = make_lane(w);
  const int L1 = L.d.L1, L2 = L.d.L2;
  if (L1 >= COUNT_ROWS || L2 >= COUNT_COLS) {  // (k_plan never buckets such a window for k_fill)
    if (u0 == 0) res[wi].status = ST_INTERNAL;
    return;
  }
  const uint8_t* mt = mbits + L.d.mt * 128;
  uint8_t* mr = mrow[slot];
  uint8_t* gc = gcol[slot];
  // rows 1..L1: the group's lanes read adjacent query bytes
  // (four rows per lane at a time: their loads are issued together)
  for (int r0 = 1 + u0; r0 <= L1; r0 += 4 * COUNT_LANES) {
    unsigned char qc[4], uc[4];
#pragma unroll
    for (int e = 0; e < 4; e++) {
      const int r = min(r0 + e * COUNT_LANES, L1);
      const int qi = L.qbase + L.qstep * (r - 1);
      qc[e] = qchar(q, qi);
      uc[e] = (unsigned char)qu[qi];
    }
#pragma unroll
    for (int e = 0; e < 4; e++) {
      const int r = r0 + e * COUNT_LANES;
      if (r <= L1) mr[r] = mt[qc[e]] | (uc[e] < 128 ? mbits[4 * 128 + uc[e]] : (uint8_t)0);
    }
  }
  // columns 1..L2: adjacent genome positions (or segment bytes)
  if (sjw) {
    const int sp = (int)sjw[wi].spos - L.gstep;  // column c is q[sp + gstep * c] (every column inside)
    for (int c = 1 + u0; c <= L2; c += COUNT_LANES) gc[c] = (uint8_t)seg_class((unsigned char)q[sp + L.gstep * c]);
  } else {
    ColStream cs;
    cs.init(L);
    for (int c0 = 1 + u0; c0 <= L2; c0 += 4 * COUNT_LANES) {
      int g[4];
#pragma unroll
      for (int e = 0; e < 4; e++) g[e] = cs.cls(blocks, nwords, min(c0 + e * COUNT_LANES, L2));
#pragma unroll
      for (int e = 0; e < 4; e++)
        if (c0 + e * COUNT_LANES <= L2) gc[c0 + e * COUNT_LANES] = (uint8_t)g[e];
    }
  }
  // the other lanes of the group read what these lanes wrote (same wave, LDS in order)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int total = R.nmismatches;
  const uint32_t* o = ops + op_off[wi];
  int r = R.bestr, c = R.bestc, m = 0;
  for (int k = 0; k < R.nops; k++) {
    const uint32_t op = o[k];
    const int cnt = (int)GSNAPDP_OP_COUNT(op);
    const uint32_t ty = GSNAPDP_OP_TYPE(op);
    if (ty == GSNAPDP_OP_DIAG) {
      for (int x = u0; x < cnt; x += COUNT_LANES) {
        const int g = gc[c - x];
        if (g < 5) m += (int)((mr[r - x] >> g) & 1u);  // '*' columns skipped (dynprog.c:2644)
      }
      r -= cnt;
      c -= cnt;
    } else if (ty == GSNAPDP_OP_VSKIP) {
      r -= cnt;
    } else {
      c -= cnt;
    }
  }
#pragma unroll
  for (int x = COUNT_LANES / 2; x > 0; x >>= 1) m += __shfl_xor(m, x, COUNT_LANES);
  if (u0 != 0) return;
  R.nmatches = m;
  R.nmismatches = total - m;
  if (sjw) R.finalscore = m * 3 - 5 * R.nmismatches + R.nopens * L.d.open + R.nindels * L.d.ext;
  if (L.d.mode == 1 && R.nmatches + 1 < R.nmismatches) {
    R.finalscore = 0;
    if (R.status == ST_OK) R.status = ST_ZEROED;
  }
  res[wi] = R;
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

// --------------------------------------------------------------- k_introns
// score_introns (stage3.c:7935-8162) for a batch of paths, one lane per path:
// the lane walks its path's introns in list order, takes the two MaxEnt site
// probabilities of each (the same maxent_prob as k_maxent; 1.0 for a site the
// splicing IIT knows, :7997-8046 / :8069-8116), sums them in that order and
// divides by the intron count, as the reference does in double precision.
// Positions are the reference's unsigned Genomicpos_T arithmetic.
__global__ void k_introns(const gsnapdp_intron_path* __restrict__ P, int npaths,
                          const gsnapdp_intron* __restrict__ I, gsnapdp_intron_scores* __restrict__ out,
                          const uint32_t* __restrict__ blocks, uint64_t nwords, const double* __restrict__ T) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npaths) return;
  const gsnapdp_intron_path x = P[p];
  const uint32_t gl1 = (uint32_t)x.genomiclength - 1u;
  double sd = 0.0, sa = 0.0;
  int nbad = 0, nin = 0;
  for (int k = 0; k < x.nintrons; k++) {
    const gsnapdp_intron t = I[x.first_intron + k];
    int md, ma;        // models of the donor and acceptor sites
    uint32_t pd, pa;   // their splicesitepos
    if (x.cdna_direction == 1) {
      if (x.watsonp) {
        md = GSNAPDP_DONOR, pd = x.chrpos + t.left_genomepos + 1u;
        ma = GSNAPDP_ACCEPTOR, pa = x.chrpos + t.right_genomepos;
      } else {
        md = GSNAPDP_ANTIDONOR, pd = x.chrpos + gl1 - t.left_genomepos;
        ma = GSNAPDP_ANTIACCEPTOR, pa = x.chrpos + gl1 - t.right_genomepos + 1u;
      }
    } else if (x.cdna_direction == -1) {
      if (x.watsonp) {
        ma = GSNAPDP_ANTIACCEPTOR, pa = x.chrpos + t.left_genomepos + 1u;
        md = GSNAPDP_ANTIDONOR, pd = x.chrpos + t.right_genomepos;
      } else {
        ma = GSNAPDP_ACCEPTOR, pa = x.chrpos + gl1 - t.left_genomepos;
        md = GSNAPDP_DONOR, pd = x.chrpos + gl1 - t.right_genomepos + 1u;
      }
    } else {
      continue;  // neither branch of the reference runs: the intron is not counted
    }
    const double d = t.known_donor ? 1.0 : maxent_prob(md, x.chroffset + pd, x.chroffset, blocks, nwords, T);
    const double a = t.known_acceptor ? 1.0 : maxent_prob(ma, x.chroffset + pa, x.chroffset, blocks, nwords, T);
    nin++;
    if (!t.knowngapp && d < 0.9 && a < 0.9) {
      if (x.cdna_direction == 1 && t.comp == '>') nbad = 1;        // FWD_CANONICAL_INTRON_COMP: set (:8048)
      if (x.cdna_direction == -1 && t.comp == '<') nbad += 1;      // REV_CANONICAL_INTRON_COMP: counted (:8119)
    }
    sd = __dadd_rn(sd, d);
    sa = __dadd_rn(sa, a);
  }
  gsnapdp_intron_scores r;
  r.avg_donor_score = nin > 0 ? __ddiv_rn(sd, (double)nin) : sd;
  r.avg_acceptor_score = nin > 0 ? __ddiv_rn(sa, (double)nin) : sa;
  r.nbadintrons = nbad;
  r.nintrons = nin;
  out[p] = r;
}

}  // namespace

// ======================================================================
// Host side: context and the C-ABI of include/gsnapdp.h
// ======================================================================
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <string>
#include <vector>

#include "gsnapdp_ctx.h"

static thread_local std::string g_err;
void gsnapdp__set_err(const std::string& s) { g_err = s; }

// the context's small area: histogram, cursors, class starts, row-lane class
// counts, END flags and tickets (zero between batches)
static constexpr size_t SMALL_WORDS = (size_t)2 * NKEYS + NCLASS + 1 + 1 + 64;

// per-wave k_fill scratch: TB_BATCH regions (see FILL_REGION_DW)
static const size_t WAVE_STRIDE_DW = (size_t)TB_BATCH * FILL_REGION_DW;

extern "C" const char* gsnapdp_last_error(void) { return g_err.c_str(); }

int gsnapdp__lds_fits(const void* fn, size_t dyn, size_t max_lds, const char* name) {
  hipFuncAttributes a;
  HIPCHK(hipFuncGetAttributes(&a, fn));
  if (a.sharedSizeBytes + dyn > max_lds) {
    g_err = std::string(name) + ": " + std::to_string(a.sharedSizeBytes) + " B of static LDS + " +
            std::to_string(dyn) + " B dynamic exceed the " + std::to_string(max_lds) +
            " B a workgroup can hold (the launch would abort the queue)";
    return -1;
  }
  return 0;
}

// this file's kernels (none takes dynamic LDS)
static int kernels_lds_check(size_t max_lds) {
  if (gsnapdp__lds_fits((const void*)&k_plan, 0, max_lds, "k_plan") ||
      gsnapdp__lds_fits((const void*)&k_scatter, 0, max_lds, "k_scatter") ||
      gsnapdp__lds_fits((const void*)&k_fill, 0, max_lds, "k_fill") ||
      gsnapdp__lds_fits((const void*)&k_maxent, 0, max_lds, "k_maxent") ||
      gsnapdp__lds_fits((const void*)&k_introns, 0, max_lds, "k_introns"))
    return -1;
  if constexpr (!FILL_MATCH)
    if (gsnapdp__lds_fits((const void*)&k_count, 0, max_lds, "k_count")) return -1;
  return 0;
}

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
  if (ctx->num_cus * 16 < RW_BIG_WAVES) {  // k_rows' big class runs on 16 waves per CU
    gsnapdp__set_err("gsnapdp needs at least " + std::to_string(RW_BIG_WAVES / 16) + " CUs; device has " +
                     std::to_string(ctx->num_cus));
    delete ctx;
    return nullptr;
  }
  {  // static + dynamic LDS of every kernel against one workgroup's LDS
    int max_lds = 0;
    if ((e = hipDeviceGetAttribute(&max_lds, hipDeviceAttributeMaxSharedMemoryPerBlock, device)) != hipSuccess)
      return fail("max LDS", e);
    if (kernels_lds_check((size_t)max_lds) || gsnapdp__ggap_lds_check((size_t)max_lds) ||
        gsnapdp__gband_lds_check((size_t)max_lds) || gsnapdp__micro_lds_check((size_t)max_lds) ||
        gsnapdp__gather_lds_check((size_t)max_lds) || gsnapdp__gwin_lds_check((size_t)max_lds)) {
      delete ctx;
      return nullptr;
    }
  }
  {
    const char* e = getenv("GSNAPDP_GGAP_ROWLANE");
    ctx->ggap_rowlane_only = (e && e[0] == '1') ? 1 : 0;
    const char* gwe = getenv("GSNAPDP_GWIN");  // 0: probability-mode windows off k_gwin (A/B tests)
    ctx->gwin_on = (gwe && gwe[0] == '0') ? 0 : 1;
    // GSNAPDP_GBAND_PROB=1: probability-mode windows on k_gband too (A/B tests;
    // off by default until it beats k_ggap, DESIGN.md §4 k_gband)
    const char* p = getenv("GSNAPDP_GBAND_PROB");
    ctx->ggap_use_band = ctx->ggap_rowlane_only ? 0 : (1 | ((p && p[0] == '1') ? 2 : 0));  // GB_USE_SCORE | GB_USE_PROB
    // a register-band wave-task (16 windows) takes ~80 us and a row-lane one (2
    // windows) ~37 us, so the band pays only once a batch fills the row-lane
    // waves several times over: smaller batches (the stage-3 pass's rounds) stay
    // on k_ggap (DESIGN.md §4 k_gband)
    const char* m = getenv("GSNAPDP_GBAND_MIN");
    if (m) ctx->gband_min = atoi(m);
    // k_gwin runs a wave-task (64 windows) in ~0.4 ms of latency-bound steps:
    // only batches that fill its waves go there (the stage-3 pass's rounds stay
    // on k_ggap; DESIGN.md §4 k_gwin)
    const char* gm = getenv("GSNAPDP_GWIN_MIN");
    if (gm) ctx->gwin_min = atoi(gm);
    // k_fill on fewer waves per SIMD when a batch gives each wave fewer than
    // this many tasks (0: always GSNAPDP_FILL_WAVES)
    const char* mt = getenv("GSNAPDP_FILL_MIN_TASKS");
    if (mt) ctx->fill_min_tasks = atoi(mt);
    // the first traceback batch of the k-th block of a CU is k * this many tasks short
    const char* sg = getenv("GSNAPDP_FILL_STAGGER");
    if (sg) ctx->fill_stagger = atoi(sg);
    // k_fill's class split: -1 small batches only, 0 never, 1 always; the per-task weight S + w
    const char* sm = getenv("GSNAPDP_FILL_SPLIT");
    if (sm) ctx->fill_split = atoi(sm);
    const char* sw = getenv("GSNAPDP_FILL_SPLIT_W");
    if (sw) ctx->fill_split_w = atoi(sw);
    const char* f = getenv("GSNAPDP_ENDS_ROWLANE");
    ctx->ends_rowlane = (f && f[0] == '1') ? 1 : 0;
  }
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
  if ((e = hipMalloc(&ctx->d_small, SMALL_WORDS * 4)) != hipSuccess) return fail("malloc small", e);
  if ((e = hipMemset(ctx->d_small, 0, SMALL_WORDS * 4)) != hipSuccess) return fail("memset small", e);

  ctx->dirpool_waves = (size_t)ctx->fill_waves;
  if ((e = hipMalloc(&ctx->d_dirpool, ctx->dirpool_waves * WAVE_STRIDE_DW * 4)) != hipSuccess)
    return fail("malloc dirpool", e);
  return ctx;
}

extern "C" void gsnapdp_destroy(gsnapdp_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  gsnapdp__s3_pool_free(ctx);
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
  (void)hipFree(ctx->d_gband_pool);
  (void)hipFree(ctx->d_gband_pool_prob);
  (void)hipFree(ctx->d_gwin_pool);
  (void)hipFree(ctx->d_gwin_probs);
  (void)hipFree(ctx->d_ggap_stage);
  (void)hipFree(ctx->d_sj_win);
  (void)hipFree(ctx->d_stage);
  (void)hipFree(ctx->d_csum);
  (void)hipFree(ctx->d_si_stage);
  if (ctx->h_small) (void)hipHostFree(ctx->h_small);
  if (ctx->h_in) (void)hipHostFree(ctx->h_in);
  if (ctx->h_mx) (void)hipHostFree(ctx->h_mx);
  (void)hipFree(ctx->d_mx_stage);
  if (ctx->compact_done) (void)hipEventDestroy(ctx->compact_done);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

extern "C" const char* gsnapdp_device_arch(gsnapdp_ctx* ctx) { return ctx ? ctx->arch.c_str() : ""; }

extern "C" int64_t gsnapdp_debug_buckets(gsnapdp_ctx* ctx, int n, int32_t* keys, int32_t* perm,
                                         int64_t perm_cap, int32_t* class_start, int32_t* class_wave,
                                         int ncls) {
  if (!ctx) return -1;
  if (!keys && !perm && !class_start && !class_wave) return NCLASS;
  if (ncls != NCLASS || n < 0 || n > ctx->cap_n) {
    g_err = "gsnapdp_debug_buckets: ncls must be " + std::to_string(NCLASS) + " and n at most the last batch";
    return -1;
  }
  std::lock_guard<std::mutex> lock(ctx->mu);
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  int32_t cs[NCLASS + 1];
  const int* class_start_d = ctx->d_small + 2 * NKEYS;  // after hist and cursor (gsnapdp__fill_pipeline)
  HIPCHK(hipMemcpy(cs, class_start_d, sizeof(cs), hipMemcpyDeviceToHost));
  const int64_t nperm = cs[NCLASS];
  if (class_start) memcpy(class_start, cs, sizeof(cs));
  if (class_wave)
    for (int c = 0; c < NCLASS; c++) class_wave[c] = 64 / CLASS_LPW[c];
  if (keys && n) HIPCHK(hipMemcpy(keys, ctx->d_keys, (size_t)n * 4, hipMemcpyDeviceToHost));
  if (perm && nperm > 0)
    HIPCHK(hipMemcpy(perm, ctx->d_perm, (size_t)std::min(nperm, perm_cap) * 4, hipMemcpyDeviceToHost));
  return nperm;
}

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

// The single/end-gap pipeline over windows already on the device: plan, bucket,
// k_fill, then k_rows for the windows the register band does not take.  sjw:
// the splice-junction records the windows were derived from (segment genome),
// or nullptr.  The caller holds ctx->mu.
int gsnapdp__fill_pipeline(gsnapdp_ctx* ctx, hipStream_t st, const gsnapdp_window* d_windows, int n,
                           const char* d_query, const char* d_query_uc, gsnapdp_result* d_results,
                           uint32_t* d_ops, const int64_t* d_op_offsets, const gsnapdp_sj_window* sjw) {
  if (n >= (1 << SCAN_PAD_SHIFT)) {  // a bucket count must fit scan_buckets' stage word
    g_err = "batch of " + std::to_string(n) + " windows: at most 2^26 - 1 per call";
    return -1;
  }
  if (ensure_capacity(ctx, n)) return -1;
  int* hist = ctx->d_small;
  int* cursor = hist + NKEYS;
  int* class_start = cursor + NKEYS;
  int* big_count = class_start + NCLASS + 1;  // RW_NCLS row-lane class counts
  // (the class counts and END flags start at zero: the context clears them once
  // and k_rows' last block after every batch)
  static_assert(ROWS_TICKET < 64, "tickets inside the context's small area");
  if (gsnapdp__rows_pools(ctx)) return -1;
  constexpr int tb = 1024;
  const int nb = (n + tb - 1) / tb;
  auto mark = [&](int stage, int end) { gsnapdp__mark(ctx, st, stage, end); };
  mark(0, 0);
  static_assert(tb == 1024, "k_plan's last block runs scan_buckets with 1024 threads");
  hipLaunchKernelGGL(k_plan, dim3(nb), dim3(tb), 0, st, d_windows, n, d_query, d_query_uc,
                     ctx->d_blocks, (uint64_t)ctx->nwords, ctx->d_prof, d_results, d_ops,
                     d_op_offsets, ctx->d_keys, hist, ctx->d_big_list, big_count,
                     ctx->cap_n, ctx->ends_rowlane ? 0 : 1, cursor, class_start, ctx->d_perm,
                     big_count + PLAN_TICKET);
  mark(0, 1);
  mark(1, 0);
  hipLaunchKernelGGL(k_scatter, dim3(nb), dim3(tb), 0, st, ctx->d_keys, n, cursor, ctx->d_perm);
  mark(1, 1);
  const int blocks = (int)(ctx->dirpool_waves / 4);
  const uint64_t nw = (uint64_t)ctx->nwords;
  // (k_fill keeps every CU busy, so k_rows runs after it on the same stream: a
  // side stream measured slower)
  mark(2, 0);
  hipLaunchKernelGGL(k_fill, dim3(blocks), dim3(256), 0, st, d_windows, ctx->d_perm, class_start,
                     d_query, d_query_uc, ctx->d_blocks, nw, ctx->d_prof, ctx->d_dirpool,
                     WAVE_STRIDE_DW, d_results, d_ops, d_op_offsets, big_count + RW_NCLS, sjw,
                     ctx->fill_min_tasks, ctx->fill_stagger, ctx->fill_split, ctx->fill_split_w);
  mark(2, 1);
  if constexpr (!FILL_MATCH) {
    mark(7, 0);
    // perm holds at most 64 entries per window (a bucket pads to whole waves)
    const size_t nperm = std::min(ctx->perm_cap, (size_t)n * 64);
    const size_t per_block = 256 / COUNT_LANES;
    hipLaunchKernelGGL(k_count, dim3((unsigned)((nperm + per_block - 1) / per_block)), dim3(256), 0, st, d_windows, ctx->d_perm, class_start, d_query,
                       d_query_uc, ctx->d_blocks, nw, ctx->d_prof, d_results, d_ops, d_op_offsets, sjw);
    mark(7, 1);
  }
#ifdef TB_PROF
  {
    unsigned long long h[8];
    HIPCHK(hipStreamSynchronize(st));
    HIPCHK(hipMemcpyFromSymbol(h, HIP_SYMBOL(tb_prof), sizeof(h)));
    fprintf(stderr, "tb_prof sweeps %llu groups %llu slow %llu lanecols %llu fill_cyc %llu trace_cyc %llu wave_cyc %llu waves %llu\n",
            h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7]);
    memset(h, 0, sizeof(h));
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(tb_prof), h, sizeof(h)));
  }
#endif
  mark(3, 0);
  // A batch that stops between k_plan and the end of k_rows would leave the
  // histogram, row-lane counts, END flags or tickets set (only the last blocks
  // of k_plan / k_rows clear them): put the whole small area back to its
  // allocation state so the next batch starts clean.
  auto recover = [&]() {
    (void)hipGetLastError();
    (void)hipMemsetAsync(ctx->d_small, 0, SMALL_WORDS * 4, st);
    return -1;
  };
  if (gsnapdp__rows_launch(ctx, st, d_windows, ctx->d_big_list, big_count, ctx->cap_n, d_query,
                           d_query_uc, d_results, d_ops, d_op_offsets, sjw))
    return recover();
  mark(3, 1);
  if (hipError_t e = hipGetLastError(); e != hipSuccess) {
    g_err = std::string("single/end-gap pipeline launch: ") + hipGetErrorString(e);
    return recover();
  }
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
  return gsnapdp__fill_pipeline(ctx, st, d_windows, n, d_query, d_query_uc, d_results, d_ops,
                                d_op_offsets, nullptr);
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
                                          "k_ggap_plan", "k_ggap", "k_gband", "k_count", "k_gwin"};
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

extern "C" int gsnapdp_score_introns_device(gsnapdp_ctx* ctx, const gsnapdp_intron_path* d_paths, int npaths,
                                            const gsnapdp_intron* d_introns, gsnapdp_intron_scores* d_out,
                                            void* stream_v) {
  if (!ctx || !ctx->d_tables) {
    gsnapdp__set_err("maxent tables not loaded");
    return -1;
  }
  if (npaths <= 0) return 0;
  hipStream_t st = stream_v ? (hipStream_t)stream_v : ctx->stream;
  hipLaunchKernelGGL(k_introns, dim3((npaths + 255) / 256), dim3(256), 0, st, d_paths, npaths, d_introns,
                     d_out, ctx->d_blocks, (uint64_t)ctx->nwords, ctx->d_tables);
  HIPCHK(hipGetLastError());
  return 0;
}

extern "C" int gsnapdp_score_introns_host(gsnapdp_ctx* ctx, const gsnapdp_intron_path* paths, int npaths,
                                          const gsnapdp_intron* introns, int nintrons,
                                          gsnapdp_intron_scores* out) {
  if (!ctx) return -1;
  if (npaths <= 0) return 0;
  for (int p = 0; p < npaths; p++)  // the kernel trusts the ranges: check them here
    if (paths[p].nintrons < 0 || paths[p].first_intron < 0 ||
        (int64_t)paths[p].first_intron + paths[p].nintrons > (int64_t)nintrons) {
      gsnapdp__set_err("score_introns: a path's introns lie outside the intron array");
      return -1;
    }
  HIPCHK(hipSetDevice(ctx->device));
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t szp = al((size_t)npaths * sizeof(gsnapdp_intron_path));
  const size_t szi = al((size_t)(nintrons > 0 ? nintrons : 1) * sizeof(gsnapdp_intron));
  const size_t szo = (size_t)npaths * sizeof(gsnapdp_intron_scores);
  std::lock_guard<std::mutex> host_lock(ctx->host_mu);
  {
    std::lock_guard<std::mutex> lock(ctx->mu);
    if (szp + szi + szo > ctx->si_cap) {
      (void)hipFree(ctx->d_si_stage);
      ctx->d_si_stage = nullptr;
      const size_t cap = szp + szi + szo + (szp + szi + szo) / 2 + 4096;
      HIPCHK(hipMalloc(&ctx->d_si_stage, cap));
      ctx->si_cap = cap;
    }
  }
  char* d = ctx->d_si_stage;
  hipStream_t st = ctx->stream;
  HIPCHK(hipMemcpyAsync(d, paths, (size_t)npaths * sizeof(gsnapdp_intron_path), hipMemcpyHostToDevice, st));
  if (nintrons > 0)
    HIPCHK(hipMemcpyAsync(d + szp, introns, (size_t)nintrons * sizeof(gsnapdp_intron), hipMemcpyHostToDevice, st));
  int rc = gsnapdp_score_introns_device(ctx, (const gsnapdp_intron_path*)d, npaths,
                                        (const gsnapdp_intron*)(d + szp),
                                        (gsnapdp_intron_scores*)(d + szp + szi), st);
  if (rc == 0) {
    HIPCHK(hipMemcpyAsync(out, d + szp + szi, szo, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
  }
  return rc;
}
