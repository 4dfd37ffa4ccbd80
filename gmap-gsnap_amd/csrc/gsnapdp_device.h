// gsnapdp_device.h -- device code shared by the single-gap kernels
// (gsnapdp_kernels.hip) and the genome-gap kernels (gsnapdp_ggap.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gsnapdp_internal.h"

namespace gsnapdp {

// ------------------------------------------------------------ per-lane view
struct Lane {
  Derived d;
  int qbase, qstep;   // query index of row r: qbase + qstep*(r-1)
  int g0, gstep;      // genomicpos of column c: g0 + gstep*(c-1)
  uint32_t base;      // chroffset + chrpos (uint32 wrap, like the reference)
  int glen;
  int watson;
  int allstar;        // chroffset+chrpos overflow or >= chrhigh (dynprog.c:415-419)
  int off1, off2;     // pair coordinate offsets
  int cdna_direction;
};

__device__ inline Lane make_lane(const gsnapdp_window& w) {
  Lane L;
  L.d = derive(w);
  L.qbase = (int)w.qpos;
  L.qstep = L.d.rev ? -1 : 1;
  L.g0 = w.offset2;
  L.gstep = L.d.rev ? -1 : 1;
  L.base = w.chroffset + w.chrpos;
  L.glen = (int)w.genomiclength;
  L.watson = w.watsonp ? 1 : 0;
  L.allstar = (L.base < w.chroffset) || (L.base >= w.chrhigh);
  L.off1 = w.offset1;
  L.off2 = w.offset2;
  L.cdna_direction = w.cdna_direction;
  return L;
}

// get_genomic_nt (dynprog.c:403-441) on the packed blocks (uncompress_one_char,
// genome.c:9325): class code 0..5 = A C G T N '*'.
__device__ inline int gclass(const uint32_t* __restrict__ blocks, uint64_t nwords, const Lane& L,
                             int gpos) {
  if (gpos < 0 || gpos >= L.glen || L.allstar) return 5;
  const uint32_t pos = L.watson ? (L.base + (uint32_t)gpos)
                                : (L.base + (uint32_t)(L.glen - 1) - (uint32_t)gpos);
  const uint64_t ptr = (uint64_t)(pos >> 5) * 3u;
  if (ptr + 2 >= nwords) return 4;  // outside the genome (outside the reference's domain)
  const uint32_t bit = pos & 31u;
  const uint32_t fl = blocks[ptr + 2];
  if ((fl >> bit) & 1u) return 4;
  const uint32_t word = bit < 16 ? blocks[ptr + 1] : blocks[ptr];
  const int code = (int)((word >> ((bit & 15u) * 2u)) & 3u);
  return L.watson ? code : 3 - code;
}

// Class of a genomic-segment byte (use_genomicseg_p): A C G T N -> 0..4, else 6
// (outside the domain: the segments of Dynprog_make_splicejunction_5/3 are ACGTN).
__device__ inline int seg_class(unsigned char a) {
  return a == 'A' ? 0 : a == 'C' ? 1 : a == 'G' ? 2 : a == 'T' ? 3 : a == 'N' ? 4 : 6;
}

// A wave's global stores made visible to its own other lanes: a workgroup-scope
// fence, which waits for the stores (the CU's vector L1 stays coherent with
// its own stores).  An agent-scope __threadfence() also writes back the XCD's
// whole L2 (buffer_wbl2 sc1) on gfx950: measured at ~0.4 ms per k_gband task.
__device__ inline void wave_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); }

__device__ inline int wave_max(int x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = max(x, __shfl_xor(x, o));
  return x;
}

__device__ inline unsigned char qchar(const char* __restrict__ q, int idx) {
  return (unsigned char)q[idx] & 127u;
}

// --------------------------------------------------------------- op writer
struct OpWriter {
  uint32_t* out;
  int cap, n;
  int run;  // pending DIAG steps
  __device__ inline void put(uint32_t op) {
    if (n < cap) out[n] = op;
    n++;
  }
  __device__ inline void flush() {
    if (run > 0) put(GSNAPDP_OP(GSNAPDP_OP_DIAG, run));
    run = 0;
  }
};

// Counts of one traceback
struct Tally {
  int nmatches, nmismatches, nopens, nindels;
  int npush;  // pairs the reference pushes (gapholders included)
};

// The match mask of a query row: bit g set when a diagonal step against genome
// class g (A C G T N) counts as a match -- the uppercase bytes are equal or
// consistent_array holds (dynprog.c:2650-2656).  prof rows as build_profile_table.
__device__ inline uint32_t row_match_mask(const uint32_t* __restrict__ prof, int mt, unsigned char c1,
                                          unsigned char u1) {
  const uint32_t a = prof[mt * 128 + (c1 & 127u)];
  const uint32_t b = u1 < 128 ? prof[4 * 128 + u1] : 0u;
  return ((a | b) >> 24) & 31u;
}

// Direction nibble: bit0 gap1==HORIZ, bit1 gap2==VERT, bit2 nogap HORIZ, bit3 nogap VERT.
// `dirs(r, c)` returns the nibble of an in-band cell with r >= 1, c >= 1.
//
// traceback (dynprog.c:2611-2712) with the reference's memset semantics for
// cells outside the band and the row-0 / column-0 initialisation
// (dynprog.c:1460-1488).
//
// `colcls(c)` is the genome class (0..5 = A C G T N *) of column c in 1..L2;
// `qmask(r)` is row r's match mask (row_match_mask).  Runs of diagonal steps
// are taken four cells at a time: the cells (r-k, c-k), k = 0..3, share the
// diagonal, so they are in the band when r, c >= 4, and their eight loads are
// independent.
// `score` (optional) is told every step of the path: diag(r, c) for a nogap
// cell and gap(dist) for a gap of dist cells, so a caller can total the path's
// score (the DP value of the start cell: every path ends at (0, 0) with 0).
struct NoScore {
  __device__ inline void diag(int, int) const {}
  __device__ inline void gap(int) const {}
};
template <class Dirs, class Col, class QMask, class Score = NoScore>
__device__ inline void traceback(const Dirs& dirs, const Lane& L, int r, int c, const QMask& qmask,
                                 const Col& colcls, Tally& t, OpWriter& ow, Score&& score = Score()) {
  const int lband = L.d.lband, rband = L.d.rband;
  auto inband = [&](int rr, int cc) {
    const int d = rr - cc + rband;
    return rr >= 1 && cc >= 1 && d >= 0 && d <= lband + rband;
  };
  auto gap1_horiz = [&](int rr, int cc) -> bool {
    if (rr == 0) return cc >= 2 && cc <= rband && cc <= L.d.L2;
    if (!inband(rr, cc)) return false;
    return dirs(rr, cc) & 1u;
  };
  auto gap2_vert = [&](int rr, int cc) -> bool {
    if (cc == 0) return rr >= 2 && rr <= lband && rr <= L.d.L1;
    if (!inband(rr, cc)) return false;
    return (dirs(rr, cc) >> 1) & 1u;
  };
  auto count = [&](int rr, int cc) {  // the nogap cell (rr, cc): one pair unless the genome is '*'
    score.diag(rr, cc);
    const int g = colcls(cc);
    if (g != 5) {
      const int m = (int)((qmask(rr) >> g) & 1u);
      t.nmatches += m;
      t.nmismatches += 1 - m;
      t.npush++;
    }
  };
  while (inband(r, c)) {
    uint32_t nib;
    if (r >= 4 && c >= 4) {
      const uint32_t n0 = dirs(r, c), n1 = dirs(r - 1, c - 1), n2 = dirs(r - 2, c - 2), n3 = dirs(r - 3, c - 3);
      if (((n0 | n1 | n2 | n3) & 12u) == 0u) {
        count(r, c);
        count(r - 1, c - 1);
        count(r - 2, c - 2);
        count(r - 3, c - 3);
        ow.run += 4;
        r -= 4;
        c -= 4;
        continue;
      }
      nib = n0;
    } else {
      nib = dirs(r, c);
    }
    count(r, c);
    ow.run++;
    if (nib & 8u) {  // VERT: query skip (add_queryskip, dynprog.c:2372)
      int dist = 1;
      r--;
      c--;
      while (gap2_vert(r, c)) {
        dist++;
        r--;
      }
      r--;
      score.gap(dist);
      ow.flush();
      ow.put(GSNAPDP_OP(GSNAPDP_OP_VSKIP, dist));
      t.npush += dist;
      t.nopens++;
      t.nindels += dist;
    } else if (nib & 4u) {  // HORIZ: genome skip (add_genomeskip, dynprog.c:2416)
      int dist = 1;
      r--;
      c--;
      while (gap1_horiz(r, c)) {
        dist++;
        c--;
      }
      c--;
      bool dashes = true;
      if (dist >= MICROINTRON_LENGTH) {
        // columns c+1 .. c+dist are skipped; left = column c+1, right = column c+dist.
        // In window-coordinate order (leftgenomecoord < rightgenomecoord) the
        // dinucleotides sit at the skip's two ends; a reversed fill runs the
        // columns backwards along the genome.
        const int cl = c + 1, cr = c + dist;
        const int rv = L.d.rev;
        const int l1 = colcls(rv ? cr : cl), l2 = colcls(rv ? cr - 1 : cl + 1);
        const int r2 = colcls(rv ? cl + 1 : cr - 1), r1 = colcls(rv ? cl : cr);
        dashes = intron_type_codes(l1, l2, r2, r1, L.cdna_direction) == 0;
      }
      score.gap(dist);
      ow.flush();
      ow.put(GSNAPDP_OP(dashes ? GSNAPDP_OP_HDASH : GSNAPDP_OP_HGAP, dist));
      t.npush += dashes ? dist : 1;
      if (dashes) {
        t.nopens++;
        t.nindels += dist;
      }
    } else {
      r--;
      c--;
    }
  }
  ow.flush();
}

// Wave-aggregated "pos = atomicAdd(&counter[key], 1)" for lanes with key >= 0
// (most lanes of a wave share a key, so one atomic per distinct key per wave).
// Every lane of the wave must call it.
__device__ inline int agg_atomic_inc(int* counter, int key) {
  const int lane = threadIdx.x & 63;
  int pos = -1;
  uint64_t todo = __ballot(key >= 0);
  while (todo) {
    const int leader = __ffsll((unsigned long long)todo) - 1;
    const int lkey = __shfl(key, leader);
    const uint64_t m = __ballot(key == lkey) & todo;
    int base = 0;
    if (lane == leader) base = atomicAdd(&counter[lkey], __popcll(m));
    base = __shfl(base, leader);
    if (key == lkey) pos = base + __popcll(m & ((1ull << lane) - 1ull));
    todo &= ~m;
  }
  return pos;
}

// Final bookkeeping shared by all paths.
__device__ inline void write_result(gsnapdp_result* res, const gsnapdp_window& w, const Lane& L,
                                    int score, int bestr, int bestc, const Tally& t,
                                    const OpWriter& ow, bool post = true) {
  gsnapdp_result R;
  R.finalscore = score;
  R.nmatches = t.nmatches;
  R.nmismatches = t.nmismatches;
  R.nopens = t.nopens;
  R.nindels = t.nindels;
  R.bestr = bestr;
  R.bestc = bestc;
  R.nops = ow.n < ow.cap ? ow.n : ow.cap;
  R.status = ow.n > ow.cap ? ST_OPS_OVERFLOW : ST_OK;
  R.length1 = L.d.L1;
  R.length2 = L.d.L2;
  R.reserved = step_dpi(w.dynprogindex);
  // (post = false: k_fill's tracebacks; k_count applies the rules below once it
  // has split the diagonal steps into matches and mismatches)
  // end gaps, QUERYEND_GAP / BEST_LOCAL: dynprog.c:5259-5262 / 5715-5718
  if (post && L.d.mode == 1 && t.nmatches + 1 < t.nmismatches) {
    R.finalscore = 0;
    if (R.status == ST_OK) R.status = ST_ZEROED;
  }
  // QUERYEND_NOGAPS rescoring: dynprog.c:5243 / 5700
  if (L.d.mode == 3) R.finalscore = t.nmatches * 3 + t.nmismatches * (-5);
  *res = R;
}

// ------------------------------------------------- row-lane window classes
// Windows the register-band kernel does not take (end gaps, wide or long
// single gaps) run on the row-lane kernel k_rows (gsnapdp_ggap.hip): rows on
// lanes, band cells (H << 4 | dirs) in LDS, or in global scratch when large.
enum { RW_SMALL = 0, RW_MID = 1, RW_LARGE = 2, RW_BIG = 3, RW_TINY = 4, RW_NCLS = 5 };
constexpr int RW_TINY_WORDS = 640;               // LDS words per window, 16-row groups (4 per wave)
constexpr int RW_SMALL_WORDS = 1280;             // LDS words per window, 32-row groups
constexpr int RW_MID_WORDS = 4096;               // LDS words per window, 64-row stripes
constexpr int RW_LARGE_WORDS = 16384;            // global words per wave (64 KB)
constexpr int RW_LARGE_WAVES_PER_CU = 16;        // enough waves to cover the latency of global scratch
constexpr size_t RW_BIG_WORDS = (size_t)2 << 20; // global words per wave
constexpr int RW_BIG_WAVES = 128;
// after the row-lane class counts and k_fill's END flags (RW_NCLS + 1 words):
// k_plan's and k_rows' last-block tickets (the context's small area, zeroed once)
constexpr int PLAN_TICKET = RW_NCLS + 2, ROWS_TICKET = RW_NCLS + 3;

// storage of one window: band cells, column classes (bytes), query (u16 per
// row) and, for more than one 64-row stripe, the boundary row (3 words per column)
__host__ __device__ inline size_t rows_words(int L1, int L2, int W) {
  const size_t stripes = ((size_t)L1 + 1 + 63) / 64;
  return (size_t)L1 * W + ((size_t)L2 + 2 + 3) / 4 + ((size_t)L1 + 1) / 2 +
         (stripes > 1 ? 3 * ((size_t)L2 + 2) : 0);
}
__host__ __device__ inline int rows_class(int L1, int L2, int W) {
  const size_t words = rows_words(L1, L2, W);
  if (L1 + 1 <= 16 && words <= (size_t)RW_TINY_WORDS) return RW_TINY;
  if (L1 + 1 <= 32 && words <= (size_t)RW_SMALL_WORDS) return RW_SMALL;
  if (words <= (size_t)RW_MID_WORDS) return RW_MID;
  if (words <= (size_t)RW_LARGE_WORDS) return RW_LARGE;
  if (words <= RW_BIG_WORDS) return RW_BIG;
  return -1;
}

// ---------------------------------------------------------------- maxent
// Maxent_hr_{donor,acceptor,antidonor,antiacceptor}_prob (maxent_hr.c:27217-27390).
// The reference's 32 shift-specialised handlers all read a k-mer `off` nt past
// startpos from the 128-bit window (low, high, nextlow, nexthigh).
__device__ inline uint32_t kmer_at(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, int bit) {
  // bits [bit, bit+32) of the little-endian 128-bit value w0 | w1<<32 | w2<<64 | w3<<96
  const uint32_t w[5] = {w0, w1, w2, w3, 0u};
  const int i = bit >> 5, sh = bit & 31;
  return sh == 0 ? w[i] : ((w[i] >> sh) | (w[i + 1] << (32 - sh)));
}

// model m: 0 donor, 1 acceptor, 2 antidonor, 3 antiacceptor; T = the 16 tables
// in the order of DESIGN.md (gsnapdp_load_maxent_tables).
__device__ inline double maxent_prob(int m, uint32_t sp, uint32_t co,
                                     const uint32_t* __restrict__ blocks, uint64_t nwords,
                                     const double* __restrict__ T) {
  // table offsets (declaration order of maxent_hr.c:25-22606)
  const double* donor_p = T;
  const double* donor_di_p = donor_p + 16384;
  const double* acc1_p = donor_di_p + 16;
  const double* acc2_p = acc1_p + 16384;
  const double* acc3_p = acc2_p + 16384;
  const double* accdi_p = acc3_p + 16384;
  const double* acc467_p = accdi_p + 16;
  const double* acc589_p = acc467_p + 16384;
  const double* donor_m = acc589_p + 16384;
  const double* donor_di_m = donor_m + 16384;
  const double* acc1_m = donor_di_m + 16;
  const double* acc2_m = acc1_m + 16384;
  const double* acc3_m = acc2_m + 16384;
  const double* accdi_m = acc3_m + 16384;
  const double* acc467_m = accdi_m + 16;
  const double* acc589_m = acc467_m + 16384;
  const uint32_t margin = (m == 0) ? 3u : (m == 1) ? 20u : (m == 2) ? 6u : 3u;
  if (sp < co + margin) return 0.0;
  const uint32_t start = sp - margin;
  const uint64_t ptr = (uint64_t)(start >> 5) * 3u;
  if (ptr + 4 >= nwords) return 0.0;  // outside the genome: outside the reference's domain
  const uint32_t high = blocks[ptr], low = blocks[ptr + 1];
  const uint32_t nexthigh = blocks[ptr + 3], nextlow = blocks[ptr + 4];
  const int b0 = 2 * (int)(start & 31u);
  auto seq = [&](int off) { return kmer_at(low, high, nextlow, nexthigh, b0 + 2 * off); };
  double odds;
  if (m == 0) {
    const uint32_t s = seq(0);
    odds = donor_p[(s & 0x3Fu) | ((s >> 4) & 0x3FC0u)] * donor_di_p[(s >> 6) & 0xFu];
  } else if (m == 2) {
    const uint32_t s = seq(0);
    odds = donor_m[(s & 0xFFu) | ((s >> 4) & 0x3F00u)] * donor_di_m[(s >> 8) & 0xFu];
  } else if (m == 1) {
    odds = acc1_p[seq(0) & 0x3FFFu];
    odds = __dmul_rn(odds, acc2_p[seq(7) & 0x3FFFu]);
    const uint32_t s = seq(14);
    odds = __dmul_rn(odds, acc3_p[(s & 0xFFu) | ((s >> 4) & 0x3F00u)]);
    odds = __dmul_rn(odds, accdi_p[(s >> 8) & 0xFu]);
    odds = __dmul_rn(odds, acc467_p[seq(4) & 0x3FFFu]);
    odds = __dmul_rn(odds, acc589_p[seq(11) & 0x3FFFu]);
  } else {
    odds = acc1_m[seq(16) & 0x3FFFu];
    odds = __dmul_rn(odds, acc2_m[seq(9) & 0x3FFFu]);
    const uint32_t s = seq(0);
    odds = __dmul_rn(odds, acc3_m[(s & 0x3Fu) | ((s >> 4) & 0x3FC0u)]);
    odds = __dmul_rn(odds, accdi_m[(s >> 6) & 0xFu]);
    odds = __dmul_rn(odds, acc467_m[seq(12) & 0x3FFFu]);
    odds = __dmul_rn(odds, acc589_m[seq(5) & 0x3FFFu]);
  }
  return __ddiv_rn(odds, __dadd_rn(1.0, odds));
}


// maxent_prob for N sites of one model at once, for latency: every site's
// genome words are loaded before any table index is formed, and every table
// load before the products (the same operations in the same order per site,
// so the values are bit-identical).  ok[i] false: out[i] = 0.0.
__device__ inline uint32_t kmer_sel(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, int bit) {
  const int i = bit >> 5;  // kmer_at without a register array (no indexed private access)
  const uint32_t lo = i == 0 ? w0 : i == 1 ? w1 : i == 2 ? w2 : w3;
  const uint32_t hi = i == 0 ? w1 : i == 1 ? w2 : i == 2 ? w3 : 0u;
  return __builtin_amdgcn_alignbit(hi, lo, (uint32_t)(bit & 31));
}
template <int N, class Seq>
__device__ inline void maxent_probs_of(int m, Seq&& seq, const bool (&v)[N], const double* __restrict__ T,
                                       double (&out)[N]);
template <int N>
__device__ inline void maxent_probs(int m, const uint32_t (&sp)[N], const bool (&ok)[N], uint32_t co,
                                    const uint32_t* __restrict__ blocks, uint64_t nwords,
                                    const double* __restrict__ T, double (&out)[N]) {
  const uint32_t margin = (m == 0) ? 3u : (m == 1) ? 20u : (m == 2) ? 6u : 3u;
  uint32_t w0[N], w1[N], w2[N], w3[N];
  int b0[N];
  bool v[N];
#pragma unroll
  for (int i = 0; i < N; i++) {
    const uint32_t start = sp[i] - margin;
    const uint64_t ptr = (uint64_t)(start >> 5) * 3u;
    v[i] = ok[i] && sp[i] >= co + margin && ptr + 4 < nwords;
    const uint64_t p = v[i] ? ptr : 0;
    w1[i] = blocks[p];  // high
    w0[i] = blocks[p + 1];  // low
    w3[i] = blocks[p + 3];  // nexthigh
    w2[i] = blocks[p + 4];  // nextlow
    b0[i] = 2 * (int)(start & 31u);
  }
  auto seq = [&](int i, int off) { return kmer_sel(w0[i], w1[i], w2[i], w3[i], b0[i] + 2 * off); };
  maxent_probs_of<N>(m, seq, v, T, out);
}

// the table part of maxent_probs: seq(i, off) = the 16-mer `off` nt past site
// i's start (startpos - margin); v[i] false: out[i] = 0.0
template <int N, class Seq>
__device__ inline void maxent_probs_of(int m, Seq&& seq, const bool (&v)[N], const double* __restrict__ T,
                                       double (&out)[N]) {
  const double* donor_p = T;
  const double* donor_di_p = donor_p + 16384;
  const double* acc1_p = donor_di_p + 16;
  const double* acc2_p = acc1_p + 16384;
  const double* acc3_p = acc2_p + 16384;
  const double* accdi_p = acc3_p + 16384;
  const double* acc467_p = accdi_p + 16;
  const double* acc589_p = acc467_p + 16384;
  const double* donor_m = acc589_p + 16384;
  const double* donor_di_m = donor_m + 16384;
  const double* acc1_m = donor_di_m + 16;
  const double* acc2_m = acc1_m + 16384;
  const double* acc3_m = acc2_m + 16384;
  const double* accdi_m = acc3_m + 16384;
  const double* acc467_m = accdi_m + 16;
  const double* acc589_m = acc467_m + 16384;
  double odds[N];
  if (m == 0 || m == 2) {
    double a[N], b[N];
#pragma unroll
    for (int i = 0; i < N; i++) {
      const uint32_t s = seq(i, 0);
      a[i] = m == 0 ? donor_p[(s & 0x3Fu) | ((s >> 4) & 0x3FC0u)] : donor_m[(s & 0xFFu) | ((s >> 4) & 0x3F00u)];
      b[i] = m == 0 ? donor_di_p[(s >> 6) & 0xFu] : donor_di_m[(s >> 8) & 0xFu];
    }
#pragma unroll
    for (int i = 0; i < N; i++) odds[i] = a[i] * b[i];
  } else {
    double a[N], b[N], c[N], d[N], e[N], f[N];
#pragma unroll
    for (int i = 0; i < N; i++) {
      if (m == 1) {
        const uint32_t s = seq(i, 14);
        a[i] = acc1_p[seq(i, 0) & 0x3FFFu];
        b[i] = acc2_p[seq(i, 7) & 0x3FFFu];
        c[i] = acc3_p[(s & 0xFFu) | ((s >> 4) & 0x3F00u)];
        d[i] = accdi_p[(s >> 8) & 0xFu];
        e[i] = acc467_p[seq(i, 4) & 0x3FFFu];
        f[i] = acc589_p[seq(i, 11) & 0x3FFFu];
      } else {
        const uint32_t s = seq(i, 0);
        a[i] = acc1_m[seq(i, 16) & 0x3FFFu];
        b[i] = acc2_m[seq(i, 9) & 0x3FFFu];
        c[i] = acc3_m[(s & 0x3Fu) | ((s >> 4) & 0x3FC0u)];
        d[i] = accdi_m[(s >> 6) & 0xFu];
        e[i] = acc467_m[seq(i, 12) & 0x3FFFu];
        f[i] = acc589_m[seq(i, 5) & 0x3FFFu];
      }
    }
#pragma unroll
    for (int i = 0; i < N; i++)
      odds[i] = __dmul_rn(__dmul_rn(__dmul_rn(__dmul_rn(__dmul_rn(a[i], b[i]), c[i]), d[i]), e[i]), f[i]);
  }
#pragma unroll
  for (int i = 0; i < N; i++) out[i] = v[i] ? __ddiv_rn(odds[i], __dadd_rn(1.0, odds[i])) : 0.0;
}

}  // namespace gsnapdp
