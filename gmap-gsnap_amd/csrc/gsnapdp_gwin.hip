// gsnapdp_gwin.hip -- Dynprog_genome_gap in probability mode (reference
// src/dynprog.c:4798-5061; the bridge's probability search :3829-4081) with
// ONE WINDOW PER LANE (k_gwin).
//
// Why.  An intron window is small (GMAP: length1 ~ 22 rows, length2 ~ 30
// columns, band ~ 23 diagonals).  The row-lane kernel k_ggap puts rows on
// lanes and sweeps a skewed wavefront, so most lane-steps fall outside the band
// (about a quarter are in band), and the bridge scans every band cell again
// from LDS.  Here each lane runs its own window's DP row by row over the band
// slots held in registers: every instruction of the fill is an in-band cell of
// some lane, no lane waits on another, and the band edges cost nothing.
//
// Layout.  Slot k of row r holds column c = r - lband + k (k < W, the band's
// width; lband = extraband_paired for the windows taken here).  Cell (r, c)
// reads its diagonal predecessor (r-1, c-1) from slot k (previous row), the
// cell above (r-1, c) from slot k+1 (previous row) and the cell to its left
// (r, c-1) from slot k-1 (this row), so a row updates the slots in place from
// k = 0 up.  Out-of-band neighbours are NEG, as the reference's initialised
// matrices read there (slot W is never computed and keeps its NEG).  Rows
// r <= lband reach columns <= 0; those slots carry NEG-like values, and the
// column-0 gap2 chain open + r*extend comes out of the recurrence itself from
// H(0,0) = 0 (dynprog.c:1460-1488).  Column data sit in LDS as [column][lane]
// bytes, so a cell's read is one conflict-free ds_read_u8 whose address is
// uniform but for the lane (every lane is at the same row and slot).
//
// The bridge (probability mode, :3905-4041) keeps, over split rows rL =
// 1..L1-1 in order, the first candidate with the largest probL + probR among
// those whose score reaches score_threshold:
//   left loop:  HL(rL, cL) - pen + intron(leftdi[cL], rightdi[rR]) + HR(rR, rR)
//   right loop: HL(rL, rL) + intron(leftdi[rL], rightdi[cR]) + HR(rR, cR) - pen
// (rR = L1 - rL; pen = 1 when the cell's nogap came from a gap).  The other
// flank's diagonal is a per-row constant, so the fills evaluate the threshold
// test in passing: the right flank is filled first (its diagonal values only),
// then the left flank (direction bits, the left loop's tests, its diagonal),
// then the right flank again (direction bits, the right loop's tests).  A row's
// passing cells become one 32-bit mask in the order of the flank's columns
// sorted by site probability (ties: the smaller column first), so the row's
// best candidate is its lowest set bit; the next bits are checked while their
// f64 sum equals the best one (a smaller column with an equal sum wins, as in
// the reference's ascending scan).  The rows are then visited in the
// reference's order with its strict `>`.
//
// The final score needs H at both chosen cells.  One of them is always on its
// flank's diagonal (stored); the other's H is the score of its traceback path,
// totalled by the shared traceback (every path ends at (0, 0) with 0).
//
// Taken here (k_ggap_plan, gwin_ok): probability mode, no splicing IIT, both
// flanks at least length1 long (so the bridge band is the fill band) and at
// most GW_L2MAX, band widths <= GW_WMAX, length1 <= GW_L1MAX, and an intron
// span that never cuts the bridge's columns.  The lanes of a wave that share
// (extraband, both widths, jump_late_p) run together; a wave with several
// such keys runs them one after another.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <type_traits>

#include "gsnapdp_ctx.h"
#include "gsnapdp_device.h"
#include "gsnapdp_ggap.h"
#include "gsnapdp_internal.h"

using namespace gsnapdp;

#define AS_GLOBAL __attribute__((address_space(1)))
#define AS_LDS __attribute__((address_space(3)))

namespace {

constexpr int GW_EXT = -3;  // SINGLE_EXTEND = PAIRED_EXTEND (dynprog.c:142-293)
static_assert(SINGLE_EXTEND == GW_EXT && PAIRED_EXTEND == GW_EXT, "one extend penalty");
constexpr int GW_NC = GW_L1MAX + GW_WMAX;  // column slots per flank in LDS: index c + lband
constexpr int GW_RANK_NONE = 31;           // rank byte of a column that is never a candidate
// LDS per wave: each flank's columns [index][lane] as u16 words packing A (4 x
// genome class, bits 0-4), C (6 x dinucleotide index, bits 5-9) and B
// (probability rank, bits 10-14); then the traceback rows [i][lane] u32
constexpr int GW_LDS_PL = 0, GW_LDS_PR = 2 * GW_NC * 64, GW_LDS_T = 4 * GW_NC * 64;
constexpr int GW_LDS_WAVE = 6 * GW_NC * 64;
constexpr uint32_t GW_COL_NONE = 4 * 5 | (uint32_t)GW_RANK_NONE << 10;  // '*', no term, no candidate
constexpr int GW_BLOCK = 256;
constexpr int GW_WAVES_PER_SIMD = 2;
// global scratch per wave, [index][lane] dwords (uint4 / double as 4 / 2 dwords)
enum {
  GS_RW = 0,                          // row words: profile word of query row r (1..L1)
  GS_QB = GS_RW + (GW_L1MAX + 1),     // row match masks by query index
  GS_DR = GS_QB + GW_L1MAX,           // HR(r, r)
  GS_DL = GS_DR + (GW_L1MAX + 1),     // HL(r, r)
  GS_ML = GS_DL + (GW_L1MAX + 1),     // left loop pass masks by rL
  GS_MR = GS_ML + (GW_L1MAX + 1),     // right loop pass masks by rR
  GS_INVL = GS_MR + (GW_L1MAX + 1),   // column of rank i, left
  GS_INVR = GS_INVL + 32,             // right
  GS_PL = GS_INVR + 32,               // direction planes, left: 3 dwords per row
  GS_PR = GS_PL + 3 * (GW_L1MAX + 1), // right
  GS_SPL = GS_PR + 3 * (GW_L1MAX + 1),  // site probabilities by rank (double), left
  GS_SPR = GS_SPL + 2 * 32,
  GS_SL = GS_SPR + 2 * 32,            // a row's best candidate: probL + probR (double), left loop by rL
  GS_SR = GS_SL + 2 * (GW_L1MAX + 1), // right loop by rR
  GS_CL = GS_SR + 2 * (GW_L1MAX + 1), // its column | 256 (an equal sum follows) | 512 (any), left
  GS_CR = GS_CL + (GW_L1MAX + 1),
  GS_DW = GS_CR + (GW_L1MAX + 1)      // dwords per lane
};
constexpr size_t GW_WAVE_DW = (size_t)GS_DW * 64;

#ifdef GW_PROF  // diagnostics: cycles per phase summed over wave-tasks (s_memtime)
__device__ unsigned long long gw_prof[16];
// (summed per wave in SGPRs, added to gw_prof once at the end: an atomic per
// phase would itself stall the wave's next memory wait)
#define GW_T(i, t0)                                                            \
  do {                                                                          \
    const uint64_t t1_ = __builtin_amdgcn_s_memtime();                          \
    gw_acc[i] += t1_ - (t0);                                                    \
    t0 = t1_;                                                                   \
  } while (0)
#else
#define GW_T(i, t0) (void)0
#endif

// dinucleotide index of a leftdi / rightdi code (0: none)
__device__ inline int left_idx(int d) {
  return d == LEFT_GT ? 1 : d == LEFT_GC ? 2 : d == LEFT_AT ? 3 : d == LEFT_CT ? 4 : 0;
}
__device__ inline int right_idx(int d) {
  return d == RIGHT_AG ? 1 : d == RIGHT_AC ? 2 : d == RIGHT_GC ? 3 : d == RIGHT_AT ? 4 : 0;
}
__device__ inline int left_code(int i) {
  return i == 1 ? LEFT_GT : i == 2 ? LEFT_GC : i == 3 ? LEFT_AT : i == 4 ? LEFT_CT : 0;
}
__device__ inline int right_code(int i) {
  return i == 1 ? RIGHT_AG : i == 2 ? RIGHT_AC : i == 3 ? RIGHT_GC : i == 4 ? RIGHT_AT : 0;
}

// The direction word of a row: four planes (gap1 extends, gap2 extends, nogap
// from gap1, nogap from gap2; a jump-late flank stores complements) of W bits,
// slot k at bit W-1-k, packed into three dwords (W <= 24).
// One flank fill over rows 1..L1max (wave-uniform), W slots with the diagonal
// in slot LB (compile-time: a wave's windows share them).  JL: the flank's tie
// rule (x wins ties iff jump_late).  MODE 0:
// only the diagonal values H(r, r) -> outD; MODE 1: also the direction planes
// and the bridge's threshold tests (the other flank's diagonal inD, intron
// terms by rw[] keyed by the other flank's dinucleotide at the diagonal).
// Where a fill reads and writes: scratch regions (GS_*, [index][lane] from the
// wave's uniform scratch base) and LDS byte arrays (offsets from the wave's LDS
// base plus the lane), so that no per-lane 64-bit pointer stays live.
//   RW: row words; Dout / Din: this / the other flank's diagonal values; P, M:
//   direction planes and pass masks; SP, INV: this flank's probabilities and
//   columns by rank; PO: the other flank's probabilities by column; S, C: the
//   row's best candidate; COL / COLO: this / the other flank's column words
//   (LDS); rev: rows read the query backwards.
struct FillIO {
  int RW, Dout, Din, P, M, SP, INV, PO, S, C;
  int COL, COLO;  // LDS byte offsets of this / the other flank's column words
  int rev;
};
struct Scr {  // the wave's scratch: [index][lane] dwords / doubles
  AS_GLOBAL uint32_t* b;  // wave-uniform
  int lane;
  __device__ inline AS_GLOBAL uint32_t& u(int region, int i) const {
    return b[(uint32_t)((region + i) * 64 + lane)];
  }
  __device__ inline AS_GLOBAL double& d(int region, int i) const {
    return ((AS_GLOBAL double*)b)[(uint32_t)(region * 32 + i * 64 + lane)];
  }
};

template <int W, int LB, int JL, int MODE>
__device__ __forceinline__ void gw_fill(int L1max, int L1, int L2, int open, int thr, const Scr& sc_, const Scr& po_,
                                        const AS_LDS uint8_t* lwb, const FillIO& io, const uint32_t (&rwd)[5]) {
  const AS_LDS uint16_t* lP = (const AS_LDS uint16_t*)(lwb + io.COL) + sc_.lane;
  const AS_LDS uint16_t* lPo = (const AS_LDS uint16_t*)(lwb + io.COLO) + sc_.lane;
  const int rev = io.rev;
  static_assert(W <= GW_WMAX && LB < W, "band shape");
  constexpr int lband = LB;
  int H[W], E[W], F[W];
  constexpr int rband = W - 1 - lband;
  const int e0 = min(rband, L2);
#pragma unroll
  for (int k = 0; k < W; k++) {  // row 0 (dynprog.c:1460-1488)
    const int c = k - lband;
    H[k] = c == 0 ? 0 : NEG;
    E[k] = (c >= 1 && c <= e0) ? open + c * GW_EXT : NEG;
    F[k] = NEG;
  }
  auto rowword = [&](int r) -> uint32_t {
    const int rr = r <= L1 ? r : L1;
    return sc_.u(io.RW, rev ? L1 + 1 - rr : rr);
  };
  // the other flank's diagonal row and its dinucleotide index for row r
  auto other = [&](int r) { return max(L1 - r, 0); };
  uint32_t rk = rowword(1);
  int Dn = 0;
  uint32_t cn = 0;
  double pOn = 0.0;
  if constexpr (MODE == 1) {
    Dn = (int)sc_.u(io.Din, other(1));
    cn = ((uint32_t)lPo[(size_t)(other(1) + lband) * 64] >> 5) & 31u;
    pOn = po_.d(io.PO, other(1));
  }
  // slot k of row r is column r - lband + k, index r + k: the slots' column
  // words shift down one slot per row, one new word entering at the top (read
  // a row ahead: no LDS wait inside the row)
  uint32_t cv[W];
#pragma unroll
  for (int k = 0; k < W; k++) cv[k] = lP[(size_t)(1 + k) * 64];
  // the previous row's best candidate, finished a row later (its loads in flight meanwhile)
  int rp = 0, ip = 31, jp = 31;
  uint32_t cp = 0;
  double spi = 0.0, spj = 0.0, pOp = 0.0;
  auto finish = [&]() {
    if (rp >= 1 && rp <= L1 - 1) {
      const double S = spi + pOp, S2 = spj + pOp;
      const bool valid = ip < 31, slow = jp < 31 && S2 == S;
      sc_.d(io.S, rp) = valid ? S : -1.0;
      sc_.u(io.C, rp) = cp | (slow ? 256u : 0u) | (valid ? 512u : 0u);
    }
  };
  for (int r = 1; r <= L1max; r++) {
    const uint32_t rkc = rk;
    rk = rowword(r + 1);  // the next row's loads in flight through this row
    int Tm1 = 0;
    uint32_t rwc = 0;
    double pOc = 0.0;
    if constexpr (MODE == 1) {
      Tm1 = thr - Dn - 1 + JL;  // x >= T, x = H - pen + term (JL: H + penraw + term >= T + 1)
      rwc = cn == 6 ? rwd[1] : cn == 12 ? rwd[2] : cn == 18 ? rwd[3] : cn == 24 ? rwd[4] : rwd[0];
      pOc = pOn;
      Dn = (int)sc_.u(io.Din, other(r + 1));
      cn = ((uint32_t)lPo[(size_t)(other(r + 1) + lband) * 64] >> 5) & 31u;
      pOn = po_.d(io.PO, other(r + 1));
    }
    const uint32_t cnext = lP[(size_t)(r + W) * 64];
    int Hl = NEG, El = NEG;  // (r, c-1) of slot 0: outside the band
    uint32_t p0 = 0, p1 = 0, p2 = 0, p3 = 0, pm = 0;
    int dg = NEG;
#pragma unroll
    for (int k = 0; k < W; k++) {
      // (r-1, c) of the last slot lies outside the band: NEG
      const int Ha = k + 1 < W ? H[k + 1] : NEG, Fa = k + 1 < W ? F[k + 1] : NEG;
      const int Hd = H[k], Ed = E[k], Fd = F[k];
      const int av = Hl + open, bv = Ha + open;
      const int En = max(El, av) + GW_EXT;
      const int Fn = max(Fa, bv) + GW_EXT;
      const int m1 = max(Hd, Ed);
      const int sc = __builtin_amdgcn_sbfe((int)rkc, (int)cv[k], 4);  // (offset: bits 0-4, A)
      const int Hn = max(m1, Fd) + sc;
      if constexpr (MODE == 1) {
        // direction signs (recurrences :1519-1561, "x wins ties iff jump_late")
        const int dE = JL ? El - av : av - El;  // gap1: extend (El) or open (H + open)
        const int dF = JL ? Fa - bv : bv - Fa;  // gap2
        const int dh = JL ? Ed - Hd : Hd - Ed;  // nogap: gap1 over H
        const int dv = JL ? Fd - m1 : m1 - Fd;  // nogap: gap2 over max(H, gap1)
        p0 = __builtin_amdgcn_alignbit(p0, (uint32_t)dE, 31u);
        p1 = __builtin_amdgcn_alignbit(p1, (uint32_t)dF, 31u);
        p2 = __builtin_amdgcn_alignbit(p2, (uint32_t)dh, 31u);
        p3 = __builtin_amdgcn_alignbit(p3, (uint32_t)dv, 31u);
        // the bridge's test on this cell: H - pen + intron term >= threshold - D
        const uint32_t penraw = JL ? ((uint32_t)(dh & dv) >> 31) : ((uint32_t)(dh | dv) >> 31);
        const int term = (int)__builtin_amdgcn_ubfe(rwc, cv[k] >> 5, 6);
        const int x = JL ? Hn + term + (int)penraw : Hn + term - (int)penraw;
        const uint32_t ok = (uint32_t)(Tm1 - x) >> 31;
        pm |= ok << (cv[k] >> 10);
      }
      if (k == lband) dg = Hn;  // the diagonal cell (r, r)
      H[k] = Hn;
      E[k] = En;
      F[k] = Fn;
      Hl = Hn;
      El = En;
    }
#pragma unroll
    for (int k = 0; k + 1 < W; k++) cv[k] = cv[k + 1];
    cv[W - 1] = cnext;
    if (r <= L1) {
      sc_.u(io.Dout, r) = (uint32_t)dg;
      if constexpr (MODE == 1) {
        // planes of W bits each, at bits 24 j of the 96-bit row word
        constexpr uint32_t m = (1u << W) - 1u;
        p0 &= m, p1 &= m, p2 &= m, p3 &= m;
        sc_.u(io.P, 3 * r) = p0 | (p1 << 24);
        sc_.u(io.P, 3 * r + 1) = (p1 >> 8) | (p2 << 16);
        sc_.u(io.P, 3 * r + 2) = (p2 >> 16) | (p3 << 8);
        sc_.u(io.M, r) = pm & 0x7FFFFFFFu;
      }
    }
    if constexpr (MODE == 1) {
      // the row's best candidate: its lowest set bit (the largest probability,
      // then the smaller column), and the next bit to tell an equal sum
      finish();
      const uint32_t mm = pm & 0x7FFFFFFFu, m2 = mm & (mm - 1u);
      rp = r;
      ip = mm ? __builtin_ctz(mm) : 31;
      jp = m2 ? __builtin_ctz(m2) : 31;
      spi = sc_.d(io.SP, ip < 31 ? ip : 0);
      spj = sc_.d(io.SP, jp < 31 ? jp : 0);
      cp = sc_.u(io.INV, ip < 31 ? ip : 0);
      pOp = pOc;
    }
  }
  if constexpr (MODE == 1) finish();
}

// The traceback of one flank for every lane at once, as a backward sweep over
// the rows: a path only ever moves to a lower row (a diagonal step, a vertical
// gap) or along its row (a horizontal gap), so the wave visits rows L1max .. 0
// once, loading each row's direction words for all lanes in one coalesced
// load (the next row's in flight meanwhile), and every lane takes the steps of
// its own path that lie in that row.  The steps, counts and op stream are the
// shared traceback's (gsnapdp_device.h, dynprog.c:2611-2712) in the same
// order; `score` totals the path (the start cell's H).
//   mode H: at a nogap cell; VR / HR: inside a vertical / horizontal gap run
//   (dist cells so far); DONE: the path left the band.
// pen0: 1 when the start cell's nogap came from a gap (the bridge's penalty).
template <class QMask, class Col, class Score>
__device__ __forceinline__ void gw_traceback(const AS_GLOBAL uint32_t* planes, int W, int lband, int cpl, int L1, int L2,
                                    int rev, int cdna_direction, int r, int c, int Rmax, const QMask& qmask,
                                    const Col& colcls, Tally& t, OpWriter& ow, Score& score, int& pen0) {
  enum { MH = 0, MVR = 1, MHR = 2, MDONE = 3 };
  const int rband = W - 1 - lband;
  const int r0 = r, c0 = c;
  auto inband = [&](int rr, int cc) {
    const int d = rr - cc + rband;
    return rr >= 1 && cc >= 1 && d >= 0 && d <= lband + rband;
  };
  int mode = MH, dist = 0;
  auto count = [&](int rr, int cc) {
    score.diag(rr, cc);
    const int g = colcls(cc);
    if (g != 5) {
      const int m = (int)((qmask(rr) >> g) & 1u);
      t.nmatches += m;
      t.nmismatches += 1 - m;
      t.npush++;
    }
  };
  // every row's words at once (one memory latency for the sweep, not one per row)
  uint32_t pw[GW_L1MAX + 1][3];
#pragma unroll
  for (int R = 1; R <= GW_L1MAX; R++)
#pragma unroll
    for (int j = 0; j < 3; j++) pw[R][j] = planes[(size_t)(3 * min(R, max(Rmax, 1)) + j) * 64];
#pragma unroll
  for (int R = GW_L1MAX; R >= 0; R--) {
    if (R > Rmax) continue;  // (wave-uniform)
    // the row's four planes (24 bits each in the 96-bit w0 | w1 << 32 | w2 << 64)
    const uint32_t n0 = R ? pw[R][0] : 0u, n1 = R ? pw[R][1] : 0u, n2 = R ? pw[R][2] : 0u;
    const uint32_t P0 = n0 & 0xFFFFFFu, P1 = (n0 >> 24) | ((n1 & 0xFFFFu) << 8);
    const uint32_t P2 = (n1 >> 16) | ((n2 & 0xFFu) << 16), P3 = n2 >> 8;
    // the direction nibble of cell (R, cc) (in band, R >= 1): bit0 gap1 extends, bit1 gap2
    // extends, bit2 nogap from gap1, bit3 nogap from gap2 (gsnapdp_device.h)
    auto dirs = [&](int cc) -> uint32_t {
      const uint32_t pos = (uint32_t)(W - 1 - (cc - R + lband));
      const uint32_t raw = (((P0 >> pos) & 1u) | (((P1 >> pos) & 1u) << 1) | (((P2 >> pos) & 1u) << 2) |
                            (((P3 >> pos) & 1u) << 3)) ^ (uint32_t)cpl;
      return (raw & 3u) | ((raw & 8u) ? 8u : (raw & 4u));
    };
    if (r != R || mode == MDONE) continue;
    if (mode == MVR) {  // gap2_vert(R, c): the vertical run goes on, or ends below row R
      const bool more = c == 0 ? (R >= 2 && R <= lband && R <= L1) : (inband(R, c) && ((dirs(c) >> 1) & 1u));
      r--;
      if (more) {
        dist++;
        continue;
      }
      score.gap(dist);
      ow.flush();
      ow.put(GSNAPDP_OP(GSNAPDP_OP_VSKIP, dist));
      t.npush += dist;
      t.nopens++;
      t.nindels += dist;
      mode = MH;
      continue;  // (at row R - 1)
    }
    if (mode == MHR) {  // gap1_horiz(R, c) along this row
      while (R == 0 ? (c >= 2 && c <= rband && c <= L2) : (inband(R, c) && (dirs(c) & 1u))) {
        dist++;
        c--;
      }
      c--;
      bool dashes = true;
      if (dist >= MICROINTRON_LENGTH) {
        const int cl = c + 1, cr = c + dist;
        const int rv = rev;
        const int l1 = colcls(rv ? cr : cl), l2 = colcls(rv ? cr - 1 : cl + 1);
        const int r2 = colcls(rv ? cl + 1 : cr - 1), r1 = colcls(rv ? cl : cr);
        dashes = intron_type_codes(l1, l2, r2, r1, cdna_direction) == 0;
      }
      score.gap(dist);
      ow.flush();
      ow.put(GSNAPDP_OP(dashes ? GSNAPDP_OP_HDASH : GSNAPDP_OP_HGAP, dist));
      t.npush += dashes ? dist : 1;
      if (dashes) {
        t.nopens++;
        t.nindels += dist;
      }
      mode = MH;  // (still at row R)
    }
    if (!inband(r, c)) {
      mode = MDONE;
      continue;
    }
    const uint32_t nib = dirs(c);
    if (r == r0 && mode == MH && c == c0) pen0 = (nib & 12u) ? 1 : 0;  // (the first step: the start cell)
    count(r, c);
    ow.run++;
    dist = 1;
    r--;
    c--;
    mode = (nib & 8u) ? MVR : (nib & 4u) ? MHR : MH;
  }
  ow.flush();
}

// Genome classes of columns 0 .. GW_L2MAX + 2 of one flank (get_genomic_nt,
// dynprog.c:403-441, as gclass): column c (1..L2) is genomic position g0 +
// gstep * (c - 1); the flank's positions are consecutive, so two packed blocks
// hold them all (one load batch instead of a chain per column).  Column 0 and
// the columns past L2 are '*'.
struct FlankBlk {
  uint32_t h0, l0, f0, h1, l1, f1;
  uint32_t b0;
  bool ok0, ok1, wrap;
};
__device__ inline uint32_t flank_pos(const Lane& L, int gp) {
  return L.watson ? (L.base + (uint32_t)gp) : (L.base + (uint32_t)(L.glen - 1) - (uint32_t)gp);
}
__device__ inline FlankBlk flank_load(const uint32_t* __restrict__ blocks, uint64_t nwords, const Lane& L, int g0,
                                      int gstep, int L2) {
  FlankBlk f;
  const uint32_t pa = flank_pos(L, g0), pb = flank_pos(L, g0 + gstep * (L2 - 1));
  const uint32_t lo = pa < pb ? pa : pb, hi = pa < pb ? pb : pa;
  f.wrap = hi - lo != (uint32_t)(L2 - 1);  // (positions wrap around 2^32: column by column)
  const uint64_t b0 = lo >> 5;
  f.b0 = (uint32_t)b0;
  f.ok0 = b0 * 3u + 2u < nwords;
  f.ok1 = (b0 + 1u) * 3u + 2u < nwords;
  const uint64_t p0 = f.ok0 ? b0 * 3u : 0u, p1 = f.ok1 ? (b0 + 1u) * 3u : 0u;
  f.h0 = blocks[p0], f.l0 = blocks[p0 + 1], f.f0 = blocks[p0 + 2];
  f.h1 = blocks[p1], f.l1 = blocks[p1 + 1], f.f1 = blocks[p1 + 2];
  return f;
}
__device__ inline void flank_classes(const FlankBlk& f, const uint32_t* __restrict__ blocks, uint64_t nwords,
                                     const Lane& L, int g0, int gstep, int L2, int (&cls)[GW_L2MAX + 3]) {
  if (f.wrap) {
#pragma unroll
    for (int c = 0; c < GW_L2MAX + 3; c++) cls[c] = (c >= 1 && c <= L2) ? gclass(blocks, nwords, L, g0 + gstep * (c - 1)) : 5;
    return;
  }
  cls[0] = 5;
#pragma unroll
  for (int c = 1; c < GW_L2MAX + 3; c++) {
    const int gp = g0 + gstep * (c - 1);
    const uint32_t pos = flank_pos(L, gp);
    const bool second = (pos >> 5) != f.b0;
    const uint32_t bit = pos & 31u;
    const uint32_t fl = second ? f.f1 : f.f0;
    const uint32_t word = bit < 16 ? (second ? f.l1 : f.l0) : (second ? f.h1 : f.h0);
    const int code = (int)((word >> ((bit & 15u) * 2u)) & 3u);
    int k = L.watson ? code : 3 - code;
    if (!(second ? f.ok1 : f.ok0) || ((fl >> bit) & 1u)) k = 4;  // outside the genome / N
    if (gp < 0 || gp >= L.glen || L.allstar) k = 5;
    cls[c] = c <= L2 ? k : 5;
  }
}

// The MaxEnt site probabilities of every list window's candidate columns
// (:3856-3903; a window here has no known sites), ahead of k_gwin: item (chunk,
// side, lane) takes list entry chunk * 64 + lane, one flank, columns
// 0..GW_L2MAX-1 (0 from L2 - 1 on), and writes them [chunk][side][column][lane]
// as k_gwin reads them.
//
// The tables' gathers are the work (about four per site, all over 1.5 MB), so
// the tables come through LDS: a block of GP_THREADS items streams the twelve
// 16384-entry tables through one 128 KB LDS buffer in their order in the
// product (maxent_hr.c's acceptor odds a*b*c*d*e*f, donor a*b), and each item
// multiplies its 32 sites' running odds by the current table's entries; the
// 16-entry dinucleotide tables stay in global memory (cached).  A flank's
// candidate sites are consecutive genome positions, so the three packed blocks
// under all of them are loaded once and each site's 16-mers are constant
// funnel shifts of that span (a line that would wrap 2^32 is computed site by
// site from global tables before the table phases).
// the k_gwin lists' 64-window chunks, numbered across the lists in order
struct GwChunks {
  int cnt[GW_NSUB], cum[GW_NSUB + 1];
};
__device__ inline GwChunks gw_chunks(const int* __restrict__ counts) {
  GwChunks q;
  q.cum[0] = 0;
#pragma unroll
  for (int l = 0; l < GW_NSUB; l++) {
    q.cnt[l] = counts[l];
    q.cum[l + 1] = q.cum[l] + (q.cnt[l] + 63) / 64;
  }
  return q;
}
__device__ inline int gw_sub(const GwChunks& q, int chunk) {
  return (chunk >= q.cum[1] ? 1 : 0) + (chunk >= q.cum[2] ? 1 : 0) + (chunk >= q.cum[3] ? 1 : 0);
}
// (selects, not a dynamically indexed private array)
__device__ inline int gw_cnt(const GwChunks& q, int l) {
  return l == 0 ? q.cnt[0] : l == 1 ? q.cnt[1] : l == 2 ? q.cnt[2] : q.cnt[3];
}
__device__ inline int gw_cum(const GwChunks& q, int l) {
  return l == 0 ? q.cum[0] : l == 1 ? q.cum[1] : l == 2 ? q.cum[2] : q.cum[3];
}
static_assert(GW_NSUB == 4, "gw_sub");

constexpr int GP_THREADS = 1024;
constexpr int GP_TABLE = 16384;  // entries of a big table
constexpr size_t GP_LDS = (size_t)GP_TABLE * sizeof(double);
// the big tables' offsets in the table buffer (gsnapdp_load_maxent_tables'
// order: donor_p, donor_di_p, acc1..3_p, accdi_p, acc467_p, acc589_p, then
// the same for the minus models), the phase's model, and the di tables
__device__ constexpr int gp_off(int t) {
  return t == 0 ? 0 : t == 1 ? 16400 : t == 2 ? 32784 : t == 3 ? 49168 : t == 4 ? 65568 : t == 5 ? 81952
       : t == 6 ? 98336 : t == 7 ? 114736 : t == 8 ? 131120 : t == 9 ? 147504 : t == 10 ? 163904 : 180288;
}
__device__ constexpr int gp_model(int t) { return t == 0 ? 0 : t <= 5 ? 1 : t == 6 ? 2 : 3; }

template <int T>
__device__ __forceinline__ void gp_phase(const uint32_t (&x_)[5], bool up, const AS_LDS double* tab,
                                         const double* __restrict__ tables, double (&odds)[GW_L2MAX]) {
  // (the span laundered per phase: the k-mers are recomputed here, not kept
  // live from another phase's identical ones)
  uint32_t x[5];
#pragma unroll
  for (int j = 0; j < 5; j++) {
    x[j] = x_[j];
    asm volatile("" : "+v"(x[j]));
  }
  // the 16-mer `off` nt past site c's start
  auto seq = [&](int c, int off) -> uint32_t {
    const int bf = 2 * (c + off), br = 2 * (GW_L2MAX - 1 - c + off);
    const uint32_t kf = __builtin_amdgcn_alignbit(x[(bf >> 5) + 1], x[bf >> 5], (uint32_t)(bf & 31));
    const uint32_t kr = __builtin_amdgcn_alignbit(x[(br >> 5) + 1], x[br >> 5], (uint32_t)(br & 31));
    return up ? kf : kr;
  };
#pragma unroll
  for (int c = 0; c < GW_L2MAX; c++) {
    if constexpr (T == 0) {  // donor: donor_p * donor_di_p
      const uint32_t s = seq(c, 0);
      odds[c] = tab[(s & 0x3Fu) | ((s >> 4) & 0x3FC0u)] * tables[16384 + ((s >> 6) & 0xFu)];
    } else if constexpr (T == 6) {  // antidonor
      const uint32_t s = seq(c, 0);
      odds[c] = tab[(s & 0xFFu) | ((s >> 4) & 0x3F00u)] * tables[114720 + ((s >> 8) & 0xFu)];
    } else if constexpr (T == 1) {
      odds[c] = tab[seq(c, 0) & 0x3FFFu];
    } else if constexpr (T == 2) {
      odds[c] = __dmul_rn(odds[c], tab[seq(c, 7) & 0x3FFFu]);
    } else if constexpr (T == 3) {  // acc3_p, then accdi_p
      const uint32_t s = seq(c, 14);
      odds[c] = __dmul_rn(__dmul_rn(odds[c], tab[(s & 0xFFu) | ((s >> 4) & 0x3F00u)]), tables[65552 + ((s >> 8) & 0xFu)]);
    } else if constexpr (T == 4) {
      odds[c] = __dmul_rn(odds[c], tab[seq(c, 4) & 0x3FFFu]);
    } else if constexpr (T == 5) {
      odds[c] = __dmul_rn(odds[c], tab[seq(c, 11) & 0x3FFFu]);
    } else if constexpr (T == 7) {
      odds[c] = tab[seq(c, 16) & 0x3FFFu];
    } else if constexpr (T == 8) {
      odds[c] = __dmul_rn(odds[c], tab[seq(c, 9) & 0x3FFFu]);
    } else if constexpr (T == 9) {  // acc3_m, then accdi_m
      const uint32_t s = seq(c, 0);
      odds[c] = __dmul_rn(__dmul_rn(odds[c], tab[(s & 0x3Fu) | ((s >> 4) & 0x3FC0u)]), tables[163888 + ((s >> 6) & 0xFu)]);
    } else if constexpr (T == 10) {
      odds[c] = __dmul_rn(odds[c], tab[seq(c, 12) & 0x3FFFu]);
    } else {
      odds[c] = __dmul_rn(odds[c], tab[seq(c, 5) & 0x3FFFu]);
    }
  }
}

__global__ __launch_bounds__(GP_THREADS) void k_gwin_probs(const gsnapdp_ggap_window* __restrict__ Wn,
                                                           const int* __restrict__ lists, int list_cap,
                                                           const int* __restrict__ counts,
                                                           const uint32_t* __restrict__ blocks, uint64_t nwords,
                                                           const double* __restrict__ tables, double* __restrict__ probs) {
  extern __shared__ double gp_tab[];
  const AS_LDS double* tab = (const AS_LDS double*)gp_tab;
  const GwChunks q = gw_chunks(counts);
  const int nitems = q.cum[GW_NSUB] * 128;
  for (int base = blockIdx.x * GP_THREADS; base < nitems; base += gridDim.x * GP_THREADS) {  // (block-uniform)
    const int t = base + (int)threadIdx.x;
    const int chunk = t >> 7, side = (t >> 6) & 1, ln = t & 63;
    const int l = gw_sub(q, chunk);
    const int k = (chunk - gw_cum(q, l)) * 64 + ln;
    double* out = probs + (size_t)chunk * 4096 + side * 2048 + ln;
    bool act = t < nitems && k < gw_cnt(q, l);
    if (t < nitems && !act)
      for (int c = 0; c < GW_L2MAX; c++) out[c * 64] = 0.0;
    int m = 0;
    bool up = true;
    uint32_t vmask = 0, x[5] = {0u, 0u, 0u, 0u, 0u};
    if (act) {
      const gsnapdp_ggap_window w = Wn[lists[(size_t)(GW_LIST + l) * list_cap + k]];
      const int L2 = side ? w.length2R : w.length2L;
      int step;
      uint32_t sp0;
      site_line(w, side, m, sp0, step);
      const uint32_t margin = (m == 0) ? 3u : (m == 1) ? 20u : (m == 2) ? 6u : 3u;
      up = step > 0;
      if (up ? sp0 <= 0xFFFFFFFFu - (GW_L2MAX - 1) && sp0 >= margin : sp0 >= (GW_L2MAX - 1) + margin) {
        // no uint32 wrap: site c starts c (or 31 - c) nt past the lowest start s0
        const uint32_t s0 = (up ? sp0 : sp0 - (uint32_t)(GW_L2MAX - 1)) - margin;
        const uint64_t blk = (uint64_t)(s0 >> 5) * 3u;
        uint32_t wv[6];
#pragma unroll
        for (int j = 0; j < 3; j++) {
          wv[2 * j] = blk + 3 * j + 1 < nwords ? blocks[blk + 3 * j + 1] : 0u;  // low
          wv[2 * j + 1] = blk + 3 * j < nwords ? blocks[blk + 3 * j] : 0u;      // high
        }
        const uint32_t sh = (s0 & 31u) * 2u, b = sh & 31u;
        const bool i0 = sh >= 32u;
#pragma unroll
        for (int j = 0; j < 4; j++)
          x[j] = __builtin_amdgcn_alignbit(i0 ? wv[j + 2] : wv[j + 1], i0 ? wv[j + 1] : wv[j], b);
#pragma unroll
        for (int c = 0; c < GW_L2MAX; c++) {
          const uint32_t sp = sp0 + (uint32_t)(step * c);
          const uint64_t ptr = (uint64_t)((sp - margin) >> 5) * 3u;
          const bool v = c < L2 - 1 && sp >= w.chroffset + margin && ptr + 4 < nwords;
          vmask |= (v ? 1u : 0u) << c;
        }
      } else {
        // (a line that wraps: site by site, from the global tables)
#pragma clang loop unroll(disable)
        for (int c = 0; c < GW_L2MAX; c++)
          out[c * 64] = c < L2 - 1 ? maxent_prob(m, sp0 + (uint32_t)(step * c), w.chroffset, blocks, nwords, tables)
                                   : 0.0;
        act = false;
      }
    }
    // the models some item of the block needs (a phase nobody needs is skipped)
    const int mm = act ? 1 << m : 0;
    const bool need0 = __syncthreads_or(mm & 1), need1 = __syncthreads_or(mm & 2);
    const bool need2 = __syncthreads_or(mm & 4), need3 = __syncthreads_or(mm & 8);
    double odds[GW_L2MAX];
#pragma unroll
    for (int c = 0; c < GW_L2MAX; c++) odds[c] = 0.0;
    auto phase = [&](auto tc) {
      constexpr int T = decltype(tc)::value;
      constexpr int M = gp_model(T);
      if (!(M == 0 ? need0 : M == 1 ? need1 : M == 2 ? need2 : need3)) return;
      __syncthreads();  // the previous table's readers are done
      // (from a laundered thread index: the addresses are invariant across
      // rounds and would be hoisted and spilled)
      int tid = (int)threadIdx.x;
      asm volatile("" : "+v"(tid));
      const double2* src = (const double2*)(tables + gp_off(T)) + tid;
      double2* dst = (double2*)gp_tab + tid;
#pragma unroll
      for (int i = 0; i < GP_TABLE / 2 / GP_THREADS; i++) dst[i * GP_THREADS] = src[i * GP_THREADS];
      __syncthreads();
      if (act && m == M) gp_phase<T>(x, up, tab, tables, odds);
    };
    phase(std::integral_constant<int, 0>());
    phase(std::integral_constant<int, 1>());
    phase(std::integral_constant<int, 2>());
    phase(std::integral_constant<int, 3>());
    phase(std::integral_constant<int, 4>());
    phase(std::integral_constant<int, 5>());
    phase(std::integral_constant<int, 6>());
    phase(std::integral_constant<int, 7>());
    phase(std::integral_constant<int, 8>());
    phase(std::integral_constant<int, 9>());
    phase(std::integral_constant<int, 10>());
    phase(std::integral_constant<int, 11>());
    if (act) {
#pragma unroll
      for (int c = 0; c < GW_L2MAX; c++)
        out[c * 64] = (vmask >> c) & 1u ? __ddiv_rn(odds[c], __dadd_rn(1.0, odds[c])) : 0.0;
    }
    __syncthreads();  // (the next round's first table overwrites the buffer)
  }
}

__global__ __launch_bounds__(GW_BLOCK) __attribute__((amdgpu_waves_per_eu(GW_WAVES_PER_SIMD, 8))) void k_gwin(
    const gsnapdp_ggap_window* __restrict__ Wn, const int* __restrict__ lists, int list_cap,
    const int* __restrict__ counts, const char* __restrict__ q, const char* __restrict__ qu, const uint32_t* __restrict__ blocks,
    uint64_t nwords, const uint32_t* __restrict__ prof, const double* __restrict__ tables,
    uint32_t* __restrict__ pool, const double* __restrict__ probs, gsnapdp_ggap_result* __restrict__ res,
    gsnapdp_ggap_trace* __restrict__ trc, uint32_t* __restrict__ ops, const int64_t* __restrict__ op_off) {
  extern __shared__ uint8_t gw_lds[];
  const int lane = threadIdx.x & 63;
  const int gw = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const int nw = (int)((gridDim.x * blockDim.x) >> 6);
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  AS_LDS uint8_t* lwb = (AS_LDS uint8_t*)(gw_lds + (size_t)wv * GW_LDS_WAVE);  // (wave-uniform)
  AS_LDS uint16_t* lPL = (AS_LDS uint16_t*)(lwb + GW_LDS_PL) + lane;
  AS_LDS uint16_t* lPR = (AS_LDS uint16_t*)(lwb + GW_LDS_PR) + lane;
  // the wave's scratch from a wave-uniform base (SGPRs) and the lane
  const Scr SC = {(AS_GLOBAL uint32_t*)pool + (size_t)__builtin_amdgcn_readfirstlane(gw) * GW_WAVE_DW, lane};
  auto S32 = [&](int region, int i) -> AS_GLOBAL uint32_t* { return &SC.u(region, i); };
  const GwChunks qc = gw_chunks(counts);
#ifdef GW_PROF
  uint64_t gw_acc[16] = {};
#endif
  for (int chunk = gw; chunk < qc.cum[GW_NSUB]; chunk += nw) {  // (wave-uniform)
    const int l = gw_sub(qc, chunk);
    const int base = (chunk - gw_cum(qc, l)) * 64;
    const int k0 = base + lane;
    // the chunk's site probabilities (k_gwin_probs): [side][column][lane] doubles
    AS_GLOBAL uint32_t* const PB_base = (AS_GLOBAL uint32_t*)(probs + (size_t)chunk * 4096);
    const bool valid = k0 < gw_cnt(qc, l);
    const int* list = lists + (size_t)(GW_LIST + l) * list_cap;
    const int wi = list[valid ? k0 : base];
    int key, L1v;
    {  // (only the key and length1 stay live across the groups; each reads the record again)
      const gsnapdp_ggap_window w = Wn[wi];
      const GGeo G = gg_geo(w);
      key = G.eb | (G.WL << 6) | (G.WR << 12) | ((w.jump_late_p ? 1 : 0) << 18);
      L1v = G.L1;
    }
    // lanes sharing (extraband, both band widths, jump_late_p) run together
    uint64_t todo = __ballot(valid);
    while (todo) {
      const int leader = __ffsll((unsigned long long)todo) - 1;
      const int lkey = __builtin_amdgcn_readfirstlane(__shfl(key, leader));  // (every lane holds it)
      const bool mine = valid && key == lkey;
      todo &= ~__ballot(mine);
      const int L1max = __builtin_amdgcn_readfirstlane(wave_max(mine ? L1v : 0));
      const int eb = lkey & 63, WL = (lkey >> 6) & 63, WR = (lkey >> 12) & 63, JLL = (lkey >> 18) & 1;
      if (!mine) continue;
#ifdef GW_PROF
      uint64_t tp = __builtin_amdgcn_s_memtime();
      gw_acc[7] += 1;
#endif
      // ---- per-window tables: column classes, dinucleotide indices, site
      // probabilities and their ranks (both flanks), row words, match masks
      // (only L1, the flank lengths, open, the threshold and the intron-term words
      // stay live through the fills; the outcome re-reads the window record)
      int ws = wi;
      asm volatile("" : "+v"(ws));
      // (the setup's scratch addresses from a laundered lane: invariant across
      // tasks, they would otherwise be hoisted out of the task loop and spilled)
      int lane1 = lane;
      asm volatile("" : "+v"(lane1));
      const Scr SC1 = {SC.b, lane1};
      const gsnapdp_ggap_window w = Wn[ws];
      const GGeo G = gg_geo(w);
      const int L1 = G.L1, L2L = G.L2L, L2R = G.L2R, open = G.open, thr = w.score_threshold;
      uint32_t rwL[5], rwR[5];
      {
      const Lane LL = side_lane(w, G, 0), LR = side_lane(w, G, 1);
      // every load the record alone addresses goes out at once, with no branch
      // between them (a dependent global round trip under load is thousands of
      // cycles): the query rows, both flanks' genome blocks, the left flank's
      // site probabilities; then the rows' profile words
      uint32_t qc[GW_L1MAX], uc[GW_L1MAX];
#pragma unroll
      for (int i = 0; i < GW_L1MAX; i++) {
        const int qi = (int)w.qpos + min(i + 1, L1) - 1;
        qc[i] = (unsigned char)q[qi];
        uc[i] = (unsigned char)qu[qi];
      }
      const FlankBlk fbL = flank_load(blocks, nwords, LL, w.offset2L, 1, L2L);
      const FlankBlk fbR = flank_load(blocks, nwords, LR, w.revoffset2R, -1, L2R);
      const Scr PB = {PB_base, lane1};
      {
        const uint32_t* ptab = prof + G.mt * 128;
        uint32_t rk[GW_L1MAX], ub[GW_L1MAX];
#pragma unroll
        for (int i = 0; i < GW_L1MAX; i++) {
          rk[i] = ptab[qc[i] & 127u];
          ub[i] = prof[4 * 128 + (uc[i] & 127u)];
        }
        // rows past L1 get row L1's words (never read)
#pragma unroll
        for (int i = 0; i < GW_L1MAX; i++) {
          SC1.u(GS_RW, i + 1) = rk[i];
          SC1.u(GS_QB, i) = ((rk[i] | (uc[i] < 128u ? ub[i] : 0u)) >> 24) & 31u;  // row_match_mask
        }
      }
      for (int side = 0; side < 2; side++) {
        const int L2 = side ? G.L2R : G.L2L;
        AS_LDS uint16_t* lP = side ? lPR : lPL;
        // classes of columns 0 .. 33 (0 and past L2: '*', never read as such)
        int cls[GW_L2MAX + 3];
        const Lane& LF = side ? LR : LL;
        FlankBlk fb;
        fb.h0 = side ? fbR.h0 : fbL.h0;
        fb.l0 = side ? fbR.l0 : fbL.l0;
        fb.f0 = side ? fbR.f0 : fbL.f0;
        fb.h1 = side ? fbR.h1 : fbL.h1;
        fb.l1 = side ? fbR.l1 : fbL.l1;
        fb.f1 = side ? fbR.f1 : fbL.f1;
        fb.b0 = side ? fbR.b0 : fbL.b0;
        fb.ok0 = side ? fbR.ok0 : fbL.ok0;
        fb.ok1 = side ? fbR.ok1 : fbL.ok1;
        fb.wrap = side ? fbR.wrap : fbL.wrap;
        flank_classes(fb, blocks, nwords, LF, side ? w.revoffset2R : w.offset2L, side ? -1 : 1, L2, cls);
        GW_T(14, tp);
        // column words at index c + eb: A = 4 x class ('*' outside 1..L2), C =
        // 6 x the leftdi / rightdi index (:3331-3373; 0 from column L2 - 1 on),
        // B (below) = the rank; outside columns 1..32 no term, no candidate
        for (int i = 0; i <= eb; i++) lP[i * 64] = (uint16_t)GW_COL_NONE;
        for (int i = eb + GW_L2MAX + 1; i < GW_NC; i++) lP[i * 64] = (uint16_t)GW_COL_NONE;
        uint32_t pk[GW_L2MAX + 1];
#pragma unroll
        for (int c = 1; c <= GW_L2MAX; c++) {
          const int d = c < L2 - 1 ? (side ? right_di(cls[c + 2], cls[c + 1]) : left_di(cls[c + 1], cls[c + 2])) : 0;
          pk[c] = (uint32_t)(4 * cls[c]) | (uint32_t)(6 * (side ? right_idx(d) : left_idx(d))) << 5;
        }
        double p[GW_L2MAX];
#pragma unroll
        for (int c = 0; c < GW_L2MAX; c++) p[c] = PB.d(side * 64, c);
        GW_T(13, tp);
        // ranks of the candidate columns 1 .. L2 - 1 by probability (larger
        // first, then the smaller column); RANK_NONE elsewhere.  Every pair is
        // compared once: c < c2 puts c first unless p[c2] > p[c] (the others
        // carry -1, below every probability, so they rank last, ranks L2 .. 30,
        // whose slots no mask bit reaches).
        const int INVG = side ? GS_INVR : GS_INVL, SPG = side ? GS_SPR : GS_SPL;
        int rank[GW_L2MAX];
#pragma unroll
        for (int c = 0; c < GW_L2MAX; c++) {
          rank[c] = 0;
          p[c] = c < L2 ? p[c] : -1.0;
        }
#pragma clang loop unroll(full)
        for (int c = 1; c < GW_L2MAX; c++)
#pragma clang loop unroll(full)
          for (int c2 = 2; c2 < GW_L2MAX; c2++) {
            if (c2 <= c) continue;
            const int x = p[c2] > p[c] ? 1 : 0;
            rank[c] += x;
            rank[c2] += 1 - x;
          }
#pragma unroll
        for (int c = 1; c < GW_L2MAX; c++) {
          SC1.u(INVG, rank[c]) = (uint32_t)c;
          SC1.d(SPG, rank[c]) = p[c];
          lP[(c + eb) * 64] = (uint16_t)(pk[c] | (uint32_t)(c < L2 ? rank[c] : GW_RANK_NONE) << 10);
        }
        lP[(GW_L2MAX + eb) * 64] = (uint16_t)(pk[GW_L2MAX] | (uint32_t)GW_RANK_NONE << 10);
        GW_T(12, tp);
      }
      // intron terms (:3148-3192) by dinucleotide index: rwL[ri] for the left
      // loop (keyed by rightdi[rR]), fields by leftdi index; rwR[li] likewise
#pragma unroll
      for (int i = 0; i < 5; i++) {
        rwL[i] = 0u;
        rwR[i] = 0u;
      }
#pragma unroll
      for (int li = 1; li < 5; li++)
#pragma unroll
        for (int ri = 1; ri < 5; ri++) {
          int it;
          const uint32_t s = (uint32_t)intron_score(it, left_code(li), right_code(ri), w.cdna_direction, G.canon,
                                                    w.finalp);
          rwL[ri] |= s << (6 * li);
          rwR[li] |= s << (6 * ri);
        }
      }
#ifdef GW_PROF
      __builtin_amdgcn_s_waitcnt(0);
#endif
      GW_T(0, tp);
      // ---- the three fills: right (diagonal only), left, right; the band
      // shape (W, lband) of the wave's windows as template arguments
      AS_GLOBAL uint32_t* const SO_base = SC.b;
      // (byte offsets of the LDS arrays from lw: A_L, A_R, B_L, B_R, C_L, C_R)
      const FillIO ioR1 = {GS_RW, GS_DR, 0, 0, 0, 0, 0, 0, 0, 0, GW_LDS_PR, GW_LDS_PL, 1};
      const FillIO ioL = {GS_RW, GS_DL, GS_DR, GS_PL, GS_ML, GS_SPL, GS_INVL, 64, GS_SL, GS_CL,
                          GW_LDS_PL, GW_LDS_PR, 0};
      const FillIO ioR2 = {GS_RW, GS_DR, GS_DL, GS_PR, GS_MR, GS_SPR, GS_INVR, 0, GS_SR, GS_CR,
                           GW_LDS_PR, GW_LDS_PL, 1};
      auto fills = [&](auto wt, auto lt) {
        constexpr int W = decltype(wt)::value, LB = decltype(lt)::value;
        int lane3 = lane;
        asm volatile("" : "+v"(lane3));
        const Scr SC = {SO_base, lane3}, PO = {PB_base, lane3};
        if (JLL) {
          gw_fill<W, LB, 0, 0>(L1max, L1, L2R, open, thr, SC, PO, lwb, ioR1, rwR);
          GW_T(4, tp);
          gw_fill<W, LB, 1, 1>(L1max, L1, L2L, open, thr, SC, PO, lwb, ioL, rwL);
          GW_T(5, tp);
          gw_fill<W, LB, 0, 1>(L1max, L1, L2R, open, thr, SC, PO, lwb, ioR2, rwR);
        } else {
          gw_fill<W, LB, 1, 0>(L1max, L1, L2R, open, thr, SC, PO, lwb, ioR1, rwR);
          GW_T(4, tp);
          gw_fill<W, LB, 0, 1>(L1max, L1, L2L, open, thr, SC, PO, lwb, ioL, rwL);
          GW_T(5, tp);
          gw_fill<W, LB, 1, 1>(L1max, L1, L2R, open, thr, SC, PO, lwb, ioR2, rwR);
        }
      };
      static_assert(GW_CLASSES == 2, "k_gwin's band shapes");
      if (WL == GW_W0) fills(std::integral_constant<int, GW_W0>(), std::integral_constant<int, GW_LB0>());
      else fills(std::integral_constant<int, GW_W1>(), std::integral_constant<int, GW_LB1>());
      GW_T(1, tp);
      // ---- the candidates in the reference's order (rL ascending, the left
      // loop before the right), strict `>` on probL + probR; each row's best of a
      // loop was found by its fill (a row whose next candidate has an equal sum
      // scans its mask here for the smallest such column)
      const Scr PB = {PB_base, lane};
      auto PL = [&](int c) -> double { return PB.d(0, c); };
      auto PR = [&](int c) -> double { return PB.d(64, c); };
      double bestp = 0.0;
      int brL = 0, bcL = 0, bcR = 0;
      auto tie_scan = [&](uint32_t m, int INVG, int SPG, double pO, double S) -> int {
        int c = (int)SC.u(INVG, __builtin_ctz(m));
        for (m &= m - 1; m; m &= m - 1) {
          const int i = __builtin_ctz(m);
          if (SC.d(SPG, i) + pO != S) break;
          const int c2 = (int)SC.u(INVG, i);
          c = c2 < c ? c2 : c;
        }
        return c;
      };
      for (int r0 = 1; r0 < L1; r0 += 8) {
        double sl[8], sr[8];
        uint32_t cl[8], cr[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {  // eight rows' records in flight at once
          const int rL = min(r0 + u, L1 - 1), rR = L1 - rL;
          sl[u] = SC.d(GS_SL, rL);
          cl[u] = SC.u(GS_CL, rL);
          sr[u] = SC.d(GS_SR, rR);
          cr[u] = SC.u(GS_CR, rR);
        }
#pragma unroll
        for (int u = 0; u < 8; u++) {
          const int rL = r0 + u, rR = L1 - rL;
          if (rL >= L1) break;
          if (cl[u] & 512u) {
            int c = (int)(cl[u] & 255u);
            if (cl[u] & 256u) c = tie_scan(SC.u(GS_ML, rL), GS_INVL, GS_SPL, PR(rR), sl[u]);
            if (sl[u] > bestp) {
              bestp = sl[u];
              brL = rL;
              bcL = c;
              bcR = rR;
            }
          }
          if (cr[u] & 512u) {
            int c = (int)(cr[u] & 255u);
            if (cr[u] & 256u) c = tie_scan(SC.u(GS_MR, rR), GS_INVR, GS_SPR, PL(rL), sr[u]);
            if (sr[u] > bestp) {
              bestp = sr[u];
              brL = rL;
              bcL = rL;
              bcR = c;
            }
          }
        }
      }
      GW_T(2, tp);
      // ---- outcome (:4043-4068, :4084-4108) and the two tracebacks
      // per query index i, for the tracebacks: the row's score nibbles (bits
      // 0..23, as the fill's profile word) and its match mask (bits 24..28), in
      // LDS over the rank arrays (dead after the fills)
      AS_LDS uint32_t* lT = (AS_LDS uint32_t*)(lwb + GW_LDS_T) + lane;
      static_assert(GW_LDS_T + GW_L1MAX * 256 <= GW_LDS_WAVE, "the traceback rows fit");
      // (scratch addresses from a laundered lane: recomputed here, not kept live
      // or spilled from the setup's identical ones; all rows' loads at once)
      int lane2 = lane;
      asm volatile("" : "+v"(lane2));
      const Scr SO = {SC.b, lane2};
      uint32_t tv[GW_L1MAX];
#pragma unroll
      for (int i = 0; i < GW_L1MAX; i++) tv[i] = (SO.u(GS_RW, i + 1) & 0xFFFFFFu) | (SO.u(GS_QB, i) << 24);
#pragma unroll
      for (int i = 0; i < GW_L1MAX; i++)
        if (i < L1) lT[i * 64] = tv[i];
      GW_T(8, tp);
      // the window record again (a laundered index: nothing of the first read is
      // kept live through the fills), only the fields the outcome needs
      int wr = wi;
      asm volatile("" : "+v"(wr));
      int o2L, r2R, off1, dpi, cdir, finalp, halfp, canon, wopen;
      {
        const gsnapdp_ggap_window w2 = Wn[wr];
        const GGeo G2 = gg_geo(w2);
        o2L = w2.offset2L;
        r2R = w2.revoffset2R;
        off1 = w2.offset1;
        dpi = w2.dynprogindex;
        cdir = w2.cdna_direction;
        finalp = w2.finalp;
        halfp = w2.halfp;
        canon = G2.canon;
        wopen = G2.open;
      }
      GW_T(6, tp);
      const int brR = L1 - brL;
      struct PathScore {  // the traceback path's score = the start cell's H
        int s;
        const AS_LDS uint32_t* rw;  // lT: query index i
        const AS_LDS uint16_t* la;  // the flank's column words (A: bits 0-4)
        int L1, eb, rev, open;
        __device__ inline void diag(int r, int c) {
          const uint32_t rk = rw[(size_t)(rev ? L1 - r : r - 1) * 64];
          s += __builtin_amdgcn_sbfe((int)rk, (int)la[(size_t)(c + eb) * 64], 4);
        }
        __device__ inline void gap(int d) { s += open + d * GW_EXT; }
      };
      int finalscore = 0, rc = -1;
      Tally t = {0, 0, 0, 0, 0};
      int nR = 0, nL = 0;
      bool over = false;
      if (bestp > 0.0) {  // (none: the reference reads uninitialised indices, :4055)
        // the right flank's traceback (reversed), then the left's, into one op
        // stream (:5000-5040); each path's score is its start cell's H.  A window
        // whose final score turns out negative returns NULL: its ops are unused.
        const int64_t o0 = op_off[wi];
        const int cap = (int)(op_off[wi + 1] - o0);
        int sR = 0, sL = 0, penR = 0, penL = 0;
        // one loop over the two flanks (one inlined sweep: two would be merged
        // by the compiler through pointers to their writers, kept in scratch)
        for (int f = 0; f < 2; f++) {
          const bool right = f == 0;
          PathScore ps = {0, lT, right ? lPR : lPL, L1, eb, right ? 1 : 0, wopen};
          int pen = 0;
          OpWriter ow = {ops + o0 + (right ? 0 : nR), right ? cap : cap - nR, 0, 0};
          // (the sweep starts at L1max, wave-uniform: the lanes' start rows are below)
          gw_traceback(S32(right ? GS_PR : GS_PL, 0), right ? WR : WL, eb, (right ? !JLL : JLL) ? 0xF : 0, L1,
                       right ? L2R : L2L, right ? 1 : 0, cdir, right ? brR : brL, right ? bcR : bcL, L1max,
                       [&](int r) -> uint32_t { return lT[(size_t)(right ? L1 - r : r - 1) * 64] >> 24; },
                       [&](int c) -> int { return ((right ? lPR : lPL)[(size_t)(c + eb) * 64] & 31) >> 2; }, t, ow,
                       ps, pen);
          const int nn = ow.n < ow.cap ? ow.n : ow.cap;
          over = over || ow.n > ow.cap;
          if (right) {
            nR = nn;
            sR = ps.s;
            penR = pen;
          } else {
            nL = nn;
            sL = ps.s;
            penL = pen;
          }
        }
        GW_T(10, tp);
        const int dl = bcL < L2L - 1 ? left_code((((int)lPL[(size_t)(bcL + eb) * 64] >> 5) & 31) / 6) : 0;
        const int dr = bcR < L2R - 1 ? right_code((((int)lPR[(size_t)(bcR + eb) * 64] >> 5) & 31) / 6) : 0;
        int it;
        const int sI = intron_score(it, dl, dr, cdir, canon, finalp);
        sL -= penL;
        sR -= penR;
        finalscore = halfp ? sL + sI + sR - sI / 2 : sL + sI + sR;
        rc = finalscore >= 0;
        GW_T(11, tp);
      }
      gsnapdp_ggap_result R;
      gsnapdp_ggap_trace X;
      memset(&R, 0, sizeof(R));
      memset(&X, 0, sizeof(X));
      R.dynprogindex = dpi;
      R.bridge_ok = 1;
      X.status = ST_OK;
      if (rc == -1) {
        R.bridge_ok = 0;
        R.returned_null = 1;
        R.finalscore = NEG;
      } else if (rc == 0) {
        R.finalscore = finalscore;
        R.returned_null = 1;
      } else {
        R.finalscore = finalscore;
        if (finalp) {  // :4104-4108: the columns below L2 - 1 were evaluated already
          if (bcL < L2L - 1 && bcR < L2R - 1) {
            R.left_prob = PL(bcL);
            R.right_prob = PR(bcR);
          } else {
            int wq = wi;
            asm volatile("" : "+v"(wq));
            const gsnapdp_ggap_window w3 = Wn[wq];
            R.left_prob = bcL < L2L - 1 ? PL(bcL) : left_site_prob(w3, bcL, blocks, nwords, tables);
            R.right_prob = bcR < L2R - 1 ? PR(bcR) : right_site_prob(w3, bcR, blocks, nwords, tables);
          }
        }
        R.new_leftgenomepos = o2L + (bcL - 1);
        R.new_rightgenomepos = r2R - (bcR - 1);
        R.exonhead = (off1 + L1 - 1) - (brR - 1);
        X.bridge_accepted = 1;
        X.brL = brL;
        X.bcL = bcL;
        X.brR = brR;
        X.bcR = bcR;
        X.nops_right = nR;
        X.nops_left = nL;
        if (over) X.status = ST_OPS_OVERFLOW;
        R.nmatches = t.nmatches;
        R.nmismatches = t.nmismatches;
        R.nopens = t.nopens;
        R.nindels = t.nindels;
        X.npairs = t.npush + 1;  // + the gapholder
        if (t.npush == 0) {      // only the gapholder: the list is dropped (:5050-5053)
          R.returned_null = 1;
          X.npairs = 0;
        }
        R.dynprogindex = step_dpi(dpi);
      }
      res[wi] = R;
      trc[wi] = X;
      GW_T(3, tp);
    }
  }
#ifdef GW_PROF
  if (lane == 0)
    for (int i = 0; i < 16; i++) atomicAdd(&gw_prof[i], (unsigned long long)gw_acc[i]);
#endif
}

}  // namespace

// Launch k_gwin over lists GW_LIST .. + GW_NSUB - 1 of a genome-gap batch
// (k_ggap_plan fills them only when the MaxEnt tables are loaded).
int gsnapdp__gwin_launch(gsnapdp_ctx* ctx, hipStream_t st, const gsnapdp_ggap_window* d_windows,
                         const int* lists, const int* counts, int list_cap, const char* d_query,
                         const char* d_query_uc, gsnapdp_ggap_result* d_results, gsnapdp_ggap_trace* d_traces,
                         uint32_t* d_ops, const int64_t* d_op_offsets) {
  const int blocks = ctx->num_cus * 2;
  const int waves = blocks * (GW_BLOCK / 64);
  if (!ctx->d_gwin_pool) HIPCHK(hipMalloc(&ctx->d_gwin_pool, (size_t)waves * GW_WAVE_DW * 4));
  // the site probabilities of up to list_cap windows (64 doubles each, by chunk)
  const size_t pcap = (((size_t)list_cap + 63) / 64 + GW_NSUB) * 4096;
  if (pcap > ctx->gwin_probs_cap) {
    (void)hipFree(ctx->d_gwin_probs);
    ctx->d_gwin_probs = nullptr;
    HIPCHK(hipMalloc(&ctx->d_gwin_probs, pcap * sizeof(double)));
    ctx->gwin_probs_cap = pcap;
  }
  hipLaunchKernelGGL(k_gwin_probs, dim3(ctx->num_cus), dim3(GP_THREADS), GP_LDS, st, d_windows, lists, list_cap,
                     counts + GW_LIST,
                     ctx->d_blocks, (uint64_t)ctx->nwords, ctx->d_tables, ctx->d_gwin_probs);
  hipLaunchKernelGGL(k_gwin, dim3(blocks), dim3(GW_BLOCK), (size_t)(GW_BLOCK / 64) * GW_LDS_WAVE, st, d_windows,
                     lists, list_cap, counts + GW_LIST, d_query, d_query_uc, ctx->d_blocks, (uint64_t)ctx->nwords,
                     ctx->d_prof, ctx->d_tables, ctx->d_gwin_pool, ctx->d_gwin_probs, d_results, d_traces, d_ops,
                     d_op_offsets);
  HIPCHK(hipGetLastError());
#ifdef GW_PROF
  {
    unsigned long long h[16];
    HIPCHK(hipStreamSynchronize(st));
    HIPCHK(hipMemcpyFromSymbol(h, HIP_SYMBOL(gw_prof), sizeof(h)));
    const double nt = h[7] ? (double)h[7] : 1.0;
    fprintf(stderr, "gw_prof tasks %llu cycles/task: setup %.0f fill1 %.0f fill2 %.0f fill3 %.0f select %.0f outcome %.0f\n",
            h[7], h[0] / nt, h[4] / nt, h[5] / nt, h[1] / nt, h[2] / nt, h[3] / nt);
    fprintf(stderr, "gw_prof detail: setup classes %.0f probs %.0f ranks %.0f | outcome reread %.0f rowsLDS %.0f trR %.0f trL %.0f score %.0f\n",
            h[14] / nt, h[13] / nt, h[12] / nt, h[6] / nt, h[8] / nt, h[9] / nt, h[10] / nt, h[11] / nt);
    memset(h, 0, sizeof(h));
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(gw_prof), h, sizeof(h)));
  }
#endif
  return 0;
}

int gsnapdp__gwin_lds_check(size_t max_lds) {
  return gsnapdp__lds_fits((const void*)&k_gwin, (size_t)(GW_BLOCK / 64) * GW_LDS_WAVE, max_lds, "k_gwin") ||
         gsnapdp__lds_fits((const void*)&k_gwin_probs, GP_LDS, max_lds, "k_gwin_probs");
}
