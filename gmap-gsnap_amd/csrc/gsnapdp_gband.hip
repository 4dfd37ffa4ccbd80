// gsnapdp_gband.hip -- Dynprog_genome_gap (reference src/dynprog.c:4798-5061)
// on the register band of k_fill, with bridge_intron_gap (:3290-4122) fused
// into the two flank fills.
//
// A genome-gap window is two banded Gotoh fills (the left flank forwards with
// jump_late_p, the right flank reversed with !jump_late_p, :4955-4990) and a
// bridge that picks the intron: for each split row rL (rR = L1 - rL) it scans
//   left loop:  HL(rL, cL) - pen + known(cL) + intronscore(leftdi[cL], rightdi[rR]) + DR(rR)
//   right loop: DL(rL) + intronscore(leftdi[rL], rightdi[cR]) + HR(rR, cR) - pen + known(cR)
// (DX(r) = HX(r, r) + known(r); pen = 1 when the cell's nogap came from a gap,
// :3715-3790), keeping the first maximum in the order (rL, loop, column).
// Inside one loop DR / DL is constant, so the bridge reduces per flank row to
// "the first column of the row with the largest partial score".  k_gband
// computes that in the fill itself: each cell packs its partial score and its
// column into one int (score << 10 | 1023 - column, so a larger int is a
// better or an earlier candidate) and each row keeps a running maximum that
// travels with the row through the band slots exactly like the gap1 value
// does.  The diagonal cells H(r, r) are written out as the fill passes them.
// After both fills, the combine step adds the other flank's diagonal to each
// row's best and takes the ordered argmax over (rL, loop): O(L1) per window
// instead of the reference's O(L1 x band) candidate scan.
//
// Everything else is k_fill's machinery (gsnapdp_band.h): the lane groups of
// S diagonals, the skewed wavefront, 16-bit offset scores, the LDS rings, the
// direction-bit scratch and the backward traceback sweep, run once per flank
// from the bridge's chosen cells.  Per-window bands are per lane here (k_fill
// buckets windows so that they are per wave); the tie rule is per wave (the
// window lists are split by jump_late_p).
//
// Scope: score mode with no IIT, reward-only known sites or site-level known
// sites (KNOWN_NONE / REWARD / SITES), flanks with length1 <= length2 <= 256
// and band width <= 48, and the intron span wide enough that the bridge's
// band is the fill band (:3720, :3760).  Every other window runs on k_ggap.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>

#include "gsnapdp_band.h"
#include "gsnapdp_ctx.h"
#include "gsnapdp_device.h"
#include "gsnapdp_ggap.h"
#include "gsnapdp_internal.h"

using namespace gsnapdp;

namespace {

constexpr int GB_EXT = -3;  // SINGLE_EXTEND == PAIRED_EXTEND: the profile folds -2*ext in
static_assert(SINGLE_EXTEND == GB_EXT && PAIRED_EXTEND == GB_EXT && -2 * GB_EXT == FILL_SC_BIAS,
              "k_gband's profile nibbles");
static_assert(FV_BIAS + 2 * PAIRED_OPEN > FV_NEG + 9u * (GB_L2MAX + 48) + 20 + 42,
              "reachable and NEG-like values stay apart with the paired open");
constexpr int GB_KEY_NONE = -(1 << 30);
constexpr int GB_PB = 8;  // rows per lane per batch of the combine
constexpr int GB_COLKEY = 1023;  // column part of a key: 1023 - c (c <= GB_L2MAX)

// per-wave scratch (dwords): the two flanks' direction words and match bytes,
// then per window group the column bytes, the row intron words, the row bests
// and the diagonal values of both flanks
constexpr int GB_COLS = GB_L2MAX + 4;   // the traceback reads whole 4-column groups
constexpr int GB_FLANK = GB_COLS * 80;  // D: 64 dwords per column, M: 64 bytes per column
constexpr int GB_RW = GB_L2MAX + 4;     // row entries of one window flank (rows 0 .. L1 <= 256)
constexpr int GB_NGMAX = 32;            // windows per wave (the classes with LPW >= 2)
constexpr int GB_CW = GB_COLS / 4 + 1;  // column bytes of one window flank, in dwords (8-byte rows)
constexpr int GB_OCI = 2 * GB_FLANK;
constexpr int GB_ORI = GB_OCI + 2 * GB_NGMAX * GB_CW;
constexpr int GB_ORB = GB_ORI + 2 * GB_NGMAX * GB_RW;
constexpr int GB_ODG = GB_ORB + 2 * GB_NGMAX * GB_RW;
// probability mode: each flank's cell values H - pen (16 bits, the fill's
// offset form), 8 per lane and column in the fill's lane order, then the site
// probabilities of each window's columns (doubles)
constexpr int GB_OCV = GB_ODG + 2 * GB_NGMAX * GB_RW;
constexpr int GB_CVF = GB_COLS * 256;
constexpr int GB_OPR = GB_OCV + 2 * GB_CVF;
// probability mode's row records, per window and flank row r: {threshold T(r),
// intron word, the partner row's site probability (a double)} for the bridge
// sweep, which overwrites each with the row's loop result {column, 0, sum}
constexpr int GB_OREC = GB_OPR + 2 * GB_NGMAX * GB_COLS * 2;
static_assert(GB_OREC + 2 * GB_NGMAX * GB_RW * 4 == GB_WAVE_DW && GB_OPR % 2 == 0 && GB_WAVE_DW % 4 == 0,
              "k_gband scratch layout");
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
enum { FL_RIGHT = 0, FL_LEFT = 1 };
#ifdef GB_CHECK
// diagnostic builds: bounds checks that record the first bad access instead of faulting
__device__ int gb_err[8];
__device__ inline uint32_t gb_chk(uint32_t idx, uint32_t lim, int site) {
  if (idx < lim) return idx;
  if (atomicCAS(&gb_err[0], 0, site) == 0) {
    gb_err[1] = (int)idx;
    gb_err[2] = (int)lim;
    gb_err[3] = (int)(threadIdx.x + 256 * blockIdx.x);
  }
  return 0;
}
#define GB_CHK(idx, lim, site) gb_chk((uint32_t)(idx), (uint32_t)(lim), site)
#else
#define GB_CHK(idx, lim, site) (idx)
#endif
#ifdef GB_PHASES
// diagnostic builds: run only the phases in GSNAPDP_GB_PHASES (bit 0 tables,
// 1 fills, 2 combine, 3 tracebacks; results are wrong when a phase is off)
__device__ int gb_phases;
#define GB_PH(b) (gb_phases & (1 << (b)))
#else
#define GB_PH(b) 1
#endif
#ifdef GB_PROF
// diagnostic builds: per-phase shader clocks summed over waves (tools/build_variant.sh)
__device__ unsigned long long gb_prof[8];
#define GB_TICK(k)                                                             \
  do {                                                                         \
    const uint64_t now_ = __builtin_amdgcn_s_memtime();                        \
    if ((threadIdx.x & 63) == 0) atomicAdd(&gb_prof[k], now_ - gb_t0);         \
    gb_t0 = now_;                                                              \
  } while (0)
#else
#define GB_TICK(k) \
  do {             \
  } while (0)
#endif

// LDS rings of one wave: k_fill's (row profile words, column bytes) plus the
// row intron words
// rows, the row intron words; staged K columns at a time, K a multiple of S so
// that only one position of the S-step unrolled column loop can stage
template <int S, int LPW>
struct GRings {
  static constexpr int K = (RING_K + S - 1) / S * S;
  static constexpr int NG = 64 / LPW;
  static constexpr int SPAN = (LPW - 1) * (S - 1);
  static constexpr int RR = pow2ceil(K + SPAN);
  static constexpr int CR = pow2ceil(K + LPW - 1);
  static constexpr int WORDS = 2 * NG * RR + (NG * CR + 3) / 4;
};
constexpr int GB_RING_WORDS = 2304;  // max GRings<S,LPW>::WORDS over the classes (checked below)

// Classes of columns c0 .. c0 + N - 1 of one flank (5 outside 1 .. L2):
// ColStream::cls on a run of consecutive genome positions, which touches at
// most two 32-nt blocks, from those two block triples.
constexpr int GB_RUN = 8;  // columns per lane per run of the per-window tables
template <int N>
__device__ inline void class_run(const ColStream& cs, const uint32_t* __restrict__ blocks,
                                 uint64_t nwords, int c0, int L2, int (&k)[N]) {
  static_assert(N <= 33, "a run spans at most two blocks");
  const uint32_t pfirst = cs.P0 + (uint32_t)(cs.PS * c0);
  const uint32_t plast = cs.P0 + (uint32_t)(cs.PS * (c0 + N - 1));
  const uint32_t b0 = (cs.PS > 0 ? pfirst : plast) >> 5;  // the run's lower block
  const uint64_t gmax = nwords >= 3 ? (nwords - 3) / 3 : 0;  // last whole block
  const uint64_t pa = ((uint64_t)b0 <= gmax ? (uint64_t)b0 : gmax) * 3u;
  const uint64_t pb = ((uint64_t)b0 + 1 <= gmax ? (uint64_t)b0 + 1 : gmax) * 3u;
  const uint32_t hi0 = blocks[pa], lo0 = blocks[pa + 1], fl0 = blocks[pa + 2];
  const uint32_t hi1 = blocks[pb], lo1 = blocks[pb + 1], fl1 = blocks[pb + 2];
#pragma unroll
  for (int i = 0; i < N; i++) {
    const int c = c0 + i;
    const uint32_t pos = cs.P0 + (uint32_t)(cs.PS * c);
    const uint32_t blk = pos >> 5, bit = pos & 31u;
    const bool second = blk != b0;
    const uint32_t word = bit < 16 ? (second ? lo1 : lo0) : (second ? hi1 : hi0);
    const uint32_t fl = second ? fl1 : fl0;
    const int code = (int)((word >> ((bit & 15u) * 2u)) & 3u) ^ cs.xorc;
    const bool ing = (uint64_t)blk <= gmax;  // outside the genome: N
    const bool inr = c >= cs.cvlo && c <= cs.cvhi;
    const int cl = !inr ? 5 : ((!ing || ((fl >> bit) & 1u)) ? 4 : code);
    k[i] = (c >= 1 && c <= L2) ? cl : 5;
  }
}

// dinucleotide codes: bits 3-5 of a column byte index these (0 = none)
__device__ inline int left_code(int di) {
  return di == LEFT_GT ? 1 : di == LEFT_GC ? 2 : di == LEFT_AT ? 3 : di == LEFT_CT ? 4 : 0;
}
__device__ inline int right_code(int di) {
  return di == RIGHT_AG ? 1 : di == RIGHT_AC ? 2 : di == RIGHT_GC ? 3 : di == RIGHT_AT ? 4 : 0;
}
__device__ inline int left_val(int k) {
  return k == 1 ? LEFT_GT : k == 2 ? LEFT_GC : k == 3 ? LEFT_AT : k == 4 ? LEFT_CT : 0;
}
__device__ inline int right_val(int k) {
  return k == 1 ? RIGHT_AG : k == 2 ? RIGHT_AC : k == 3 ? RIGHT_GC : k == 4 ? RIGHT_AT : 0;
}

// The fill of one flank over a wave's window groups (compute_scores_lookup_fwd
// / _rev, dynprog.c:1424-1736), with the bridge's per-row maxima.  k_fill's
// fill_group restated for per-lane bands; see gsnapdp_kernels.hip for the
// register layout, the offset scores and the band-edge argument.  JL is this
// flank's tie rule (jump_late_p for the left flank, its negation for the right).
//
// Not inlined: each flank fill gets its own register allocation.  The scratch,
// query and LDS bases are wave-uniform (SGPRs) and every per-lane access is a
// 32-bit offset from them, so no 64-bit per-lane pointer is kept live.
template <class T>
__device__ inline T* wave_uniform(T* p) {
  const uint64_t x = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(x >> 32));
  return (T*)(((uint64_t)hi << 32) | lo);
}
// dst = (lane's bit of m) ? b : a, with the lane mask in an SGPR pair (an explicit
// select: a chain of ternaries over a register array becomes an indexed
// scratch access)
__device__ inline uint32_t sel_mask(uint32_t a, uint32_t b, uint64_t m) {
  uint32_t d;
  asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "s"(m));
  return d;
}
// base[byte offset] with a 32-bit offset, so that a wave-uniform base stays in
// SGPRs (global_load / global_store with saddr)
template <class T>
__device__ inline T& at_b(T* base, uint32_t boff) {
  return *(T*)((char*)base + boff);
}

template <int S, int LPW, int JL, int FL, bool PM>
__device__ __noinline__ void gband_fill(int L1, int L2, int lband, int rband, int open, int mtoff,
                                        int qbase, int qstep, AS_GLOBAL uint32_t* wpool1,
                                        const AS_GLOBAL char* q1, const AS_GLOBAL char* qu1,
                                        const AS_LDS uint32_t* sprof3, AS_LDS uint32_t* ring3) {
  using RG = GRings<S, LPW>;
  static_assert(RG::WORDS <= GB_RING_WORDS, "LDS ring budget");
  constexpr int WMAX = S * LPW;
  constexpr int NG = 64 / LPW;
  const int lane = threadIdx.x & 63;
  const int j = lane % LPW;
  const int g = lane / LPW;
  const uint32_t* __restrict__ wpool = wave_uniform((uint32_t*)wpool1);
  const unsigned char* __restrict__ q = wave_uniform((const unsigned char*)q1);
  const unsigned char* __restrict__ qu = wave_uniform((const unsigned char*)qu1);
  const uint32_t* sprof = (const uint32_t*)sprof3;
  uint32_t* ring = (uint32_t*)ring3;
  uint32_t* __restrict__ D = (uint32_t*)wpool + (uint32_t)(FL * GB_FLANK);
  uint8_t* __restrict__ M = (uint8_t*)(D + GB_COLS * 64);
  u32x4* __restrict__ CV = (u32x4*)((uint32_t*)wpool + GB_OCV + FL * GB_CVF);
  // this group's tables and outputs: byte offsets from the wave's scratch
  const uint8_t* __restrict__ wb = (const uint8_t*)wpool;
  const uint32_t ci_b = 4u * (uint32_t)(GB_OCI + (FL * GB_NGMAX + g) * GB_CW);
  const uint32_t ri_b = 4u * (uint32_t)(GB_ORI + (FL * GB_NGMAX + g) * GB_RW);
  const uint32_t rb_b = 4u * (uint32_t)(GB_ORB + (FL * GB_NGMAX + g) * GB_RW);
  const uint32_t dg_b = 4u * (uint32_t)(GB_ODG + (FL * GB_NGMAX + g) * GB_RW);
  uint32_t* __restrict__ wout = (uint32_t*)wpool;
  const int stop = WMAX - (lband + rband + 1);
  const int maxL2 = __builtin_amdgcn_readfirstlane(wave_max(L2));
  const int row0 = j * S - stop - rband;  // row of local slot 0 at column 0
  // the diagonal cell H(c, c): global slot stop + rband, i.e. lane jd, slot sd
  const int gsd = stop + rband;
  const int jd = gsd / S, sd = gsd - jd * S;
  const bool dlane = j == jd;
  // loop-invariant lane masks (SGPR pairs): slot s holds the diagonal cell;
  // slot s lies above the band (its nogap is held at NEG, see k_fill)
  uint64_t dmask[S], amask[S];
#pragma unroll
  for (int s = 0; s < S; s++) {
    dmask[s] = __ballot(sd == s);
    amask[s] = __ballot(j * S + s < stop);
  }
  // per-lane step thresholds: column c = t - j is a bridge column while t < L2 + j;
  // lane 0's slot-0 row (row t - xr) leaves the band while xr + 1 <= t < xr + L1;
  // the diagonal lane writes H(c, c) while t < L1 + j
  const int t_ck = L2 + j;
  const int xr = j == 0 ? 1 + rband + stop : (1 << 28);
  const int t_dg = dlane ? L1 + j : -(1 << 28);
  const uint32_t nrx = (uint32_t)max(L1 - 1, 0);  // rows 1 .. L1-1 (none for a shadow group)

  auto row_word = [&](int r) -> uint32_t {
    uint32_t qb = 0u, ub = 255u;
    if (r >= 1 && r <= L1) {
      const uint32_t qi = (uint32_t)(qbase + qstep * (r - 1));
      qb = q[qi] & 127u;
      ub = qu[qi];
    }
    return sprof[mtoff + qb] | sprof[UTAB + ub];
  };

  FV H[S], E[S], F[S];
  uint32_t P[S], RI[S];
  int A[S];  // the row's best key so far
  const uint64_t* mlut = (const uint64_t*)(sprof + MLUT);
  constexpr uint64_t MB_KEEP = 0x0101010101ull * ((1u << (S - 1)) - 1u);
  auto row_spread = [&](uint32_t pw) -> uint64_t { return mlut[(pw >> 24) & 31u] >> (8 - S); };
  uint64_t MB = 0;
#pragma unroll
  for (int s = 0; s < S; s++) {
    const int r = row0 + s;
    H[s] = (r == 0) ? FV_BIAS : FV_NEG;
    E[s] = FV_NEG;
    F[s] = (r >= 1) ? FV_BIAS + open : FV_NEG;
    P[s] = row_word(r);
    if constexpr (!PM) RI[s] = (r >= 1 && r <= L1) ? at_b(wpool, ri_b + 4u * (uint32_t)r) : 0u;
    else RI[s] = 0u;
    A[s] = GB_KEY_NONE;
    MB = ((MB >> 1) & MB_KEEP) | row_spread(P[s]);
  }
  // rings (k_fill's staging, plus the row intron words)
  uint32_t* rr = ring + g * RG::RR;
  uint32_t* rri = ring + RG::NG * RG::RR + g * RG::RR;
  uint8_t* cr = (uint8_t*)(ring + 2 * RG::NG * RG::RR) + g * RG::CR;
  const int rbase = S - 1 - stop - rband;
  auto stage = [&](auto nrows_tag, int rlo, int clo) {
    constexpr int NR = decltype(nrows_tag)::value;
    constexpr int ER = (NR + LPW - 1) / LPW, EC = (RG::K + LPW - 1) / LPW;
    uint32_t qb[ER], ub[ER], iw[ER], cb[EC];
#pragma unroll
    for (int e = 0; e < ER; e++) {
      const int r = rlo + e * LPW + j;
      const int rc = (r >= 1 && r <= L1) ? r : 1;
      const uint32_t qi = (uint32_t)(qbase + qstep * (rc - 1));
      qb[e] = q[qi];
      ub[e] = qu[qi];
      if constexpr (!PM) iw[e] = at_b(wpool, ri_b + 4u * (uint32_t)((r >= 0 && r <= L1) ? r : 0));
    }
#pragma unroll
    for (int e = 0; e < EC; e++) {
      const int c = clo + e * LPW + j;
      cb[e] = wb[ci_b + (uint32_t)(c < 0 ? 0 : (c > L2 + 1 ? L2 + 1 : c))];
    }
#pragma unroll
    for (int e = 0; e < ER; e++) {
      const int r = rlo + e * LPW + j;
      const bool ok = r >= 1 && r <= L1;
      const uint32_t w = sprof[mtoff + (ok ? (qb[e] & 127u) : 0u)] | sprof[UTAB + (ok ? ub[e] : 255u)];
      if (e * LPW + j < NR) {
        rr[r & (RG::RR - 1)] = w;
        if constexpr (!PM) rri[r & (RG::RR - 1)] = ok ? iw[e] : 0u;
      }
    }
#pragma unroll
    for (int e = 0; e < EC; e++) {
      const int c = clo + e * LPW + j;
      if (e * LPW + j < RG::K) cr[c & (RG::CR - 1)] = (uint8_t)cb[e];
    }
    __builtin_amdgcn_s_waitcnt(0);
  };
  stage(std::integral_constant<int, RG::K + RG::SPAN>(), 1 + rbase, 1);
  uint32_t pnext = rr[(1 + j * (S - 1) + rbase) & (RG::RR - 1)];
  uint32_t inext = PM ? 0u : rri[(1 + j * (S - 1) + rbase) & (RG::RR - 1)];
  uint32_t gnext = cr[(1 - j) & (RG::CR - 1)];
  const uint32_t lane_off = (uint32_t)((LPW - 1 - j) * 64 + j * NG + g);
  // column part of a key: ((c * ext + known * 20) << 10) + 1023 - c, with
  // ext = -3; a jump-late flank's pen is 1 - (both signs set), its -1 rides here
  const int ck0 = GB_COLKEY + (JL ? -(1 << 10) : 0);

  // the unrolled position u of the rotating loop (which starts at t = LPW) whose
  // step can be a staging step
  constexpr int USTAGE = (S - LPW % S) % S;
  auto step = [&](auto masked, auto rot, int t) {
    constexpr bool MASKED = decltype(masked)::value;
    constexpr int ROT = decltype(rot)::value;
    constexpr bool MAYSTAGE = ROT < 0 || ROT == USTAGE;
    static_assert(!MASKED || ROT < 0, "rotating steps are full steps");
    auto pslot = [&](int s) -> uint32_t { return ROT < 0 ? P[s] : P[(s + ROT + 1) % S]; };
    auto islot = [&](int s) -> uint32_t { return ROT < 0 ? RI[s] : RI[(s + ROT + 1) % S]; };
    const int c = t - j;
    const bool act = !MASKED || (c >= 1 && c <= L2);
    FV hp = FV_NEG, fp = FV_NEG;
    if (LPW > 1) {
      const FV h = (FV)from_lane_above((int)H[S - 1]), f = (FV)from_lane_above((int)F[S - 1]);
      if (j != 0) {
        hp = h;
        fp = f;
      }
    }
    uint32_t av = 0u, ah = 0u, af = 0u, ae = 0u, gsh = 0u, csh = 0u;
    int ck = GB_KEY_NONE;
    uint32_t cv[S];  // probability mode: the cells' H - pen
    auto cell = [&](int s, FV Hr, FV Er, int Ar) {
      const FV Hd = H[s], Ed = E[s], Fd = F[s];
      const uint32_t pw = pslot(s);
      const FV a = Hr + open;
      const FV b = hp + open;
      const FV m1 = fv_max(Hd, Ed);
      const FV sc = (FV)__builtin_amdgcn_ubfe(pw, gsh, 4);
      const FV hn = sel_mask(fv_max(m1, Fd) + sc, FV_NEG, amask[s]);
      const int dv = JL ? (int)(Fd - m1) : (int)(m1 - Fd);
      const int dh = JL ? (int)(Ed - Hd) : (int)(Hd - Ed);
      const int df = JL ? (int)(fp - b) : (int)(b - fp);
      const int de = JL ? (int)(Er - a) : (int)(a - Er);
      av = push_sign(av, dv);
      ah = push_sign(ah, dh);
      af = push_sign(af, df);
      ae = push_sign(ae, de);
      if constexpr (PM) {
        // H - pen for the bridge scan; pen = the nogap came from gap1 or gap2 (dynprog.c:3723)
        const int npen = JL ? (int)((uint32_t)(dv & dh) >> 31) - 1 : ((dv | dh) >> 31);
        cv[s] = (uint32_t)((int)hn + npen);
      } else {
        // this cell as a bridge candidate: H - pen + intron score (+ column terms in
        // ck; a jump-late flank's -1 rides there)
        const int npen = JL ? (int)((uint32_t)(dv & dh) >> 31) : ((dv | dh) >> 31);
        const int sI = (int)__builtin_amdgcn_ubfe(islot(s), csh, 6);
        const int key = (((int)hn + sI + npen) << 10) + ck;
        A[s] = max(Ar, key);
      }
      E[s] = fv_max(a, Er);
      const FV f = fv_max(b, fp);
      F[s] = f;
      H[s] = hn;
      hp = hn;
      fp = f;
    };
    uint32_t macc = 0u;
    if (act) {
      if constexpr (ROT < 0) {
#pragma unroll
        for (int s = 0; s < S - 1; s++) {
          P[s] = P[s + 1];
          RI[s] = RI[s + 1];
        }
        P[S - 1] = pnext;
        RI[S - 1] = inext;
      } else {
        P[ROT] = pnext;
        RI[ROT] = inext;
      }
      MB = ((MB >> 1) & MB_KEEP) | row_spread(pnext);
      const uint32_t gc = gnext & 7u;
      gsh = 4u * gc;
      macc = (uint32_t)(MB >> (8u * gc));
      if constexpr (!PM) {
        csh = __builtin_amdgcn_ubfe(gnext, 3, 3) * 6u;
        // column L2 is not a bridge column (:3704, :3753)
        const int ckc = (int)((gnext & 64u) * 320u) + ck0 - __mul24(c, 3 * 1024 + 1);
        ck = t < t_ck ? ckc : GB_KEY_NONE;
        // the row leaving the band through lane 0's slot 0 (above the band for
        // `stop` columns already) is complete: slot 1's row overwrites it now
        const int r0 = t - xr;
        if ((uint32_t)(r0 - 1) < nrx) at_b(wout, rb_b + 4u * GB_CHK(r0, GB_RW, 2)) = (uint32_t)A[0];
      }
      cell(0, H[1], E[1], A[1]);
    }
    FV hb = FV_NEG, eb = FV_NEG;
    int ab = GB_KEY_NONE;
    if (LPW > 1) {
      const FV h = (FV)from_lane_below((int)H[0]), e = (FV)from_lane_below((int)E[0]);
      const int x = PM ? GB_KEY_NONE : from_lane_below(A[0]);
      if (j != LPW - 1) {
        hb = h;
        eb = e;
        ab = x;
      }
    }
    if (act) {
#pragma unroll
      for (int s = 1; s < S - 1; s++) cell(s, H[s + 1], E[s + 1], A[s + 1]);
      cell(S - 1, hb, eb, ab);
      const uint32_t acc = (((((av << S) | ah) << S) | af) << S) | ae;
      const uint32_t o = GB_CHK((uint32_t)(t - (LPW - 1)) * 64u + lane_off, GB_COLS * 64, 1);
      at_b(D, 4u * o) = acc;
      at_b(M, o) = (uint8_t)macc;
#ifdef GB_EXP_NOCV
      if constexpr (false) {  // ablation: no cell values (wrong results, timing only)
#else
      if constexpr (PM) {
#endif
        static_assert(S <= 8, "8 cell values per lane and column");
        uint32_t pk[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int s = 0; s < S; s++) pk[s >> 1] |= cv[s] << (16 * (s & 1));
        u32x4 x = {pk[0], pk[1], pk[2], pk[3]};
        at_b(CV, 16u * o) = x;
      }
      // the diagonal cell H(c, c) of this column, for the other flank's bridge loop
      uint32_t dv = H[0];
#pragma unroll
      for (int s = 1; s < S; s++) dv = sel_mask(dv, H[s], dmask[s]);
      if (t < t_dg) at_b(wout, dg_b + 4u * GB_CHK(c, GB_RW, 3)) = dv;
    }
    if (MAYSTAGE && t % RG::K == 0) stage(std::integral_constant<int, RG::K>(), t + 1 + rbase + RG::SPAN, t + 1);
    pnext = rr[(t + 1 + j * (S - 1) + rbase) & (RG::RR - 1)];
    if constexpr (!PM) inext = rri[(t + 1 + j * (S - 1) + rbase) & (RG::RR - 1)];
    gnext = cr[(t + 1 - j) & (RG::CR - 1)];
  };
  using Masked = std::integral_constant<bool, true>;
  using Full = std::integral_constant<bool, false>;
  using Shift = std::integral_constant<int, -1>;
  const int minL2 = __builtin_amdgcn_readfirstlane(-wave_max(L1 > 0 ? -L2 : -maxL2));
  int t = 1;
  for (; t < LPW && t < maxL2 + LPW; t++) step(Masked(), Shift(), t);
  for (; t + S - 1 <= minL2; t += S)
    unroll_seq(std::make_integer_sequence<int, S>(),
               [&](auto u) { step(Full(), u, t + decltype(u)::value); });
  for (; t <= minL2; t++) step(Full(), Shift(), t);
  for (; t < maxL2 + LPW; t++) step(Masked(), Shift(), t);
  // the rows still in the band at column L2
  if (!PM && L1 > 0) {
#pragma unroll
    for (int s = 0; s < S; s++) {
      const int r = L2 - rband + j * S + s - stop;
      if (r >= 1 && r < L1) at_b(wout, rb_b + 4u * GB_CHK(r, GB_RW, 4)) = (uint32_t)A[s];
    }
  }
}


// Probability mode's bridge loops over one flank (bridge_intron_gap
// :3905-4041), after both fills: for every flank row r, the first column c of
// its band (c ascending, the reference's order) with the largest
// probC(c) + probOther(r) among the cells whose score reaches score_threshold,
//   H(r, c) - pen + known(c) + intronscore + D_other(L1 - r) >= threshold,
// i.e. v + c * ext + known(c) * 20 + sI(code(c), word(r)) >= T(r) on the fill's
// 16-bit cell values v.  The sweep visits the columns in order with the fill's
// lane layout: a lane reads back its own cell values of column c (one coalesced
// 16-byte load per lane), slot s holds row row0 + s + c, and each row's best so
// far moves down one slot per column and from lane j + 1 to lane j, like the
// fill's gap values.  A row's result replaces its record when it leaves the
// band (lane 0, slot 0) or at the end.
template <int S, int LPW, int FL>
__device__ __noinline__ void gband_sweep(int L1, int L2, int lband, int rband, AS_GLOBAL uint32_t* wpool1) {
  constexpr int WMAX = S * LPW;
  constexpr int NG = 64 / LPW;
  const int lane = threadIdx.x & 63;
  const int j = lane % LPW;
  const int g = lane / LPW;
  uint32_t* __restrict__ wpool = wave_uniform((uint32_t*)wpool1);
  const u32x4* __restrict__ CV = (const u32x4*)(wpool + GB_OCV + FL * GB_CVF);
  u32x4* __restrict__ rec = (u32x4*)(wpool + GB_OREC + 4 * (FL * GB_NGMAX + g) * GB_RW);
  const double* __restrict__ prc = (const double*)(wpool + GB_OPR + 2 * (FL * GB_NGMAX + g) * GB_COLS);
  const uint8_t* __restrict__ cib = (const uint8_t*)(wpool + GB_OCI + (FL * GB_NGMAX + g) * GB_CW);
  const int stop = WMAX - (lband + rband + 1);
  const int row0 = j * S - stop - rband;
  const int cend = __builtin_amdgcn_readfirstlane(wave_max(L1 > 0 ? L2 : 0)) - 1;  // bridge columns 1 .. L2 - 1
  int T[S], bc[S];
  uint32_t Wd[S];
  double pO[S], bs[S];
  bool inb[S];
  auto load_row = [&](int r, int& t, uint32_t& w, double& po) {
    const bool ok = r >= 1 && r < L1;
    const u32x4 x = rec[GB_CHK(ok ? r : 0, GB_RW, 22)];
    t = ok ? (int)x.x : 0x7fffffff;
    w = x.y;
    po = __hiloint2double((int)x.w, (int)x.z);
  };
  auto put_row = [&](int r, int c, double sum) {
    if (r >= 1 && r < L1) {
      u32x4 x = {(uint32_t)c, 0u, (uint32_t)__double2loint(sum), (uint32_t)__double2hiint(sum)};
      rec[GB_CHK(r, GB_RW, 23)] = x;
    }
  };
  // The loads of step c (the lane's cell values of column c, the record of the
  // row entering slot S - 1, the column's probability and byte) are issued S
  // steps ahead of their use.  No register moves with the rows: logical slot s
  // at column c lives in register (s + c) % S, so the loop runs S columns per
  // iteration with every index a constant (column c = 1 + kS + u: slot s in
  // register (s + 1 + u) % S; the row leaving slot 0 and the one entering slot
  // S - 1 share register u).
  struct Pre {
    u32x4 e, r;
    double pc;
    uint32_t cb;
  };
  auto issue = [&](int c, Pre& q) {
    const int cl = c <= cend ? c : cend;
    q.e = CV[GB_CHK(cl * 64 + j * NG + g, GB_COLS * 64, 24)];
    const int r = row0 + S - 1 + c;
    q.r = rec[GB_CHK(r >= 1 && r < L1 ? r : 0, GB_RW, 22)];
    const int cc = c <= L2 - 1 ? c : 0;
    q.pc = c <= L2 - 1 ? prc[cc] : -2.0;  // past the window's bridge columns: never a candidate
    q.cb = cib[cc];
  };
  auto step = [&](auto ut, int c, const Pre& q) {
    constexpr int U = decltype(ut)::value;
    if (c > 1) {
      // the row in slot 0 moves to lane j - 1 (lane 0: it leaves the band, complete)
      if (j == 0) put_row(row0 + c - 1, bc[U], bs[U]);
      const int ilo = from_lane_below(__double2loint(bs[U])), ihi = from_lane_below(__double2hiint(bs[U]));
      const int icc = from_lane_below(bc[U]);
      const bool top = j == LPW - 1;
      bs[U] = top ? 0.0 : __hiloint2double(ihi, ilo);
      bc[U] = top ? -1 : icc;
      const int r = row0 + S - 1 + c;
      T[U] = r >= 1 && r < L1 ? (int)q.r.x : 0x7fffffff;
      Wd[U] = q.r.y;
      pO[U] = __hiloint2double((int)q.r.w, (int)q.r.z);
    }
    const int colt = c * GB_EXT + (int)((q.cb >> 6) & 1u) * KNOWN_REWARD;
    const uint32_t csh = ((q.cb >> 3) & 7u) * 6u;
#pragma unroll
    for (int s = 0; s < S; s++) {
      const int p = (s + 1 + U) % S;
      const uint32_t word = s < 2 ? q.e.x : s < 4 ? q.e.y : s < 6 ? q.e.z : q.e.w;
      const int v = (int)((word >> (16 * (s & 1))) & 0xffffu);
      const int sI = (int)__builtin_amdgcn_ubfe(Wd[p], csh, 6);
      const double sum = q.pc + pO[p];
      const bool take = inb[s] && v + colt + sI >= T[p] && sum > bs[p];
      bs[p] = take ? sum : bs[p];
      bc[p] = take ? c : bc[p];
    }
  };
#pragma unroll
  for (int s = 0; s < S; s++) {
    const int p = (s + 1) % S;
    inb[s] = j * S + s >= stop;
    load_row(row0 + s + 1, T[p], Wd[p], pO[p]);
    bs[p] = 0.0;  // bestprob starts at 0.0 (:3905): a row's sum must exceed it
    bc[p] = -1;
  }
  Pre pq[S];
#pragma unroll
  for (int d = 0; d < S; d++) issue(1 + d, pq[d]);
  for (int c = 1; c <= cend; c += S) {
    unroll_seq(std::make_integer_sequence<int, S>(), [&](auto ut) {
      constexpr int U = decltype(ut)::value;
      if (c + U <= cend) step(ut, c + U, pq[U]);
      issue(c + U + S, pq[U]);
    });
  }
  // the rows still in the band after the last column cl: register p holds
  // logical slot (p - cl) mod S
  const int cl = max(cend, 1);
#pragma unroll
  for (int p = 0; p < S; p++) {
    const int sl = ((p - cl) % S + S) % S;
    put_row(row0 + sl + cl, bc[p], bs[p]);
  }
}

struct GCand {  // a bridge candidate: total score, scan order 2*rL + loop, the two cells' columns
  int score, key, cL, cR;
};

// One wave-task of NG windows.  Not inlined (the same code for both tie
// rules); the LDS pointers keep their address space through the call.
#ifdef GB_INLINE
#define GB_GROUP_ATTR __attribute__((always_inline)) inline  // diagnostic builds
#else
#define GB_GROUP_ATTR __noinline__
#endif
template <int S, int LPW, int JL, bool PM>
__device__ GB_GROUP_ATTR void gband_group(const AS_GLOBAL gsnapdp_ggap_window* Wn1, int wi,
                                         bool active, int lane, AS_GLOBAL uint32_t* wpool1,
                                         const AS_GLOBAL char* q1, const AS_GLOBAL char* qu1,
                                         const AS_GLOBAL uint32_t* blocks1, uint64_t nwords,
                                         const AS_LDS uint32_t* sprof, AS_LDS uint32_t* ring,
                                         const AS_GLOBAL double* tables1,
                                         AS_GLOBAL gsnapdp_ggap_result* res1,
                                         AS_GLOBAL gsnapdp_ggap_trace* trc1,
                                         AS_GLOBAL uint32_t* ops1,
                                         const AS_GLOBAL int64_t* op_off1) {
  // address-space-qualified parameters: the tables, combine and tracebacks
  // compile to global_* accesses (generic pointers made them flat_*, each use
  // a full vmcnt(0) lgkmcnt(0) drain)
  const gsnapdp_ggap_window* __restrict__ Wn = (const gsnapdp_ggap_window*)Wn1;
  uint32_t* __restrict__ wpool = (uint32_t*)wpool1;
  const char* __restrict__ q = (const char*)q1;
  const char* __restrict__ qu = (const char*)qu1;
  const uint32_t* __restrict__ blocks = (const uint32_t*)blocks1;
  const double* __restrict__ tables = (const double*)tables1;
  gsnapdp_ggap_result* __restrict__ res = (gsnapdp_ggap_result*)res1;
  gsnapdp_ggap_trace* __restrict__ trc = (gsnapdp_ggap_trace*)trc1;
  uint32_t* __restrict__ ops = (uint32_t*)ops1;
  const int64_t* __restrict__ op_off = (const int64_t*)op_off1;
  constexpr int NG = 64 / LPW;
  static_assert(NG <= GB_NGMAX, "k_gband groups");
  const int j = lane % LPW, g = lane / LPW;
#ifdef GB_PROF
  uint64_t gb_t0 = __builtin_amdgcn_s_memtime();
#endif
  const gsnapdp_ggap_window w = Wn[wi];
  GGeo G = gg_geo(w);
  if (!active) G.L1 = G.L2L = G.L2R = 0;
  const int L1 = G.L1;
  const int km = active ? w.known_mode : GSNAPDP_KNOWN_NONE;
  const unsigned char* krec = (const unsigned char*)q + w.qpos + L1;
  Lane LL = side_lane(w, G, 0), LR = side_lane(w, G, 1);
  // a shadow group (L1 = 0) still stages query row 1 (its loads are clamped,
  // not skipped): keep that address inside the buffer (the right flank's
  // qpos + L1 - 1 would be qpos - 1)
  if (!active) LR.qbase = LL.qbase = (int)w.qpos;
  uint8_t* ci[2];
  uint32_t* ri[2];
  int* rb[2];
  uint32_t* dg[2];
  double* pr[2];  // probability mode: the site probabilities of the window's columns
#pragma unroll
  for (int f = 0; f < 2; f++) {
    pr[f] = (double*)(wpool + GB_OPR + 2 * (f * GB_NGMAX + g) * GB_COLS);
    ci[f] = (uint8_t*)(wpool + GB_OCI + (f * GB_NGMAX + g) * GB_CW);
    ri[f] = wpool + GB_ORI + (f * GB_NGMAX + g) * GB_RW;
    rb[f] = (int*)(wpool + GB_ORB + (f * GB_NGMAX + g) * GB_RW);
    dg[f] = wpool + GB_ODG + (f * GB_NGMAX + g) * GB_RW;
  }
  ColStream csR, csL;
  csR.init(LR);
  csL.init(LL);
  // intron_score (:3148-3192) tabulated per window: sL[k] = the left flank's
  // row word (6 bits per left code) against right code k, sR[k] the right
  // flank's against left code k
  uint32_t sL[5], sR[5];
#pragma unroll
  for (int k = 0; k < 5; k++) {
    sL[k] = sR[k] = 0u;
#pragma unroll
    for (int m = 1; m <= 4; m++) {
      int it;
      sL[k] |= (uint32_t)intron_score(it, left_val(m), right_val(k), w.cdna_direction, G.canon, w.finalp) << (6 * m);
      sR[k] |= (uint32_t)intron_score(it, left_val(k), right_val(m), w.cdna_direction, G.canon, w.finalp) << (6 * m);
    }
  }
  // ---- per-window tables in the wave's scratch, read by the fills' ring
  // staging.  Lane j takes runs of GB_RUN consecutive columns (run j, j + LPW,
  // ...) and decodes each flank's classes (get_genomic_nt, :403-441) for the
  // run plus two columns of look-ahead from the two block triples that hold
  // them; from those come each column's byte: class | dinucleotide code << 3 |
  // known << 6 (:3331-3550).  Row r's bridge partner is column L1 - r of the
  // other flank, so the lane also writes the intron-score words of the rows
  // whose partners fall in its run.
  const int L2f[2] = {G.L2R, G.L2L};
#ifdef GB_EXP_NOPRE
  const int cmaxw = -1;  // ablation: no per-window tables (wrong results, timing only)
#else
  const int cmaxw = GB_PH(0) ? __builtin_amdgcn_readfirstlane(wave_max(max(G.L2L, G.L2R) + 1)) : -1;
#endif
  for (int cb = GB_RUN * j; cb <= cmaxw; cb += GB_RUN * LPW) {
    int code[2][GB_RUN];
#pragma unroll
    for (int f = 0; f < 2; f++) {
      const int L2 = L2f[f];
      int k[GB_RUN + 2];
      class_run(f == FL_RIGHT ? csR : csL, blocks, nwords, cb, L2, k);
      const unsigned char* kf = krec + (f == FL_RIGHT ? G.L2L : 0);
      uint64_t packed = 0;
#pragma unroll
      for (int i = 0; i < GB_RUN; i++) {
        const int c = cb + i;
        int cd = 0;
        if (c < L2 - 1) cd = f == FL_LEFT ? left_code(left_di(k[i + 1], k[i + 2])) : right_code(right_di(k[i + 2], k[i + 1]));
        const int known = (km != GSNAPDP_KNOWN_NONE && c < L2 && kf[c] != 0) ? 1 : 0;
        code[f][i] = cd;
        packed |= (uint64_t)(k[i] | cd << 3 | known << 6) << (8 * i);
      }
      if (cb <= L2 + 1) *(uint64_t*)(ci[f] + GB_CHK(cb, GB_CW * 4 - 7, 5)) = packed;  // bytes past L2 + 1 are never read
      if constexpr (PM) {
        // :3856-3903: a known site has probability 1.0, column L2 - 1 none (calloc)
        if (tables != nullptr && cb < L2) {
          int m, step;
          uint32_t sp0;
          site_line(w, f == FL_RIGHT, m, sp0, step);
          uint32_t sp[GB_RUN];
          bool ok[GB_RUN], kn[GB_RUN];
          double pv[GB_RUN];
#pragma unroll
          for (int i = 0; i < GB_RUN; i++) {
            const int c = cb + i;
            kn[i] = c < L2 - 1 && km != GSNAPDP_KNOWN_NONE && kf[c] != 0;
            ok[i] = c < L2 - 1 && !kn[i];
            sp[i] = sp0 + (uint32_t)(step * c);
          }
          maxent_probs<GB_RUN>(m, sp, ok, w.chroffset, blocks, nwords, tables, pv);
#pragma unroll
          for (int i = 0; i < GB_RUN; i++) {
            const int c = cb + i;
            if (c < L2) pr[f][GB_CHK(c, GB_COLS, 18)] = kn[i] ? 1.0 : pv[i];  // column L2 - 1: 0.0
          }
        }
      }
    }
#pragma unroll
    for (int i = 0; i < GB_RUN; i++) {
      const int r = L1 - (cb + i);  // the row whose partner is column cb + i
      if (r >= 0) {
        const bool inner = r >= 1 && r < L1;
        const int cR = code[FL_RIGHT][i], cL = code[FL_LEFT][i];
        ri[FL_LEFT][GB_CHK(r, GB_RW, 6)] = inner ? (cR == 1 ? sL[1] : cR == 2 ? sL[2] : cR == 3 ? sL[3] : cR == 4 ? sL[4] : sL[0]) : 0u;
        ri[FL_RIGHT][GB_CHK(r, GB_RW, 15)] = inner ? (cL == 1 ? sR[1] : cL == 2 ? sR[2] : cL == 3 ? sR[3] : cL == 4 ? sR[4] : sR[0]) : 0u;
      }
    }
  }
  wave_fence();
  const int rmaxw = __builtin_amdgcn_readfirstlane(wave_max(L1));
  GB_TICK(0);
  // ---- the two fills: right flank reversed with !jump_late_p, left forwards
  uint32_t* Dr = wpool + FL_RIGHT * GB_FLANK;
  uint32_t* Dl = wpool + FL_LEFT * GB_FLANK;
  uint8_t* Mr = (uint8_t*)(Dr + GB_COLS * 64);
  uint8_t* Ml = (uint8_t*)(Dl + GB_COLS * 64);
#ifndef GB_EXP_NOFILL
  if (GB_PH(1)) {
  gband_fill<S, LPW, 1 - JL, FL_RIGHT, PM>(L1, G.L2R, G.lbR, G.rbR, G.open, G.mt * 128, LR.qbase, LR.qstep,
                                       (AS_GLOBAL uint32_t*)wpool, (const AS_GLOBAL char*)q,
                                       (const AS_GLOBAL char*)qu, sprof, ring);
  GB_TICK(1);
  gband_fill<S, LPW, JL, FL_LEFT, PM>(L1, G.L2L, G.lbL, G.rbL, G.open, G.mt * 128, LL.qbase, LL.qstep,
                                  (AS_GLOBAL uint32_t*)wpool, (const AS_GLOBAL char*)q,
                                  (const AS_GLOBAL char*)qu, sprof, ring);
  }
#endif
  wave_fence();

  GB_TICK(2);
  // ---- combine (bridge_intron_gap's scan order, :3698-4081): per split row,
  // the left loop's best plus DR, then DL plus the right loop's best
  GCand best = {BRIDGE_INIT, 0x7fffffff, 0, 0};
  const int bias = (int)FV_BIAS;
  // probability mode: a flank cell's H - pen (dynprog.c:3723) from the fill's
  // cell values (lane jj = G / S, slot G % S of column c, G = r - c + WMAX - 1 - lband)
  auto cellv = [&](int f, int r, int c) -> int {
    const int lb = f == FL_LEFT ? G.lbL : G.lbR;
    const int gs = r - c + S * LPW - 1 - lb;
    const int jj = gs / S, sl = gs - jj * S;
    const uint32_t wd = wpool[GB_OCV + f * GB_CVF + GB_CHK(4 * (c * 64 + jj * NG + g) + (sl >> 1), GB_CVF, 19)];
    return (int)((wd >> (16 * (sl & 1))) & 0xffffu) - bias + (r + c) * GB_EXT;
  };
  double pbest = 0.0;  // probability mode: bestprob (:3905)
  if constexpr (PM) {
    // bridge_intron_gap's probability mode (:3905-4041): the row records, the
    // two flank sweeps (gband_sweep), then the ordered argmax over (rL, loop)
    int thr_i = wi;
    asm volatile("" : "+v"(thr_i));
    const int thr = Wn[thr_i].score_threshold;
    for (int r = 1 + j; r < (GB_PH(2) ? rmaxw : 0); r += LPW) {
      if (r >= L1) continue;
      const int rp = L1 - r;  // the partner row of the other flank
      const int npl = km != GSNAPDP_KNOWN_NONE ? krec[rp] : 0, npr = km != GSNAPDP_KNOWN_NONE ? krec[G.L2L + rp] : 0;
      // D_other of the partner: H(rp, rp) + known(rp) (:3727, :3767)
      const int DRp = ((int)dg[FL_RIGHT][GB_CHK(rp, GB_RW, 20)] - bias) + 2 * rp * GB_EXT + (npr != 0 ? KNOWN_REWARD : 0);
      const int DLp = ((int)dg[FL_LEFT][GB_CHK(rp, GB_RW, 21)] - bias) + 2 * rp * GB_EXT + (npl != 0 ? KNOWN_REWARD : 0);
      const double pRp = rp < G.L2R - 1 ? pr[FL_RIGHT][rp] : 0.0;
      const double pLp = rp < G.L2L - 1 ? pr[FL_LEFT][rp] : 0.0;
      u32x4 xl = {(uint32_t)(thr - DRp + bias - r * GB_EXT), ri[FL_LEFT][r], (uint32_t)__double2loint(pRp),
                  (uint32_t)__double2hiint(pRp)};
      u32x4 xr = {(uint32_t)(thr - DLp + bias - r * GB_EXT), ri[FL_RIGHT][r], (uint32_t)__double2loint(pLp),
                  (uint32_t)__double2hiint(pLp)};
      *(u32x4*)(wpool + GB_OREC + 4 * ((FL_LEFT * GB_NGMAX + g) * GB_RW + r)) = xl;
      *(u32x4*)(wpool + GB_OREC + 4 * ((FL_RIGHT * GB_NGMAX + g) * GB_RW + r)) = xr;
    }
    wave_fence();
    if (GB_PH(2)) {
      gband_sweep<S, LPW, FL_LEFT>(L1, G.L2L, G.lbL, G.rbL, (AS_GLOBAL uint32_t*)wpool);
      gband_sweep<S, LPW, FL_RIGHT>(L1, G.L2R, G.lbR, G.rbR, (AS_GLOBAL uint32_t*)wpool);
    }
    wave_fence();
    for (int rL = 1 + j; rL < (GB_PH(2) ? rmaxw : 0); rL += LPW) {
      if (rL >= L1) continue;
      const int rR = L1 - rL;
      const u32x4 xl = *(const u32x4*)(wpool + GB_OREC + 4 * ((FL_LEFT * GB_NGMAX + g) * GB_RW + rL));
      const u32x4 xr = *(const u32x4*)(wpool + GB_OREC + 4 * ((FL_RIGHT * GB_NGMAX + g) * GB_RW + rR));
      const double sl = __hiloint2double((int)xl.w, (int)xl.z), sr = __hiloint2double((int)xr.w, (int)xr.z);
      if (sl > pbest) {  // left loop of row rL (cR = rR)
        pbest = sl;
        best.key = 2 * rL;
        best.cL = (int)xl.x;
        best.cR = rR;
      }
      if (sr > pbest) {  // right loop (cL = rL)
        pbest = sr;
        best.key = 2 * rL + 1;
        best.cL = rL;
        best.cR = (int)xr.x;
      }
    }
#pragma unroll
    for (int o = LPW / 2; o > 0; o >>= 1) {
      const double xp = __shfl_xor(pbest, o);
      const int xk = __shfl_xor(best.key, o), xl = __shfl_xor(best.cL, o), xr = __shfl_xor(best.cR, o);
      if (xp > pbest || (xp == pbest && xk < best.key)) {
        pbest = xp;
        best.key = xk;
        best.cL = xl;
        best.cR = xr;
      }
    }
  }
  for (int r0 = 1; r0 < (!PM && GB_PH(2) ? rmaxw : 0); r0 += GB_PB * LPW) {
    int kl[GB_PB], kr[GB_PB], hl[GB_PB], hr[GB_PB], nl[GB_PB], nr[GB_PB];
#pragma unroll
    for (int e = 0; e < GB_PB; e++) {
      const int rL = r0 + e * LPW + j;
      const int rLc = rL < L1 ? rL : 1, rRc = max(0, L1 - rLc);
      kl[e] = rb[FL_LEFT][GB_CHK(rLc, GB_RW, 7)];
      kr[e] = rb[FL_RIGHT][GB_CHK(rRc, GB_RW, 8)];
      hl[e] = (int)dg[FL_LEFT][GB_CHK(rLc, GB_RW, 16)];
      hr[e] = (int)dg[FL_RIGHT][GB_CHK(rRc, GB_RW, 17)];
      nl[e] = km != GSNAPDP_KNOWN_NONE ? krec[rLc] : 0;  // left_known[rL], right_known[rR]
      nr[e] = km != GSNAPDP_KNOWN_NONE ? krec[G.L2L + rRc] : 0;
    }
#pragma unroll
    for (int e = 0; e < GB_PB; e++) {
      const int rL = r0 + e * LPW + j, rR = L1 - rL;
      if (rL >= L1) continue;
      const int DR = (hr[e] - bias) + 2 * rR * GB_EXT + (nr[e] != 0 ? KNOWN_REWARD : 0);
      const int DL = (hl[e] - bias) + 2 * rL * GB_EXT + (nl[e] != 0 ? KNOWN_REWARD : 0);
      const int totL = (kl[e] >> 10) - bias + rL * GB_EXT + DR;
      const int totR = DL + (kr[e] >> 10) - bias + rR * GB_EXT;
      if (totL > best.score) best = {totL, 2 * rL, GB_COLKEY - (kl[e] & 1023), rR};
      if (totR > best.score) best = {totR, 2 * rL + 1, rL, GB_COLKEY - (kr[e] & 1023)};
    }
  }
#pragma unroll
  for (int o = PM ? 0 : LPW / 2; o > 0; o >>= 1) {
    GCand x;
    x.score = __shfl_xor(best.score, o);
    x.key = __shfl_xor(best.key, o);
    x.cL = __shfl_xor(best.cL, o);
    x.cR = __shfl_xor(best.cR, o);
    if (x.score > best.score || (x.score == best.score && x.key < best.key)) best = x;
  }
  const int rLb = best.key >> 1, rRb = L1 - rLb;

  // ---- outcome (:4084-4108) on the group leader
  gsnapdp_ggap_result R;
  gsnapdp_ggap_trace X;
  memset(&R, 0, sizeof(R));
  memset(&X, 0, sizeof(X));
  int rc = 0;
  const bool lead = active && j == 0;
  // The outcome re-reads the window record instead of keeping the fields it
  // needs live across both fills (the laundered index defeats CSE with the
  // first load).  Round 3: with gband_group inlined, a build kept offset2L
  // live across the fills and traceback and stored a corrupted value for
  // jump-late windows (DESIGN.md §4 k_gband); the short live range removes
  // that exposure in every build.
  int wo_i = wi;
  asm volatile("" : "+v"(wo_i));
  const gsnapdp_ggap_window wo = Wn[wo_i];
  if (lead) {
    R.dynprogindex = wo.dynprogindex;
    R.bridge_ok = 1;
    X.status = ST_OK;
    // the chosen columns' dinucleotides and known flags (:3331-3550)
    const int cL = best.cL, cR = best.cR;
    const int dl = cL < G.L2L - 1 ? left_di(csL.cls(blocks, nwords, cL + 1), csL.cls(blocks, nwords, cL + 2)) : 0;
    const int dr = cR < G.L2R - 1 ? right_di(csR.cls(blocks, nwords, cR + 2), csR.cls(blocks, nwords, cR + 1)) : 0;
    const bool kL = km != GSNAPDP_KNOWN_NONE && cL < G.L2L && krec[cL] != 0;
    const bool kR = km != GSNAPDP_KNOWN_NONE && cR < G.L2R && krec[G.L2L + cR] != 0;
    int it;
    const int sI = intron_score(it, dl, dr, wo.cdna_direction, G.canon, wo.finalp);
    int finalscore = 0;
    if constexpr (PM) {
      // :4043-4068: the chosen cells' scores, both with their pen
      if (!(pbest > 0.0)) {
        rc = -1;  // no candidate: the reference reads uninitialised indices (:4055)
      } else {
        const int sL = cellv(FL_LEFT, rLb, cL) + (kL ? KNOWN_REWARD : 0);
        const int sR = cellv(FL_RIGHT, rRb, cR) + (kR ? KNOWN_REWARD : 0);
        finalscore = wo.halfp ? sL + sI + sR - sI / 2 : sL + sI + sR;
        rc = finalscore >= 0 ? 1 : 0;
      }
    } else {
      finalscore = wo.halfp ? best.score - sI / 2 : best.score;
      R.introntype = best.score > BRIDGE_INIT ? it : 0;
      rc = finalscore >= 0 ? 1 : 0;
    }
    // novel splicing off with a site-level IIT: both chosen sites must be known (:4090-4096)
    if (rc == 1 && km == GSNAPDP_KNOWN_SITES)
      rc = kL && kR;
    if ((PM || wo.finalp) && tables == nullptr) rc = -2;
    if (rc == -2) {
      X.status = ST_UNSUPPORTED;
      R.returned_null = 1;
      R.finalscore = NEG;
    } else if (rc == -1) {
      R.bridge_ok = 0;
      R.returned_null = 1;
      R.finalscore = NEG;
    } else {
      R.finalscore = finalscore;
      R.returned_null = rc == 0;
    }
    // guard: the chosen cells lie inside both flanks (a violated invariant is
    // reported, never traced: the sweep's loads are bounded by these columns)
    if (rc == 1 && ((uint32_t)cL > (uint32_t)G.L2L || (uint32_t)cR > (uint32_t)G.L2R ||
                    (uint32_t)rLb > (uint32_t)L1)) {
      X.status = ST_INTERNAL;
      rc = -3;
    }
    if (rc == 1) {
      if (wo.finalp) {  // :4104-4108 (a known site has probability 1.0, :3215, :3255)
        // probability mode's tables hold these sites already (the same model at the
        // same position, columns below L2 - 1)
        R.left_prob = kL ? 1.0 : (PM && cL < G.L2L - 1) ? pr[FL_LEFT][cL] : left_site_prob(wo, cL, blocks, nwords, tables);
        R.right_prob =
            kR ? 1.0 : (PM && cR < G.L2R - 1) ? pr[FL_RIGHT][cR] : right_site_prob(wo, cR, blocks, nwords, tables);
      }
      R.new_leftgenomepos = wo.offset2L + (best.cL - 1);
      R.new_rightgenomepos = wo.revoffset2R - (best.cR - 1);
      R.exonhead = (wo.offset1 + L1 - 1) - (rRb - 1);
      X.bridge_accepted = 1;
      X.brL = rLb;
      X.bcL = best.cL;
      X.brR = rRb;
      X.bcR = best.cR;
    }
  }
  // ---- the two tracebacks (right flank, the gapholder, then the left flank,
  // :5000-5040), each a backward sweep over its flank's scratch
  GB_TICK(3);
  const bool tr = lead && rc == 1;
#ifdef GB_CHECK
  if (tr) {
    best.cR = (int)GB_CHK(best.cR, GB_COLS - 3, 9);
    best.cL = (int)GB_CHK(best.cL, GB_COLS - 3, 10);
    GB_CHK(rLb, (uint32_t)L1 + 1, 11);
    GB_CHK(rRb, (uint32_t)L1 + 1, 12);
  }
#endif
  const int maxCR = __builtin_amdgcn_readfirstlane(wave_max(tr ? best.cR : 0));
  const int maxCL = __builtin_amdgcn_readfirstlane(wave_max(tr ? best.cL : 0));
#ifdef GB_PROF
  if (!lead) {
    GB_TICK(5);
    return;
  }
#else
  if (!lead) return;
#endif
#if defined(GB_EXP_NOTRACE) || defined(GB_EXP_NOFILL)
  if (false) {
#else
  if (tr && GB_PH(3)) {
#endif
    const int64_t o0 = op_off[wi];
    const int cap = (int)(op_off[wi + 1] - o0);
    Tally t = {0, 0, 0, 0, 0};
    OpWriter owR = {ops + o0, cap, 0, 0};
    band_traceback<S, LPW>(Dr, Mr, g, rRb, best.cR, maxCR, G.lbR, G.rbR, S * LPW - G.WR, csR.cvlo,
                           csR.cvhi, 1 - JL, LR, blocks, nwords, t, owR);
    const int nR = owR.n < cap ? owR.n : cap;
    OpWriter owL = {ops + o0 + nR, cap - nR, 0, 0};
    band_traceback<S, LPW>(Dl, Ml, g, rLb, best.cL, maxCL, G.lbL, G.rbL, S * LPW - G.WL, csL.cvlo,
                           csL.cvhi, JL, LL, blocks, nwords, t, owL);
    X.nops_right = nR;
    X.nops_left = owL.n < owL.cap ? owL.n : owL.cap;
    if (owR.n > cap || owL.n > owL.cap) X.status = ST_OPS_OVERFLOW;
    R.nmatches = t.nmatches;
    R.nmismatches = t.nmismatches;
    R.nopens = t.nopens;
    R.nindels = t.nindels;
    const int npush = t.nmatches + t.nmismatches + t.nindels + t.npush;
    X.npairs = npush + 1;  // + the gapholder
    if (npush == 0) {      // only the gapholder: the list is dropped (:5050-5053)
      R.returned_null = 1;
      X.npairs = 0;
    }
    R.dynprogindex = step_dpi(wo.dynprogindex);
  }
  res[wi] = R;
  trc[wi] = X;
  GB_TICK(4);
}

// This wave's wave-tasks of one band class (both tie-rule lists; __noinline__
// for its own register allocation, as k_fill's fill_tasks).
template <int S, int LPW, bool PM>
__device__ __noinline__ void gband_tasks(int cls, int t0, int t1, int stride, int ntask0,
                                         const AS_GLOBAL gsnapdp_ggap_window* Wn1,
                                         const AS_GLOBAL int* lists1, const AS_GLOBAL int* counts1,
                                         int list_cap, const AS_GLOBAL char* q1, const AS_GLOBAL char* qu1,
                                         const AS_GLOBAL uint32_t* blocks1, uint64_t nwords,
                                         const AS_LDS uint32_t* sprof3, AS_LDS uint32_t* ring3,
                                         AS_GLOBAL uint32_t* wpool1, const AS_GLOBAL uint32_t* prof1,
                                         const AS_GLOBAL double* tables1,
                                         AS_GLOBAL gsnapdp_ggap_result* res1,
                                         AS_GLOBAL gsnapdp_ggap_trace* trc1, AS_GLOBAL uint32_t* ops1,
                                         const AS_GLOBAL int64_t* op_off1) {
  constexpr int NG = 64 / LPW;
  const int lane = threadIdx.x & 63;
  const int g = lane / LPW;
  // list (cls, jl) holds counts[GB_LIST0 + 2*cls + jl] windows; its tasks are
  // [0, ntask0) for jl = 0 and [ntask0, ...) for jl = 1
  for (int t = t0; t < t1; t += stride) {
    const int jl = t >= ntask0 ? 1 : 0;
    const int lt = t - (jl ? ntask0 : 0);
    const int li = (PM ? GP_LIST0 : GB_LIST0) + 2 * cls + jl;
    const int* list = (const int*)lists1 + (size_t)li * list_cap;
    const int n = ((const int*)counts1)[li];
    const int k = lt * NG + g;
    const bool active = k < n;
    const int wi = list[active ? k : lt * NG];
#ifdef GB_CHECK
    GB_CHK(li, GG_NLISTS, 13);
    GB_CHK(wi, list_cap * 4, 14);
#endif
    if (jl)
      gband_group<S, LPW, 1, PM>(Wn1, wi, active, lane, wpool1, q1, qu1, blocks1, nwords, sprof3, ring3,
                             tables1, res1, trc1, ops1, op_off1);
    else
      gband_group<S, LPW, 0, PM>(Wn1, wi, active, lane, wpool1, q1, qu1, blocks1, nwords, sprof3, ring3,
                             tables1, res1, trc1, ops1, op_off1);
  }
}

// All band classes in one persistent launch (k_fill's scheme): the wave-tasks
// of the lists form one index space, class by class.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(GB_WAVES_PER_SIMD, 8))) void k_gband(
    const gsnapdp_ggap_window* __restrict__ Wn, const int* __restrict__ lists,
    const int* __restrict__ counts, int list_cap, const char* __restrict__ q,
    const char* __restrict__ qu, const uint32_t* __restrict__ blocks, uint64_t nwords,
    const uint32_t* __restrict__ prof, const double* __restrict__ tables, uint32_t* __restrict__ pool,
    uint32_t wave_dw, gsnapdp_ggap_result* __restrict__ res, gsnapdp_ggap_trace* __restrict__ trc,
    uint32_t* __restrict__ ops, const int64_t* __restrict__ op_off) {
  __shared__ alignas(8) uint32_t sprof[SPROF_WORDS];
  __shared__ uint32_t rings[4][GB_RING_WORDS];
  {  // no register-band window in the batch (a probability-mode batch on k_gwin): no table staging
    int any = 0;
#pragma unroll
    for (int k = GB_LIST0; k < GB_LIST0 + 4 * (NCLASS - 1); k++) any |= counts[k];
    if (any == 0) return;  // (block-uniform)
  }
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
  uint32_t* wpool = pool + (size_t)gw * wave_dw;  // GB_OCV dwords, or GB_WAVE_DW with probability-mode lists
  // tasks of list pair k: score mode for k < NCLASS - 1, then probability mode
  // (band class k % (NCLASS - 1) + 1 of k_fill's table), both tie-rule lists
  static_assert(GP_LIST0 == GB_LIST0 + 2 * (NCLASS - 1), "k_gband's list pairs");
  constexpr int NK = 2 * (NCLASS - 1);
  int tfirst[NK + 1], ntask0[NK];
  tfirst[0] = 0;
#pragma unroll
  for (int k = 0; k < NK; k++) {
    const int ng = 64 / CLASS_LPW[k % (NCLASS - 1) + 1];
    const int n0 = counts[GB_LIST0 + 2 * k], n1 = counts[GB_LIST0 + 2 * k + 1];
    ntask0[k] = (n0 + ng - 1) / ng;
    tfirst[k + 1] = tfirst[k] + ntask0[k] + (n1 + ng - 1) / ng;
  }
#define GBAND_CLASS(K, PM)                                                                       \
  {                                                                                              \
    constexpr int KK = K + (PM ? NCLASS - 1 : 0);                                                \
    const int lo = tfirst[KK], hi = tfirst[KK + 1];                                              \
    const int tau0 = gw >= lo ? gw : gw + (lo - gw + nw - 1) / nw * nw;                          \
    if (tau0 < hi)                                                                               \
      gband_tasks<CLASS_S[K + 1], CLASS_LPW[K + 1], PM>(                                        \
          K, tau0 - lo, hi - lo, nw, ntask0[KK], (const AS_GLOBAL gsnapdp_ggap_window*)Wn,        \
          (const AS_GLOBAL int*)lists, (const AS_GLOBAL int*)counts, list_cap,                    \
          (const AS_GLOBAL char*)q, (const AS_GLOBAL char*)qu, (const AS_GLOBAL uint32_t*)blocks, \
          nwords, (const AS_LDS uint32_t*)sprof, (AS_LDS uint32_t*)ring,                         \
          (AS_GLOBAL uint32_t*)wpool, (const AS_GLOBAL uint32_t*)prof,                           \
          (const AS_GLOBAL double*)tables, (AS_GLOBAL gsnapdp_ggap_result*)res,                  \
          (AS_GLOBAL gsnapdp_ggap_trace*)trc, (AS_GLOBAL uint32_t*)ops,                          \
          (const AS_GLOBAL int64_t*)op_off);                                                     \
  }
  static_assert(NCLASS == 7, "k_gband dispatches classes 1..6");
  GBAND_CLASS(0, false) GBAND_CLASS(1, false) GBAND_CLASS(2, false)
  GBAND_CLASS(3, false) GBAND_CLASS(4, false) GBAND_CLASS(5, false)
  GBAND_CLASS(0, true) GBAND_CLASS(1, true) GBAND_CLASS(2, true)
  GBAND_CLASS(3, true) GBAND_CLASS(4, true) GBAND_CLASS(5, true)
#undef GBAND_CLASS
}

}  // namespace

// Launch k_gband over the register-band lists of a genome-gap batch (the
// lists and counts k_ggap_plan filled; list GB_LIST0 + 2*k + jl).
int gsnapdp__gband_launch(gsnapdp_ctx* ctx, hipStream_t st, const gsnapdp_ggap_window* d_windows,
                          const int* lists, const int* counts, int list_cap, const char* d_query,
                          const char* d_query_uc, gsnapdp_ggap_result* d_results,
                          gsnapdp_ggap_trace* d_traces, uint32_t* d_ops, const int64_t* d_op_offsets,
                          int use_band) {
  const int waves = ctx->num_cus * 4 * GB_WAVES_PER_SIMD;
  // score mode needs the scratch up to GB_OCV only; probability-mode lists
  // (use_band & GB_USE_PROB) the whole layout, in a pool of their own made on
  // first use (1.3 MB per wave against 0.4 MB)
  const bool prob = (use_band & gsnapdp::GB_USE_PROB) != 0;
  const uint32_t wave_dw = prob ? (uint32_t)GB_WAVE_DW : (uint32_t)GB_OCV;
  uint32_t** poolp = prob ? &ctx->d_gband_pool_prob : &ctx->d_gband_pool;
  if (!*poolp) HIPCHK(hipMalloc(poolp, (size_t)waves * wave_dw * 4));
#ifdef GB_PHASES
  {
    const char* e = getenv("GSNAPDP_GB_PHASES");
    const int ph = e ? atoi(e) : 15;
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(gb_phases), &ph, sizeof(ph)));
  }
#endif
  hipLaunchKernelGGL(k_gband, dim3(waves / 4), dim3(256), 0, st, d_windows, lists, counts, list_cap,
                     d_query, d_query_uc, ctx->d_blocks, (uint64_t)ctx->nwords, ctx->d_prof,
                     ctx->d_tables, *poolp, wave_dw, d_results, d_traces, d_ops, d_op_offsets);
  HIPCHK(hipGetLastError());
#ifdef GB_CHECK
  {
    int e[8];
    HIPCHK(hipStreamSynchronize(st));
    HIPCHK(hipMemcpyFromSymbol(e, HIP_SYMBOL(gb_err), sizeof(e)));
    fprintf(stderr, "gb_check site %d idx %d lim %d thread %d\n", e[0], e[1], e[2], e[3]);
    memset(e, 0, sizeof(e));
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(gb_err), e, sizeof(e)));
  }
#endif
#ifdef GB_PROF
  unsigned long long h[8];
  HIPCHK(hipStreamSynchronize(st));
  HIPCHK(hipMemcpyFromSymbol(h, HIP_SYMBOL(gb_prof), sizeof(h)));
  fprintf(stderr, "gb_prof cycles/wave-task: pre %.0f fillR %.0f fillL %.0f combine %.0f trace %.0f\n",
          (double)h[0], (double)h[1], (double)h[2], (double)h[3], (double)h[4]);
  memset(h, 0, sizeof(h));
  HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(gb_prof), h, sizeof(h)));
#endif
  return 0;
}

int gsnapdp__gband_lds_check(size_t max_lds) { return gsnapdp__lds_fits((const void*)&k_gband, 0, max_lds, "k_gband"); }
