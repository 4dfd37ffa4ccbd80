// gsnapdp_ggap.hip -- Dynprog_genome_gap (reference src/dynprog.c:4798-5061)
// on gfx950: the two flank fills (compute_scores_lookup_fwd / _rev,
// :1424-1736), bridge_intron_gap (:3290-4122, splicing_iit == NULL, score
// and probability modes), the MaxEnt site probabilities (:3195-3287) and the
// two tracebacks (:2611-2712) of every intron window, batched.
//
// Layout.  Intron windows are small (GMAP: length1 = 2 x maxpeelback ~ 22,
// length2 = length1 + 8), so a window's query rows map onto the lanes of a
// lane group (RL = 32 rows: two windows per wave; RL = 64: one).  Lane rho
// holds row rho, and at step t it computes column t - rho (a skewed wavefront).
// The inputs from row r-1 come from the lane above by a DPP wave shift.  Each
// band cell's nogap score and its four direction bits are packed into one
// dword (H << 4 | nibble) and kept in LDS, band-compressed per row, for both
// flanks.  The bridge then scans rows in parallel (lane = rL) from LDS, and an
// ordered argmax over the group reproduces the reference's sequential
// strict-`>` scan.  The group leader walks both tracebacks with the shared
// traceback template (gsnapdp_device.h) and emits the op stream.
//
// Windows whose rows or band storage exceed the LDS classes run the same code
// with one window per wave, rows in stripes of 64 (the row above a stripe comes
// from a boundary buffer), and storage in a per-wave global scratch.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string.h>

#include <mutex>
#include <type_traits>

#include "gsnapdp_ctx.h"
#include "gsnapdp_device.h"
#include "gsnapdp_ggap.h"
#include "gsnapdp_internal.h"

using namespace gsnapdp;

#define AS_GLOBAL __attribute__((address_space(1)))
#define AS_LDS __attribute__((address_space(3)))

namespace {

// window classes of the batch
enum { GG_SMALL = 0, GG_MID = 1, GG_BIG = 2, GG_NCLS = 3 };
static_assert(GB_LIST0 == GG_NCLS && GG_NLISTS <= 32, "genome-gap lists (the counts buffer holds 32)");
#ifndef GG_SMALL_WORDS_CFG
#define GG_SMALL_WORDS_CFG 1280
#endif
#ifndef GG_WAVES
#define GG_WAVES 4  // C4 prob k_ggap: 4 waves 1.62 ms; 2: 2.17, 3: 2.16, 5: 2.24, 6: 2.72
#endif
constexpr int GG_SMALL_WORDS = GG_SMALL_WORDS_CFG;  // LDS words per window, RL = 32 (2 per wave)
constexpr int GG_SMALL_BLOCKS = 160 * 1024 / (8 * GG_SMALL_WORDS * 4);  // blocks per CU that fit in LDS
constexpr int GG_MID_WORDS = 4096;        // LDS words per window, RL = 64
constexpr size_t GG_BIG_WORDS = (size_t)4 << 20;  // global words per wave of the large path
constexpr int GG_BIG_WAVES = 32;

template <class P>
struct CellDirs {  // direction nibble of an in-band cell (r >= 1, c >= 1)
  P H;
  int W, lband;
  __device__ inline uint32_t operator()(int r, int c) const {
    return (uint32_t)H[(r - 1) * W + (c - r + lband)] & 0xFu;
  }
};

__device__ inline int from_above(int v) {  // lane i receives lane i-1's v (DPP wave_shr:1)
  return __builtin_amdgcn_update_dpp(v, v, 0x138, 0xF, 0xF, false);
}

// The same shift into a fresh register: lane 0 of the wave reads 0 (bound_ctrl),
// which gg_fill never uses (a group's first lane is row 0 or reads the stripe's
// boundary row instead).
__device__ inline int from_above_fresh(int v) {
  return __builtin_amdgcn_mov_dpp(v, 0x138, 0xF, 0xF, true);
}

template <class P>
struct Side {
  P H;              // L1 x W dwords: H << 4 | nibble (bit0 gap1 HORIZ, bit1 gap2 VERT,
                    // bit2 nogap HORIZ, bit3 nogap VERT)
  int L2, lband, rband, W;
};

// One flank fill (compute_scores_lookup_fwd / _rev, dynprog.c:1424-1736) over
// the rows of the lane group, in stripes of RL rows.  Every lane of the wave
// calls it (the DPP shift spans the wave); `T` and `NS` are wave-uniform.
// One flank fill (compute_scores_lookup_fwd / _rev, dynprog.c:1424-1736, or
// with CD the genome-row _12 fills of Dynprog_cdna_gap, :1742-2044) over the
// rows of the lane group, in stripes of RL rows.  `rowkey(r)` is the row's
// profile word (query rows: pairdistance of the query char against genome
// classes A C G T N * as signed nibbles), or with CD 4 x the genome row's
// class; `colv[c]` is column c's genome class, or with CD the profile word of
// its query char.  Every lane of the wave calls it (the DPP shift spans the
// wave); `T` and `NS` are wave-uniform.
template <int RL, bool GMEM, bool CD, class P, class PC, class RK>
__device__ void gg_fill(const Side<P>& sd, PC colv, P bnd, int L1, int rho, int open, int ext,
                        int jl, const RK& rowkey, int T, int NS) {
  const int lband = sd.lband, rband = sd.rband, L2 = sd.L2, W = sd.W;
  for (int s = 0; s < NS; s++) {
    const int r = s * RL + rho;
    const uint32_t rk = rowkey((r >= 1 && r <= L1) ? r : 1);
    // this row's band columns [cmin, cmax] (empty for row 0 and rows past L1)
    const int cmin0 = max(1, r - lband), cmax = min(L2, r + rband);
    const bool rowok = r >= 1 && r <= L1 && cmax >= cmin0;
    const int cmin = rowok ? cmin0 : (1 << 30);  // c - cmin < 0: never in band
    const uint32_t cspan = rowok ? (uint32_t)(cmax - cmin0) : 0u;
    // initial values (dynprog.c:1460-1488): row 0 E = open + c*extend for
    // 1 <= c <= rband, H(0,0) = 0; column 0 F = open + r*extend for r <= lband
    const uint32_t e0span = r == 0 ? (uint32_t)min(rband, L2) : 0u;  // c - 1 < e0span
    const int hz = r == 0 ? 0 : -(1 << 30);                           // H(r, c) = 0 iff c == hz
    const int F0 = (r >= 1 && r <= lband && r <= L1) ? open + r * ext : NEG;
    // store slot: row r's band starts at column r - lband
    const int sbase = (r - 1) * W - r + lband;
    int Hc = NEG, Ec = NEG, Fc = NEG;      // (r, c-1)
    int Hup = NEG, Eup = NEG, Fup = NEG;   // (r-1, c-1)
    int erun = open - rho * ext;           // open + c * extend, c = t - rho
    uint32_t g = (uint32_t)colv[max(0, min(L2 + 1, -rho))];
    // Per step: every value is computed, then selected (no per-lane branch but
    // the in-band store).  Out of band a cell takes its initial value
    // (dynprog.c:1460-1488) or NEG; row 0 and column 0 are never in band.
    const bool top = rho == 0 && s > 0;  // this lane reads the stripe's boundary row
    // the column loop, unswitched on whether the window is striped (NS > 1)
    auto columns = [&](auto striped) {
    constexpr bool STRIPED = decltype(striped)::value;
    auto step = [&](int t) {
      const int c = t - rho;
      const uint32_t gn = (uint32_t)colv[max(0, min(L2 + 1, c + 1))];  // next column's value
      int Hn = from_above_fresh(Hc), En = from_above_fresh(Ec), Fn = from_above_fresh(Fc);  // (r-1, c)
      if (STRIPED && s > 0) {  // wave-uniform: only striped windows read a boundary row
        const bool ok = top && c >= 0 && c <= L2;
        const int cc = ok ? c : 0;
        const int bh = (int)bnd[3 * cc], be = (int)bnd[3 * cc + 1], bf = (int)bnd[3 * cc + 2];
        Hn = top ? (ok ? bh : NEG) : Hn;
        En = top ? (ok ? be : NEG) : En;
        Fn = top ? (ok ? bf : NEG) : Fn;
      }
      // the recurrences (:1519-1561), each with the tie rule "x wins ties iff jump_late"
      const int a = Hc + open;
      const bool tE = Ec > a - jl;
      const int Er = (tE ? Ec : a) + ext;
      const int b = Hn + open;
      const bool tF = Fn > b - jl;
      const int Fr = (tF ? Fn : b) + ext;
      const bool hE = Eup > Hup - jl;
      const int m1 = hE ? Eup : Hup;
      const bool hF = Fup > m1 - jl;
      const int sc = CD ? __builtin_amdgcn_sbfe((int)g, (int)rk, 4) : __builtin_amdgcn_sbfe((int)rk, 4 * (int)g, 4);
      const int Hr = (hF ? Fup : m1) + sc;
      const bool inb = (uint32_t)(c - cmin) <= cspan;
      const int Ho = c == hz ? 0 : NEG;
      const int Eo = (uint32_t)(c - 1) < e0span ? erun : NEG;
      const int Fo = c == 0 ? F0 : NEG;
      const int H = inb ? Hr : Ho;
      const int E = inb ? Er : Eo;
      const int F = inb ? Fr : Fo;
      const uint32_t nib = (tE ? 1u : 0u) | (tF ? 2u : 0u) | (hF ? 8u : (hE ? 4u : 0u));
      const uint32_t word = ((uint32_t)H << 4) | nib;
      if (inb) sd.H[sbase + c] = word;
      if (STRIPED && rho == RL - 1 && c >= 0 && c <= L2) {
        bnd[3 * c] = (uint32_t)H;
        bnd[3 * c + 1] = (uint32_t)E;
        bnd[3 * c + 2] = (uint32_t)F;
      }
      Hup = Hn;
      Eup = En;
      Fup = Fn;
      Hc = H;
      Ec = E;
      Fc = F;
      erun += ext;
      g = gn;
    };
    // two steps per iteration: the (r-1, c-1) values rotate without register copies
    int t = 0;
    for (; t + 1 < T; t += 2) {
      step(t);
      step(t + 1);
    }
    if (t < T) step(t);
    };
    if (NS > 1) columns(std::true_type{});
    else columns(std::false_type{});
    // the boundary row is read by the next stripe's lane 0
    if constexpr (GMEM) wave_fence();
    else __builtin_amdgcn_s_waitcnt(0xc07f);
  }
}

struct Cand {  // a bridge candidate (dynprog.c:3698-4081)
  int score;     // scoreL + scoreI + scoreR
  double prob;   // probL + probR (probability mode)
  int key;       // scan order: 2*rL + (right loop)
  int rL, cL, rR, cR, sI, itype;
};

__device__ inline bool better(const Cand& x, const Cand& y, bool probmode) {
  // x replaces y in the sequential scan's outcome
  if (probmode) return x.prob > y.prob || (x.prob == y.prob && x.key < y.key);
  return x.score > y.score || (x.score == y.score && x.key < y.key);
}

template <int RL>
__device__ inline Cand group_best(Cand c, bool probmode) {
#pragma unroll
  for (int o = RL / 2; o > 0; o >>= 1) {
    Cand x;
    x.score = __shfl_xor(c.score, o);
    x.prob = __shfl_xor(c.prob, o);
    x.key = __shfl_xor(c.key, o);
    x.rL = __shfl_xor(c.rL, o);
    x.cL = __shfl_xor(c.cL, o);
    x.rR = __shfl_xor(c.rR, o);
    x.cR = __shfl_xor(c.cR, o);
    x.sI = __shfl_xor(c.sI, o);
    x.itype = __shfl_xor(c.itype, o);
    if (better(x, c, probmode)) c = x;
  }
  return c;
}

template <int RL, bool GMEM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(GG_WAVES, 8))) void k_ggap(
    const gsnapdp_ggap_window* __restrict__ Wn, const int* __restrict__ list,
    const int* __restrict__ count, const char* __restrict__ q, const char* __restrict__ qu,
    const uint32_t* __restrict__ blocks, uint64_t nwords, const uint32_t* __restrict__ prof,
    const double* __restrict__ tables, uint32_t* __restrict__ pool, size_t stride,
    gsnapdp_ggap_result* __restrict__ res, gsnapdp_ggap_trace* __restrict__ trc,
    uint32_t* __restrict__ ops, const int64_t* __restrict__ op_off) {
  extern __shared__ uint32_t smem[];
  using P = typename std::conditional<GMEM, AS_GLOBAL uint32_t*, AS_LDS uint32_t*>::type;
  using PB = typename std::conditional<GMEM, AS_GLOBAL uint8_t*, AS_LDS uint8_t*>::type;
  using PD = typename std::conditional<GMEM, AS_GLOBAL double*, AS_LDS double*>::type;
  constexpr int NGW = 64 / RL;
  const int lane = threadIdx.x & 63, grp = lane / RL, rho = lane % RL;
  const int gw = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const int nw = (int)((gridDim.x * blockDim.x) >> 6);
  P region;
  if constexpr (GMEM) {
    region = (P)(pool + (size_t)gw * stride);
  } else {
    region = (P)(smem + ((threadIdx.x >> 6) * NGW + grp) * stride);
  }
  const int n = *count;
  for (int base = gw * NGW; base < n; base += nw * NGW) {
    const int k = base + grp;
    const bool act = k < n;
    const int wi = list[act ? k : base];
    const gsnapdp_ggap_window w = Wn[wi];
    GGeo G = gg_geo(w);
    if (!act) G.L1 = 0;  // a shadow group: no rows, no stores
    const P HL = region;
    const P HR = region + G.oHR;
    const PB clsL = (PB)(region + G.oClsL);
    const PB clsR = (PB)(region + G.oClsR);
    const PD lp = (PD)(region + G.oProbL);
    const PD rp = (PD)(region + G.oProbR);
    const P bnd = region + G.oBnd;
    // the constrained known-intron mode precedes (and ignores) probability mode (:3552)
    const bool probmode = w.use_probabilities_p != 0 && w.known_mode != GSNAPDP_KNOWN_INTRONS;
    // known splice sites (a splicing IIT, dynprog.c:3375-3550): the caller's
    // record follows the query rows (include/gsnapdp.h, gsnapdp_ggap_window)
    const int km = act ? w.known_mode : GSNAPDP_KNOWN_NONE;
    const unsigned char* krec = (const unsigned char*)q + w.qpos + (act ? G.L1 : 0);
    // column genome classes (get_genomic_nt, dynprog.c:403-441), both flanks
    const Lane LL = side_lane(w, G, 0), LR = side_lane(w, G, 1);
    if (act) {
      for (int c = rho; c <= G.L2L + 1; c += RL)
        clsL[c] = (uint8_t)((c >= 1 && c <= G.L2L) ? gclass(blocks, nwords, LL, w.offset2L + c - 1) : 5);
      for (int c = rho; c <= G.L2R + 1; c += RL)
        clsR[c] = (uint8_t)((c >= 1 && c <= G.L2R) ? gclass(blocks, nwords, LR, w.revoffset2R + 1 - c) : 5);
#ifdef GG_EXP_NOPROB  // timing experiment only: no MaxEnt evaluation (wrong probabilities)
      if (probmode) {
        for (int c = rho; c < G.L2L; c += RL) lp[c] = 0.01 * (double)(c & 63);
        for (int c = rho; c < G.L2R; c += RL) rp[c] = 0.01 * (double)(c & 31);
      }
      if (false) {
#else
      if (probmode) {  // :3856-3903 (a known site has probability 1.0)
#endif
        for (int c = rho; c < G.L2L; c += RL)
          lp[c] = c < G.L2L - 1 ? (kflag(krec, km, c) ? 1.0 : left_site_prob(w, c, blocks, nwords, tables)) : 0.0;
        for (int c = rho; c < G.L2R; c += RL)
          rp[c] = c < G.L2R - 1 ? (kflag(krec + G.L2L, km, c) ? 1.0 : right_site_prob(w, c, blocks, nwords, tables))
                                : 0.0;
      }
    }
    using PH = typename std::conditional<GMEM, AS_GLOBAL uint16_t*, AS_LDS uint16_t*>::type;
    const PB diL = (PB)(region + G.oDiL);
    const PB diR = (PB)(region + G.oDiR);
    const PH itab = (PH)(region + G.oItab);
    const PH qb = (PH)(region + G.oQ);
    if (act) {
      for (int i = rho; i < G.L1; i += RL)  // the traceback's per-row match masks
        qb[i] = (uint16_t)row_match_mask(prof, G.mt, (unsigned char)q[w.qpos + i], (unsigned char)qu[w.qpos + i]);
      for (int t = rho; t < 64; t += RL) {  // intron_score by leftdi & rightdi (:3148-3192)
        int it;
        const int sI = intron_score(it, t, 0x3F, w.cdna_direction, G.canon, w.finalp);
        itab[t] = (uint16_t)(sI | (it << 8));
      }
    }
    if constexpr (GMEM) wave_fence();
    else __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the class bytes are in LDS
    if (act) {  // leftdi / rightdi (:3331-3373); 0 past the scanned columns (calloc);
                // bit 7: left_known / right_known (:3375-3550)
      for (int c = rho; c <= G.L2L; c += RL)
        diL[c] = (uint8_t)((c < G.L2L - 1 ? left_di(clsL[c + 1], clsL[c + 2]) : 0) |
                           (c < G.L2L && kflag(krec, km, c) ? KNOWN_BIT : 0));
      for (int c = rho; c <= G.L2R; c += RL)
        diR[c] = (uint8_t)((c < G.L2R - 1 ? right_di(clsR[c + 2], clsR[c + 1]) : 0) |
                           (c < G.L2R && kflag(krec + G.L2L, km, c) ? KNOWN_BIT : 0));
    }
    // wave-uniform step and stripe counts
    const int L2max = max(G.L2L, G.L2R);
    // the last row's lane reaches column L2 at step L2 + L1; a striped window's
    // last lane writes the boundary row through step L2 + RL - 1
    const int T = __builtin_amdgcn_readfirstlane(
        wave_max(act ? L2max + (G.L1 + 1 > RL ? RL : G.L1 + 1) : 0));
    const int NS = __builtin_amdgcn_readfirstlane(wave_max(act ? G.L1 + 1 : 1) + RL - 1) / RL;
    const uint32_t* ptab = prof + G.mt * 128;
    const Side<P> SL = {HL, G.L2L, G.lbL, G.rbL, G.WL};
    const Side<P> SR = {HR, G.L2R, G.lbR, G.rbR, G.WR};
    // left flank forward with jump_late_p, right flank reversed with !jump_late_p (:4955-4990)
    const int jl = w.jump_late_p ? 1 : 0;
#ifndef GG_EXP_NOFILL
    gg_fill<RL, GMEM, false>(SL, clsL, bnd, G.L1, rho, G.open, G.ext, jl,
                             [&](int r) { return ptab[(unsigned char)q[(int)w.qpos + r - 1] & 127u]; }, T, NS);
#endif
#ifndef GG_EXP_NOFILL
    gg_fill<RL, GMEM, false>(SR, clsR, bnd, G.L1, rho, G.open, G.ext, 1 - jl,
                             // (a shadow group has L1 = 0: clamp to the window's first query byte)
                             [&](int r) { return ptab[(unsigned char)q[(int)w.qpos + max(0, G.L1 - r)] & 127u]; },
                             T, NS);
#endif
    if constexpr (GMEM) wave_fence();
    else __builtin_amdgcn_s_waitcnt(0xc07f);

    // ---- bridge_intron_gap (dynprog.c:3290-4122), lane = rL
    const int leftoffset = w.offset2L, rightoffset = w.revoffset2R;
    const int lbandB = G.eb, rbandBL = G.L2L - G.L1 + G.eb, rbandBR = G.L2R - G.L1 + G.eb;
    if constexpr (GMEM) wave_fence();
    else __builtin_amdgcn_s_waitcnt(0xc07f);  // the dinucleotide codes are in LDS
    auto HLv = [&](int r, int c) { return (int)HL[(r - 1) * G.WL + (c - r + G.lbL)]; };
    auto HRv = [&](int r, int c) { return (int)HR[(r - 1) * G.WR + (c - r + G.lbR)]; };
    auto pen = [](int v) { return (v & 12) ? 1 : 0; };  // nogap dir HORIZ or VERT
    Cand best;
    best.score = BRIDGE_INIT;
    best.prob = 0.0;
    best.key = 0x7fffffff;
    best.rL = best.cL = best.rR = best.cR = 0;
    best.sI = BRIDGE_INIT;
    best.itype = 0;
#ifdef GG_EXP_NOBRIDGE
    const int rows = 0;
#else
    const int rows = __builtin_amdgcn_readfirstlane(wave_max(act ? G.L1 : 0));
#endif
    const int span = rightoffset - leftoffset;  // cR < span - cL (:3720, 3760)
    for (int r0 = 0; r0 < rows; r0 += RL) {
      const int rL = r0 + rho;
      if (rL < 1 || rL >= G.L1) continue;
      const int rR = G.L1 - rL;
      const int cloL = max(1, rL - lbandB), chighL = min(min(G.L2L - 1, rL + rbandBL), span - rR - 1);
      const int cloR = max(1, rR - lbandB), chighR = min(min(G.L2R - 1, rR + rbandBR), span - rL - 1);
      const int rdR = diR[rR], ldL = diL[rL];
      // (rR, rR): on the right band's main diagonal; + right_known[rR] (:3727)
      const int DR = (HRv(rR, rR) >> 4) + kreward(rdR);
      const int DL = (HLv(rL, rL) >> 4) + kreward(ldL);
      const int baseL = (rL - 1) * G.WL - rL + G.lbL, baseR = (rR - 1) * G.WR - rR + G.lbR;
      if (km == GSNAPDP_KNOWN_INTRONS) {  // constrain to given introns (:3552-3697)
        if (rdR & KNOWN_BIT) {
          for (int cL = cloL; cL <= chighL; cL++) {  // indel on left, cR = rR
            if (!(diL[cL] & KNOWN_BIT)) continue;
            const int v = (int)HL[baseL + cL];
            const int tot = (v >> 4) - pen(v) + (DR - KNOWN_REWARD);
            if (tot > best.score && known_intron(krec + G.L2L + G.L2R, cL, rR)) {
              best.score = tot;
              best.key = 2 * rL;
              best.sI = 0;
              best.cL = cL;
              best.cR = rR;
            }
          }
        }
        if (ldL & KNOWN_BIT) {
          for (int cR = cloR; cR <= chighR; cR++) {  // indel on right, cL = rL
            if (!(diR[cR] & KNOWN_BIT)) continue;
            const int v = (int)HR[baseR + cR];
            const int tot = (DL - KNOWN_REWARD) + (v >> 4) - pen(v);
            if (tot > best.score && known_intron(krec + G.L2L + G.L2R, rL, cR)) {
              best.score = tot;
              best.key = 2 * rL + 1;
              best.sI = 0;
              best.cL = rL;
              best.cR = cR;
            }
          }
        }
      } else if (probmode) {
        const double pR = rR < G.L2R - 1 ? rp[rR] : 0.0;
        const double pL = rL < G.L2L - 1 ? lp[rL] : 0.0;
        for (int cL = cloL; cL <= chighL; cL++) {  // indel on left, cR = rR
          const double p = lp[cL] + pR;
          if (!(p > best.prob)) continue;
          const int v = (int)HL[baseL + cL], d = diL[cL];
          const int tot = (v >> 4) - pen(v) + kreward(d) + (itab[d & rdR & DI_MASK] & 255) + DR;
          if (tot >= w.score_threshold) {
            best.prob = p;
            best.key = 2 * rL;
            best.cL = cL;
            best.cR = rR;
          }
        }
        for (int cR = cloR; cR <= chighR; cR++) {  // indel on right, cL = rL
          const double p = pL + rp[cR];
          if (!(p > best.prob)) continue;
          const int v = (int)HR[baseR + cR], d = diR[cR];
          const int tot = DL + (itab[ldL & d & DI_MASK] & 255) + (v >> 4) - pen(v) + kreward(d);
          if (tot >= w.score_threshold) {
            best.prob = p;
            best.key = 2 * rL + 1;
            best.cL = rL;
            best.cR = cR;
          }
        }
      } else {
        for (int cL = cloL; cL <= chighL; cL++) {  // indel on left, cR = rR
          const int v = (int)HL[baseL + cL], d = diL[cL];
          const int e = itab[d & rdR & DI_MASK];
          const int tot = (v >> 4) - pen(v) + kreward(d) + (e & 255) + DR;
          if (tot > best.score) {
            best.score = tot;
            best.key = 2 * rL;
            best.sI = e;  // score | type << 8 until the reduction
            best.cL = cL;
            best.cR = rR;
          }
        }
        for (int cR = cloR; cR <= chighR; cR++) {  // indel on right, cL = rL
          const int v = (int)HR[baseR + cR], d = diR[cR];
          const int e = itab[ldL & d & DI_MASK];
          const int tot = DL + (e & 255) + (v >> 4) - pen(v) + kreward(d);
          if (tot > best.score) {
            best.score = tot;
            best.key = 2 * rL + 1;
            best.sI = e;
            best.cL = rL;
            best.cR = cR;
          }
        }
      }
    }
    // the lane's rows of its best candidate
    if (best.key != 0x7fffffff) {
      best.rL = best.key >> 1;
      best.rR = G.L1 - best.rL;
      if (!probmode) {
        best.itype = best.sI >> 8;
        best.sI &= 255;
      }
    }
    best = group_best<RL>(best, probmode);

    // ---- outcome and probabilities (group leader), then the two tracebacks
    int do_tr = 0;
    if (act && rho == 0) {
      gsnapdp_ggap_result R;
      gsnapdp_ggap_trace X;
      memset(&R, 0, sizeof(R));
      memset(&X, 0, sizeof(X));
      R.dynprogindex = w.dynprogindex;
      R.bridge_ok = 1;
      X.status = ST_OK;
      const bool tables_ok = tables != nullptr || !ggap_needs_tables(w);
      int finalscore = 0, rc;
      if (!tables_ok) {
        rc = -2;
      } else if (probmode) {
        if (!(best.prob > 0.0)) {
          rc = -1;  // no candidate: the reference reads uninitialised indices (:4055)
        } else {
          const int vl = HLv(best.rL, best.cL), vr = HRv(best.rR, best.cR);
          const int dl = diL[best.cL], dr = diR[best.cR];
          int it;
          const int sI = intron_score(it, dl & DI_MASK, dr & DI_MASK, w.cdna_direction, G.canon,
                                      w.finalp);
          const int sL = (vl >> 4) - pen(vl) + kreward(dl), sR = (vr >> 4) - pen(vr) + kreward(dr);
          finalscore = w.halfp ? sL + sI + sR - sI / 2 : sL + sI + sR;
          rc = finalscore >= 0;
        }
      } else if (km == GSNAPDP_KNOWN_INTRONS) {
        finalscore = best.score;  // no intron score, no halfp (:3694-3695)
        rc = finalscore >= 0;
      } else {
        finalscore = w.halfp ? best.score - best.sI / 2 : best.score;
        R.introntype = best.score > BRIDGE_INIT ? best.itype : 0;
        rc = finalscore >= 0;
      }
      // novel splicing off with a site-level IIT: both chosen sites must be known (:4090-4096)
      if (rc == 1 && km == GSNAPDP_KNOWN_SITES)
        rc = (diL[best.cL] & KNOWN_BIT) && (diR[best.cR] & KNOWN_BIT);
      if (rc == -2) {
        X.status = ST_UNSUPPORTED;
        R.returned_null = 1;
        R.finalscore = NEG;
      } else if (rc == -1) {
        R.bridge_ok = 0;
        R.returned_null = 1;
        R.finalscore = NEG;
      } else if (rc == 0) {
        R.finalscore = finalscore;
        R.returned_null = 1;
      } else {
        R.finalscore = finalscore;
        if (w.finalp) {  // :4104-4108 (get_splicesite_probs: a known site is 1.0, :3215, :3255)
          // probability mode evaluated these sites already (lp / rp: the same model at the
          // same position, columns below L2 - 1); the leader re-evaluates only the others
          R.left_prob = (diL[best.cL] & KNOWN_BIT)              ? 1.0
                        : (probmode && best.cL < G.L2L - 1) ? (double)lp[best.cL]
                                                            : left_site_prob(w, best.cL, blocks, nwords, tables);
          R.right_prob = (diR[best.cR] & KNOWN_BIT)              ? 1.0
                         : (probmode && best.cR < G.L2R - 1) ? (double)rp[best.cR]
                                                             : right_site_prob(w, best.cR, blocks, nwords, tables);
        }
        R.new_leftgenomepos = w.offset2L + (best.cL - 1);
        R.new_rightgenomepos = w.revoffset2R - (best.cR - 1);
        R.exonhead = (w.offset1 + G.L1 - 1) - (best.rR - 1);
        X.bridge_accepted = 1;
        X.brL = best.rL;
        X.bcL = best.cL;
        X.brR = best.rR;
        X.bcR = best.cR;
        do_tr = 1;  // the counts and op totals follow from the tracebacks below
      }
      res[wi] = R;
      trc[wi] = X;
    }
    // The right flank (reversed), the gapholder, then the left flank (:5000-5040).
    // Lanes 0 and 1 of the group trace the two flanks at once (one traceback
    // each, same code, lane-selected flank): the right flank's ops at the
    // window's op offset, the left flank's at L1 + L2R + 2 (past the most a
    // right traceback emits), then lane 0 moves them down behind the right
    // flank's.  An op capacity below 2*L1 + L2L + L2R + 4 traces both flanks on
    // lane 0, one after the other.
    do_tr = __shfl(do_tr, lane - rho);
    if (act && do_tr && rho < 2) {
      const int64_t o0 = op_off[wi];
      const int cap = (int)(op_off[wi + 1] - o0);
      const int offL = G.L1 + G.L2R + 2;
      const bool split = cap >= 2 * G.L1 + G.L2L + G.L2R + 4;  // (wave-uniform per group)
      const int L1 = G.L1;
      Tally t = {0, 0, 0, 0, 0};
      int nR = 0, nL = 0;
      bool over = false;
      if (split) {
        const bool right = rho == 0;
        OpWriter ow = {ops + o0 + (right ? 0 : offL), right ? offL : cap - offL, 0, 0};
#ifndef GG_EXP_NOTRACE
        const P Hs = right ? HR : HL;
        const PB cls = right ? clsR : clsL;
        const int qa = right ? L1 : -1, qs = right ? -1 : 1;
        traceback(CellDirs<P>{Hs, right ? G.WR : G.WL, right ? G.lbR : G.lbL}, right ? LR : LL,
                  right ? best.rR : best.rL, right ? best.cR : best.cL,
                  [&](int r) -> uint32_t { return qb[qa + qs * r]; }, [&](int c) -> int { return cls[c]; }, t, ow);
#endif
        // lane 1 moves its own ops behind lane 0's (a lane reads back only its own
        // stores; nR <= offL, so the forward move never overwrites an unread op)
        const int n0 = __shfl(ow.n, lane - rho), c0 = __shfl(ow.cap, lane - rho);
        const int n1 = __shfl(ow.n, lane - rho + 1), c1 = __shfl(ow.cap, lane - rho + 1);
        nR = n0 < c0 ? n0 : c0;
        nL = n1 < c1 ? n1 : c1;
        if (!right)
          for (int i = 0; i < nL; i++) ops[o0 + nR + i] = ops[o0 + offL + i];
        const Tally t1 = {__shfl(t.nmatches, lane - rho + 1), __shfl(t.nmismatches, lane - rho + 1),
                          __shfl(t.nopens, lane - rho + 1), __shfl(t.nindels, lane - rho + 1),
                          __shfl(t.npush, lane - rho + 1)};
        if (right) {
          over = n0 > c0 || n1 > c1;
          t.nmatches += t1.nmatches;
          t.nmismatches += t1.nmismatches;
          t.nopens += t1.nopens;
          t.nindels += t1.nindels;
          t.npush += t1.npush;
        }
      } else if (rho == 0) {
        OpWriter owR = {ops + o0, cap, 0, 0};
#ifndef GG_EXP_NOTRACE
        traceback(CellDirs<P>{HR, G.WR, G.lbR}, LR, best.rR, best.cR,
                  [&](int r) -> uint32_t { return qb[L1 - r]; }, [&](int c) -> int { return clsR[c]; },
                  t, owR);
#endif
        nR = owR.n < cap ? owR.n : cap;
        OpWriter owL = {ops + o0 + nR, cap - nR, 0, 0};
#ifndef GG_EXP_NOTRACE
        traceback(CellDirs<P>{HL, G.WL, G.lbL}, LL, best.rL, best.cL,
                  [&](int r) -> uint32_t { return qb[r - 1]; }, [&](int c) -> int { return clsL[c]; },
                  t, owL);
#endif
        nL = owL.n < owL.cap ? owL.n : owL.cap;
        over = owR.n > cap || owL.n > owL.cap;
      }
      if (rho == 0) {
        gsnapdp_ggap_result R = res[wi];
        gsnapdp_ggap_trace X = trc[wi];
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
        R.dynprogindex = step_dpi(w.dynprogindex);
        res[wi] = R;
        trc[wi] = X;
      }
    }
  }
}

// Every window the register-band kernel does not take: end gaps (all
// endpoint modes but QUERYEND_NOGAPS, which k_plan finishes) and single gaps
// with W > 48 or L2 > 640.  Fill as in k_ggap (one flank, forward or reversed),
// then the endpoint -- (L1, L2) for a single gap, find_best_endpoint
// (dynprog.c:2235-2290) or find_best_endpoint_to_queryend_indels (:2293-2355)
// for end gaps, as a row-parallel scan with an ordered argmax -- and the
// traceback (:2611-2712) by the group leader.
//
// SEG: the splice-junction end gaps (Dynprog_end5/3_splicejunction,
// :5412-5553 / :5869-6057).  Wn then holds the end-gap records k_sj_plan
// derived (endalign QUERYEND_INDELS), the genome of column c is the caller's
// segment byte at sjw[wi].spos (use_genomicseg_p, :1535 / :1690), and the
// final score is recomputed from the counts (:5541 / :6045).
//
// One class's share of the windows for wave gw of nw (wave wv of its block
// for the LDS regions).
template <int RL, bool GMEM, bool SEG>
__device__ __forceinline__ void rows_class(
    const gsnapdp_window* __restrict__ Wn, const int* __restrict__ list,
    const int* __restrict__ count, const char* __restrict__ q, const char* __restrict__ qu,
    const uint32_t* __restrict__ blocks, uint64_t nwords, const uint32_t* __restrict__ prof,
    uint32_t* __restrict__ pool, size_t stride, gsnapdp_result* __restrict__ res,
    uint32_t* __restrict__ ops, const int64_t* __restrict__ op_off,
    const gsnapdp_sj_window* __restrict__ sjw, int gw, int nw, int wv) {
  extern __shared__ uint32_t smem[];
  using P = typename std::conditional<GMEM, AS_GLOBAL uint32_t*, AS_LDS uint32_t*>::type;
  using PB = typename std::conditional<GMEM, AS_GLOBAL uint8_t*, AS_LDS uint8_t*>::type;
  using PH = typename std::conditional<GMEM, AS_GLOBAL uint16_t*, AS_LDS uint16_t*>::type;
  constexpr int NGW = 64 / RL;
  const int lane = threadIdx.x & 63, grp = lane / RL, rho = lane % RL;
  P region;
  if constexpr (GMEM) {
    region = (P)(pool + (size_t)gw * stride);
  } else {
    region = (P)(smem + (wv * NGW + grp) * stride);
  }
  const int n = *count;
  for (int base = gw * NGW; base < n; base += nw * NGW) {
    const int k = base + grp;
    const bool act = k < n;
    const int wi = list[act ? k : base];
    const gsnapdp_window w = Wn[wi];
    const Lane L = make_lane(w);
    const Derived& d = L.d;
    const int L1 = act ? d.L1 : 0, L2 = d.L2, W = d.W;
    const P H = region;
    const PB cls = (PB)(region + L1 * W);
    const PH qb = (PH)(region + L1 * W + (L2 + 2 + 3) / 4);
    const P bnd = region + L1 * W + (L2 + 2 + 3) / 4 + (L1 + 1) / 2;
    if (act) {
      if constexpr (SEG) {
        const int sp = (int)sjw[wi].spos;
        for (int c = rho; c <= L2 + 1; c += RL)
          cls[c] = (uint8_t)((c >= 1 && c <= L2) ? seg_class((unsigned char)q[sp + L.gstep * (c - 1)]) : 5);
      } else {
        for (int c = rho; c <= L2 + 1; c += RL)
          cls[c] = (uint8_t)((c >= 1 && c <= L2) ? gclass(blocks, nwords, L, L.g0 + L.gstep * (c - 1)) : 5);
      }
      for (int i = rho; i < L1; i += RL) {
        const int qi = L.qbase + L.qstep * i;
        qb[i] = (uint16_t)row_match_mask(prof, d.mt, (unsigned char)q[qi], (unsigned char)qu[qi]);
      }
    }
    if constexpr (GMEM) wave_fence();
    else __builtin_amdgcn_s_waitcnt(0xc07f);
    const int T = __builtin_amdgcn_readfirstlane(wave_max(act ? L2 + (L1 + 1 > RL ? RL : L1 + 1) : 0));
    const int NS = __builtin_amdgcn_readfirstlane(wave_max(act ? L1 + 1 : 1) + RL - 1) / RL;
    const Side<P> sd = {H, L2, d.lband, d.rband, W};
    const uint32_t* ptab = prof + d.mt * 128;
    gg_fill<RL, GMEM, false>(sd, cls, bnd, L1, rho, d.open, d.ext, d.jl,
                             [&](int r) { return ptab[(unsigned char)q[L.qbase + L.qstep * (r - 1)] & 127u]; },
                             T, NS);
    if constexpr (GMEM) wave_fence();
    else __builtin_amdgcn_s_waitcnt(0xc07f);
    // ---- endpoint: a row-parallel scan, then the first (or, with jump_late,
    // the last) best cell in row-major order
    const int jl = d.jl;
    int best, key;  // key = r * (L2 + 1) + c
    if (d.mode == 1) {
      best = 0;  // find_best_endpoint starts at (0, 0) with 0 (:2243)
      key = 0;
    } else {
      best = NEG;  // queryend_indels starts at (L1, 0) with NEG_INFINITY (:2302)
      key = L1 * (L2 + 1);
    }
    const int rows = __builtin_amdgcn_readfirstlane(wave_max(act && d.mode != 0 ? L1 : 0));
    for (int r0 = 0; r0 < rows; r0 += RL) {
      const int r = r0 + rho + 1;
      if (r > L1 || (d.mode == 2 && r != L1)) continue;
      // mode 1: the unwidened band |r - c| <= extraband; mode 2: the widened band
      const int clo = max(1, d.mode == 1 ? r - d.eb : r - d.lband);
      const int chi = min(L2, d.mode == 1 ? r + d.eb : r + d.rband);
      const int rb = (r - 1) * W - r + d.lband;
      for (int c = clo; c <= chi; c++) {
        const int v = (int)H[rb + c] >> 4;
        if (v > best - jl) {
          best = v;
          key = r * (L2 + 1) + c;
        }
      }
    }
#pragma unroll
    for (int o = RL / 2; o > 0; o >>= 1) {
      const int ob = __shfl_xor(best, o), ok = __shfl_xor(key, o);
      if (ob > best || (ob == best && (jl ? ok > key : ok < key))) {
        best = ob;
        key = ok;
      }
    }
    if (act && rho == 0) {
      int br, bc, score;
      if (d.mode == 0) {
        br = L1;
        bc = L2;
        score = (int)H[(L1 - 1) * W + (L2 - L1 + d.lband)] >> 4;  // matrix[L1][L2].nogap (:4534)
      } else {
        br = key / (L2 + 1);
        bc = key - br * (L2 + 1);
        score = best;
      }
      Tally t = {0, 0, 0, 0, 0};
      OpWriter ow = {ops + op_off[wi], (int)(op_off[wi + 1] - op_off[wi]), 0, 0};
      traceback(CellDirs<P>{H, W, d.lband}, L, br, bc,
                [&](int r) -> uint32_t { return qb[r - 1]; }, [&](int c) -> int { return cls[c]; },
                t, ow);
      if constexpr (SEG)
        score = t.nmatches * 3 - 5 * t.nmismatches + t.nopens * d.open + t.nindels * d.ext;
      write_result(&res[wi], w, L, score, br, bc, t, ow);
    }
  }
}

// All five row-lane classes in one launch of one 16-wave block per CU (the
// whole 160 KB of LDS): the LDS classes in turn, a block barrier between two
// of them since their regions overlap, then the global-scratch classes.  A
// batch with no row-lane windows (most single-gap batches) pays for one
// launch instead of five.
template <bool SEG>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(GG_WAVES, 8))) void k_rows(
    const gsnapdp_window* __restrict__ Wn, const int* __restrict__ lists, int list_cap,
    int* __restrict__ counts, const char* __restrict__ q, const char* __restrict__ qu,
    const uint32_t* __restrict__ blocks, uint64_t nwords, const uint32_t* __restrict__ prof,
    uint32_t* __restrict__ largepool, uint32_t* __restrict__ bigpool,
    gsnapdp_result* __restrict__ res, uint32_t* __restrict__ ops,
    const int64_t* __restrict__ op_off, const gsnapdp_sj_window* __restrict__ sjw) {
  const int wv = (int)(threadIdx.x >> 6), nb = (int)gridDim.x;
  const int gw = (int)blockIdx.x * 16 + wv, nw = nb * 16;
  rows_class<16, false, SEG>(Wn, lists + (size_t)RW_TINY * list_cap, counts + RW_TINY, q, qu,
                             blocks, nwords, prof, nullptr, RW_TINY_WORDS, res, ops, op_off, sjw,
                             gw, nw, wv);
  __syncthreads();
  rows_class<32, false, SEG>(Wn, lists + (size_t)RW_SMALL * list_cap, counts + RW_SMALL, q, qu,
                             blocks, nwords, prof, nullptr, RW_SMALL_WORDS, res, ops, op_off, sjw,
                             gw, nw, wv);
  __syncthreads();
  if (wv < 8)  // 8 regions of RW_MID_WORDS
    rows_class<64, false, SEG>(Wn, lists + (size_t)RW_MID * list_cap, counts + RW_MID, q, qu,
                               blocks, nwords, prof, nullptr, RW_MID_WORDS, res, ops, op_off, sjw,
                               (int)blockIdx.x * 8 + wv, nb * 8, wv);
  rows_class<64, true, SEG>(Wn, lists + (size_t)RW_LARGE * list_cap, counts + RW_LARGE, q, qu,
                            blocks, nwords, prof, largepool, RW_LARGE_WORDS, res, ops, op_off, sjw,
                            gw, nw, wv);
  if (gw < RW_BIG_WAVES)
    rows_class<64, true, SEG>(Wn, lists + (size_t)RW_BIG * list_cap, counts + RW_BIG, q, qu,
                              blocks, nwords, prof, bigpool, RW_BIG_WORDS, res, ops, op_off, sjw,
                              gw, RW_BIG_WAVES, wv);
  // the last block out clears the class counts and END flags for the next batch
  // (every wave read its counts before its block's ticket; wave 0 takes the
  // ticket and clears -- no static LDS beside the 160 KB of regions)
  __syncthreads();
  if (wv == 0) {
    int t = 0;
    if (threadIdx.x == 0)
      t = __hip_atomic_fetch_add(counts + ROWS_TICKET, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (__shfl(t, 0) == (int)gridDim.x - 1) {
      if (threadIdx.x <= RW_NCLS) counts[threadIdx.x] = 0;
      if (threadIdx.x == 0) counts[ROWS_TICKET] = 0;
    }
  }
}

// Dynprog_end5/3_splicejunction windows -> the end-gap records k_rows runs
// (QUERYEND_INDELS: find_best_endpoint_to_queryend_indels, ENDQ, END
// open/extend, the reversed fill's !jump_late_p), early returns (:5446-5461)
// and the row-lane class of each window.  Segments outside A C G T N (never
// produced by Dynprog_make_splicejunction_5/3) are marked unsupported.
__global__ void k_sj_plan(const gsnapdp_sj_window* __restrict__ S, int n,
                          const char* __restrict__ q, const char* __restrict__ qu,
                          gsnapdp_window* __restrict__ Wn, gsnapdp_result* __restrict__ res) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const gsnapdp_sj_window s = S[i];
    gsnapdp_window w;
    memset(&w, 0, sizeof(w));
    w.kind = s.kind == GSNAPDP_END5_GAP ? GSNAPDP_END5_GAP : GSNAPDP_END3_GAP;
    w.length1 = s.length1;
    w.length2 = s.length2;
    w.offset1 = s.offset1;
    w.offset2 = s.offset2_anchor;
    w.qpos = s.qpos;
    w.cdna_direction = s.cdna_direction;
    w.extraband = s.extraband_end;
    w.dynprogindex = s.dynprogindex;
    w.maxlength1 = s.maxlength1;
    w.maxlength2 = s.maxlength2;
    w.defect_rate = s.defect_rate;
    w.watsonp = s.watsonp;
    w.jump_late_p = s.jump_late_p;
    w.widebandp = 1;
    w.endalign = GSNAPDP_QUERYEND_INDELS;
    Wn[i] = w;
    int status = ST_OK;
    if (s.length1 <= 0 || s.length1 > s.maxlength1 || s.length2 <= 0 || s.length2 > s.maxlength2) {
      status = ST_EARLY;  // NULL, finalscore 0, counts 0, *dynprogindex untouched
    } else if (s.kind != GSNAPDP_END5_GAP && s.kind != GSNAPDP_END3_GAP) {
      status = ST_UNSUPPORTED;
    } else {
      const Derived d = derive(w);
      const int step = s.kind == GSNAPDP_END5_GAP ? -1 : 1;
      if (d.status != ST_OK) status = ST_UNSUPPORTED;
      // the segment's bytes [lo, lo + length2) (either direction): A C G T N and
      // the same in both buffers; a dword at a time where both are aligned
      const int lo = step > 0 ? (int)s.spos : (int)s.spos - (s.length2 - 1);
      const unsigned char* a = (const unsigned char*)q + lo;
      const unsigned char* b = (const unsigned char*)qu + lo;
      auto byte_ok = [](unsigned x, unsigned y) { return x == y && seg_class((unsigned char)x) <= 4; };
      bool ok = d.status == ST_OK;
      int k = 0;
      for (; ok && k < s.length2 && ((uintptr_t)(a + k) & 3u); k++) ok = byte_ok(a[k], b[k]);
      if (((uintptr_t)(b + k) & 3u) == 0) {
        for (; ok && k + 4 <= s.length2; k += 4) {
          const uint32_t x = *(const uint32_t*)(a + k), y = *(const uint32_t*)(b + k);
          ok = x == y && seg_class(x & 255u) <= 4 && seg_class((x >> 8) & 255u) <= 4 &&
               seg_class((x >> 16) & 255u) <= 4 && seg_class(x >> 24) <= 4;
        }
      }
      for (; ok && k < s.length2; k++) ok = byte_ok(a[k], b[k]);
      if (!ok) status = ST_UNSUPPORTED;
    }
    if (status != ST_OK) {
      gsnapdp_result R = {};
      R.status = status;
      R.length1 = s.length1;
      R.length2 = s.length2;
      R.reserved = s.dynprogindex;
      res[i] = R;
      Wn[i].kind = KIND_SKIP;  // finished here: the fill pipeline's planner skips it
    }
  }
}

// Parameters, early returns (dynprog.c:4843-4870) and the class of every
// window; windows that reach the fills are appended to their class list.
__global__ void k_ggap_plan(const gsnapdp_ggap_window* __restrict__ Wn, int n,
                            gsnapdp_ggap_result* __restrict__ res,
                            gsnapdp_ggap_trace* __restrict__ trc, int* __restrict__ lists,
                            int* __restrict__ counts, int cap, int use_band) {
  __shared__ int lcnt[GG_NLISTS], lbase[GG_NLISTS];  // block-local list appends
  if (threadIdx.x < GG_NLISTS) lcnt[threadIdx.x] = 0;
  __syncthreads();
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  int cls = -1;
  if (i < n) {
    const gsnapdp_ggap_window w = Wn[i];
    const GGeo G = gg_geo(w);
    gsnapdp_ggap_result R;
    gsnapdp_ggap_trace X;
    memset(&R, 0, sizeof(R));
    memset(&X, 0, sizeof(X));
    R.dynprogindex = w.dynprogindex;
    R.bridge_ok = 1;
    X.status = ST_EARLY;
    bool done = true;
    if (G.L1 <= 1) {  // :4855-4858
      R.finalscore = NEG;
      R.returned_null = 1;
    } else if (G.L1 > w.maxlength1 || G.L2L > w.maxlength2 || G.L2R > w.maxlength2) {
      R.new_leftgenomepos = w.offset2L - 1;  // :4898-4909
      R.new_rightgenomepos = w.revoffset2R + 1;
      R.exonhead = w.offset1 + G.L1 - 1;
      R.dynprogindex = step_dpi(w.dynprogindex);
      R.finalscore = NEG;
      R.returned_null = 1;
    } else if (G.L2L <= 0 || G.L2R <= 0 || G.eb < 0 || G.L2L < G.L1 - 1 || G.L2R < G.L1 - 1 ||
               w.known_mode > GSNAPDP_KNOWN_INTRONS) {
      // the reference aborts (Matrix3_alloc :495) or, with a flank shorter than
      // length1 - 1, reads the bridge's diagonal cells past its matrix rows
      // (or: an unknown known-site mode)
      R.finalscore = NEG;
      R.returned_null = 1;
      X.status = ST_UNSUPPORTED;
    } else {
      done = false;
      cls = (use_band & GW_USE) && gwin_ok(w, G) ? gwin_list(w, G) : gband_list(w, G, use_band);  // k_gwin / k_gband when they can
      const int bndw = G.L1 + 1 > 64 ? 3 * (max(G.L2L, G.L2R) + 2) : 0;  // stripe boundary row
      if (cls >= 0) {
      } else if (G.L1 + 1 <= 32 && G.words <= GG_SMALL_WORDS) cls = GG_SMALL;
      else if (G.words + bndw <= GG_MID_WORDS) cls = GG_MID;
      else if ((size_t)G.words + bndw <= GG_BIG_WORDS) cls = GG_BIG;
      else {
        done = true;
        R.finalscore = NEG;
        R.returned_null = 1;
        X.status = ST_UNSUPPORTED;  // beyond the large path's scratch
      }
    }
    if (done) {
      res[i] = R;
      trc[i] = X;
    }
  }
  // one global reservation per non-empty list per block (list order is free:
  // every window writes its own result slot)
  const int slot = cls >= 0 ? atomicAdd(&lcnt[cls], 1) : 0;
  __syncthreads();
  if (threadIdx.x < GG_NLISTS)
    lbase[threadIdx.x] = lcnt[threadIdx.x] > 0 ? atomicAdd(counts + threadIdx.x, lcnt[threadIdx.x]) : 0;
  __syncthreads();
  if (cls >= 0) lists[(size_t)cls * cap + lbase[cls] + slot] = i;
}


// ------------------------------------------------------------------ cDNA gaps
constexpr int CDNA_OPEN = -10, CDNA_EXTEND = -7;  // dynprog.c:229-235 (every bin)
constexpr int INSERT_PAIRS = 9;                   // :140

// traceback_cdna (dynprog.c:2716-2812): genome rows, query columns.  Every
// nogap cell pushes a pair (no '*' test); the consistency test is swapped
// (consistent_array[genome][query]); HORIZ runs skip query (add_queryskip with
// cdna_gap_p, :2372) and VERT runs skip genome (add_genomeskip_cdna, :2516,
// with the intron test).  Ops: DIAG runs, VSKIP = query skip, HDASH / HGAP =
// genome skip.  `grow(r)` is genome row r's class, `qcol(c)` column c's
// query byte | uppercase byte << 8.
template <class Dirs, class GRow, class QCol>
__device__ inline void traceback_cdna(const Dirs& dirs, int lband, int rband, int Lr, int Lc,
                                      int rev, int cdna_direction, int r, int c, const GRow& grow,
                                      const QCol& qcol, const uint32_t* __restrict__ cons_sw,
                                      Tally& t, OpWriter& ow) {
  auto inband = [&](int rr, int cc) {
    const int d = rr - cc + rband;
    return rr >= 1 && cc >= 1 && d >= 0 && d <= lband + rband;
  };
  auto gap1_horiz = [&](int rr, int cc) -> bool {
    if (rr == 0) return cc >= 2 && cc <= rband && cc <= Lc;
    if (!inband(rr, cc)) return false;
    return dirs(rr, cc) & 1u;
  };
  auto gap2_vert = [&](int rr, int cc) -> bool {
    if (cc == 0) return rr >= 2 && rr <= lband && rr <= Lr;
    if (!inband(rr, cc)) return false;
    return (dirs(rr, cc) >> 1) & 1u;
  };
  while (inband(r, c)) {
    const uint32_t nib = dirs(r, c);
    const int g = grow(r);
    const uint32_t qq = qcol(c);
    const unsigned char c1 = (unsigned char)(qq & 127u), u1 = (unsigned char)(qq >> 8);
    if (u1 == (unsigned char)("ACGTN*"[g]) || (g < 5 && ((cons_sw[c1] >> (24 + g)) & 1u)))
      t.nmatches++;
    else
      t.nmismatches++;
    t.npush++;
    ow.run++;
    if (nib & 8u) {  // VERT: genome skip
      int dist = 1;
      r--;
      c--;
      while (gap2_vert(r, c)) {
        dist++;
        r--;
      }
      r--;
      bool dashes = true;
      if (dist >= MICROINTRON_LENGTH) {  // rows r+1 .. r+dist are skipped
        const int rl = r + 1, rh = r + dist;
        const int l1 = grow(rev ? rh : rl), l2 = grow(rev ? rh - 1 : rl + 1);
        const int r2 = grow(rev ? rl + 1 : rh - 1), r1 = grow(rev ? rl : rh);
        dashes = intron_type_codes(l1, l2, r2, r1, cdna_direction) == 0;
      }
      ow.flush();
      ow.put(GSNAPDP_OP(dashes ? GSNAPDP_OP_HDASH : GSNAPDP_OP_HGAP, dist));
      t.npush += dashes ? dist : 1;
      if (dashes) {
        t.nopens++;
        t.nindels += dist;
      }
    } else if (nib & 4u) {  // HORIZ: query skip
      int dist = 1;
      r--;
      c--;
      while (gap1_horiz(r, c)) {
        dist++;
        c--;
      }
      c--;
      ow.flush();
      ow.put(GSNAPDP_OP(GSNAPDP_OP_VSKIP, dist));
      t.npush += dist;
      t.nopens++;
      t.nindels += dist;
    } else {
      r--;
      c--;
    }
  }
  ow.flush();
}

struct CGeo {
  int G, L1L, L1R, eb, mt;
  int lbL, rbL, WL, lbR, rbR, WR;
  int oHR, oCwL, oCwR, oQL, oQR, oGL, oGR, oBnd, words, bndw;
};

__device__ inline CGeo cg_geo(const gsnapdp_cgap_window& w) {
  CGeo C;
  C.G = w.length2;
  C.L1L = w.length1L;
  C.L1R = w.length1R;
  C.eb = w.extraband_paired;
  const double dr = (double)w.defect_rate;  // :4622-4641
  C.mt = dr < 0.003 ? MT_HIGHQ : (dr < 0.014 ? MT_MEDQ : MT_LOWQ);
  fill_bands(C.G, C.L1L, C.eb, C.lbL, C.rbL);  // rows = genome, columns = query
  fill_bands(C.G, C.L1R, C.eb, C.lbR, C.rbR);
  C.WL = C.lbL + C.rbL + 1;
  C.WR = C.lbR + C.rbR + 1;
  const int g = C.G > 0 ? C.G : 0, l1 = C.L1L > 0 ? C.L1L : 0, l2 = C.L1R > 0 ? C.L1R : 0;
  C.oHR = g * C.WL;
  C.oCwL = C.oHR + g * C.WR;     // column profile words, 0 .. L1+1
  C.oCwR = C.oCwL + l1 + 2;
  C.oQL = C.oCwR + l2 + 2;       // column query | uc << 8 (u16), 0 .. L1+1
  C.oQR = C.oQL + (l1 + 3) / 2;
  C.oGL = C.oQR + (l2 + 3) / 2;  // genome row classes (bytes), 0 .. G+1
  C.oGR = C.oGL + (g + 2 + 3) / 4;
  C.oBnd = C.oGR + (g + 2 + 3) / 4;
  C.words = C.oBnd;
  C.bndw = C.G + 1 > 64 ? 3 * (max(l1, l2) + 2) : 0;
  return C;
}

template <int RL, bool GMEM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(GG_WAVES, 8))) void k_cgap(
    const gsnapdp_cgap_window* __restrict__ Wn, const int* __restrict__ list,
    const int* __restrict__ count, const char* __restrict__ q, const char* __restrict__ qu,
    const uint32_t* __restrict__ blocks, uint64_t nwords, const uint32_t* __restrict__ prof,
    uint32_t* __restrict__ pool, size_t stride, gsnapdp_cgap_result* __restrict__ res,
    uint32_t* __restrict__ ops, const int64_t* __restrict__ op_off) {
  extern __shared__ uint32_t smem[];
  using P = typename std::conditional<GMEM, AS_GLOBAL uint32_t*, AS_LDS uint32_t*>::type;
  using PB = typename std::conditional<GMEM, AS_GLOBAL uint8_t*, AS_LDS uint8_t*>::type;
  using PH = typename std::conditional<GMEM, AS_GLOBAL uint16_t*, AS_LDS uint16_t*>::type;
  constexpr int NGW = 64 / RL;
  const int lane = threadIdx.x & 63, grp = lane / RL, rho = lane % RL;
  const int gw = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const int nw = (int)((gridDim.x * blockDim.x) >> 6);
  P region;
  if constexpr (GMEM) {
    region = (P)(pool + (size_t)gw * stride);
  } else {
    region = (P)(smem + ((threadIdx.x >> 6) * NGW + grp) * stride);
  }
  const int n = *count;
  for (int base = gw * NGW; base < n; base += nw * NGW) {
    const int k = base + grp;
    const bool act = k < n;
    const int wi = list[act ? k : base];
    const gsnapdp_cgap_window w = Wn[wi];
    CGeo C = cg_geo(w);
    if (!act) C.G = 0;
    const P HL = region, HR = region + C.oHR;
    const P cwL = region + C.oCwL, cwR = region + C.oCwR;
    const PH qL = (PH)(region + C.oQL), qR = (PH)(region + C.oQR);
    const PB gL = (PB)(region + C.oGL), gR = (PB)(region + C.oGR);
    const P bnd = region + C.oBnd;
    const int revoffset2 = w.offset2 + w.length2 - 1;
    // the genome rows of both fills (get_genomic_nt), the query columns
    Lane LG;  // genome view for gclass
    LG.base = w.chroffset + w.chrpos;
    LG.glen = (int)w.genomiclength;
    LG.watson = w.watsonp ? 1 : 0;
    LG.allstar = (LG.base < w.chroffset) || (LG.base >= w.chrhigh);
    const uint32_t* ptab = prof + C.mt * 128;
    if (act) {
      for (int r = rho; r <= C.G + 1; r += RL) {
        const bool in = r >= 1 && r <= C.G;
        gL[r] = (uint8_t)(in ? gclass(blocks, nwords, LG, w.offset2 + r - 1) : 5);
        gR[r] = (uint8_t)(in ? gclass(blocks, nwords, LG, revoffset2 + 1 - r) : 5);
      }
      for (int c = rho; c <= C.L1L + 1; c += RL) {
        const bool in = c >= 1 && c <= C.L1L;
        const int qi = (int)w.qposL + c - 1;
        const unsigned a = in ? (unsigned char)q[qi] : 0u, u = in ? (unsigned char)qu[qi] : 0u;
        cwL[c] = ptab[a & 127u];
        qL[c] = (uint16_t)(a | (u << 8));
      }
      for (int c = rho; c <= C.L1R + 1; c += RL) {
        const bool in = c >= 1 && c <= C.L1R;
        const int qi = (int)w.qposR + 1 - c;  // revsequence1R[1 - c]
        const unsigned a = in ? (unsigned char)q[qi] : 0u, u = in ? (unsigned char)qu[qi] : 0u;
        cwR[c] = ptab[a & 127u];
        qR[c] = (uint16_t)(a | (u << 8));
      }
    }
    if constexpr (GMEM) wave_fence();
    else __builtin_amdgcn_s_waitcnt(0xc07f);
    const int L1max = max(C.L1L, C.L1R);
    const int T = __builtin_amdgcn_readfirstlane(wave_max(act ? L1max + (C.G + 1 > RL ? RL : C.G + 1) : 0));
    const int NS = __builtin_amdgcn_readfirstlane(wave_max(act ? C.G + 1 : 1) + RL - 1) / RL;
    const int jl = w.jump_late_p ? 1 : 0;
    const Side<P> SR = {HR, C.L1R, C.lbR, C.rbR, C.WR};
    const Side<P> SL = {HL, C.L1L, C.lbL, C.rbL, C.WL};
    // right side reversed with !jump_late_p, left side forward (:4680-4710)
    gg_fill<RL, GMEM, true>(SR, cwR, bnd, C.G, rho, CDNA_OPEN, CDNA_EXTEND, 1 - jl,
                            [&](int r) { return 4u * (uint32_t)gR[r]; }, T, NS);
    gg_fill<RL, GMEM, true>(SL, cwL, bnd, C.G, rho, CDNA_OPEN, CDNA_EXTEND, jl,
                            [&](int r) { return 4u * (uint32_t)gL[r]; }, T, NS);
    if constexpr (GMEM) wave_fence();
    else __builtin_amdgcn_s_waitcnt(0xc07f);

    // ---- bridge_cdna_gap (dynprog.c:3068-3146), lane = rL; scan order rL,
    // rR descending, cL, cR, strict >.  rR = 0 never wins: row 0's nogap is
    // NEG_INFINITY over the whole range the bridge reads.
    const int span = w.revoffset1R - w.offset1L;  // cR < span - cL
    const int rbandBL = C.L1L - C.G + C.eb, rbandBR = C.L1R - C.G + C.eb;
    int best = BRIDGE_INIT, bkey = 0x7fffffff, bcL = 0, bcR = 0, brR = 0;
    const int rows = __builtin_amdgcn_readfirstlane(wave_max(act ? C.G : 0));
    for (int r0 = 0; r0 < rows; r0 += RL) {
      const int rL = r0 + rho;
      if (rL < 1 || rL >= C.G) continue;
      const int cloL = max(1, rL - C.eb), chighL = min(C.L1L - 1, rL + rbandBL);
      const int baseL = (rL - 1) * C.WL - rL + C.lbL;
      for (int rR = C.G - rL; rR >= 1; rR--) {
        const int pen = rR == C.G - rL ? 0 : CDNA_OPEN;
        const int cloR = max(1, rR - C.eb), chighR = min(C.L1R - 1, rR + rbandBR);
        const int baseR = (rR - 1) * C.WR - rR + C.lbR;
        for (int cL = cloL; cL <= chighL; cL++) {
          const int sL = (int)HL[baseL + cL] >> 4;
          const int hi = min(chighR, span - cL - 1);
          for (int cR = cloR; cR <= hi; cR++) {
            const int tot = sL + ((int)HR[baseR + cR] >> 4) + pen;
            if (tot > best) {
              best = tot;
              bkey = rL;
              bcL = cL;
              bcR = cR;
              brR = rR;
            }
          }
        }
      }
    }
#pragma unroll
    for (int o = RL / 2; o > 0; o >>= 1) {
      const int ob = __shfl_xor(best, o), ok = __shfl_xor(bkey, o);
      const int ocL = __shfl_xor(bcL, o), ocR = __shfl_xor(bcR, o), orR = __shfl_xor(brR, o);
      if (ob > best || (ob == best && ok < bkey)) {
        best = ob;
        bkey = ok;
        bcL = ocL;
        bcR = ocR;
        brR = orR;
      }
    }
    if (act && rho == 0) {
      gsnapdp_cgap_result R;
      memset(&R, 0, sizeof(R));
      R.dynprogindex = w.dynprogindex;
      R.finalscore = best;
      R.finalscore_set = 1;
      if (bkey == 0x7fffffff) {
        R.status = 5;  // no candidate: the reference traces back from uninitialised indices
        R.returned_null = 1;
      } else {
        const int brL = bkey;
        R.brL = brL;
        R.bcL = bcL;
        R.brR = brR;
        R.bcR = bcR;
        const int64_t o0 = op_off[wi];
        const int cap = (int)(op_off[wi + 1] - o0);
        Tally t = {0, 0, 0, 0, 0};
        OpWriter owR = {ops + o0, cap, 0, 0};
        const uint32_t* cons_sw = prof + PROF_CONS_SWAPPED;
        traceback_cdna(CellDirs<P>{HR, C.WR, C.lbR}, C.lbR, C.rbR, C.G, C.L1R, 1, w.cdna_direction,
                       brR, bcR, [&](int r) -> int { return gR[r]; },
                       [&](int c) -> uint32_t { return qR[c]; }, cons_sw, t, owR);
        const int nR = owR.n < cap ? owR.n : cap;
        OpWriter owL = {ops + o0 + nR, cap - nR, 0, 0};
        traceback_cdna(CellDirs<P>{HL, C.WL, C.lbL}, C.lbL, C.rbL, C.G, C.L1L, 0, w.cdna_direction,
                       brL, bcL, [&](int r) -> int { return gL[r]; },
                       [&](int c) -> uint32_t { return qL[c]; }, cons_sw, t, owL);
        R.nops_right = nR;
        R.nops_left = owL.n < owL.cap ? owL.n : owL.cap;
        if (owR.n > cap || owL.n > owL.cap) R.status = ST_OPS_OVERFLOW;
        const int qj = (w.revoffset1R - bcR) - (w.offset1L + bcL) + 1;
        const int gj = (revoffset2 - brR) - (w.offset2 + brL) + 1;
        R.insert_pairs = qj == INSERT_PAIRS && gj == INSERT_PAIRS;  // :4730
        R.incompletep = !R.insert_pairs;
        R.npairs = t.npush + (R.insert_pairs ? qj + gj : 1);
        if (R.npairs == 1) {  // only the gapholder (:4779)
          R.npairs = 0;
          R.returned_null = 1;
        }
        R.dynprogindex = step_dpi(w.dynprogindex);
      }
      res[wi] = R;
    }
  }
}

// Early returns (dynprog.c:4605, 4651-4675) and the class of every cDNA-gap window
__global__ void k_cgap_plan(const gsnapdp_cgap_window* __restrict__ Wn, int n,
                            gsnapdp_cgap_result* __restrict__ res, int* __restrict__ lists,
                            int* __restrict__ counts, int cap) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  int cls = -1;
  if (i < n) {
    const gsnapdp_cgap_window w = Wn[i];
    const CGeo C = cg_geo(w);
    gsnapdp_cgap_result R;
    memset(&R, 0, sizeof(R));
    R.dynprogindex = w.dynprogindex;
    R.status = ST_EARLY;
    R.returned_null = 1;
    bool done = true;
    if (C.G <= 1) {
      // NULL, nothing written
    } else if (C.G > w.maxlength1 || C.L1R > w.maxlength2 || C.L1L > w.maxlength2) {
      R.dynprogindex = step_dpi(w.dynprogindex);
    } else if (C.L1L <= 0 || C.L1R <= 0 || C.eb < 0) {
      R.status = ST_UNSUPPORTED;  // the reference aborts (Matrix3_alloc :495)
    } else {
      done = false;
      if (C.G + 1 <= 32 && C.words <= GG_SMALL_WORDS) cls = GG_SMALL;
      else if (C.words + C.bndw <= GG_MID_WORDS) cls = GG_MID;
      else if ((size_t)C.words + C.bndw <= GG_BIG_WORDS) cls = GG_BIG;
      else {
        done = true;
        R.status = ST_UNSUPPORTED;
      }
    }
    if (done) res[i] = R;
  }
#pragma unroll
  for (int c = 0; c < GG_NCLS; c++) {
    const int pos = agg_atomic_inc(counts + c, cls == c ? 0 : -1);
    if (cls == c) lists[(size_t)c * cap + pos] = i;
  }
}

}  // namespace

// ======================================================================
// Host side (include/gsnapdp.h: gsnapdp_ggap_*; k_rows for gsnapdp_run_device)
// ======================================================================
// global scratch of the row-lane classes that do not fit LDS, on first use
int gsnapdp__rows_pools(gsnapdp_ctx* ctx) {
  if (!ctx->d_bigpool) HIPCHK(hipMalloc(&ctx->d_bigpool, (size_t)RW_BIG_WAVES * RW_BIG_WORDS * 4));
  if (!ctx->d_largepool)
    HIPCHK(hipMalloc(&ctx->d_largepool,
                     (size_t)ctx->num_cus * RW_LARGE_WAVES_PER_CU * RW_LARGE_WORDS * 4));
  return 0;
}

// k_rows takes every byte of a CU's LDS as dynamic LDS, so it must declare no
// static __shared__ of its own (round 5: a 4-byte static ticket beside the
// 160 KB made group_seg_size 163844 and aborted the queue)
constexpr size_t RW_DYN_LDS = (size_t)160 * 1024;

int gsnapdp__ggap_lds_check(size_t max_lds) {
  const size_t small = (size_t)8 * GG_SMALL_WORDS * 4, mid = (size_t)4 * GG_MID_WORDS * 4;
  if (gsnapdp__lds_fits((const void*)&k_rows<false>, RW_DYN_LDS, max_lds, "k_rows") ||
      gsnapdp__lds_fits((const void*)&k_rows<true>, RW_DYN_LDS, max_lds, "k_rows<SEG>") ||
      gsnapdp__lds_fits((const void*)&k_sj_plan, 0, max_lds, "k_sj_plan") ||
      gsnapdp__lds_fits((const void*)&k_ggap_plan, 0, max_lds, "k_ggap_plan") ||
      gsnapdp__lds_fits((const void*)&k_ggap<32, false>, small, max_lds, "k_ggap<32>") ||
      gsnapdp__lds_fits((const void*)&k_ggap<64, false>, mid, max_lds, "k_ggap<64>") ||
      gsnapdp__lds_fits((const void*)&k_ggap<64, true>, 0, max_lds, "k_ggap<64, striped>") ||
      gsnapdp__lds_fits((const void*)&k_cgap_plan, 0, max_lds, "k_cgap_plan") ||
      gsnapdp__lds_fits((const void*)&k_cgap<32, false>, small, max_lds, "k_cgap<32>") ||
      gsnapdp__lds_fits((const void*)&k_cgap<64, false>, mid, max_lds, "k_cgap<64>") ||
      gsnapdp__lds_fits((const void*)&k_cgap<64, true>, 0, max_lds, "k_cgap<64, striped>"))
    return -1;
  return 0;
}

// the row-lane classes, one launch each (lists[c * list_cap ...], counts[c])
template <bool SEG>
static int rows_launch(gsnapdp_ctx* ctx, hipStream_t st, const gsnapdp_window* dw, const int* lists,
                       int* counts, int list_cap, const char* d_query, const char* d_query_uc,
                       gsnapdp_result* d_results, uint32_t* d_ops, const int64_t* d_op_offsets,
                       const gsnapdp_sj_window* sjw) {
  const uint64_t nw = (uint64_t)ctx->nwords;
  // k_rows: one 16-wave block per CU, every class in turn (the LDS classes at
  // their old occupancy: tiny 64 windows, small 32, mid 8 per CU)
  static_assert(64 * RW_TINY_WORDS * 4 <= 160 * 1024 && 32 * RW_SMALL_WORDS * 4 <= 160 * 1024 &&
                    8 * RW_MID_WORDS * 4 <= 160 * 1024 && RW_LARGE_WAVES_PER_CU == 16 &&
                    RW_BIG_WAVES % 16 == 0,
                "k_rows regions");
  // (gsnapdp_create checked num_cus * 16 >= RW_BIG_WAVES and the static + dynamic LDS)
  hipLaunchKernelGGL((k_rows<SEG>), dim3(ctx->num_cus), dim3(1024), RW_DYN_LDS, st, dw, lists,
                     list_cap, counts, d_query, d_query_uc, ctx->d_blocks, nw, ctx->d_prof,
                     ctx->d_largepool, ctx->d_bigpool, d_results, d_ops, d_op_offsets, sjw);
  HIPCHK(hipGetLastError());
  return 0;
}

int gsnapdp__rows_launch(gsnapdp_ctx* ctx, hipStream_t st, const gsnapdp_window* d_windows,
                         const int* lists, int* counts, int list_cap, const char* d_query,
                         const char* d_query_uc, gsnapdp_result* d_results, uint32_t* d_ops,
                         const int64_t* d_op_offsets, const gsnapdp_sj_window* sjw) {
  if (sjw)
    return rows_launch<true>(ctx, st, d_windows, lists, counts, list_cap, d_query, d_query_uc,
                             d_results, d_ops, d_op_offsets, sjw);
  return rows_launch<false>(ctx, st, d_windows, lists, counts, list_cap, d_query, d_query_uc,
                            d_results, d_ops, d_op_offsets, nullptr);
}

// ======================================================================
// Host side (include/gsnapdp.h: gsnapdp_sj_*)
// ======================================================================
extern "C" int gsnapdp_sj_run_device(gsnapdp_ctx* ctx, const gsnapdp_sj_window* d_windows, int n,
                                     const char* d_query, const char* d_query_uc,
                                     gsnapdp_result* d_results, uint32_t* d_ops,
                                     const int64_t* d_op_offsets, void* stream_v) {
  if (!ctx) return -1;
  if (n <= 0) return 0;
  hipStream_t st = stream_v ? (hipStream_t)stream_v : ctx->stream;
  std::lock_guard<std::mutex> lock(ctx->mu);
  HIPCHK(hipSetDevice(ctx->device));
  if (n > ctx->sj_cap) {
    const int cap = n + n / 4 + 1024;
    (void)hipFree(ctx->d_sj_win);
    ctx->d_sj_win = nullptr;
    HIPCHK(hipMalloc(&ctx->d_sj_win, (size_t)cap * sizeof(gsnapdp_window)));
    ctx->sj_cap = cap;
  }
  gsnapdp_window* dw = ctx->d_sj_win;
  // the end-gap windows of the records (early returns finished here), then the
  // single/end-gap pipeline on their segments: the register band (k_fill's
  // END = 2 fill) or k_rows in segment mode
  hipLaunchKernelGGL(k_sj_plan, dim3((n + 255) / 256), dim3(256), 0, st, d_windows, n, d_query,
                     d_query_uc, dw, d_results);
  return gsnapdp__fill_pipeline(ctx, st, dw, n, d_query, d_query_uc, d_results, d_ops, d_op_offsets,
                                d_windows);
}

extern "C" int gsnapdp_sj_run_host(gsnapdp_ctx* ctx, const gsnapdp_sj_window* windows, int n,
                                   const char* query, const char* query_uc, size_t query_bytes,
                                   gsnapdp_result* results, uint32_t* ops,
                                   const int64_t* op_offsets) {
  if (!ctx) return -1;
  if (n <= 0) return 0;
  // one host round trip at a time: the staging buffer is the context's
  std::lock_guard<std::mutex> host_lock(ctx->host_mu);
  HIPCHK(hipSetDevice(ctx->device));
  const size_t nops = (size_t)op_offsets[n];
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t szw = al((size_t)n * sizeof(gsnapdp_sj_window));
  const size_t szq = al(query_bytes + 4);
  const size_t szr = al((size_t)n * sizeof(gsnapdp_result));
  const size_t szo = al((nops + 1) * 4);
  const size_t szoff = al((size_t)(n + 1) * 8);
  const size_t total = szw + 2 * szq + szr + szo + szoff;
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
  gsnapdp_sj_window* dw = (gsnapdp_sj_window*)b;
  char* dq = b + szw;
  char* du = dq + szq;
  gsnapdp_result* dr = (gsnapdp_result*)(du + szq);
  uint32_t* dops = (uint32_t*)((char*)dr + szr);
  int64_t* doff = (int64_t*)((char*)dops + szo);
  hipStream_t st = ctx->stream;
  HIPCHK(hipMemcpyAsync(dw, windows, (size_t)n * sizeof(gsnapdp_sj_window), hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(dq, query, query_bytes, hipMemcpyHostToDevice, st));
  // a caller that passes one buffer for both (query already upper case) pays one copy
  if (query_uc == query) du = dq;
  else HIPCHK(hipMemcpyAsync(du, query_uc, query_bytes, hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(doff, op_offsets, (size_t)(n + 1) * 8, hipMemcpyHostToDevice, st));
  if (gsnapdp_sj_run_device(ctx, dw, n, dq, du, dr, dops, doff, st)) return -1;
  HIPCHK(hipMemcpyAsync(results, dr, (size_t)n * sizeof(gsnapdp_result), hipMemcpyDeviceToHost, st));
  if (nops) HIPCHK(hipMemcpyAsync(ops, dops, nops * 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  return 0;
}

// ======================================================================
// Host side (include/gsnapdp.h: gsnapdp_ggap_*)
// ======================================================================
static int ggap_capacity(gsnapdp_ctx* ctx, int n) {
  if (n > ctx->ggap_cap) {
    const int cap = n + n / 4 + 1024;
    (void)hipFree(ctx->d_ggap_lists);
    ctx->d_ggap_lists = nullptr;
    HIPCHK(hipMalloc(&ctx->d_ggap_lists, (size_t)GG_NLISTS * cap * 4));
    ctx->ggap_cap = cap;
  }
  if (!ctx->d_ggap_counts) HIPCHK(hipMalloc(&ctx->d_ggap_counts, 128));
  return 0;
}

extern "C" int gsnapdp_ggap_run_device(gsnapdp_ctx* ctx, const gsnapdp_ggap_window* d_windows,
                                       int n, const char* d_query, const char* d_query_uc,
                                       gsnapdp_ggap_result* d_results, gsnapdp_ggap_trace* d_traces,
                                       uint32_t* d_ops, const int64_t* d_op_offsets, void* stream_v) {
  if (!ctx) return -1;
  if (n <= 0) return 0;
  hipStream_t st = stream_v ? (hipStream_t)stream_v : ctx->stream;
  std::lock_guard<std::mutex> lock(ctx->mu);
  HIPCHK(hipSetDevice(ctx->device));
  if (ggap_capacity(ctx, n)) return -1;
  if (!ctx->d_ggap_pool)
    HIPCHK(hipMalloc(&ctx->d_ggap_pool, (size_t)GG_BIG_WAVES * GG_BIG_WORDS * 4));
  const uint64_t nw = (uint64_t)ctx->nwords;
  int* counts = ctx->d_ggap_counts;
  int* lists = ctx->d_ggap_lists;
  const int cap = ctx->ggap_cap;
  HIPCHK(hipMemsetAsync(counts, 0, 4 * GG_NLISTS, st));
  gsnapdp__mark(ctx, st, 4, 0);
  // k_gwin takes probability-mode windows of batches of at least gwin_min
  // windows when the MaxEnt tables are loaded (GSNAPDP_GWIN=0: k_ggap / k_gband
  // as before, for A/B tests)
  const int use_gwin =
      ctx->gwin_on && ctx->d_tables && !ctx->ggap_rowlane_only && n >= ctx->gwin_min ? GW_USE : 0;
  const int use_band = (n >= ctx->gband_min ? ctx->ggap_use_band : 0) | use_gwin;
  hipLaunchKernelGGL(k_ggap_plan, dim3((n + 255) / 256), dim3(256), 0, st, d_windows, n,
                     d_results, d_traces, lists, counts, cap, use_band);
  gsnapdp__mark(ctx, st, 4, 1);
  gsnapdp__mark(ctx, st, 6, 0);
  if ((use_band & (GB_USE_SCORE | GB_USE_PROB)) &&
      gsnapdp__gband_launch(ctx, st, d_windows, lists, counts, cap, d_query, d_query_uc, d_results, d_traces,
                            d_ops, d_op_offsets, use_band))
    return -1;
  gsnapdp__mark(ctx, st, 6, 1);
  // (k_gwin timed as a stage of its own, not inside k_gband's)
  gsnapdp__mark(ctx, st, 8, 0);
  if (use_gwin && gsnapdp__gwin_launch(ctx, st, d_windows, lists, counts, cap, d_query, d_query_uc, d_results,
                                       d_traces, d_ops, d_op_offsets))
    return -1;
  gsnapdp__mark(ctx, st, 8, 1);
  gsnapdp__mark(ctx, st, 5, 0);
  // small windows: 4 waves x 2 windows per block, as many blocks per CU as LDS holds
  hipLaunchKernelGGL((k_ggap<32, false>), dim3(ctx->num_cus * GG_SMALL_BLOCKS), dim3(256),
                     (size_t)8 * GG_SMALL_WORDS * 4, st, d_windows, lists, counts + GG_SMALL,
                     d_query, d_query_uc, ctx->d_blocks, nw, ctx->d_prof, ctx->d_tables,
                     (uint32_t*)nullptr, (size_t)GG_SMALL_WORDS, d_results, d_traces, d_ops,
                     d_op_offsets);
  // rows 32..63: one window per wave, 2 blocks per CU
  hipLaunchKernelGGL((k_ggap<64, false>), dim3(ctx->num_cus * 2), dim3(256),
                     (size_t)4 * GG_MID_WORDS * 4, st, d_windows, lists + (size_t)GG_MID * cap,
                     counts + GG_MID, d_query, d_query_uc, ctx->d_blocks, nw, ctx->d_prof,
                     ctx->d_tables, (uint32_t*)nullptr, (size_t)GG_MID_WORDS, d_results, d_traces,
                     d_ops, d_op_offsets);
  // the rest: stripes of 64 rows, storage in global scratch
  hipLaunchKernelGGL((k_ggap<64, true>), dim3(GG_BIG_WAVES), dim3(64), 0, st, d_windows,
                     lists + (size_t)GG_BIG * cap, counts + GG_BIG, d_query, d_query_uc,
                     ctx->d_blocks, nw, ctx->d_prof, ctx->d_tables, ctx->d_ggap_pool,
                     GG_BIG_WORDS, d_results, d_traces, d_ops, d_op_offsets);
  gsnapdp__mark(ctx, st, 5, 1);
  HIPCHK(hipGetLastError());
  return 0;
}

extern "C" int gsnapdp_ggap_run_host(gsnapdp_ctx* ctx, const gsnapdp_ggap_window* windows, int n,
                                     const char* query, const char* query_uc, size_t query_bytes,
                                     gsnapdp_ggap_result* results, gsnapdp_ggap_trace* traces,
                                     uint32_t* ops, const int64_t* op_offsets) {
  if (!ctx) return -1;
  if (n <= 0) return 0;
  HIPCHK(hipSetDevice(ctx->device));
  const size_t nops = (size_t)op_offsets[n];
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t szw = al((size_t)n * sizeof(gsnapdp_ggap_window));
  const size_t szq = al(query_bytes + 4);
  const size_t szr = al((size_t)n * sizeof(gsnapdp_ggap_result));
  const size_t szt = al((size_t)n * sizeof(gsnapdp_ggap_trace));
  const size_t szo = al((nops + 1) * 4);
  const size_t szoff = al((size_t)(n + 1) * 8);
  const bool alias = query_uc == query;  // one buffer for both (query already upper case): one copy
  // inputs first (windows, query, query_uc, op offsets), then the outputs
  const size_t in_bytes = szw + (alias ? 1 : 2) * szq + szoff;
  const size_t total = in_bytes + szr + szt + szo;
  const bool small = in_bytes <= ((size_t)1 << 20);  // one packed H2D copy (the per-call drop-in)
  // one host round trip at a time per context (the staging buffers are shared)
  std::lock_guard<std::mutex> host_lock(ctx->host_mu);
  {
    std::lock_guard<std::mutex> lock(ctx->mu);
    if (total > ctx->ggap_stage_cap) {
      (void)hipFree(ctx->d_ggap_stage);
      ctx->d_ggap_stage = nullptr;
      HIPCHK(hipMalloc(&ctx->d_ggap_stage, total));
      ctx->ggap_stage_cap = total;
    }
    if (small && in_bytes > ctx->h_in_cap) {
      if (ctx->h_in) (void)hipHostFree(ctx->h_in);
      ctx->h_in = nullptr;
      HIPCHK(hipHostMalloc(&ctx->h_in, (size_t)1 << 20));
      ctx->h_in_cap = (size_t)1 << 20;
    }
  }
  char* b = (char*)ctx->d_ggap_stage;
  const size_t o_q = szw, o_u = szw + szq, o_off = o_u + (alias ? 0 : szq);
  gsnapdp_ggap_window* dw = (gsnapdp_ggap_window*)b;
  char* dq = b + o_q;
  char* du = alias ? dq : b + o_u;
  int64_t* doff = (int64_t*)(b + o_off);
  gsnapdp_ggap_result* dr = (gsnapdp_ggap_result*)(b + in_bytes);
  gsnapdp_ggap_trace* dt = (gsnapdp_ggap_trace*)((char*)dr + szr);
  uint32_t* dops = (uint32_t*)((char*)dt + szt);
  hipStream_t st = ctx->stream;
  if (small) {
    char* h = (char*)ctx->h_in;
    memcpy(h, windows, (size_t)n * sizeof(gsnapdp_ggap_window));
    memcpy(h + o_q, query, query_bytes);
    if (!alias) memcpy(h + o_u, query_uc, query_bytes);
    memcpy(h + o_off, op_offsets, (size_t)(n + 1) * 8);
    HIPCHK(hipMemcpyAsync(b, h, o_off + (size_t)(n + 1) * 8, hipMemcpyHostToDevice, st));
  } else {
    HIPCHK(hipMemcpyAsync(dw, windows, (size_t)n * sizeof(gsnapdp_ggap_window), hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(dq, query, query_bytes, hipMemcpyHostToDevice, st));
    if (!alias) HIPCHK(hipMemcpyAsync(du, query_uc, query_bytes, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(doff, op_offsets, (size_t)(n + 1) * 8, hipMemcpyHostToDevice, st));
  }
  if (gsnapdp_ggap_run_device(ctx, dw, n, dq, du, dr, dt, dops, doff, st)) return -1;
  HIPCHK(hipMemcpyAsync(results, dr, (size_t)n * sizeof(gsnapdp_ggap_result), hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(traces, dt, (size_t)n * sizeof(gsnapdp_ggap_trace), hipMemcpyDeviceToHost, st));
  if (nops) HIPCHK(hipMemcpyAsync(ops, dops, nops * 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  return 0;
}

extern "C" int gsnapdp_cgap_run_device(gsnapdp_ctx* ctx, const gsnapdp_cgap_window* d_windows,
                                       int n, const char* d_query, const char* d_query_uc,
                                       gsnapdp_cgap_result* d_results, uint32_t* d_ops,
                                       const int64_t* d_op_offsets, void* stream_v) {
  if (!ctx) return -1;
  if (n <= 0) return 0;
  hipStream_t st = stream_v ? (hipStream_t)stream_v : ctx->stream;
  std::lock_guard<std::mutex> lock(ctx->mu);
  HIPCHK(hipSetDevice(ctx->device));
  if (ggap_capacity(ctx, n)) return -1;
  if (!ctx->d_ggap_pool)
    HIPCHK(hipMalloc(&ctx->d_ggap_pool, (size_t)GG_BIG_WAVES * GG_BIG_WORDS * 4));
  const uint64_t nw = (uint64_t)ctx->nwords;
  int* counts = ctx->d_ggap_counts;
  int* lists = ctx->d_ggap_lists;
  const int cap = ctx->ggap_cap;
  HIPCHK(hipMemsetAsync(counts, 0, 4 * GG_NCLS, st));
  hipLaunchKernelGGL(k_cgap_plan, dim3((n + 255) / 256), dim3(256), 0, st, d_windows, n, d_results,
                     lists, counts, cap);
  hipLaunchKernelGGL((k_cgap<32, false>), dim3(ctx->num_cus * GG_SMALL_BLOCKS), dim3(256),
                     (size_t)8 * GG_SMALL_WORDS * 4, st, d_windows, lists, counts + GG_SMALL,
                     d_query, d_query_uc, ctx->d_blocks, nw, ctx->d_prof, (uint32_t*)nullptr,
                     (size_t)GG_SMALL_WORDS, d_results, d_ops, d_op_offsets);
  hipLaunchKernelGGL((k_cgap<64, false>), dim3(ctx->num_cus * 2), dim3(256),
                     (size_t)4 * GG_MID_WORDS * 4, st, d_windows, lists + (size_t)GG_MID * cap,
                     counts + GG_MID, d_query, d_query_uc, ctx->d_blocks, nw, ctx->d_prof,
                     (uint32_t*)nullptr, (size_t)GG_MID_WORDS, d_results, d_ops, d_op_offsets);
  hipLaunchKernelGGL((k_cgap<64, true>), dim3(GG_BIG_WAVES), dim3(64), 0, st, d_windows,
                     lists + (size_t)GG_BIG * cap, counts + GG_BIG, d_query, d_query_uc,
                     ctx->d_blocks, nw, ctx->d_prof, ctx->d_ggap_pool, GG_BIG_WORDS, d_results,
                     d_ops, d_op_offsets);
  HIPCHK(hipGetLastError());
  return 0;
}

extern "C" int gsnapdp_cgap_run_host(gsnapdp_ctx* ctx, const gsnapdp_cgap_window* windows, int n,
                                     const char* query, const char* query_uc, size_t query_bytes,
                                     gsnapdp_cgap_result* results, uint32_t* ops,
                                     const int64_t* op_offsets) {
  if (!ctx) return -1;
  if (n <= 0) return 0;
  // one host round trip at a time: the staging buffer is the context's
  std::lock_guard<std::mutex> host_lock(ctx->host_mu);
  HIPCHK(hipSetDevice(ctx->device));
  const size_t nops = (size_t)op_offsets[n];
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t szw = al((size_t)n * sizeof(gsnapdp_cgap_window));
  const size_t szq = al(query_bytes + 4);
  const size_t szr = al((size_t)n * sizeof(gsnapdp_cgap_result));
  const size_t szo = al((nops + 1) * 4);
  const size_t szoff = al((size_t)(n + 1) * 8);
  const size_t total = szw + 2 * szq + szr + szo + szoff;
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
  gsnapdp_cgap_window* dw = (gsnapdp_cgap_window*)b;
  char* dq = b + szw;
  char* du = dq + szq;
  gsnapdp_cgap_result* dr = (gsnapdp_cgap_result*)(du + szq);
  uint32_t* dops = (uint32_t*)((char*)dr + szr);
  int64_t* doff = (int64_t*)((char*)dops + szo);
  hipStream_t st = ctx->stream;
  HIPCHK(hipMemcpyAsync(dw, windows, (size_t)n * sizeof(gsnapdp_cgap_window), hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(dq, query, query_bytes, hipMemcpyHostToDevice, st));
  // a caller that passes one buffer for both (query already upper case) pays one copy
  if (query_uc == query) du = dq;
  else HIPCHK(hipMemcpyAsync(du, query_uc, query_bytes, hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(doff, op_offsets, (size_t)(n + 1) * 8, hipMemcpyHostToDevice, st));
  if (gsnapdp_cgap_run_device(ctx, dw, n, dq, du, dr, dops, doff, st)) return -1;
  HIPCHK(hipMemcpyAsync(results, dr, (size_t)n * sizeof(gsnapdp_cgap_result), hipMemcpyDeviceToHost, st));
  if (nops) HIPCHK(hipMemcpyAsync(ops, dops, nops * 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  return 0;
}
