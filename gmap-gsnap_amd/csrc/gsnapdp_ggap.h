// gsnapdp_ggap.h -- Dynprog_genome_gap pieces shared by the row-lane kernel
// k_ggap (gsnapdp_ggap.hip) and the register-band kernel k_gband
// (gsnapdp_gband.hip): constants, window geometry, intron scores, known-site
// flags, dinucleotide codes, MaxEnt site probabilities and the per-flank Lane.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gsnapdp_device.h"
#include "gsnapdp_internal.h"

namespace gsnapdp {

// dynprog.c:142-293, intron.h:10-29
constexpr int SINGLE_OPEN = -10, SINGLE_EXTEND = -3, PAIRED_OPEN = -18, PAIRED_EXTEND = -3;
constexpr int GCAG_INTRON = 15, ATAC_INTRON = 12, FINAL_GCAG_INTRON = 20, FINAL_ATAC_INTRON = 12;
constexpr int LEFT_GT = 0x21, LEFT_GC = 0x10, LEFT_AT = 0x08, LEFT_CT = 0x06;
constexpr int RIGHT_AG = 0x30, RIGHT_AC = 0x0C, RIGHT_GC = 0x02, RIGHT_AT = 0x01;
constexpr int GTAG_FWD = 0x20, GCAG_FWD = 0x10, ATAC_FWD = 0x08;
constexpr int GTAG_REV = 0x04, GCAG_REV = 0x02, ATAC_REV = 0x01;
constexpr int BRIDGE_INIT = -100000;  // bestscore / bestscoreI start (:3302)

__device__ inline bool ggap_needs_tables(const gsnapdp_ggap_window& w) {
  return w.use_probabilities_p || w.finalp;
}

// Window geometry: widened fill bands (dynprog.c:1442-1454 with widebandp) and
// the storage layout of one window (words): H|dirs of the left flank (L1 x WL),
// of the right flank (L1 x WR), the column classes of both flanks (bytes), the
// site probabilities (probability mode, doubles) and the stripe boundary row.
struct GGeo {
  int L1, L2L, L2R, eb;
  int lbL, rbL, WL, lbR, rbR, WR;
  int mt, open, ext, canon;
  int oHR, oClsL, oClsR, oDiL, oDiR, oItab, oQ, oProbL, oProbR, oBnd, words;
};

__device__ __host__ inline void fill_bands(int L1, int L2, int eb, int& lb, int& rb) {
  if (L2 >= L1) {
    rb = L2 - L1 + eb;
    lb = eb;
  } else {
    lb = L1 - L2 + eb;
    rb = eb;
  }
}

__device__ inline GGeo gg_geo(const gsnapdp_ggap_window& w) {
  GGeo G;
  G.L1 = w.length1;
  G.L2L = w.length2L;
  G.L2R = w.length2R;
  G.eb = w.extraband_paired;
  fill_bands(G.L1, G.L2L, G.eb, G.lbL, G.rbL);
  fill_bands(G.L1, G.L2R, G.eb, G.lbR, G.rbR);
  G.WL = G.lbL + G.rbL + 1;
  G.WR = G.lbR + G.rbR + 1;
  const double dr = (double)w.defect_rate;  // dynprog.c:4871-4886
  G.mt = dr < 0.003 ? MT_HIGHQ : (dr < 0.014 ? MT_MEDQ : MT_LOWQ);
  if (G.L1 > w.maxpeelback * 4) {  // :4888-4896
    G.open = SINGLE_OPEN;
    G.ext = SINGLE_EXTEND;
  } else {
    G.open = PAIRED_OPEN;
    G.ext = PAIRED_EXTEND;
  }
  const int canon[3] = {10, 16, 22}, fcanon[3] = {30, 36, 42};  // :277-283
  G.canon = !w.splicingp ? 0 : (w.finalp ? fcanon[G.mt] : canon[G.mt]);
  const int l1 = G.L1 > 0 ? G.L1 : 0;
  G.oHR = l1 * G.WL;
  G.oClsL = G.oHR + l1 * G.WR;
  G.oClsR = G.oClsL + (G.L2L + 2 + 3) / 4;
  G.oDiL = G.oClsR + (G.L2R + 2 + 3) / 4;     // leftdi[0 .. L2L]   (bytes)
  G.oDiR = G.oDiL + (G.L2L + 1 + 3) / 4;      // rightdi[0 .. L2R]  (bytes)
  G.oItab = G.oDiR + (G.L2R + 1 + 3) / 4;     // intron score | type << 8 by leftdi & rightdi (64 x u16)
  G.oQ = G.oItab + 32;                        // query | uppercase << 8 per query index (u16)
  int o = G.oQ + (l1 + 1) / 2;
  o = (o + 1) & ~1;
  G.oProbL = o;
  G.oProbR = o + 2 * G.L2L;
  if (w.use_probabilities_p) o += 2 * (G.L2L + G.L2R);
  G.oBnd = o;
  G.words = o;
  return G;
}

// intron_score (dynprog.c:3148-3192), non-PMAP
__device__ inline int intron_score(int& introntype, int leftdi, int rightdi, int cdna_direction,
                                   int canonical_reward, int finalp) {
  const int t = leftdi & rightdi;
  const int gcag = finalp ? FINAL_GCAG_INTRON : GCAG_INTRON;
  const int atac = finalp ? FINAL_ATAC_INTRON : ATAC_INTRON;
  introntype = t;
  if (t == 0) return 0;
  if (cdna_direction > 0) {
    if (t == GTAG_FWD) return canonical_reward;
    if (t == GCAG_FWD) return gcag;
    if (t == ATAC_FWD) return atac;
  } else if (cdna_direction < 0) {
    if (t == GTAG_REV) return canonical_reward;
    if (t == GCAG_REV) return gcag;
    if (t == ATAC_REV) return atac;
  } else {
    if (t == GTAG_FWD || t == GTAG_REV) return canonical_reward;
    if (t == GCAG_FWD || t == GCAG_REV) return gcag;
    if (t == ATAC_FWD || t == ATAC_REV) return atac;
  }
  introntype = 0;
  return 0;
}

// Known splice sites: bit 7 of a leftdi / rightdi byte (the dinucleotide codes
// use 6 bits, intron.h:10-18) carries left_known / right_known.
constexpr int KNOWN_BIT = 0x80, DI_MASK = 0x3F;
constexpr int KNOWN_REWARD = 20;  // KNOWN_SPLICESITE_REWARD (dynprog.c:285)
__device__ inline int kreward(int d) { return (d >> 7) * KNOWN_REWARD; }
__device__ inline bool kflag(const unsigned char* f, int km, int c) { return km != 0 && f[c] != 0; }
// IIT_exists_with_divno_signed on the intron (cL, cR) (:3598-3612), from the
// caller's pair list
__device__ inline bool known_intron(const unsigned char* p, int cL, int cR) {
  const int n = p[0] | (p[1] << 8);
  for (int i = 0; i < n; i++) {
    const unsigned char* e = p + 2 + 4 * i;
    if ((e[0] | (e[1] << 8)) == cL && (e[2] | (e[3] << 8)) == cR) return true;
  }
  return false;
}

// leftdi / rightdi (dynprog.c:3331-3373) from two genome class codes
__device__ inline int left_di(int a, int b) {
  if (a == 2 && b == 3) return LEFT_GT;
  if (a == 2 && b == 1) return LEFT_GC;
  if (a == 0 && b == 3) return LEFT_AT;
  if (a == 1 && b == 3) return LEFT_CT;
  return 0;
}
__device__ inline int right_di(int b, int a) {
  if (b == 0 && a == 2) return RIGHT_AG;
  if (b == 0 && a == 1) return RIGHT_AC;
  if (b == 2 && a == 1) return RIGHT_GC;
  if (b == 0 && a == 3) return RIGHT_AT;
  return 0;
}

// Maxent site probability of a left / right splice column
// (get_splicesite_probs :3195-3287, probability precompute :3856-3903).
__device__ inline double left_site_prob(const gsnapdp_ggap_window& w, int cL,
                                        const uint32_t* blocks, uint64_t nwords, const double* T) {
  const int cdir = w.cdna_direction;
  uint32_t pos;
  if (w.watsonp) {
    pos = w.chrpos + (uint32_t)w.offset2L + (uint32_t)cL;
    return maxent_prob(cdir > 0 ? GSNAPDP_DONOR : GSNAPDP_ANTIACCEPTOR, w.chroffset + pos,
                       w.chroffset, blocks, nwords, T);
  }
  pos = w.chrpos + (uint32_t)(w.genomiclength - 1) - (uint32_t)w.offset2L - (uint32_t)cL + 1u;
  return maxent_prob(cdir > 0 ? GSNAPDP_ANTIDONOR : GSNAPDP_ACCEPTOR, w.chroffset + pos,
                     w.chroffset, blocks, nwords, T);
}
__device__ inline double right_site_prob(const gsnapdp_ggap_window& w, int cR,
                                         const uint32_t* blocks, uint64_t nwords, const double* T) {
  const int cdir = w.cdna_direction;
  uint32_t pos;
  if (w.watsonp) {
    pos = w.chrpos + (uint32_t)w.revoffset2R - (uint32_t)cR + 1u;
    return maxent_prob(cdir > 0 ? GSNAPDP_ACCEPTOR : GSNAPDP_ANTIDONOR, w.chroffset + pos,
                       w.chroffset, blocks, nwords, T);
  }
  pos = w.chrpos + (uint32_t)(w.genomiclength - 1) - (uint32_t)w.revoffset2R + (uint32_t)cR;
  return maxent_prob(cdir > 0 ? GSNAPDP_ANTIACCEPTOR : GSNAPDP_DONOR, w.chroffset + pos,
                     w.chroffset, blocks, nwords, T);
}

// The model and position line of one flank's splice columns: column c's site
// is sp0 + step * c with model m, as left_site_prob / right_site_prob compute
// them (uint32 arithmetic, the same wrap-around).
__device__ inline void site_line(const gsnapdp_ggap_window& w, int right, int& m, uint32_t& sp0, int& step) {
  const int cdir = w.cdna_direction;
  const uint32_t last = (uint32_t)(w.genomiclength - 1);
  if (!right) {
    if (w.watsonp) {
      m = cdir > 0 ? GSNAPDP_DONOR : GSNAPDP_ANTIACCEPTOR;
      sp0 = w.chroffset + (w.chrpos + (uint32_t)w.offset2L);
      step = 1;
    } else {
      m = cdir > 0 ? GSNAPDP_ANTIDONOR : GSNAPDP_ACCEPTOR;
      sp0 = w.chroffset + (w.chrpos + last - (uint32_t)w.offset2L + 1u);
      step = -1;
    }
  } else {
    if (w.watsonp) {
      m = cdir > 0 ? GSNAPDP_ACCEPTOR : GSNAPDP_ANTIDONOR;
      sp0 = w.chroffset + (w.chrpos + (uint32_t)w.revoffset2R + 1u);
      step = -1;
    } else {
      m = cdir > 0 ? GSNAPDP_ANTIACCEPTOR : GSNAPDP_DONOR;
      sp0 = w.chroffset + (w.chrpos + last - (uint32_t)w.revoffset2R);
      step = 1;
    }
  }
}

// The per-side view the shared traceback template expects (gsnapdp_device.h).
__device__ inline Lane side_lane(const gsnapdp_ggap_window& w, const GGeo& G, int right) {
  Lane L;
  L.d.L1 = G.L1;
  L.d.L2 = right ? G.L2R : G.L2L;
  L.d.lband = right ? G.lbR : G.lbL;
  L.d.rband = right ? G.rbR : G.rbL;
  L.d.W = L.d.lband + L.d.rband + 1;
  L.d.mode = 0;
  L.d.eb = G.eb;
  L.d.open = G.open;
  L.d.ext = G.ext;
  L.d.mt = G.mt;
  L.d.jl = 0;
  L.d.rev = right;
  L.d.status = ST_OK;
  L.d.early_score = 0;
  L.d.early_dpi_step = 0;
  // right flank: query read backwards from sequence1[length1-1] (dynprog.c:4960)
  L.qbase = right ? (int)w.qpos + G.L1 - 1 : (int)w.qpos;
  L.qstep = right ? -1 : 1;
  L.g0 = right ? w.revoffset2R : w.offset2L;
  L.gstep = right ? -1 : 1;
  L.base = w.chroffset + w.chrpos;
  L.glen = (int)w.genomiclength;
  L.watson = w.watsonp ? 1 : 0;
  L.allstar = (L.base < w.chroffset) || (L.base >= w.chrhigh);
  L.off1 = w.offset1;
  L.off2 = right ? w.revoffset2R : w.offset2L;
  L.cdna_direction = w.cdna_direction;
  return L;
}


// ---- k_gband (gsnapdp_gband.hip): the register-band path of score- and
// probability-mode windows.  Lists of a genome-gap batch: 0..2 the row-lane
// classes of k_ggap, then GB_LIST0 + 2*k + jump_late_p (score mode) and
// GP_LIST0 + 2*k + jump_late_p (probability mode) for k_fill's band classes
// k + 1 = 1..6.
constexpr int GB_L2MAX = 256;            // longest flank on the register band
constexpr int GB_LIST0 = 3;
constexpr int GP_LIST0 = GB_LIST0 + 2 * (NCLASS - 1);
// k_gwin (gsnapdp_gwin.hip): probability-mode windows with one window per
// lane, lists GW_LIST + 2 * shape + jump_late_p (a wave's 64 windows share the
// band shape and the tie rule)
constexpr int GW_LIST = GP_LIST0 + 2 * (NCLASS - 1);
constexpr int GW_NSUB = 4;
constexpr int GG_NLISTS = GW_LIST + GW_NSUB;
constexpr int GW_WMAX = 24;   // widest band of either flank
// the band shapes k_gwin is built for: width 2 * extraband + 9 with extraband
// 7 and 3 (GMAP's length2 = length1 + 8, stage3.c:5793); both flanks alike
constexpr int GW_CLASSES = 2, GW_W0 = 23, GW_LB0 = 7, GW_W1 = 15, GW_LB1 = 3;
constexpr int GW_L1MAX = 24;  // rows
constexpr int GW_L2MAX = 32;  // columns of a flank (their probability ranks fit bits 0..30)
#ifndef GB_WAVES_PER_SIMD
#define GB_WAVES_PER_SIMD 2  // k_gband (256 VGPRs): C4 score 0.65 ms; 3 waves 0.70, 4 waves 0.95 (spills)
#endif
// per-wave scratch of k_gband in dwords (layout in gsnapdp_gband.hip): the
// score-mode part, then probability mode's cell values (4 dwords per lane and
// column, both flanks), site probabilities (doubles per window and column) and
// row records (4 dwords per window and row)
constexpr int GB_WAVE_DW = 2 * (GB_L2MAX + 4) * 80 + 2 * 32 * ((GB_L2MAX + 4) / 4 + 1) +
                           3 * 2 * 32 * (GB_L2MAX + 4) + 2 * (GB_L2MAX + 4) * 256 + 2 * 32 * (GB_L2MAX + 4) * 2 +
                           2 * 32 * (GB_L2MAX + 4) * 4;
// use_band bits of k_ggap_plan (GW_USE: probability-mode windows on k_gwin)
enum { GB_USE_SCORE = 1, GB_USE_PROB = 2, GW_USE = 4 };

// The register-band list of a window that reached the fills, or -1 for k_ggap:
// no constrained known-intron bridge, both flanks at least length1 long (so the
// bridge's band is the fill band, :3716-3760) and at most GB_L2MAX, band width
// <= FAST_WMAX, and an intron span that never cuts the bridge's columns
// (cL < span - rR, cR < span - rL; :3720, :3760).
__device__ inline int gband_list(const gsnapdp_ggap_window& w, const GGeo& G, int use_band) {
  if (w.known_mode == GSNAPDP_KNOWN_INTRONS) return -1;
  if (!(use_band & (w.use_probabilities_p ? GB_USE_PROB : GB_USE_SCORE))) return -1;
  if (G.L2L < G.L1 || G.L2R < G.L1 || G.L2L > GB_L2MAX || G.L2R > GB_L2MAX) return -1;
  const int W = G.WL > G.WR ? G.WL : G.WR;
  if (W > FAST_WMAX) return -1;
  const int span = w.revoffset2R - w.offset2L;
  if (span - G.L1 - 1 < (G.rbL > G.rbR ? G.rbL : G.rbR)) return -1;
  const int k = class_of_w(W);
  return (w.use_probabilities_p ? GP_LIST0 : GB_LIST0) + 2 * (k > 0 ? k - 1 : 0) + (w.jump_late_p ? 1 : 0);
}

// A window k_gwin takes (its fills and bridge assume all of this): probability
// mode without a splicing IIT, both flanks at least length1 long (the bridge's
// band is then the fill band, :3716-3760) and at most GW_L2MAX, band widths
// <= GW_WMAX, length1 <= GW_L1MAX, and an intron span that never cuts the
// bridge's columns (cL < span - rR, cR < span - rL; :3720, :3760).
__device__ inline bool gwin_ok(const gsnapdp_ggap_window& w, const GGeo& G) {
  if (!w.use_probabilities_p || w.known_mode != GSNAPDP_KNOWN_NONE) return false;
  if (G.L1 < 2 || G.L1 > GW_L1MAX) return false;
  if (G.L2L < G.L1 || G.L2R < G.L1 || G.L2L > GW_L2MAX || G.L2R > GW_L2MAX) return false;
  if (G.WL != G.WR || G.lbL != G.lbR) return false;
  if (!((G.WL == GW_W0 && G.lbL == GW_LB0) || (G.WL == GW_W1 && G.lbL == GW_LB1))) return false;
  const int span = w.revoffset2R - w.offset2L;
  return span - G.L1 - 1 >= (G.rbL > G.rbR ? G.rbL : G.rbR);
}
// the k_gwin list of a window gwin_ok takes: its band shape and tie rule
__device__ inline int gwin_list(const gsnapdp_ggap_window& w, const GGeo& G) {
  return GW_LIST + (G.WL == GW_W0 ? 0 : 2) + (w.jump_late_p ? 1 : 0);
}

}  // namespace gsnapdp
