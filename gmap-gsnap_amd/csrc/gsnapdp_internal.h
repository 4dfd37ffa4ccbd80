// gsnapdp_internal.h -- shared between the HIP kernels (gsnapdp_kernels.hip)
// and the host-side code (gsnapdp_host.cpp).  Not part of the public ABI.
#pragma once
#include <stdint.h>

#include "../../include/gsnapdp.h"

#if defined(__HIPCC__)
#define GSNAPDP_HD_CONST __host__ __device__ constexpr
#else
#define GSNAPDP_HD_CONST constexpr
#endif

namespace gsnapdp {

constexpr int NEG = -1000000;          // NEG_INFINITY, dynprog.c:119
constexpr int MICROINTRON_LENGTH = 9;  // dynprog.c:139
constexpr int FAST_L2MAX = 640;        // longest genome span handled by the register-band kernel
// band-width classes of k_fill: W in (CLASS_W[c-1], CLASS_W[c]].
// A window of class c is spread over CLASS_LPW[c] lanes of CLASS_S[c] diagonals
// each (CLASS_S * CLASS_LPW = CLASS_W), so a wave carries 64 / LPW windows.
constexpr int NCLASS = 7;
constexpr int CLASS_W[NCLASS] = {8, 16, 24, 28, 32, 40, 48};
constexpr int CLASS_S[NCLASS] = {8, 8, 6, 7, 8, 5, 6};
constexpr int CLASS_LPW[NCLASS] = {1, 2, 4, 4, 4, 8, 8};
constexpr int FAST_WMAX = 48;
GSNAPDP_HD_CONST inline int class_low(int c) { return c == 0 ? 1 : CLASS_W[c - 1] + 1; }
GSNAPDP_HD_CONST inline bool classes_ok() {
  for (int c = 0; c < NCLASS; c++)
    if (CLASS_S[c] * CLASS_LPW[c] != CLASS_W[c] || (c > 0 && CLASS_W[c] <= CLASS_W[c - 1])) return false;
  return CLASS_W[NCLASS - 1] == FAST_WMAX;
}
static_assert(classes_ok(), "k_fill class table");
GSNAPDP_HD_CONST inline int class_of_w(int W) {
  int c = 0;
  while (c < NCLASS - 1 && W > CLASS_W[c]) c++;
  return c;
}
// k_fill bucket key = ((W(W-1)/2 + lband) * 2 + jl) * 3 + end: W-major over
// the (W, lband < W) triangle (W <= 48; jl the fill's tie rule; end: 0 a single
// gap, 1 an end gap scanned by find_best_endpoint, 2 one scanned by
// find_best_endpoint_to_queryend_indels -- end gaps' open/extend differ)
constexpr int NEND = 3;
GSNAPDP_HD_CONST inline int key_tri(int W) { return W * (W - 1) / 2; }
constexpr int NKEYS = key_tri(FAST_WMAX + 1) * 2 * NEND;
GSNAPDP_HD_CONST inline int fill_key(int W, int lband, int jl, int end) {
  return ((key_tri(W) + lband) * 2 + jl) * NEND + end;
}
GSNAPDP_HD_CONST inline int first_key_of_w(int W) { return key_tri(W) * 2 * NEND; }
// gsnapdp_window.kind of a window the planner skips (its result is already written)
constexpr int KIND_SKIP = 0x5c;
GSNAPDP_HD_CONST inline int w_of_key(int k) {  // the W whose keys hold k
  int W = 1;
  while (W < FAST_WMAX && first_key_of_w(W + 1) <= k) W++;
  return W;
}

// Mismatch types (dynprog.c:150)
enum { MT_HIGHQ = 0, MT_MEDQ = 1, MT_LOWQ = 2, MT_ENDQ = 3 };

// Window status (gsnapdp_result.status)
// ST_INTERNAL: a kernel invariant failed (k_gband's bridge cells outside the
// flanks); the window is not traced and every host path reports an error
enum { ST_OK = 0, ST_EARLY = 1, ST_OPS_OVERFLOW = 2, ST_ZEROED = 3, ST_UNSUPPORTED = 4, ST_INTERNAL = 6 };

// Derived per-window parameters (device + host), restating the parameter
// selection of Dynprog_single_gap (dynprog.c:4471-4519) and
// Dynprog_end5/3_gap (:5127-5163, 5589-5623).
struct Derived {
  int L1, L2;          // effective lengths (after end-gap chopping)
  int lband, rband;    // fill band (dynprog.c:1442-1454)
  int W;               // lband + rband + 1
  int mode;            // 0 endpoint (L1,L2); 1 best local; 2 queryend indels; 3 nogaps
  int eb;              // extraband
  int open, ext, mt, jl, rev;
  int status;          // ST_OK or an early-return / unsupported status
  int early_score;     // finalscore for early returns
  int early_dpi_step;  // 1 if *dynprogindex is stepped on the early return
};

#if defined(__HIPCC__)
#define GSNAPDP_HD __host__ __device__
#else
#define GSNAPDP_HD
#endif

GSNAPDP_HD inline Derived derive(const gsnapdp_window& w) {
  Derived d;
  d.L1 = w.length1;
  d.L2 = w.length2;
  d.eb = w.extraband;
  d.status = ST_OK;
  d.early_score = 0;
  d.early_dpi_step = 0;
  d.rev = (w.kind == GSNAPDP_END5_GAP) ? 1 : 0;
  int wide = 1;
  if (w.kind == GSNAPDP_SINGLE_GAP) {
    const double dr = (double)w.defect_rate;  // DEFECT_HIGHQ/MEDQ, dynprog.h:27-28
    d.mt = dr < 0.003 ? MT_HIGHQ : (dr < 0.014 ? MT_MEDQ : MT_LOWQ);
    d.open = -10;
    d.ext = -3;
    d.jl = w.jump_late_p ? 1 : 0;
    d.mode = 0;
    wide = w.widebandp ? 1 : 0;
    if (d.L1 > w.maxlength1 || d.L2 > w.maxlength2) {
      d.status = ST_EARLY;
      d.early_score = -10000;
      d.early_dpi_step = 1;
    } else if (d.L1 <= 0 || d.L2 <= 0) {
      d.status = ST_UNSUPPORTED;  // reference aborts (Matrix3_alloc, dynprog.c:495-498)
    } else if (!wide && (d.L2 - d.L1 > d.eb || d.L1 - d.L2 > d.eb)) {
      d.status = ST_UNSUPPORTED;  // reference writes past the matrix (dynprog.c:1504)
    }
  } else {
    d.mt = MT_ENDQ;
    d.open = -12;
    d.ext = -1;
    d.jl = (d.rev ? !w.jump_late_p : w.jump_late_p) ? 1 : 0;
    if (w.endalign == GSNAPDP_QUERYEND_NOGAPS) d.mode = 3;
    else if (w.endalign == GSNAPDP_QUERYEND_INDELS) d.mode = 2;
    else if (w.endalign == GSNAPDP_QUERYEND_GAP || w.endalign == GSNAPDP_BEST_LOCAL) d.mode = 1;
    else d.status = ST_UNSUPPORTED;  // reference aborts (dynprog.c:5215)
    if (d.L1 <= 0 || d.L2 <= 0) {
      d.status = ST_EARLY;
      d.early_score = 0;
      d.early_dpi_step = 0;
    } else if (d.mode != 3) {
      if (d.L1 > w.maxlength1) d.L1 = w.maxlength1;
      if (d.L2 > w.maxlength2) d.L2 = w.maxlength2;
    }
  }
  if (!wide) {
    d.lband = d.eb;
    d.rband = d.eb;
  } else if (d.L2 >= d.L1) {
    d.rband = d.L2 - d.L1 + d.eb;
    d.lband = d.eb;
  } else {
    d.lband = d.L1 - d.L2 + d.eb;
    d.rband = d.eb;
  }
  if (d.eb < 0) d.status = ST_UNSUPPORTED;
  d.W = d.lband + d.rband + 1;
  return d;
}

GSNAPDP_HD inline int step_dpi(int dpi) { return dpi + (dpi > 0 ? 1 : -1); }

// Intron_type (intron.c:18-180, non-PMAP) on genome class codes
// 0..5 = A C G T N *
GSNAPDP_HD inline int intron_type_codes(int l1, int l2, int r2, int r1, int cdna_direction) {
  int leftdi, rightdi, t;
  if (l1 == 2 && l2 == 3) leftdi = 0x21;       // GT
  else if (l1 == 2 && l2 == 1) leftdi = 0x10;  // GC
  else if (l1 == 0 && l2 == 3) leftdi = 0x08;  // AT
  else if (l1 == 1 && l2 == 3) leftdi = 0x06;  // CT
  else return 0;
  if (r2 == 0 && r1 == 2) rightdi = 0x30;       // AG
  else if (r2 == 0 && r1 == 1) rightdi = 0x0C;  // AC
  else if (r2 == 2 && r1 == 1) rightdi = 0x02;  // GC
  else if (r2 == 0 && r1 == 3) rightdi = 0x01;  // AT
  else return 0;
  if ((t = leftdi & rightdi) == 0) return 0;
  if (cdna_direction > 0) return t < 0x08 ? 0 : t;
  if (cdna_direction < 0) return t > 0x04 ? 0 : t;
  return 0;
}

}  // namespace gsnapdp

// Host-side helpers implemented in gsnapdp_host.cpp
namespace gsnapdp {
// Profile words prof[mt*128 + c]: bits 4g..4g+3 = pairdistance[mt][c][class g] as a
// signed 4-bit field (g = A C G T N *), bits 24..28 = consistent_array[c][class g].
// prof[4*128 + u]: bit 24+g set when the uppercase query byte u equals "ACGTN"[g]
// (the `rsequenceuc[r] == c2` half of the match test, dynprog.c:2650).
// prof[5*128 + c]: bit 24+g = consistent_array[class g][c], the swapped test of
// traceback_cdna (dynprog.c:2760; consistent_array is asymmetric in the CMET modes).
constexpr int PROF_WORDS = 6 * 128;
constexpr int PROF_CONS_SWAPPED = 5 * 128;
void build_profile_table(int mode, uint32_t prof[PROF_WORDS]);
int host_pairdistance(int mt, int c1, int c2);
int host_consistent(int c1, int c2);
}  // namespace gsnapdp
