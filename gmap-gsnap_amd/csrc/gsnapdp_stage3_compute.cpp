// gsnapdp_stage3_compute.cpp -- path_compute (stage3.c:8586-9220) from pass 2A
// for many queries at once: passes 2A-6 (gsnapdp_stage3_compute) and 2A-10
// (gsnapdp_stage3_path_compute).
//
// Every query runs the reference's sequence: build_pairs_singles (2A), the
// adjacent-indel fix, build_pairs_singles again (2C), the defect rate,
// Smooth_pairs_by_size with build_pairs_dualintrons and the build_pairs_introns
// iterations (3a-3c), the end chop by changepoint, the two HMM filters (4),
// remove_indel_gaps and build_dual_breaks (5), and the final build_pairs_introns
// (6); then the dual breaks at the ends (7), the adjacent indels (7b, 7C), the
// end extensions (8), assign_gap_types and the BEST_LOCAL extensions (9) and
// the noncanonical end-exon trims (10).  The host steps between the DP passes
// are restated here on each query's
// list (a vector of gsnapdp_s3_pair in list order); the DP passes of all the
// queries that have reached one run as ONE gsnapdp_stage3_pass, whatever pass
// each query is at, so the GPU sees every query's windows of a round together.
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <memory>
#include <vector>

#include "../../include/gsnapdp.h"
#include "gsnapdp_internal.h"
#include "gsnapdp_stage3.h"

extern "C" const uint32_t* gsnapdp__host_blocks(gsnapdp_ctx* ctx);
extern "C" size_t gsnapdp__host_nwords(gsnapdp_ctx* ctx);
void gsnapdp__set_err(const std::string& s);  // gsnapdp_kernels.hip

namespace {

using List = std::vector<gsnapdp_s3_pair>;  // list order: [0] is the head

// stage3.c:42-44, smooth.c:20-36, stage3.c:74-75, changepoint.c:11-12
constexpr int MAXITER_SMOOTH_BY_SIZE = 2, MAXITER_INTRONS = 2;
constexpr double DELETE_THRESHOLD = 0.1, MARK_THRESHOLD = 1e-7;
// smooth.c:30-35: GSNAP "allows more intron predictions in ends of short reads"
constexpr double SHORTEXONPROB_END_GMAP = 0.05, SHORTEXONPROB_END_GSNAP = 0.10;
constexpr int SHORTEXONLEN_END = 10, STAGE2_INDEXSIZE = 6;
constexpr double THETA_SLACK = 0.10, TRIM_END_PVALUE = 1e-4, NPSEUDO = 12.0, CP_SLACK = 0.10;
enum { KEEP = 0, DELETE = 1, MARK = 2 };

bool gapp(const gsnapdp_s3_pair& p) { return (p.flags & GSNAPDP_S3_GAPP) != 0; }
bool knowngapp(const gsnapdp_s3_pair& p) { return (p.flags & GSNAPDP_S3_KNOWNGAPP) != 0; }
bool unknown_base(char c) {  // pair.c
  switch (c) {
    case 'A': case 'C': case 'G': case 'T': case 'U':
    case 'a': case 'c': case 'g': case 't': case 'u': return false;
    default: return true;
  }
}
void reverse(List& l) { std::reverse(l.begin(), l.end()); }

// Pairpool_push_gapholder (pairpool.c:352-410), knownp false
gsnapdp_s3_pair gapholder(int queryjump, int genomejump) {
  gsnapdp_s3_pair g;
  memset(&g, 0, sizeof(g));
  g.querypos = -1;
  g.genomepos = -1;
  g.queryjump = queryjump;
  g.genomejump = genomejump;
  g.src = -1;
  g.cdna = g.comp = g.genome = ' ';
  g.flags = GSNAPDP_S3_GAPP;
  return g;
}

// insert_gapholders (stage3.c:817-925): pairs -> path (the reversed list, with
// the unknown gaps dropped and one gapholder per jump; the first and the last
// gapholder made are end introns)
List insert_gapholders(const List& pairs, bool reversed = true) {
  List st;  // the path as a stack: back() is its head
  st.reserve(pairs.size() + pairs.size() / 8 + 4);
  const gsnapdp_s3_pair* left = nullptr;  // the last pair kept
  int gappair = -1;  // the last gapholder made (its index in st)
  bool firstp = true;
  for (const gsnapdp_s3_pair& pair : pairs) {
    if (!(knowngapp(pair) || !gapp(pair))) continue;  // old gapholders are dropped
    if (!left) {
      st.push_back(pair);
      left = &pair;
      continue;
    }
    int queryjump = pair.querypos - left->querypos - 1;
    int genomejump = (int)((uint32_t)pair.genomepos - (uint32_t)left->genomepos - 1u);  // Genomicpos_T
    if (left->cdna == ' ') queryjump++;
    if (left->genome == ' ') genomejump++;
    if (knowngapp(pair) || knowngapp(*left) || (queryjump <= 0 && genomejump <= 0)) {
      st.push_back(pair);
    } else {
      st.push_back(gapholder(queryjump, genomejump));
      gappair = (int)st.size() - 1;
      if (firstp) {
        st.back().flags |= GSNAPDP_S3_END_INTRON;
        firstp = false;
      }
      st.push_back(pair);
    }
    left = &pair;
  }
  if (gappair >= 0) st[(size_t)gappair].flags |= GSNAPDP_S3_END_INTRON;
  if (reversed) reverse(st);  // (reversed false: the caller's List_reverse of the result, done)
  return st;
}

// fix_adjacent_indels (stage3.c:1660-1882): pairs -> path, dropping an indel
// that directly follows another indel token (the pops are the reference's)
bool fix_adjacent_indels(const List& pairs, List* out, std::string* err) {
  List st;  // path as a stack
  st.reserve(pairs.size());
  bool in_exon = false;
  int M = 0, I = 0, D = 0;
  char last_type = ' ';
  int last_len = 0;
  auto pop = [&](int n) {
    for (int i = 0; i < n; i++) {
      if (st.empty()) return false;  // Pairpool_pop on NULL: the reference crashes
      st.pop_back();
    }
    return true;
  };
  for (const gsnapdp_s3_pair& t : pairs) {
    if (gapp(t)) {
      if (in_exon) {
        if (M > 0) {
          last_type = 'M', last_len = M;
        } else if (I > 0) {
          if (last_type == 'I' || last_type == 'D') {
            if (!pop(last_len + I)) return *err = "fix_adjacent_indels popped an empty path", false;
            last_type = 'I', last_len = 0;
          } else {
            last_type = 'I', last_len = I;
          }
        } else if (D > 0) {
          if (last_type == 'I' || last_type == 'D') {
            if (!pop(last_len + D)) return *err = "fix_adjacent_indels popped an empty path", false;
            last_type = 'D', last_len = 0;
          } else {
            last_type = 'D', last_len = D;
          }
        }
        M = I = D = 0;
        in_exon = false;
      }
    } else if (t.comp == '.') {  // INTRONGAP_COMP
    } else {
      if (!in_exon) {
        if (last_type != ' ') last_type = 'N', last_len = 0;
        in_exon = true;
      }
      if (t.comp == '-' || t.comp == '~') {
        if (t.genome == ' ') {
          if (M > 0) {
            last_type = 'M', last_len = M, M = 0;
          } else if (D > 0) {
            if (last_type == 'I' || last_type == 'D') {
              if (!pop(last_len + D)) return *err = "fix_adjacent_indels popped an empty path", false;
              last_type = 'D', last_len = 0;  // D is not reset here (:1745-1751)
            } else {
              last_type = 'D', last_len = D, D = 0;
            }
          }
          I++;
        } else if (t.cdna == ' ') {
          if (M > 0) {
            last_type = 'M', last_len = M, M = 0;
          } else if (I > 0) {
            if (last_type == 'I' || last_type == 'D') {
              if (!pop(last_len + I)) return *err = "fix_adjacent_indels popped an empty path", false;
              last_type = 'I', last_len = 0;
            } else {
              last_type = 'I', last_len = I;
            }
            I = 0;
          }
          D++;
        } else {
          return *err = "fix_adjacent_indels: an indel with neither side blank (the reference exits)", false;
        }
      } else {
        if (I > 0) {
          if (last_type == 'I' || last_type == 'D') {
            if (!pop(last_len + I)) return *err = "fix_adjacent_indels popped an empty path", false;
            last_type = 'I', last_len = 0;
          } else {
            last_type = 'I', last_len = I;
          }
          I = 0;
        } else if (D > 0) {
          if (last_type == 'I' || last_type == 'D') {
            if (!pop(last_len + D)) return *err = "fix_adjacent_indels popped an empty path", false;
            last_type = 'D', last_len = 0;
          } else {
            last_type = 'D', last_len = D;
          }
          D = 0;
        }
        M++;
      }
    }
    st.push_back(t);
  }
  if (M > 0) {
  } else if (I > 0) {
    if ((last_type == 'I' || last_type == 'D') && !pop(last_len + I))
      return *err = "fix_adjacent_indels popped an empty path", false;
  } else if (D > 0) {
    if ((last_type == 'I' || last_type == 'D') && !pop(last_len + D))
      return *err = "fix_adjacent_indels popped an empty path", false;
  }
  reverse(st);
  *out = std::move(st);
  return true;
}

// Pair_fracidentity (pair.c:5426-5505) with cdna_direction 0: the defect rate
// mismatches / (matches + mismatches) of path_compute (:8723, :8808)
bool defect_rate(const List& pairs, double* rate, std::string* err) {
  int matches = 0, mismatches = 0;
  const gsnapdp_s3_pair* prev = nullptr;
  for (const gsnapdp_s3_pair& t : pairs) {
    if (!gapp(t)) {
      if (t.comp == '-' || t.comp == '~') {
        if (t.cdna != ' ' && t.genome != ' ') return *err = "Pair_fracidentity: cannot parse comp (abort)", false;
      } else if (unknown_base(t.cdna) || unknown_base(t.genome) || t.comp == ':') {
      } else if (t.comp == '|' || t.comp == '*' || t.comp == ':') {
        matches++;
      } else if (t.comp == ' ') {
        mismatches++;
      } else {
        return *err = "Pair_fracidentity: cannot parse comp (abort)", false;
      }
    }
    prev = &t;
  }
  (void)prev;
  *rate = (double)mismatches / (double)(matches + mismatches);
  return true;
}

// ---- Smooth_pairs_by_size (smooth.c:535-614), bysizep: every gap is big
double compute_prob(int exonlen, int intronlen, int indexsize) {  // smooth.c:176-186
  if (exonlen < indexsize) return 1.0;
  return 1 - pow(1.0 - pow(4.0, (double)-exonlen), (double)intronlen);
}
void exon_lengths(const List& pairs, std::vector<int>* matches) {  // get_exonlengths (:88-133)
  matches->clear();
  size_t i = 0;
  int nmatches = 0;
  while (i < pairs.size()) {
    const gsnapdp_s3_pair& pair = pairs[i];
    if (gapp(pair)) {
      matches->push_back(nmatches);
      i++;
      if (i < pairs.size()) nmatches = 0;
    } else {
      if (pair.comp == '|' || pair.comp == '*') nmatches++;
      i++;
    }
  }
  matches->push_back(nmatches);
}
void intron_lengths(const List& pairs, std::vector<int>* v) {  // get_intronlengths (:135-170)
  v->clear();
  for (const gsnapdp_s3_pair& p : pairs)
    if (gapp(p)) {
      const int length = p.genomejump - p.queryjump;
      v->push_back(length < 0 ? -length : length);
    }
}
// delete_and_mark_exons (:368-462), bysizep
List delete_and_mark(const List& pairs, const std::vector<int>& status, bool markp) {
  List st;  // newpairs as a stack
  st.reserve(pairs.size());
  size_t i = 0;
  int curr = status[0];
  for (const gsnapdp_s3_pair& p : pairs) {
    if (gapp(p)) {
      const int prev = curr;
      curr = status[++i];
      if (prev != DELETE && curr != DELETE) st.push_back(p);
    } else if (curr == KEEP) {
      st.push_back(p);
    } else if (curr == MARK) {
      st.push_back(p);
      if (markp) st.back().flags |= GSNAPDP_S3_SHORTEXON;
    }
  }
  // "Remove gaps at end / beginning": the loop pops while the pair it last
  // popped was a gap, so it also takes the first non-gap after the gaps
  auto strip = [](List& s) {
    if (s.empty()) return;
    gsnapdp_s3_pair pair = s.back();
    while (!s.empty() && gapp(pair)) {
      pair = s.back();
      s.pop_back();
    }
  };
  strip(st);                         // the list's end (newpairs' head)
  List fwd(st.rbegin(), st.rend());  // List_reverse(newpairs): back() is the list's head now
  strip(fwd);
  reverse(fwd);  // list order
  return fwd;
}
List smooth_by_size(bool* shortp, bool* deletep, List pairs, bool gsnap) {
  const double SHORTEXONPROB_END = gsnap ? SHORTEXONPROB_END_GSNAP : SHORTEXONPROB_END_GMAP;
  *shortp = *deletep = false;
  for (gsnapdp_s3_pair& p : pairs) p.flags &= (uint8_t)~GSNAPDP_S3_SHORTEXON;  // smooth_reset
  std::vector<int> em, il, status;
  if (!pairs.empty()) {  // trim_ends (:327-365)
    exon_lengths(pairs, &em);
    intron_lengths(pairs, &il);
    const int nexons = (int)em.size();
    status.assign((size_t)nexons, KEEP);
    bool delete1p = false;
    bool sh = true;
    for (int i = 0; i < nexons - 1 && sh; i++) {
      if (em[(size_t)i] < SHORTEXONLEN_END &&
          !(compute_prob(em[(size_t)i], il[(size_t)i], 0) < SHORTEXONPROB_END)) {
        delete1p = true;
        status[(size_t)i] = DELETE;
      } else {
        sh = false;
      }
    }
    sh = true;
    for (int i = nexons - 1; i > 0 && sh; --i) {
      if (em[(size_t)i] < SHORTEXONLEN_END &&
          !(compute_prob(em[(size_t)i], il[(size_t)i - 1], 0) < SHORTEXONPROB_END)) {
        delete1p = true;
        status[(size_t)i] = DELETE;
      } else {
        sh = false;
      }
    }
    if (delete1p) {
      *deletep = true;
      pairs = delete_and_mark(pairs, status, false);
    }
  }
  if (!pairs.empty()) {  // find_internal_shorts_by_size (:295-323)
    exon_lengths(pairs, &em);
    intron_lengths(pairs, &il);
    const int nexons = (int)em.size();
    status.assign((size_t)nexons, KEEP);
    bool delete2p = false;
    for (int i = 1; i < nexons - 1; i++) {
      const double prob = compute_prob(em[(size_t)i] + 4, il[(size_t)i - 1] + il[(size_t)i], STAGE2_INDEXSIZE);
      if (prob > DELETE_THRESHOLD) {
        delete2p = true;
        status[(size_t)i] = DELETE;
      } else if (prob > MARK_THRESHOLD) {
        *shortp = true;
        status[(size_t)i] = MARK;
      }
    }
    if (delete2p) *deletep = true;
    if (delete2p || *shortp) pairs = delete_and_mark(pairs, status, true);
  }
  return pairs;
}

// ---- chop_ends_by_changepoint (stage3.c:2130-2306)
// Changepoint_left / Changepoint_right (changepoint.c:23-246)
int changepoint_left(int* nmatches_left, int* ntotal_left, const std::vector<int>& ms) {
  const int length = (int)ms.size();
  int edge = 0;
  *nmatches_left = *ntotal_left = 0;
  int x = 0, y = 0;
  for (int s : ms) x += s == 1, y += s == 0;
  const int n = x + y;
  double min_rss_sep, rss;
  min_rss_sep = rss = (double)x * (double)y / (double)n;
  if (rss == 0.0) return 0;
  const double theta = (double)x / (double)n, x_pseudo = NPSEUDO * theta;
  int x_past = 0, y_past = 0, n_past = 0, x_future = x, y_future = y, n_future = n;
  for (int pos = length - 1; pos > 0; --pos) {
    if (ms[(size_t)pos] < 0) continue;
    if (ms[(size_t)pos] == 1) x_past++, x_future--;
    else y_past++, y_future--;
    n_past++, n_future--;
    const double tp = ((double)x_past + x_pseudo) / ((double)n_past + NPSEUDO);
    const double tf = ((double)x_future + x_pseudo) / ((double)n_future + NPSEUDO);
    const double rp = (double)x_past * (1.0 - tp) * (1.0 - tp) + (double)y_past * tp * tp;
    const double rf = (double)x_future * (1.0 - tf) * (1.0 - tf) + (double)y_future * tf * tf;
    const double rss_sep = rp + rf;
    if (rss_sep == 0.0) continue;
    if (tf < tp - CP_SLACK && rss_sep < min_rss_sep) {
      min_rss_sep = rss_sep;
      edge = pos;
      *nmatches_left = x_future;
      *ntotal_left = n_future;
    }
  }
  return edge;
}
int changepoint_right(int* nmatches_right, int* ntotal_right, const std::vector<int>& ms) {
  const int length = (int)ms.size();
  int edge = length;
  *nmatches_right = *ntotal_right = 0;
  int x = 0, y = 0;
  for (int s : ms) x += s == 1, y += s == 0;
  const int n = x + y;
  double min_rss_sep, rss;
  min_rss_sep = rss = (double)x * (double)y / (double)n;
  if (rss == 0.0) return length;
  const double theta = (double)x / (double)n, x_pseudo = NPSEUDO * theta;
  int x_past = 0, y_past = 0, n_past = 0, x_future = x, y_future = y, n_future = n;
  for (int pos = 1; pos < length; pos++) {
    if (ms[(size_t)pos] < 0) continue;
    if (ms[(size_t)pos] == 1) x_past++, x_future--;
    else y_past++, y_future--;
    n_past++, n_future--;
    const double tp = ((double)x_past + x_pseudo) / ((double)n_past + NPSEUDO);
    const double tf = ((double)x_future + x_pseudo) / ((double)n_future + NPSEUDO);
    const double rp = (double)x_past * (1.0 - tp) * (1.0 - tp) + (double)y_past * tp * tp;
    const double rf = (double)x_future * (1.0 - tf) * (1.0 - tf) + (double)y_future * tf * tf;
    const double rss_sep = rp + rf;
    if (rss_sep == 0.0) continue;
    if (tf < tp - CP_SLACK && rss_sep < min_rss_sep) {
      min_rss_sep = rss_sep;
      edge = pos;
      *nmatches_right = x_future;
      *ntotal_right = n_future;
    }
  }
  return edge;
}
// ---- Pbinom (pbinom.c:1680): GSL 1.8's binomial CDF P(X <= k) as the
// reference carries it (gsl_cdf_binomial_P :1634 -> gsl_cdf_beta_Q :1617 ->
// beta_inc_AXPY :1563, beta_cont_frac :1465, gsl_sf_lnbeta :1419), restated for
// the arguments chop_ends_by_changepoint passes: a = k + 1 and b = n - k are
// integers >= 1 and 0.1 <= theta < 1, so lngamma is the Lanczos sum (or exactly 0
// at 1 and 2, :1146-1160) and gammastar its Chebyshev / Stirling branches for
// x >= 1 (:1315-1350).  The operations are the reference's, in its order, so the
// doubles are its doubles; tests/test_pbinom.py compares them bit for bit with
// the reference's own pbinom.c.
constexpr double PB_EPS = 2.2204460492503131e-16, PB_DBL_MIN = 2.2250738585072014e-308;
constexpr double PB_ROOT4_EPS = 1.2207031250000000e-04, PB_ROOT6_EPS = 2.4607833005759251e-03;
constexpr double PB_E = 2.71828182845904523536028747135, PB_SQRT2 = 1.41421356237309504880168872421;
constexpr double PB_SQRTPI = 1.77245385090551602729816748334, PB_LOGROOT2PI = 0.9189385332046727418;

// the Chebyshev series (coefficients c[0..order], interval [-1, 1]) by Clenshaw's recurrence (:146-168)
double pb_cheb(const double* c, int order, double x) {
  double d = 0.0, dd = 0.0;
  const double y = (2.0 * x - -1.0 - 1.0) / (1.0 - -1.0), y2 = 2.0 * y;
  for (int j = order; j >= 1; j--) {
    const double t = d;
    d = y2 * d - dd + c[j];
    dd = t;
  }
  return y * d - dd + 0.5 * c[0];
}
// Lanczos coefficients, gamma = 7, kmax = 8 (:650-659)
const double PB_LANCZOS[9] = {0.99999999999980993227684700473478,  676.520368121885098567009190444019,
                              -1259.13921672240287047156078755283, 771.3234287776530788486528258894,
                              -176.61502916214059906584551354,     12.507343278686904814458936853,
                              -0.13857109526572011689554707,       9.984369578019570859563e-6,
                              1.50563273514931155834e-7};
double pb_lngamma(double x) {  // x >= 1 (:1146-1160, :661-678)
  if (fabs(x - 1.0) < 0.01 || fabs(x - 2.0) < 0.01) return 0.0 * x;  // the Pade forms at eps = 0: exactly 0
  x -= 1.0;
  double ag = PB_LANCZOS[0];
  for (int k = 1; k <= 8; k++) ag += PB_LANCZOS[k] / (x + k);
  const double t1 = (x + 0.5) * log((x + 7.5) / PB_E);
  const double t2 = PB_LOGROOT2PI + log(ag);
  return t1 + (t2 - 7.0);
}
// Gamma*(x) Chebyshev data for [0.5, 2) and [2, 10) (:1187-1260)
const double PB_GSTAR_A[30] = {
    2.16786447866463034423060819465,     -0.05533249018745584258035832802,    0.01800392431460719960888319748,
    -0.00580919269468937714480019814,    0.00186523689488400339978881560,     -0.00059746524113955531852595159,
    0.00019125169907783353925426722,     -0.00006124996546944685735909697,    0.00001963889633130842586440945,
    -6.3067741254637180272515795142e-06, 2.0288698405861392526872789863e-06,  -6.5384896660838465981983750582e-07,
    2.1108698058908865476480734911e-07,  -6.8260714912274941677892994580e-08, 2.2108560875880560555583978510e-08,
    -7.1710331930255456643627187187e-09, 2.3290892983985406754602564745e-09,  -7.5740371598505586754890405359e-10,
    2.4658267222594334398525312084e-10,  -8.0362243171659883803428749516e-11, 2.6215616826341594653521346229e-11,
    -8.5596155025948750540420068109e-12, 2.7970831499487963614315315444e-12,  -9.1471771211886202805502562414e-13,
    2.9934720198063397094916415927e-13,  -9.8026575909753445931073620469e-14, 3.2116773667767153777571410671e-14,
    -1.0518035333878147029650507254e-14, 3.4144405720185253938994854173e-15,  -1.0115153943081187052322643819e-15};
const double PB_GSTAR_B[30] = {
    0.0057502277273114339831606096782,   0.0004496689534965685038254147807,   -0.0001672763153188717308905047405,
    0.0000615137014913154794776670946,   -0.0000223726551711525016380862195,  8.0507405356647954540694800545e-06,
    -2.8671077107583395569766746448e-06, 1.0106727053742747568362254106e-06,  -3.5265558477595061262310873482e-07,
    1.2179216046419401193247254591e-07,  -4.1619640180795366971160162267e-08, 1.4066283500795206892487241294e-08,
    -4.6982570380537099016106141654e-09, 1.5491248664620612686423108936e-09,  -5.0340936319394885789686867772e-10,
    1.6084448673736032249959475006e-10,  -5.0349733196835456497619787559e-11, 1.5357154939762136997591808461e-11,
    -4.5233809655775649997667176224e-12, 1.2664429179254447281068538964e-12,  -3.2648287937449326771785041692e-13,
    7.1528272726086133795579071407e-14,  -9.4831735252566034505739531258e-15, -2.3124001991413207293120906691e-15,
    2.8406613277170391482590129474e-15,  -1.7245370321618816421281770927e-15, 8.6507923128671112154695006592e-16,
    -3.9506563665427555895391869919e-16, 1.6779342132074761078792361165e-16,  -6.0483153034414765129837716260e-17};
double pb_gammastar(double x) {  // x >= 1 (:1315-1350; the x < 0.5 branch is not reached)
  if (x < 2.0) return pb_cheb(PB_GSTAR_A, 29, 4.0 / 3.0 * (x - 0.5) - 1.0);
  if (x < 10.0) return pb_cheb(PB_GSTAR_B, 29, 0.25 * (x - 2.0) - 1.0) / (x * x) + 1.0 + 1.0 / (12.0 * x);
  if (x < 1.0 / PB_ROOT4_EPS) {  // the Stirling series of the log correction (:1295-1311)
    const double y = 1.0 / (x * x);
    const double c0 = 1.0 / 12.0, c1 = -1.0 / 360.0, c2 = 1.0 / 1260.0, c3 = -1.0 / 1680.0, c4 = 1.0 / 1188.0,
                 c5 = -691.0 / 360360.0, c6 = 1.0 / 156.0, c7 = -3617.0 / 122400.0;
    const double ser = c0 + y * (c1 + y * (c2 + y * (c3 + y * (c4 + y * (c5 + y * (c6 + y * c7))))));
    return exp(ser / x);
  }
  if (x < 1.0 / PB_EPS) {
    const double xi = 1.0 / x;
    return 1.0 + xi / 12.0 * (1.0 + xi / 24.0 * (1.0 - xi * (139.0 / 180.0 + 571.0 / 8640.0 * xi)));
  }
  return 1.0;
}
// log(1 + x)/x Chebyshev data (:1363-1386)
const double PB_LOPX[21] = {
    2.16647910664395270521272590407,     -0.28565398551049742084877469679,    0.01517767255690553732382488171,
    -0.00200215904941415466274422081,    0.00019211375164056698287947962,     -0.00002553258886105542567601400,
    2.9004512660400621301999384544e-06,  -3.8873813517057343800270917900e-07, 4.7743678729400456026672697926e-08,
    -6.4501969776090319441714445454e-09, 8.2751976628812389601561347296e-10,  -1.1260499376492049411710290413e-10,
    1.4844576692270934446023686322e-11,  -2.0328515972462118942821556033e-12, 2.7291231220549214896095654769e-13,
    -3.7581977830387938294437434651e-14, 5.1107345870861673561462339876e-15,  -7.0722150011433276578323272272e-16,
    9.7089758328248469219003866867e-17,  -1.3492637457521938883731579510e-17, 1.8657327910677296608121390705e-18};
double pb_log1plusx(double x) {  // 0 < x < 0.2 here (:1389-1414)
  if (fabs(x) < PB_ROOT6_EPS) {
    const double c1 = -0.5, c2 = 1.0 / 3.0, c3 = -1.0 / 4.0, c4 = 1.0 / 5.0, c5 = -1.0 / 6.0, c6 = 1.0 / 7.0,
                 c7 = -1.0 / 8.0, c8 = 1.0 / 9.0, c9 = -1.0 / 10.0;
    const double t = c5 + x * (c6 + x * (c7 + x * (c8 + x * c9)));
    return x * (1.0 + x * (c1 + x * (c2 + x * (c3 + x * (c4 + x * t)))));
  }
  if (fabs(x) < 0.5) return x * pb_cheb(PB_LOPX, 20, 0.5 * (8.0 * x + 1.0) / (x + 2.0));
  return log(1.0 + x);
}
double pb_lnbeta(double x, double y) {  // x, y >= 1 (:1419-1458)
  const double max = x > y ? x : y, min = x < y ? x : y, rat = min / max;
  if (rat < 0.2) {  // min << max: through Gamma*
    const double gsx = pb_gammastar(x), gsy = pb_gammastar(y), gsxy = pb_gammastar(x + y);
    const double lnopr = pb_log1plusx(rat);
    const double lnpre = log(gsx * gsy / gsxy * PB_SQRT2 * PB_SQRTPI);
    const double t1 = min * log(rat), t2 = 0.5 * log(min), t3 = (x + y - 0.5) * lnopr;
    return lnpre + (t1 - t2 - t3);
  }
  return pb_lngamma(x) + pb_lngamma(y) - pb_lngamma(x + y);
}
// the continued fraction of the incomplete beta function (:1465-1557); false
// where the reference aborts
bool pb_cont_frac(double a, double b, double x, double epsabs, double* cf_out) {
  const double cutoff = 2.0 * PB_DBL_MIN;
  double num = 1.0, den = 1.0 - (a + b) * x / (a + 1.0);
  if (fabs(den) < cutoff) return false;
  den = 1.0 / den;
  double cf = den;
  unsigned iter = 0;
  for (; iter < 512; iter++) {
    const int k = (int)iter + 1;
    double coeff = k * (b - k) * x / (((a - 1.0) + 2 * k) * (a + 2 * k));
    den = 1.0 + coeff * den;
    num = 1.0 + coeff / num;
    if (fabs(den) < cutoff || fabs(num) < cutoff) return false;
    den = 1.0 / den;
    double delta = den * num;
    cf *= delta;
    coeff = -(a + k) * (a + b + k) * x / ((a + 2 * k) * (a + 2 * k + 1.0));
    den = 1.0 + coeff * den;
    num = 1.0 + coeff / num;
    if (fabs(den) < cutoff || fabs(num) < cutoff) return false;
    den = 1.0 / den;
    delta = den * num;
    cf *= delta;
    if (fabs(delta - 1.0) < 2.0 * PB_EPS) break;
    if (cf * fabs(delta - 1.0) < epsabs) break;
  }
  if (iter >= 512) return false;
  *cf_out = cf;
  return true;
}
// Pbinom(k, n, theta) = gsl_cdf_binomial_P(k, theta, n) (k and n as the
// reference's unsigned ints) = gsl_cdf_beta_Q(theta, k + 1, n - k) =
// beta_inc_AXPY(-1, 1, a, b, theta); false where the reference aborts
bool pbinom(int k, int n, double theta, double* p) {
  if (theta > 1.0 || theta < 0.0) return false;
  if ((unsigned)k >= (unsigned)n) return *p = 1.0, true;
  const double a = (double)(unsigned)k + 1.0, b = (double)(unsigned)n - (unsigned)k, x = theta;
  if (x >= 1.0) return *p = 0.0, true;
  if (x <= 0.0) return *p = 1.0, true;
  if (a < 1.0 || b < 1.0) return false;  // (not reached: unsigned k < n)
  const double A = -1.0, Y = 1.0;
  const double ln_pre = -pb_lnbeta(a, b) + a * log(x) + b * log1p(-x);
  const double prefactor = exp(ln_pre);
  double cf;
  if (x < (a + 1.0) / (a + b + 2.0)) {
    const double epsabs = fabs(Y / (A * prefactor / a)) * PB_EPS;
    if (!pb_cont_frac(a, b, x, epsabs, &cf)) return false;
    *p = A * (prefactor * cf / a) + Y;
  } else {
    const double epsabs = fabs((A + Y) / (A * prefactor / b)) * PB_EPS;
    if (!pb_cont_frac(b, a, 1.0 - x, epsabs, &cf)) return false;
    *p = -A * (prefactor * cf / b);  // A == -Y
  }
  return true;
}
bool chop_ends_by_changepoint(List& pairs, std::string* err) {
  if (pairs.empty()) return true;
  // Pair_matchscores_list (pair.c:5785-5818)
  std::vector<int> ms;
  ms.reserve(pairs.size());
  int nmatches = 0, ntotal = 0;
  for (const gsnapdp_s3_pair& t : pairs) {
    if (gapp(t) || t.comp == ' ' || t.comp == ':') ms.push_back(0), ntotal++;
    else if (t.comp == '-') ms.push_back(-1);
    else ms.push_back(1), nmatches++, ntotal++;
  }
  const int length = (int)ms.size();
  int nml, ntl, nmr, ntr;
  const int left_edge = changepoint_left(&nml, &ntl, ms);
  const int right_edge = changepoint_right(&nmr, &ntr, ms);
  auto chop_left = [&](List& l) { l.erase(l.begin(), l.begin() + std::min((size_t)left_edge, l.size())); };
  auto chop_right = [&](List& l) {
    const size_t n = std::min((size_t)(length - right_edge), l.size());
    l.erase(l.end() - (ptrdiff_t)n, l.end());
  };
  if (right_edge <= left_edge) {
    int side;
    if (ntl == 0 || ntotal - ntl <= 0) side = +1;
    else if (ntr == 0 || ntotal - ntr <= 0) side = -1;
    else side = ntl < ntr ? -1 : +1;  // the shorter side
    if (side == -1) chop_left(pairs);
    else chop_right(pairs);
    return true;
  }
  auto theta_of = [&](int m, int t) {
    double theta = (double)(nmatches - m) / (double)(ntotal - t) - THETA_SLACK;
    return theta < 0.10 ? 0.10 : theta;
  };
  double p;
  if (!(ntl == 0 || ntotal - ntl <= 0)) {
    if (!pbinom(nml, ntl, theta_of(nml, ntl), &p)) return *err = "Pbinom: the reference aborts", false;
    if (!(p > TRIM_END_PVALUE)) chop_left(pairs);
  }
  if (!(ntr == 0 || ntotal - ntr <= 0)) {
    if (!pbinom(nmr, ntr, theta_of(nmr, ntr), &p)) return *err = "Pbinom: the reference aborts", false;
    if (!(p > TRIM_END_PVALUE)) chop_right(pairs);
  }
  return true;
}

// ---- filter_goodness_hmm / filter_indels_hmm (stage3.c:8166-8339): the
// Viterbi path of a two-state HMM over the list; BAD pairs are dropped
List viterbi_filter(const List& pairs, bool goodness, double defect) {
  if (goodness && defect == 0.0) defect = 0.001;
  const size_t n = pairs.size();
  std::vector<uint8_t> vgood(n), vbad(n);  // the previous state each state came from (1 GOOD)
  // A pair's emissions take one of two values (match / mismatch, or indel / not),
  // so its four log sums are tabulated once per call: the same operands in the
  // same order as per pair, so the same doubles.
  double GG[2], BG[2], GBd[2], BBd[2];
  for (int m = 0; m < 2; m++) {  // m = 1: a match (goodness) or an indel
    double eg, eb, tgg, tbg, tgb, tbb;
    if (goodness) {
      eg = m ? 1.0 - defect : defect;
      eb = m ? 0.25 : 0.75;
      tgg = 0.99, tbg = 0.10, tgb = 0.01, tbb = 0.90;
    } else {
      eg = m ? 0.0001 : 0.9999;
      eb = 0.5;
      tgg = 0.9999, tbg = 0.25, tgb = 0.0001, tbb = 0.75;
    }
    GG[m] = log(eg) + log(tgg);
    BG[m] = log(eg) + log(tbg);
    GBd[m] = log(eb) + log(tgb);
    BBd[m] = log(eb) + log(tbb);
  }
  double pg = 0.0, pb = 0.0;
  for (size_t i = 0; i < n; i++) {
    const gsnapdp_s3_pair& p = pairs[i];
    const int m = goodness ? (p.comp == '|' || p.comp == '*' || p.comp == ':') : (p.comp == '-');
    double gi = GG[m], bi = BG[m], vg, vb;
    if (pg + gi > pb + bi) vg = pg + gi, vgood[i] = 1;
    else vg = pb + bi, vgood[i] = 0;
    gi = GBd[m], bi = BBd[m];
    if (pg + gi > pb + bi) vb = pg + gi, vbad[i] = 1;
    else vb = pb + bi, vbad[i] = 0;
    pg = vg, pb = vb;
  }
  bool good = pg > pb;
  List kept;
  kept.reserve(n);
  for (size_t j = n; j-- > 0;) {  // backwards along List_reverse(pairs)
    if (good) {
      kept.push_back(pairs[j]);  // List_transfer_one onto the result: it ends in list order
      good = vgood[j] != 0;
    } else {
      good = vbad[j] != 0;
    }
  }
  reverse(kept);
  return kept;
}

// remove_indel_gaps (stage3.c:1266-1343): path -> pairs
List remove_indel_gaps(const List& path, int min_intronlength) {
  List st;  // pairs as a stack
  st.reserve(path.size());
  for (size_t i = 0; i < path.size(); i++) {
    gsnapdp_s3_pair pair = path[i];
    const bool more = i + 1 < path.size();
    if (!gapp(pair)) {
      st.push_back(pair);
    } else if (st.empty() || !more) {  // the initial / terminal gap is discarded
    } else if (pair.queryjump == 0 && pair.genomejump == 0) {
    } else if (pair.genomejump == 0) {  // a cDNA insertion
    } else if (pair.queryjump > 0) {  // a dual break
      pair.comp = '#';  // DUALBREAK_COMP
      st.push_back(pair);
    } else {
      const gsnapdp_s3_pair& left = path[i + 1];  // path->first
      const gsnapdp_s3_pair& right = st.back();   // pairs->first
      int leftgenomepos = left.genomepos;
      if (left.genome == ' ') leftgenomepos--;
      const int intronlength = right.genomepos - leftgenomepos - 1;
      if (!(intronlength < min_intronlength)) st.push_back(pair);
    }
  }
  reverse(st);
  return st;
}

// ---- passes 7-10 (stage3.c:8885-9212)

// A pair's donor_prob / acceptor_prob: assign_gap_types writes them on the
// intron gaps (stage3.c:1131-1244); every other pair keeps what
// Pairpool_push / Pairpool_push_gapholder gave it (pairpool.c:213-214,
// 385-391: 2.0 for a known gap, else 0.0).  The pipeline's lists carry a
// pair's row in the query's table in `src` (-1: none).
struct Probs {
  double d = 0.0, a = 0.0;
};

bool match_comp(char c) { return c == '|' || c == '*' || c == ':'; }  // MATCH, DYNPROG_MATCH, AMBIGUOUS

// dualbreak_p (stage3.c:2586-2598)
bool dualbreak_p(const List& l) {
  for (const gsnapdp_s3_pair& p : l)
    if (gapp(p) && p.queryjump > 0 && p.genomejump > 0) return true;
  return false;
}
// dualbreak_distance_from_end (:2601-2640): the pairs up to and including the
// first dual break, and its query jump weighed against the matches before it
int dualbreak_distance(int* npairs, int* totaljump, const List& l) {
  *totaljump = 0;
  if (l.empty()) return 0;
  int nmatches = 0, nmismatches = 0;
  size_t i = 0;
  const gsnapdp_s3_pair* pair = &l[0];
  *npairs = 0;
  while (i < l.size() && (!gapp(*pair) || pair->queryjump == 0 || pair->genomejump == 0)) {
    if (gapp(*pair)) {
    } else if (pair->comp == ' ' || pair->comp == '-') {
      nmismatches++;
    } else {
      nmatches++;
    }
    if (++i < l.size()) pair = &l[i];
    (*npairs)++;
  }
  if (gapp(*pair) && pair->queryjump > 0 && pair->genomejump > 0) {
    (*npairs)++;
    *totaljump = 10 * pair->queryjump;  // DUALBREAK_QUERYJUMP_FACTOR
  }
  return nmatches - nmismatches;
}
List reversed(const List& l) { return List(l.rbegin(), l.rend()); }

// pass 7 (:8885-8925): remove the dual breaks nearer an end than their query
// jump is worth.  pairs (pass 6's) -> pairs.
bool remove_end_dual_breaks(const List& pairs6, List* out, std::string* err) {
  List path = insert_gapholders(pairs6);
  List pairs;
  if (path.empty()) {
    if (!pairs6.empty())  // every pair an unknown gap: the reference keeps a list insert_gapholders re-linked
      return *err = "pass 7: a path of gaps only (the reference returns a stale list)", false;
    out->clear();
    return true;
  }
  for (;;) {
    if (path.empty()) break;  // (pairs as the last trim left it)
    if (!dualbreak_p(path)) {
      pairs = reversed(path);
      break;
    }
    int n3 = 0, t3, n5 = 0, t5;
    const int d3 = dualbreak_distance(&n3, &t3, path);
    pairs = reversed(path);
    const int d5 = dualbreak_distance(&n5, &t5, pairs);
    bool trim5;
    if (t5 < d5 && t3 < d3) break;  // keep the dual breaks
    if (t5 > d5 && t3 > d3) trim5 = d5 < d3;
    else trim5 = t5 > d5;
    if (trim5) {  // trim_npairs(pairs, npairs5)
      pairs.erase(pairs.begin(), pairs.begin() + n5);
      path = reversed(pairs);
    } else {  // path = List_reverse(pairs); trim_npairs(path, npairs3)
      const gsnapdp_s3_pair head = pairs[0];
      path = reversed(pairs);
      path.erase(path.begin(), path.begin() + n3);
      // the reversal left pairs' old head cell last in path, its rest NULL:
      // if the trim took all of path, `pairs` is that one cell
      if (path.empty()) pairs.assign(1, head);
    }
  }
  *out = std::move(pairs);
  return true;
}

// remove_adjacent_ins_del (:1889-1971): an insertion run directly followed by
// a deletion run (or the reverse) is dropped, both sides.  pairs -> pairs (the
// reference's path, List_reverse'd by path_compute).
bool remove_adjacent_ins_del(bool* foundp, const List& pairs, List* out, std::string* err) {
  auto indel = [](const gsnapdp_s3_pair& p) { return p.comp == '-' || p.comp == '~'; };  // INDEL, SHORTGAP
  enum { NORMAL = 0, INSERTION = 1, DELETION = -1 };
  List st;  // path as a stack
  st.reserve(pairs.size());
  int state = NORMAL;
  *foundp = false;
  size_t i = 0;
  while (i < pairs.size()) {
    const gsnapdp_s3_pair& t = pairs[i++];
    if (!indel(t)) {
      st.push_back(t);
      state = NORMAL;
    } else if (t.genome == ' ') {
      if (state != DELETION) {
        st.push_back(t);
        state = INSERTION;
      } else {
        while (!st.empty() && indel(st.back()) && st.back().cdna == ' ') st.pop_back();
        while (i < pairs.size() && indel(pairs[i]) && pairs[i].genome == ' ') i++;
        *foundp = true;
        state = NORMAL;
      }
    } else if (t.cdna == ' ') {
      if (state != INSERTION) {
        st.push_back(t);
        state = DELETION;
      } else {
        while (!st.empty() && indel(st.back()) && st.back().genome == ' ') st.pop_back();
        while (i < pairs.size() && indel(pairs[i]) && pairs[i].cdna == ' ') i++;
        *foundp = true;
        state = NORMAL;
      }
    } else {
      return *err = "remove_adjacent_ins_del: an indel with neither side blank (the reference aborts)", false;
    }
  }
  *out = std::move(st);  // List_reverse(path): the stack bottom first
  return true;
}

// clean_pairs_end5_gap_indels / clean_path_end3_gap_indels (:2056-2126): pop
// gaps and indels off the list's head
void clean_end_gap_indels(List& l) {
  size_t n = 0;
  while (n < l.size() && (gapp(l[n]) || l[n].comp == '-')) n++;
  l.erase(l.begin(), l.begin() + (ptrdiff_t)n);
}

// enough_matches (:2655-2692), canonicalp (:2695-2720), sufficient_splice_prob_local (:2724-2744)
bool enough_matches(int matches, int genomejump) {
  if (genomejump > 100000) return matches >= 10;
  if (genomejump > 32000) return matches >= 9;
  if (genomejump > 8000) return matches >= 8;
  if (genomejump > 2000) return matches >= 7;
  return matches >= 6;
}
bool canonicalp(bool known, char comp, int cdna_direction) {
  const bool fwd = comp == '>' || comp == ')' || comp == ']';
  const bool rev = comp == '<' || comp == '(' || comp == '[';
  if (known) return true;
  if (cdna_direction > 0) return fwd;
  if (cdna_direction < 0) return rev;
  return fwd || rev;
}
bool sufficient_splice_prob_local(int support, int nmismatches, double distal) {
  support -= 2 * nmismatches;
  if (support < 0) return false;
  if (support < 7) return distal > 0.95;
  if (support < 11) return distal > 0.90;
  if (support < 15) return distal > 0.85;
  if (support < 19) return distal > 0.50;
  return true;
}

// the options and tables the host steps of passes 7-10 read
struct Env {
  gsnapdp_s3_path_opts o;
  const uint32_t* blocks = nullptr;
  size_t nwords = 0;
  const gsnapdp_iit* iit = nullptr;
  const char* query = nullptr;
  bool full = false;  // passes 7-10 too (gsnapdp_stage3_path_compute)
};

// one site probability assign_gap_types needs
struct Site {
  int row, acceptor;  // the query's table row, donor (0) or acceptor (1)
  uint8_t model;
  uint32_t pos, chroffset;
};

// ---- one query through the passes
enum Step {
  Q_2A,       // waiting for build_pairs_singles (2A)
  Q_2C,       // ... (2C)
  Q_3B,       // build_pairs_dualintrons
  Q_3C,       // build_pairs_introns, not final
  Q_5,        // build_dual_breaks
  Q_6,        // build_pairs_introns, final
  Q_7C,       // build_pairs_singles (7C)
  Q_8_5,      // build_pairs_end5, QUERYEND_GAP (8)
  Q_8_3,      // build_path_end3, QUERYEND_GAP (8)
  Q_GT_9,     // parked: assign_gap_types before 9a, its MaxEnt sites pending
  Q_9A,       // build_pairs_end5, BEST_LOCAL, maxpeelback 0 (9a)
  Q_9B,       // build_path_end3 (9b)
  Q_GT_10,    // parked: assign_gap_types before pass 10
  Q_10_5,     // build_pairs_end5, QUERYEND_NOGAPS (10)
  Q_10_3,     // build_path_end3, QUERYEND_NOGAPS (10)
  Q_DONE
};
struct Query {
  gsnapdp_s3_call* c = nullptr;
  List list;       // the list the pending pass gets, or the result
  int step = Q_2A;
  bool failed = false;
  std::string why;
  double defect = 0.0;
  int iter1 = 0, iter2 = 0;
  bool shortp = false, deletep = false, shiftp = false, incompletep = false;
  int minor = 0, major = 0, nintrons = 0, nnonintrons = 0, intronlen = 0, nonintronlen = 0;
  int ub = 0;
  int passes[6] = {0, 0, 0, 0, 0, 0};
  gsnapdp_s3_call k;        // the pending pass's call (its pairs are list)
  std::vector<Probs> probs; // assign_gap_types' rows
  std::vector<Site> sites;  // parked: the rows' MaxEnt sites
  int iter10 = 0;           // pass 10's iterations
  bool trim5p = true, trim3p = true;
};
void fail(Query& q, const std::string& why) {
  if (!q.failed) q.why = why;
  q.failed = true;
  q.step = Q_DONE;
}
Probs probs_of(const Query& q, const gsnapdp_s3_pair& p) {
  if (p.src >= 0) return q.probs[(size_t)p.src];
  Probs r;
  if (gapp(p) && knowngapp(p)) r.d = r.a = 2.0;
  return r;
}

// Pairpool_push (pairpool.c:169-230) of a pair assign_gap_types makes
gsnapdp_s3_pair new_pair(int querypos, int genomepos, char cdna, char comp, char genome) {
  gsnapdp_s3_pair p;
  memset(&p, 0, sizeof(p));
  p.querypos = querypos;
  p.genomepos = genomepos;
  p.cdna = cdna;
  p.comp = comp;
  p.genome = genome;
  p.src = -1;
  return p;
}

// assign_gap_types (stage3.c:1015-1260) with no genomic segment: path -> pairs.
// The intron gaps get their type and a table row whose MaxEnt probabilities
// are queued in q.sites (1.0 at once for a site the splicing IIT knows).
bool assign_gap_types(Query& q, const Env& E, const List& path, List* out, std::string* err) {
  const gsnapdp_s3_call& c = *q.c;
  auto nt = [&](int gpos) { return gsnapdp::s3_genomic_nt(E.blocks, E.nwords, c, gpos); };
  auto cls = [](char ch) { return ch == 'A' ? 0 : ch == 'C' ? 1 : ch == 'G' ? 2 : ch == 'T' ? 3 : 4; };
  List st;  // pairs as a stack
  st.reserve(path.size() + 16);
  for (size_t i = 0; i < path.size(); i++) {
    gsnapdp_s3_pair pair = path[i];
    if (!gapp(pair)) {
      st.push_back(pair);
      continue;
    }
    if (st.empty() || i + 1 == path.size()) continue;  // the initial / terminal gap is discarded
    const int queryjump = pair.queryjump, genomejump = pair.genomejump;
    if (queryjump == 0 && genomejump == 0) continue;
    const gsnapdp_s3_pair& left = path[i + 1];  // path->first
    const gsnapdp_s3_pair right = st.back();    // pairs->first
    int leftquerypos = left.querypos, leftgenomepos = left.genomepos;
    if (left.cdna == ' ') leftquerypos--;
    if (genomejump == 0) {  // a cDNA insertion: its query bytes as indel pairs
      for (int cur = right.querypos - 1; cur > leftquerypos; --cur) {
        if (cur < 0 || cur >= c.querylength) return *err = "assign_gap_types: an insertion outside the query", false;
        st.push_back(new_pair(cur, right.genomepos, E.query[(size_t)c.qpos + (size_t)cur], '-', ' '));
      }
      continue;
    }
    if (queryjump > 0) {  // a dual break
      pair.comp = '#';
      st.push_back(pair);
      continue;
    }
    if (left.genome == ' ') leftgenomepos--;
    const int rightquerypos = right.querypos, rightgenomepos = right.genomepos;
    const int introntype = gsnapdp::intron_type_codes(cls(nt(leftgenomepos + 1)), cls(nt(leftgenomepos + 2)),
                                                      cls(nt(rightgenomepos - 2)), cls(nt(rightgenomepos - 1)),
                                                      c.cdna_direction);
    const int intronlength = rightgenomepos - leftgenomepos - 1;
    if (intronlength < E.o.min_intronlength) {  // too short for an intron: the genome as gap pairs
      for (int gpos = rightgenomepos - 1; gpos > leftgenomepos; --gpos)
        st.push_back(new_pair(rightquerypos, gpos, ' ', '~', nt(gpos)));
      continue;
    }
    const bool fwd = c.cdna_direction >= 0;
    switch (introntype) {
      case 0x20: pair.comp = fwd ? '>' : 0; break;  // GTAG_FWD
      case 0x10: pair.comp = fwd ? ')' : 0; break;  // GCAG_FWD
      case 0x08: pair.comp = fwd ? ']' : 0; break;  // ATAC_FWD
      case 0x01: pair.comp = fwd ? 0 : '['; break;  // ATAC_REV
      case 0x02: pair.comp = fwd ? 0 : '('; break;  // GCAG_REV
      case 0x04: pair.comp = fwd ? 0 : '<'; break;  // GTAG_REV
      default: pair.comp = '='; break;              // NONINTRON
    }
    if (!pair.comp) return *err = "assign_gap_types: unexpected intron type (the reference exits)", false;
    // the site probabilities (:1135-1244): donor at the left for fwd, at the right for rev
    const uint32_t gl1 = (uint32_t)c.genomiclength - 1U;
    const uint32_t lpos = c.watsonp ? c.chrpos + (uint32_t)leftgenomepos + 1U : c.chrpos + gl1 - (uint32_t)leftgenomepos;
    const uint32_t rpos = c.watsonp ? c.chrpos + (uint32_t)rightgenomepos
                                    : c.chrpos + gl1 - (uint32_t)rightgenomepos + 1U;
    gsnapdp_intron kn;
    memset(&kn, 0, sizeof(kn));
    kn.left_genomepos = (uint32_t)leftgenomepos;
    kn.right_genomepos = (uint32_t)rightgenomepos;
    if (E.iit && (c.cdna_direction == 1 || c.cdna_direction == -1) &&
        gsnapdp_introns_known(E.iit, c.chrnum, c.chrpos, c.genomiclength, c.cdna_direction, c.watsonp, &kn, 1))
      return *err = "assign_gap_types: the splicing IIT query failed", false;
    const int row = (int)q.probs.size();
    q.probs.emplace_back();
    pair.src = row;
    uint8_t dmodel, amodel;
    uint32_t dpos, apos;
    if (fwd) {
      dmodel = c.watsonp ? GSNAPDP_DONOR : GSNAPDP_ANTIDONOR, dpos = lpos;
      amodel = c.watsonp ? GSNAPDP_ACCEPTOR : GSNAPDP_ANTIACCEPTOR, apos = rpos;
    } else {
      amodel = c.watsonp ? GSNAPDP_ANTIACCEPTOR : GSNAPDP_ACCEPTOR, apos = lpos;
      dmodel = c.watsonp ? GSNAPDP_ANTIDONOR : GSNAPDP_DONOR, dpos = rpos;
    }
    if (kn.known_donor) q.probs.back().d = 1.0;
    else q.sites.push_back(Site{row, 0, dmodel, c.chroffset + dpos, c.chroffset});
    if (kn.known_acceptor) q.probs.back().a = 1.0;
    else q.sites.push_back(Site{row, 1, amodel, c.chroffset + apos, c.chroffset});
    st.push_back(pair);
  }
  *out = reversed(st);
  return true;
}

// trim_noncanonical_end5_exons (:2793-3014) on pairs / trim_noncanonical_end3_exons
// (:3021-3243) on path: the end exon up to and including the first gap, kept or
// trimmed by its matches against the gap's type, length and site probabilities.
// Returns the rest of the list reversed, after the kept exon (pairs -> path,
// path -> pairs).
bool trim_noncanonical_end(bool end5, bool* trimp, const List& l, const Query& q, const Env& E, List* out,
                           std::string* err) {
  const gsnapdp_s3_call& c = *q.c;
  out->clear();
  if (l.empty()) {
    *trimp = false;
    return true;
  }
  const gsnapdp_s3_pair* pair = &l[0];
  bool bingop = false;
  if (end5 ? E.o.paired_favor_mode < 0 : E.o.paired_favor_mode > 0) {
    const int insertlength = end5 ? pair->genomepos + c.querylength - E.o.zero_offset
                                  : (c.genomiclength - pair->genomepos) + c.querylength - E.o.zero_offset;
    if (insertlength > E.o.expected_pairlength - E.o.pairlength_deviation &&
        insertlength < E.o.expected_pairlength + E.o.pairlength_deviation)
      bingop = true;
  }
  size_t i = 0;  // the exon is l[0, i): up to and including the first gap
  int nmatches = 0, nmismatches = -1;  // -1 because of the gap
  while (i < l.size() && !gapp(*pair)) {
    pair = &l[i++];
    if (match_comp(pair->comp)) nmatches++;
    else nmismatches++;
  }
  bool nearindelp = false;
  for (size_t j = i, n = 0; j < l.size() && n < 6; j++, n++)  // NEARBY_INDEL medial to the gap
    if (!match_comp(l[j].comp) && l[j].comp == '-') nearindelp = true;
  for (ptrdiff_t j = (ptrdiff_t)i - 2, n = 0; j >= 0 && n < 6; j--, n++)  // distal, after the gap itself
    if (!match_comp(l[(size_t)j].comp) && l[(size_t)j].comp == '-') nearindelp = true;
  const Probs pr = probs_of(q, *pair);
  if (nearindelp) {
    nmismatches += pr.d >= 0.90 ? 0 : (pr.d >= 0.80 ? 1 : 3);
    nmismatches += pr.a >= 0.90 ? 0 : (pr.a >= 0.80 ? 1 : 3);
  }
  const bool is_canonical = canonicalp(knowngapp(*pair), pair->comp, c.cdna_direction);
  if (!is_canonical) nmismatches += 2;
  const int nrest = (int)(l.size() - i);
  bool keep;
  if (nrest == 0) {
    keep = true;
  } else if (knowngapp(*pair) && nmismatches == 0) {
    keep = true;
  } else if (i == 0) {  // the list starts with a gap: exon->rest dereferences NULL
    return *err = "trim_noncanonical_end_exons: the list starts with a gap (the reference crashes)", false;
  } else if (i >= 2 && (l[i - 2].flags & GSNAPDP_S3_DISALLOWED)) {
    keep = false;
  } else if ((int)i - 1 > nrest) {  // more than halfway across
    keep = true;
  } else if (pair->genomejump > E.o.maxintronlen_bound) {
    keep = false;
  } else if (bingop && is_canonical && nmismatches <= 1) {
    keep = true;
  } else if (nearindelp && nmatches < 12) {  // INDEL_SPLICE_ENDLENGTH
    keep = false;
  } else if (!enough_matches(nmatches - nmismatches, pair->genomejump)) {
    keep = false;
  } else if (sufficient_splice_prob_local((int)i, nmismatches,
                                          (c.cdna_direction >= 0) == end5 ? pr.d : pr.a)) {
    keep = E.o.gsnap ? true : (pr.d >= 0.9 || pr.a >= 0.9);  // :2968-2983
  } else {
    keep = false;
  }
  *trimp = nrest != 0 && !keep;
  // Pairpool_transfer(exon or NULL, the rest): the rest reversed onto the kept exon
  out->reserve(l.size());
  for (size_t j = l.size(); j-- > i;) out->push_back(l[j]);
  if (keep)
    for (size_t j = i; j-- > 0;) out->push_back(l[j]);
  return true;
}

// the loops of path_compute between DP passes (:8711-9212), from the list the
// last pass returned (q.list) to the next pass's input, a parked
// assign_gap_types, or the end
void advance(Query& q, const Env& E) {
  std::string err;
  List pairs = std::move(q.list);
  switch (q.step) {
    case Q_2A: {  // 2B: fix adjacent indels; then 2C on the gapholders
      List path;
      if (!fix_adjacent_indels(pairs, &path, &err)) return fail(q, err);
      reverse(path);
      q.list = insert_gapholders(path);
      q.step = Q_2C;
      return;
    }
    case Q_2C:
      if (!defect_rate(pairs, &q.defect, &err)) return fail(q, err);
      q.iter1 = 0;
      q.shortp = true;
      break;  // into pass 3
    case Q_3B:
      q.iter2 = 0;
      q.shiftp = q.incompletep = true;
      break;
    case Q_3C:
      q.iter2++;
      break;
    case Q_5: {
      List path = insert_gapholders(pairs, false);  // the path that ends iteration 0 (:8848), and pass 6's
                                                    // pairs = List_reverse(path)
      if (q.c->finalp) {
        q.list = insert_gapholders(path);
        q.step = Q_6;
        return;
      }
      if (!E.full) {
        q.list = std::move(path);
        q.step = Q_DONE;
        return;
      }
      pairs = std::move(path);  // pass 7 on pass 6's pairs
    }
      [[fallthrough]];
    case Q_6: {
      if (!E.full) {
        q.list = std::move(pairs);
        q.step = Q_DONE;
        return;
      }
      List p7;  // 7: dual breaks at the ends; 7b: adjacent insertions / deletions
      bool adjacent;
      if (!remove_end_dual_breaks(pairs, &p7, &err) || !remove_adjacent_ins_del(&adjacent, p7, &pairs, &err))
        return fail(q, err);
      if (adjacent) {  // 7C
        q.list = insert_gapholders(pairs);
        q.step = Q_7C;
        return;
      }
    }
      [[fallthrough]];
    case Q_7C: {  // remove_indel_gaps; 8: extend to the 5' end
      pairs = remove_indel_gaps(insert_gapholders(pairs), E.o.min_intronlength);
      clean_end_gap_indels(pairs);
      q.list = std::move(pairs);
      q.step = Q_8_5;
      return;
    }
    case Q_8_5: {  // 8: extend to the 3' end
      List path = reversed(pairs);
      clean_end_gap_indels(path);
      q.list = std::move(path);
      q.step = Q_8_3;
      return;
    }
    case Q_8_3:  // 9: gapholders, then assign_gap_types (parked for its sites)
    case Q_9B: {
      List path = insert_gapholders(reversed(pairs));
      const int next = q.step == Q_8_3 ? Q_GT_9 : Q_GT_10;
      q.sites.clear();
      if (!assign_gap_types(q, E, path, &q.list, &err)) return fail(q, err);
      q.step = next;
      return;
    }
    case Q_GT_9:  // 9a (knownsplice5p is false: every end pass here ran Dynprog_end5_gap)
      q.list = std::move(pairs);
      q.step = Q_9A;
      return;
    case Q_9A:  // 9b
      q.list = reversed(pairs);
      q.step = Q_9B;
      return;
    case Q_GT_10:  // pass 10
      q.iter10 = 0;
      q.trim5p = q.trim3p = true;
      break;
    case Q_10_5:
      if (q.trim3p) {
        q.list = reversed(pairs);
        q.step = Q_10_3;
        return;
      }
      q.iter10++;
      break;
    case Q_10_3:
      pairs = reversed(pairs);
      q.iter10++;
      break;
    default: return;
  }
  if (q.step >= Q_GT_10) {  // pass 10's loop (:9139-9212)
    while (q.iter10 < 5 && (q.trim5p || q.trim3p)) {
      List path;
      if (!q.trim5p) path = reversed(pairs);
      else if (!trim_noncanonical_end(true, &q.trim5p, pairs, q, E, &path, &err)) return fail(q, err);
      if (!q.trim3p) pairs = reversed(path);
      else if (!trim_noncanonical_end(false, &q.trim3p, path, q, E, &pairs, &err)) return fail(q, err);
      if (q.trim5p) {
        q.list = std::move(pairs);
        q.step = Q_10_5;
        return;
      }
      if (q.trim3p) {
        q.list = reversed(pairs);
        q.step = Q_10_3;
        return;
      }
      q.iter10++;
    }
    q.list = std::move(pairs);
    q.step = Q_DONE;
    return;
  }
  // pass 3: while (shortp && iter1 < MAXITER_SMOOTH_BY_SIZE) { 3a, 3b, 3c }
  for (;;) {
    if (q.step == Q_3B || q.step == Q_3C) {  // inside 3c's loop
      if ((q.shiftp || q.incompletep) && q.iter2 < MAXITER_INTRONS) {
        q.list = insert_gapholders(pairs);
        q.step = Q_3C;
        return;
      }
      q.iter1++;
    }
    if (!(q.shortp && q.iter1 < MAXITER_SMOOTH_BY_SIZE)) break;
    {  // 3a: smoothing by size
      List path = insert_gapholders(pairs, false);  // List_reverse(insert_gapholders(..))
      pairs = smooth_by_size(&q.shortp, &q.deletep, std::move(path), E.o.gsnap != 0);
    }
    if (q.shortp || q.deletep) {  // 3b: dual introns
      q.list = insert_gapholders(pairs);
      q.step = Q_3B;
      return;
    }
    q.iter2 = 0;  // 3c
    q.shiftp = q.incompletep = true;
    q.step = Q_3B;  // (as if 3b had run: 3c's loop next)
  }
  // 3b': chop_ends_by_changepoint; 4: the HMM filters on a fresh defect rate
  if (!chop_ends_by_changepoint(pairs, &err)) return fail(q, err);
  if (!defect_rate(pairs, &q.defect, &err)) return fail(q, err);
  pairs = viterbi_filter(pairs, true, q.defect);
  pairs = viterbi_filter(pairs, false, 0.0);
  // 5: remove_indel_gaps, then build_dual_breaks on the reversed list
  List gaps = remove_indel_gaps(insert_gapholders(pairs), E.o.min_intronlength);
  reverse(gaps);
  q.list = std::move(gaps);
  q.step = Q_5;
}

int pass_of(int step) {
  switch (step) {
    case Q_2A:
    case Q_2C:
    case Q_7C: return GSNAPDP_S3_SINGLES;
    case Q_3B: return GSNAPDP_S3_DUALINTRONS;
    case Q_5: return GSNAPDP_S3_DUALBREAKS;
    case Q_8_5:
    case Q_9A:
    case Q_10_5: return GSNAPDP_S3_END5;
    case Q_8_3:
    case Q_9B:
    case Q_10_3: return GSNAPDP_S3_END3;
    default: return GSNAPDP_S3_INTRONS;
  }
}

// the pipeline as the pass's driver: a query's next pass starts as soon as its
// last one has ended, in the same round, so queries at different passes share
// every round's batches.  A query that reaches assign_gap_types parks (its
// MaxEnt sites go to the next batch of all parked queries' sites).
class Pipeline final : public gsnapdp::S3Driver {
 public:
  Pipeline(std::vector<Query>& qs, const Env& env) : qs_(qs), env_(env) {}
  void set_map(const std::vector<int>* map) { map_ = map; }
  // the query's next pass call (q.list is its input), or nullptr when it is done or parked
  gsnapdp_s3_call* call_for(Query& q) {
    if (q.failed || q.step == Q_DONE || q.step == Q_GT_9 || q.step == Q_GT_10) return nullptr;
    gsnapdp_s3_call& k = q.k;
    k = *q.c;
    k.pass = pass_of(q.step);
    k.first_pair = 0;
    k.npairs = (int32_t)q.list.size();
    k.finalp = q.step == Q_6 ? 1 : 0;
    // 2A / 2C / 7C run with defect_rate 0.0 (:8676, :8705, :8944); the rest with the running rate
    k.defect_rate = (q.step == Q_2A || q.step == Q_2C || q.step == Q_7C) ? 0.0 : q.defect;
    if (k.pass == GSNAPDP_S3_END5 || k.pass == GSNAPDP_S3_END3) {
      // 8: QUERYEND_GAP; 9a / 9b: maxpeelback 0 and BEST_LOCAL (GSNAP: QUERYEND_NOGAPS); 10: QUERYEND_NOGAPS
      const bool nine = q.step == Q_9A || q.step == Q_9B;
      k.endalign = (q.step == Q_8_5 || q.step == Q_8_3)
                       ? GSNAPDP_QUERYEND_GAP
                       : (nine && !env_.o.gsnap ? GSNAPDP_BEST_LOCAL : GSNAPDP_QUERYEND_NOGAPS);
      if (nine) k.maxpeelback = 0;
    }
    k.in_minor = q.minor;
    k.in_major = q.major;
    k.in_nintrons = q.nintrons;
    k.in_nnonintrons = q.nnonintrons;
    k.in_intronlen = q.intronlen;
    k.in_nonintronlen = q.nonintronlen;
    q.passes[k.pass]++;
    return &k;
  }
  gsnapdp_s3_call* next(int i, gsnapdp_s3_call* k, std::vector<gsnapdp_s3_pair>& list,
                        const gsnapdp_s3_pair** pairs, int* n) override {
    Query& q = qs_[(size_t)(map_ ? (*map_)[(size_t)i] : i)];
    if (k->status) {
      fail(q, "a DP pass failed on the path (status -1)");
      return nullptr;
    }
    q.list.swap(list);  // (the pass's buffer takes the old list's storage for its next use; a
                        // driven pass returns each input pair with its own src: the table row)
    q.minor = k->out_minor;
    q.major = k->out_major;
    q.ub |= k->ub;
    if (k->pass == GSNAPDP_S3_INTRONS) {
      q.nintrons = k->out_nintrons;
      q.nnonintrons = k->out_nnonintrons;
      q.intronlen = k->out_intronlen;
      q.nonintronlen = k->out_nonintronlen;
      q.shiftp = k->shiftp != 0;
      q.incompletep = k->incompletep != 0;
    }
    advance(q, env_);
    gsnapdp_s3_call* c = call_for(q);
    if (c) {
      *pairs = q.list.data();
      *n = (int)q.list.size();
    }
    return c;
  }

 private:
  std::vector<Query>& qs_;
  const Env& env_;
  const std::vector<int>* map_ = nullptr;
};

int compute(gsnapdp_ctx* ctx, gsnapdp_s3_call* queries, int nqueries, const gsnapdp_s3_pair* paths_in,
            int64_t npairs_in, const char* query, const char* query_uc, size_t query_bytes, const gsnapdp_iit* iit,
            const Env& env, gsnapdp_s3_pair* out, int64_t out_cap, double* probs_out,
            gsnapdp_s3_compute_stats* stats) {
  using clock = std::chrono::steady_clock;
  const auto t0 = clock::now();
  const char* fn = env.full ? "gsnapdp_stage3_path_compute" : "gsnapdp_stage3_compute";
  if (!ctx || nqueries < 0 || npairs_in < 0 || (nqueries > 0 && (!queries || !query || !query_uc || !out))) {
    gsnapdp__set_err(std::string(fn) + ": bad arguments");
    return -1;
  }
  gsnapdp_s3_compute_stats st;
  memset(&st, 0, sizeof(st));
  std::vector<Query> qs((size_t)nqueries);
  std::vector<gsnapdp_s3_call> first((size_t)nqueries);
  Pipeline pipe(qs, env);
  for (int i = 0; i < nqueries; i++) {
    gsnapdp_s3_call& c = queries[i];
    if (c.first_pair < 0 || c.npairs < 0 || (int64_t)c.first_pair + c.npairs > npairs_in || c.qpos < 0 ||
        c.querylength < 0 || (uint64_t)c.qpos + (uint64_t)c.querylength > (uint64_t)query_bytes) {
      gsnapdp__set_err(std::string(fn) + ": query " + std::to_string(i) + " outside the buffers");
      return -1;
    }
  }
  gsnapdp::s3_parallel_for(nqueries, 16, [&](int i) {
    gsnapdp_s3_call& c = queries[i];
    Query& q = qs[(size_t)i];
    q.c = &c;
    q.list.assign(paths_in + c.first_pair, paths_in + c.first_pair + c.npairs);
    for (gsnapdp_s3_pair& p : q.list) p.src = -1;
    q.minor = c.in_minor;
    q.major = c.in_major;
    q.nintrons = c.in_nintrons;
    q.nnonintrons = c.in_nnonintrons;
    q.intronlen = c.in_intronlen;
    q.nonintronlen = c.in_nonintronlen;
    first[(size_t)i] = *pipe.call_for(q);  // pass 2A; its list is paths_in[first_pair ..]
    first[(size_t)i].first_pair = c.first_pair;
  });
  if (getenv("GSNAPDP_S3_COMPUTE_DUMP")) {  // debugging: the first pass's calls
    char path[4096];
    snprintf(path, sizeof(path), "%s/pass_000_calls.bin", getenv("GSNAPDP_S3_COMPUTE_DUMP"));
    if (FILE* f = fopen(path, "wb")) fwrite(first.data(), sizeof(first[0]), first.size(), f), fclose(f);
  }
  gsnapdp_s3_stats ps;
  if (gsnapdp::s3_run_driven(ctx, first.data(), nqueries, paths_in, npairs_in, query, query_uc, query_bytes, iit,
                             &pipe, &ps))
    return -1;
  double gpu_s = ps.seconds[1];
  auto add = [&](const gsnapdp_s3_stats& s) {
    st.passes++;
    st.rounds += s.rounds;
    for (int f = 0; f < 4; f++) st.windows[f] += s.windows[f];
  };
  add(ps);
  // the parked queries' assign_gap_types: one MaxEnt batch for all their sites,
  // then their next passes in one more driven pass, until none parks
  std::vector<int> map;
  // the parked queries' lists for their next driven pass: a buffer that is
  // copied into, never value-initialised (a resize would zero ~30 B per pair)
  std::unique_ptr<gsnapdp_s3_pair[]> phase_in;
  size_t phase_cap = 0;
  std::vector<uint8_t> model;
  std::vector<uint32_t> pos, chroff;
  std::vector<double> prob;
  std::vector<int64_t> soff, loff;
  std::vector<gsnapdp_s3_call*> next;
  for (;;) {
    map.clear();
    for (int i = 0; i < nqueries; i++) {
      const Query& q = qs[(size_t)i];
      if (!q.failed && (q.step == Q_GT_9 || q.step == Q_GT_10)) map.push_back(i);
    }
    if (map.empty()) break;
    const int nm = (int)map.size();
    soff.assign((size_t)nm + 1, 0);
    for (int j = 0; j < nm; j++) soff[(size_t)j + 1] = soff[(size_t)j] + (int64_t)qs[(size_t)map[(size_t)j]].sites.size();
    const size_t nsites = (size_t)soff[(size_t)nm];
    model.resize(nsites), pos.resize(nsites), chroff.resize(nsites), prob.resize(nsites);
    gsnapdp::s3_parallel_for(nm, 64, [&](int j) {
      size_t at = (size_t)soff[(size_t)j];
      for (const Site& s : qs[(size_t)map[(size_t)j]].sites)
        model[at] = s.model, pos[at] = s.pos, chroff[at] = s.chroffset, at++;
    });
    if (nsites) {
      const auto t1 = clock::now();
      if (gsnapdp_maxent_host(ctx, model.data(), pos.data(), chroff.data(), prob.data(), (int)nsites)) return -1;
      gpu_s += std::chrono::duration<double>(clock::now() - t1).count();
      st.sites += (int32_t)nsites;
    }
    // each parked query's probabilities, its host steps up to its next pass
    next.assign((size_t)nm, nullptr);
    gsnapdp::s3_parallel_for(nm, 4, [&](int j) {
      Query& q = qs[(size_t)map[(size_t)j]];
      size_t at = (size_t)soff[(size_t)j];
      for (const Site& s : q.sites) {
        Probs& p = q.probs[(size_t)s.row];
        (s.acceptor ? p.a : p.d) = prob[at++];
      }
      q.sites.clear();
      advance(q, env);
      next[(size_t)j] = pipe.call_for(q);
    });
    std::vector<gsnapdp_s3_call> calls;
    std::vector<int> cmap;
    loff.clear();
    int64_t tot = 0;
    for (int j = 0; j < nm; j++) {
      if (!next[(size_t)j]) continue;
      calls.push_back(*next[(size_t)j]);
      calls.back().first_pair = (int32_t)tot;
      loff.push_back(tot);
      tot += (int64_t)qs[(size_t)map[(size_t)j]].list.size();
      cmap.push_back(map[(size_t)j]);
    }
    if (calls.empty()) continue;
    if ((size_t)tot > phase_cap) {
      phase_cap = (size_t)tot + (size_t)tot / 8;
      phase_in.reset(new gsnapdp_s3_pair[phase_cap]);  // (default-initialised: no zeroing)
    }
    gsnapdp::s3_parallel_for((int)cmap.size(), 16, [&](int j) {
      const List& l = qs[(size_t)cmap[(size_t)j]].list;
      std::copy(l.begin(), l.end(), phase_in.get() + loff[(size_t)j]);
    });
    pipe.set_map(&cmap);
    const int rc = gsnapdp::s3_run_driven(ctx, calls.data(), (int)calls.size(), phase_in.get(), tot, query,
                                          query_uc, query_bytes, iit, &pipe, &ps);
    pipe.set_map(nullptr);
    if (rc) return -1;
    gpu_s += ps.seconds[1];
    add(ps);
  }
  // the returned lists, in the caller's buffer (offsets, then the copies)
  std::vector<int64_t> ooff((size_t)nqueries + 1, 0);
  for (int i = 0; i < nqueries; i++) {
    const Query& q = qs[(size_t)i];
    for (int p = 0; p < 6; p++) st.pass_calls[p] += q.passes[p];
    ooff[(size_t)i + 1] = ooff[(size_t)i] + (q.failed ? 0 : (int64_t)q.list.size());
    if (q.failed) {
      st.failed++;
      if (getenv("GSNAPDP_S3_DEBUG"))
        fprintf(stderr, "%s: query %d (tag %d) failed: %s\n", fn, i, q.c->invocation, q.why.c_str());
    }
  }
  if (ooff[(size_t)nqueries] > out_cap) {
    gsnapdp__set_err(std::string(fn) + ": the output is too small");
    return -1;
  }
  gsnapdp::s3_parallel_for(nqueries, 16, [&](int i) {
    Query& q = qs[(size_t)i];
    gsnapdp_s3_call& c = *q.c;
    const int64_t at = ooff[(size_t)i];
    c.status = q.failed ? -1 : 0;
    c.first_out = (int32_t)at;
    c.nout = (int32_t)(ooff[(size_t)i + 1] - at);
    if (q.failed) return;
    for (int64_t j = 0; j < c.nout; j++) {
      gsnapdp_s3_pair p = q.list[(size_t)j];
      if (probs_out) {
        const Probs r = probs_of(q, p);
        probs_out[2 * (at + j)] = r.d;
        probs_out[2 * (at + j) + 1] = r.a;
      }
      p.src = -1;
      out[at + j] = p;
    }
    c.out_minor = q.minor;
    c.out_major = q.major;
    c.out_nintrons = q.nintrons;
    c.out_nnonintrons = q.nnonintrons;
    c.out_intronlen = q.intronlen;
    c.out_nonintronlen = q.nonintronlen;
    c.shiftp = q.shiftp ? 1 : 0;
    c.incompletep = q.incompletep ? 1 : 0;
    c.defect_rate = q.defect;
    c.ub = q.ub;
  });
  st.seconds[1] = gpu_s;  // the time the host waited for the GPU
  st.seconds[2] = std::chrono::duration<double>(clock::now() - t0).count();
  st.seconds[0] = st.seconds[2] - st.seconds[1];
  if (stats) *stats = st;
  return 0;
}

}  // namespace

extern "C" int gsnapdp_stage3_compute(gsnapdp_ctx* ctx, gsnapdp_s3_call* queries, int nqueries,
                                      const gsnapdp_s3_pair* paths_in, int64_t npairs_in, const char* query,
                                      const char* query_uc, size_t query_bytes, const gsnapdp_iit* iit,
                                      int min_intronlength, gsnapdp_s3_pair* out, int64_t out_cap,
                                      gsnapdp_s3_compute_stats* stats) {
  Env env;
  memset(&env.o, 0, sizeof(env.o));
  env.o.min_intronlength = min_intronlength;
  return compute(ctx, queries, nqueries, paths_in, npairs_in, query, query_uc, query_bytes, iit, env, out, out_cap,
                 nullptr, stats);
}

extern "C" int gsnapdp_stage3_path_compute(gsnapdp_ctx* ctx, gsnapdp_s3_call* queries, int nqueries,
                                           const gsnapdp_s3_pair* paths_in, int64_t npairs_in, const char* query,
                                           const char* query_uc, size_t query_bytes, const gsnapdp_iit* iit,
                                           const gsnapdp_s3_path_opts* opts, gsnapdp_s3_pair* out, int64_t out_cap,
                                           double* probs_out, gsnapdp_s3_compute_stats* stats) {
  if (!opts || (nqueries > 0 && !query)) {
    gsnapdp__set_err("gsnapdp_stage3_path_compute: bad arguments");
    return -1;
  }
  Env env;
  env.o = *opts;
  env.full = true;
  env.blocks = gsnapdp__host_blocks(ctx);
  env.nwords = gsnapdp__host_nwords(ctx);
  env.iit = iit;
  env.query = query;
  return compute(ctx, queries, nqueries, paths_in, npairs_in, query, query_uc, query_bytes, iit, env, out, out_cap,
                 probs_out, stats);
}

// Pbinom as chop_ends_by_changepoint computes it (host; tests/test_pbinom.py)
extern "C" int gsnapdp_pbinom(int k, int n, double theta, double* p) { return pbinom(k, n, theta, p) ? 0 : -1; }
