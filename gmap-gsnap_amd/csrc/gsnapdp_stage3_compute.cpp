// gsnapdp_stage3_compute.cpp -- passes 2A to 6 of path_compute (stage3.c:8639-8876)
// for many queries at once.
//
// Every query runs the reference's sequence: build_pairs_singles (2A), the
// adjacent-indel fix, build_pairs_singles again (2C), the defect rate,
// Smooth_pairs_by_size with build_pairs_dualintrons and the build_pairs_introns
// iterations (3a-3c), the end chop by changepoint, the two HMM filters (4),
// remove_indel_gaps and build_dual_breaks (5), and the final build_pairs_introns
// (6).  The host steps between the DP passes are restated here on each query's
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
#include <vector>

#include "../../include/gsnapdp.h"
#include "gsnapdp_stage3.h"

void gsnapdp__set_err(const std::string& s);  // gsnapdp_kernels.hip

namespace {

using List = std::vector<gsnapdp_s3_pair>;  // list order: [0] is the head

// stage3.c:42-44, smooth.c:20-36, stage3.c:74-75, changepoint.c:11-12
constexpr int MAXITER_SMOOTH_BY_SIZE = 2, MAXITER_INTRONS = 2;
constexpr double DELETE_THRESHOLD = 0.1, MARK_THRESHOLD = 1e-7, SHORTEXONPROB_END = 0.05;
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
List smooth_by_size(bool* shortp, bool* deletep, List pairs) {
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
// Pbinom (pbinom.c:1680, GSL's binomial CDF P(X <= k)): only compared with
// TRIM_END_PVALUE here, so it is computed as an exact sum of the terms in
// long double (log-space), not with GSL's incomplete-beta continued fraction
double pbinom(int k, int n, double theta) {
  if (k >= n) return 1.0;
  if (k < 0) return 0.0;
  const long double lt = logl((long double)theta), l1t = log1pl(-(long double)theta);
  long double mx = -INFINITY, sum = 0.0L;
  std::vector<long double> terms((size_t)k + 1);
  for (int i = 0; i <= k; i++) {
    const long double t = lgammal((long double)n + 1) - lgammal((long double)i + 1) - lgammal((long double)(n - i) + 1) +
                          (theta > 0 ? (long double)i * lt : (i ? -INFINITY : 0.0L)) +
                          (theta < 1 ? (long double)(n - i) * l1t : (n - i ? -INFINITY : 0.0L));
    terms[(size_t)i] = t;
    if (t > mx) mx = t;
  }
  if (mx == -INFINITY) return 0.0;
  for (long double t : terms) sum += expl(t - mx);
  return (double)(expl(mx) * sum);
}
List chop_ends_by_changepoint(List pairs) {
  if (pairs.empty()) return pairs;
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
    return pairs;
  }
  auto theta_of = [&](int m, int t) {
    double theta = (double)(nmatches - m) / (double)(ntotal - t) - THETA_SLACK;
    return theta < 0.10 ? 0.10 : theta;
  };
  if (!(ntl == 0 || ntotal - ntl <= 0) && !(pbinom(nml, ntl, theta_of(nml, ntl)) > TRIM_END_PVALUE)) chop_left(pairs);
  if (!(ntr == 0 || ntotal - ntr <= 0) && !(pbinom(nmr, ntr, theta_of(nmr, ntr)) > TRIM_END_PVALUE)) chop_right(pairs);
  return pairs;
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

// ---- one query through the passes
enum Step {
  Q_2A,       // waiting for build_pairs_singles (2A)
  Q_2C,       // ... (2C)
  Q_3B,       // build_pairs_dualintrons
  Q_3C,       // build_pairs_introns, not final
  Q_5,        // build_dual_breaks
  Q_6,        // build_pairs_introns, final
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
  gsnapdp_s3_call k;  // the pending pass's call (its pairs are list)
};
void fail(Query& q, const std::string& why) {
  if (!q.failed) q.why = why;
  q.failed = true;
  q.step = Q_DONE;
}

// the loops of path_compute between DP passes (:8711-8876), from the list the
// last pass returned (q.list) to the next pass's input, or to the end
void advance(Query& q, int min_intronlength) {
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
      } else {
        q.list = std::move(path);
        q.step = Q_DONE;
      }
      return;
    }
    case Q_6:
      q.list = std::move(pairs);
      q.step = Q_DONE;
      return;
    default: return;
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
      pairs = smooth_by_size(&q.shortp, &q.deletep, std::move(path));
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
  pairs = chop_ends_by_changepoint(std::move(pairs));
  if (!defect_rate(pairs, &q.defect, &err)) return fail(q, err);
  pairs = viterbi_filter(pairs, true, q.defect);
  pairs = viterbi_filter(pairs, false, 0.0);
  // 5: remove_indel_gaps, then build_dual_breaks on the reversed list
  List gaps = remove_indel_gaps(insert_gapholders(pairs), min_intronlength);
  reverse(gaps);
  q.list = std::move(gaps);
  q.step = Q_5;
}

int pass_of(int step) {
  switch (step) {
    case Q_2A:
    case Q_2C: return GSNAPDP_S3_SINGLES;
    case Q_3B: return GSNAPDP_S3_DUALINTRONS;
    case Q_5: return GSNAPDP_S3_DUALBREAKS;
    default: return GSNAPDP_S3_INTRONS;
  }
}

// the pipeline as the pass's driver: a query's next pass starts as soon as its
// last one has ended, in the same round, so queries at different passes share
// every round's batches
class Pipeline final : public gsnapdp::S3Driver {
 public:
  Pipeline(std::vector<Query>& qs, int min_intronlength) : qs_(qs), min_intronlength_(min_intronlength) {}
  // the query's next pass call (q.list is its input), or nullptr when it is done
  gsnapdp_s3_call* call_for(Query& q) {
    if (q.failed || q.step == Q_DONE) return nullptr;
    gsnapdp_s3_call& k = q.k;
    k = *q.c;
    k.pass = pass_of(q.step);
    k.first_pair = 0;
    k.npairs = (int32_t)q.list.size();
    k.finalp = q.step == Q_6 ? 1 : 0;
    // 2A / 2C run with defect_rate 0.0 (:8676, :8705); the rest with the running rate
    k.defect_rate = (q.step == Q_2A || q.step == Q_2C) ? 0.0 : q.defect;
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
    Query& q = qs_[(size_t)i];
    if (k->status) {
      fail(q, "a DP pass failed on the path (status -1)");
      return nullptr;
    }
    q.list.swap(list);  // (the pass's buffer takes the old list's storage for its next use)
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
    advance(q, min_intronlength_);
    gsnapdp_s3_call* c = call_for(q);
    if (c) {
      *pairs = q.list.data();
      *n = (int)q.list.size();
    }
    return c;
  }

 private:
  std::vector<Query>& qs_;
  int min_intronlength_;
};

}  // namespace

extern "C" int gsnapdp_stage3_compute(gsnapdp_ctx* ctx, gsnapdp_s3_call* queries, int nqueries,
                                      const gsnapdp_s3_pair* paths_in, int64_t npairs_in, const char* query,
                                      const char* query_uc, size_t query_bytes, const gsnapdp_iit* iit,
                                      int min_intronlength, gsnapdp_s3_pair* out, int64_t out_cap,
                                      gsnapdp_s3_compute_stats* stats) {
  using clock = std::chrono::steady_clock;
  const auto t0 = clock::now();
  if (!ctx || nqueries < 0 || npairs_in < 0 || (nqueries > 0 && (!queries || !query || !query_uc || !out))) {
    gsnapdp__set_err("gsnapdp_stage3_compute: bad arguments");
    return -1;
  }
  gsnapdp_s3_compute_stats st;
  memset(&st, 0, sizeof(st));
  std::vector<Query> qs((size_t)nqueries);
  std::vector<gsnapdp_s3_call> first((size_t)nqueries);
  Pipeline pipe(qs, min_intronlength);
  for (int i = 0; i < nqueries; i++) {
    gsnapdp_s3_call& c = queries[i];
    if (c.first_pair < 0 || c.npairs < 0 || (int64_t)c.first_pair + c.npairs > npairs_in || c.qpos < 0 ||
        c.querylength < 0 || (uint64_t)c.qpos + (uint64_t)c.querylength > (uint64_t)query_bytes) {
      gsnapdp__set_err("gsnapdp_stage3_compute: query " + std::to_string(i) + " outside the buffers");
      return -1;
    }
    Query& q = qs[(size_t)i];
    q.c = &c;
    q.list.assign(paths_in + c.first_pair, paths_in + c.first_pair + c.npairs);
    q.minor = c.in_minor;
    q.major = c.in_major;
    q.nintrons = c.in_nintrons;
    q.nnonintrons = c.in_nnonintrons;
    q.intronlen = c.in_intronlen;
    q.nonintronlen = c.in_nonintronlen;
    first[(size_t)i] = *pipe.call_for(q);  // pass 2A; its list is paths_in[first_pair ..]
    first[(size_t)i].first_pair = c.first_pair;
  }
  if (getenv("GSNAPDP_S3_COMPUTE_DUMP")) {  // debugging: the first pass's calls
    char path[4096];
    snprintf(path, sizeof(path), "%s/pass_000_calls.bin", getenv("GSNAPDP_S3_COMPUTE_DUMP"));
    if (FILE* f = fopen(path, "wb")) fwrite(first.data(), sizeof(first[0]), first.size(), f), fclose(f);
  }
  gsnapdp_s3_stats ps;
  if (gsnapdp::s3_run_driven(ctx, first.data(), nqueries, paths_in, npairs_in, query, query_uc, query_bytes, iit,
                             &pipe, &ps))
    return -1;
  st.passes = 1;
  st.rounds = ps.rounds;
  for (int f = 0; f < 4; f++) st.windows[f] = ps.windows[f];
  // the lists after pass 6, in the caller's buffer
  int64_t at = 0;
  for (int i = 0; i < nqueries; i++) {
    Query& q = qs[(size_t)i];
    for (int p = 0; p < 6; p++) st.pass_calls[p] += q.passes[p];
    gsnapdp_s3_call& c = *q.c;
    c.status = q.failed ? -1 : 0;
    c.first_out = (int32_t)at;
    c.nout = q.failed ? 0 : (int32_t)q.list.size();
    if (q.failed) {
      st.failed++;
      if (getenv("GSNAPDP_S3_DEBUG"))
        fprintf(stderr, "gsnapdp_stage3_compute: query %d (tag %d) failed: %s\n", i, c.invocation, q.why.c_str());
      continue;
    }
    if (at + c.nout > out_cap) {
      gsnapdp__set_err("gsnapdp_stage3_compute: the output is too small");
      return -1;
    }
    for (int64_t j = 0; j < c.nout; j++) {
      gsnapdp_s3_pair p = q.list[(size_t)j];
      p.src = -1;
      out[at + j] = p;
    }
    at += c.nout;
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
  }
  st.seconds[1] = ps.seconds[1];  // the time the host waited for the GPU
  st.seconds[2] = std::chrono::duration<double>(clock::now() - t0).count();
  st.seconds[0] = st.seconds[2] - st.seconds[1];
  if (stats) *stats = st;
  return 0;
}
