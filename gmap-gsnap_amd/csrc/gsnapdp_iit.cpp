// gsnapdp_iit.cpp -- the splicing IIT as the DP path asks it (include/gsnapdp.h
// "splicing IIT"): an in-memory IIT over plain intervals, the known-site record
// of a genome-gap window (bridge_intron_gap's IIT queries, dynprog.c:3375-3612)
// and score_introns' known-site verdicts (stage3.c:7995-8116).  Host code.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <tuple>
#include <utility>
#include <vector>

#include "../../include/gsnapdp.h"

void gsnapdp__set_err(const std::string& s);

namespace {

// Each query the reference makes is an existence test on exact interval ends
// (iit-read.c:3770, 3808, 3973, 4011), so the set is four sorted key lists.
struct IntervalSet {
  gsnapdp_iit iit;  // first: the handle the caller holds is this object
  std::vector<std::tuple<int, uint32_t, uint32_t, int, int>> typed;  // chrnum, low, high, type, sign
  std::vector<std::tuple<int, uint32_t, uint32_t, int>> exact;       // chrnum, low, high, sign
  std::vector<std::tuple<int, uint32_t, int>> lows, highs;           // chrnum, end, sign
};

template <class V, class K>
bool has(const V& v, const K& k) {
  return std::binary_search(v.begin(), v.end(), k);
}
int q_typed(void* u, int chrnum, uint32_t x, uint32_t y, int type, int sign) {
  return has(((IntervalSet*)u)->typed, std::make_tuple(chrnum, x, y, type, sign)) ? 1 : 0;
}
int q_low(void* u, int chrnum, uint32_t x, int sign) {
  return has(((IntervalSet*)u)->lows, std::make_tuple(chrnum, x, sign)) ? 1 : 0;
}
int q_high(void* u, int chrnum, uint32_t x, int sign) {
  return has(((IntervalSet*)u)->highs, std::make_tuple(chrnum, x, sign)) ? 1 : 0;
}
int q_exact(void* u, int chrnum, uint32_t x, uint32_t y, int sign) {
  return has(((IntervalSet*)u)->exact, std::make_tuple(chrnum, x, y, sign)) ? 1 : 0;
}

template <class V>
void sort_unique(V& v) {
  std::sort(v.begin(), v.end());
  v.erase(std::unique(v.begin(), v.end()), v.end());
}

}  // namespace

extern "C" gsnapdp_iit* gsnapdp_iit_from_intervals(const gsnapdp_iit_interval* iv, int n) {
  if (n < 0 || (n > 0 && !iv)) {
    gsnapdp__set_err("gsnapdp_iit_from_intervals: bad arguments");
    return nullptr;
  }
  IntervalSet* s = new IntervalSet;
  bool donor = false, acceptor = false;
  for (int i = 0; i < n; i++) {
    const gsnapdp_iit_interval& x = iv[i];
    const uint32_t lo = std::min(x.start, x.end), hi = std::max(x.start, x.end);
    const int sign = x.start < x.end ? +1 : (x.start > x.end ? -1 : 0);  // Interval_new (interval.c:22-40)
    if (x.type == GSNAPDP_DONOR || x.type == GSNAPDP_ACCEPTOR) s->typed.emplace_back(x.chrnum, lo, hi, x.type, sign);
    donor |= x.type == GSNAPDP_DONOR;
    acceptor |= x.type == GSNAPDP_ACCEPTOR;
    s->exact.emplace_back(x.chrnum, lo, hi, sign);
    s->lows.emplace_back(x.chrnum, lo, sign);
    s->highs.emplace_back(x.chrnum, hi, sign);
  }
  sort_unique(s->typed);
  sort_unique(s->exact);
  sort_unique(s->lows);
  sort_unique(s->highs);
  memset(&s->iit, 0, sizeof(s->iit));
  s->iit.user = s;
  s->iit.site_level = donor && acceptor ? 1 : 0;  // IIT_typeint "donor" and "acceptor" (gmap.c:3730)
  s->iit.typed = q_typed;
  s->iit.low = q_low;
  s->iit.high = q_high;
  s->iit.exact = q_exact;
  return &s->iit;
}

extern "C" void gsnapdp_iit_free(gsnapdp_iit* iit) {
  if (iit && iit->typed == q_typed) delete (IntervalSet*)iit->user;
}

// bridge_intron_gap's known-site arrays (dynprog.c:3375-3550: left_known[cL],
// right_known[cR] per case of IIT kind, strand and direction) and, for an
// intron-level IIT without novel splicing, the (cL, cR) pairs the constrained
// bridge may take (:3598-3612).
extern "C" int gsnapdp_known_site_record(const gsnapdp_iit* iit, int novelsplicingp, int chrnum, uint32_t chrpos,
                                         uint32_t genomiclength, int leftoffset, int rightoffset, int L2L,
                                         int L2R, int cdna_direction, int watsonp, char* rec, int cap,
                                         int* len) {
  if (!iit || !rec || !len || L2L < 0 || L2R < 0) {
    gsnapdp__set_err("gsnapdp_known_site_record: bad arguments");
    return -1;
  }
  const bool sites = iit->site_level != 0;
  const bool fwd = cdna_direction > 0;
  const unsigned gl1 = genomiclength - 1U;
  const size_t base = (size_t)L2L + (size_t)L2R + 2;
  *len = (int)std::min(base, (size_t)0x7fffffff);
  if (base > (size_t)cap) return -1;
  int n = (int)base;
  memset(rec, 0, (size_t)n);
  char* left = rec;
  char* right = rec + L2L;
  for (int cL = 0; cL < L2L - 1; cL++) {  // :3379-3530, left half of each case
    const unsigned pos = watsonp ? chrpos + leftoffset + cL : chrpos + gl1 - leftoffset - cL + 1U;
    int k;
    if (sites)
      k = iit->typed(iit->user, chrnum, pos, pos + 1U, fwd ? GSNAPDP_DONOR : GSNAPDP_ACCEPTOR,
                     watsonp ? (fwd ? +1 : -1) : (fwd ? -1 : +1));
    else if (watsonp)
      k = iit->low(iit->user, chrnum, pos, fwd ? +1 : -1);
    else
      k = iit->high(iit->user, chrnum, pos + 1U, fwd ? -1 : +1);
    left[cL] = k ? 1 : 0;
  }
  for (int cR = 0; cR < L2R - 1; cR++) {  // right half of each case
    const unsigned pos = watsonp ? chrpos + rightoffset - cR + 1U : chrpos + gl1 - rightoffset + cR;
    int k;
    if (sites)
      k = iit->typed(iit->user, chrnum, pos, pos + 1U, fwd ? GSNAPDP_ACCEPTOR : GSNAPDP_DONOR,
                     watsonp ? (fwd ? +1 : -1) : (fwd ? -1 : +1));
    else if (watsonp)
      k = iit->high(iit->user, chrnum, pos + 1U, fwd ? +1 : -1);
    else
      k = iit->low(iit->user, chrnum, pos, fwd ? -1 : +1);
    right[cR] = k ? 1 : 0;
  }
  const int mode = novelsplicingp ? GSNAPDP_KNOWN_REWARD : (sites ? GSNAPDP_KNOWN_SITES : GSNAPDP_KNOWN_INTRONS);
  int npairs = 0;
  if (mode == GSNAPDP_KNOWN_INTRONS) {
    for (int cL = 0; cL < L2L - 1; cL++) {
      if (!left[cL]) continue;
      for (int cR = 0; cR < L2R - 1; cR++) {
        if (!right[cR]) continue;
        const int ok = watsonp ? iit->exact(iit->user, chrnum, chrpos + leftoffset + cL,
                                            chrpos + rightoffset - cR + 1U + 1U, cdna_direction)
                               : iit->exact(iit->user, chrnum, chrpos + gl1 - rightoffset + cR,
                                            chrpos + gl1 - leftoffset - cL + 1U + 1U, -cdna_direction);
        if (!ok) continue;
        if (npairs == 0xffff) {
          gsnapdp__set_err("gsnapdp_known_site_record: too many known introns for the record");
          *len = -1;
          return -1;
        }
        if (n + 4 <= cap) {  // past cap the pairs are only counted: *len says what the record needs
          unsigned char* e = (unsigned char*)rec + n;
          e[0] = (unsigned char)(cL & 255), e[1] = (unsigned char)(cL >> 8);
          e[2] = (unsigned char)(cR & 255), e[3] = (unsigned char)(cR >> 8);
        }
        n += 4;
        npairs++;
      }
    }
  }
  rec[L2L + L2R] = (char)(npairs & 255);
  rec[L2L + L2R + 1] = (char)(npairs >> 8);
  *len = n;
  if (n > cap) {
    gsnapdp__set_err("gsnapdp_known_site_record: the record needs " + std::to_string(n) + " bytes");
    return -1;
  }
  return mode;
}

// score_introns (stage3.c:7995-8046 for cdna_direction +1, :8069-8116 for -1):
// the donor and acceptor positions of each intron and the order of the queries
extern "C" int gsnapdp_introns_known(const gsnapdp_iit* iit, int chrnum, uint32_t chrpos, int genomiclength,
                                     int cdna_direction, int watsonp, gsnapdp_intron* introns, int n) {
  if (!iit || (n > 0 && !introns)) {
    gsnapdp__set_err("gsnapdp_introns_known: bad arguments");
    return -1;
  }
  const unsigned gl1 = (unsigned)genomiclength - 1U;
  for (int i = 0; i < n; i++) {
    gsnapdp_intron& t = introns[i];
    unsigned pd, pa;
    int sign;
    if (cdna_direction == +1) {
      pd = watsonp ? chrpos + t.left_genomepos + 1U : chrpos + gl1 - t.left_genomepos;
      pa = watsonp ? chrpos + t.right_genomepos : chrpos + gl1 - t.right_genomepos + 1U;
      sign = watsonp ? +1 : -1;
      t.known_donor = iit->typed(iit->user, chrnum, pd, pd + 1U, GSNAPDP_DONOR, sign) ? 1 : 0;
      t.known_acceptor = iit->typed(iit->user, chrnum, pa, pa + 1U, GSNAPDP_ACCEPTOR, sign) ? 1 : 0;
    } else if (cdna_direction == -1) {
      pa = watsonp ? chrpos + t.left_genomepos + 1U : chrpos + gl1 - t.left_genomepos;
      pd = watsonp ? chrpos + t.right_genomepos : chrpos + gl1 - t.right_genomepos + 1U;
      sign = watsonp ? -1 : +1;
      t.known_acceptor = iit->typed(iit->user, chrnum, pa, pa + 1U, GSNAPDP_ACCEPTOR, sign) ? 1 : 0;
      t.known_donor = iit->typed(iit->user, chrnum, pd, pd + 1U, GSNAPDP_DONOR, sign) ? 1 : 0;
    }
  }
  return 0;
}
