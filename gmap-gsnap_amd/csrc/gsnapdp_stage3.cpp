// gsnapdp_stage3.cpp -- the stage-3 DP passes of path_compute for many paths
// at once, over the batched gap families: build_pairs_introns (stage3.c:7735),
// build_pairs_singles (:7454), build_pairs_dualintrons (:7592) and the end
// extensions build_pairs_end5 / build_path_end3 (:7351 / :7236).
//
// Each path is the reference's list: the pass keeps the same cells and the
// same list operations (Pairpool_pop / List_push_existing / Pairpool_transfer,
// pairpool.c:471-519), so every peel, put-back and transfer leaves the lists
// exactly as the reference leaves them.  What changes is the control flow
// around the DP: a path runs until it needs a gap filled, parks its window,
// and resumes when its round's batch has run.  The paths are split into two
// cohorts with one round each in flight (gsnapdp_stage3.h): while the GPU runs
// one cohort's windows, a persistent pool of host threads resumes the other's
// paths, so the host work hides behind the batches instead of adding to them.
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/gsnapdp.h"
#include "gsnapdp_internal.h"
#include "gsnapdp_stage3.h"

extern "C" const uint32_t* gsnapdp__host_blocks(gsnapdp_ctx* ctx);
extern "C" size_t gsnapdp__host_nwords(gsnapdp_ctx* ctx);
void gsnapdp__set_err(const std::string& s);  // gsnapdp_kernels.hip

namespace {

using gsnapdp::ST_EARLY;
using gsnapdp::ST_INTERNAL;
using gsnapdp::ST_OK;
using gsnapdp::ST_OPS_OVERFLOW;
using gsnapdp::ST_UNSUPPORTED;

// stage3.c:50-70, dynprog.h:27-30, scores.h:7-8, intron.h:22-28
constexpr int SINGLESLEN = 9, MININTRONLEN = 9, MININTRONLEN_FINAL = 50, EXTRAQUERYGAP = 10;
constexpr int SUFFCONSECUTIVE = 5;
constexpr int UNKNOWNJUMP = -1000000;
constexpr int QOPEN = -5, QINDEL = -2, MISMATCH = -3, DUAL_HALFCANONICAL_POINTS = 4;  // scores.h:6-13
constexpr double DEFECT_HIGHQ = 0.003, DEFECT_MEDQ = 0.014;
constexpr int NONINTRON = 0, GTAG_FWD = 0x20, GTAG_REV = 0x04;
constexpr int BIG = 0x3fffffff;  // a workspace limit no window reaches

enum Fam { F_GAP = 0, F_GGAP = 1, F_CGAP = 2, F_MICRO = 3, F_N = 4, F_NONE = -1 };

float bin(double defect_rate) {  // dynprog.c:4471-4486: only the bin matters
  return defect_rate < 0.003 ? 0.001f : (defect_rate < 0.014 ? 0.01f : 0.5f);
}

// UPPERCASE_U2T (complement.h:36) as peel_* compares pairs (stage3.c:4884)
char upper_u2t(char c) {
  if (c >= 'a' && c <= 'z') c = (char)(c - 'a' + 'A');
  return c == 'U' ? 'T' : c;
}
bool unknown_base(char c) {  // pair.c
  switch (c) {
    case 'A': case 'C': case 'G': case 'T': case 'U':
    case 'a': case 'c': case 'g': case 't': case 'u': return false;
    default: return true;
  }
}

// One path's pairs and list cells.  The caller's pairs are read in place:
// pair j < nin is pairs_in[j] (only its DISALLOWED flag can change, kept in
// `dis`), cell j < nin starts as the input list's j-th cell (pair j, next
// j + 1), and the pairs and cells the pass makes are appended after them.
// Cells are never freed; a cell's pair never changes (List_push_existing
// re-links the cell itself).
//
// The input cells' links are stored sparsely, so a path costs its gaps, not
// its pairs: a cell whose link was written is in `links` (sorted by cell); a
// cell inside a reversed stretch (`rev`, [a, b): the scan's move of an
// untouched run a .. b - 1 onto `pairs`) links to cell - 1; any other still
// links to cell + 1, as the input list does (-1 after the last).  The gap
// pairs among the input pairs are `gaps` (ascending), the caller's or derived
// from the flags.
// a pair record that a resize leaves uninitialised (list_of writes every field)
struct RawPair {
  gsnapdp_s3_pair p;
  RawPair() {}
};

struct Link {
  int cell, next;
};

struct Arena {
  const gsnapdp_s3_pair* in = nullptr;
  int nin = 0;
  const int32_t* gaps = nullptr;  // the input pairs with GAPP, ascending
  int ngaps = 0;
  std::vector<int32_t> own_gaps;       // gaps derived from the flags (no caller list)
  std::vector<Link> links;             // written links of input cells, by cell
  std::vector<std::pair<int, int>> rev;  // reversed stretches [a, b), ascending, disjoint
  std::vector<int> dis;                // the input pairs the pass disallowed, ascending
  std::vector<RawPair> extra;          // pair nin + i
  std::vector<int> cp;                 // pair of cell nin + i
  std::vector<int> cnx;                // next cell of cell nin + i
  void init(const gsnapdp_s3_pair* pairs, int n, const int32_t* g, int ng) {
    in = pairs;
    nin = n;
    if (g) {
      gaps = g;
      ngaps = ng;
    } else {  // the gap pairs from the flags (one pass over the path)
      own_gaps.clear();
      for (int j = 0; j < n; j++)
        if (pairs[j].flags & GSNAPDP_S3_GAPP) own_gaps.push_back(j);
      gaps = own_gaps.data();
      ngaps = (int)own_gaps.size();
    }
    links.clear();
    rev.clear();
    dis.clear();
    extra.clear();
    cp.clear();
    cnx.clear();
  }
  // the first gap pair at or after input pair x (nin when none)
  int next_gap(int x) const {
    const int32_t* g = std::lower_bound(gaps, gaps + ngaps, x);
    return g == gaps + ngaps ? nin : *g;
  }
  bool is_dis(int p) const { return !dis.empty() && std::binary_search(dis.begin(), dis.end(), p); }
  // the flags of input pair p as the pass left them
  uint8_t in_flags(int p) const { return (uint8_t)(in[p].flags | (is_dis(p) ? GSNAPDP_S3_DISALLOWED : 0)); }
  // the reversed stretch holding c strictly inside (a < c < b), or nullptr
  const std::pair<int, int>* rev_of(int c) const {
    auto it = std::upper_bound(rev.begin(), rev.end(), c,
                               [](int x, const std::pair<int, int>& r) { return x < r.first; });
    if (it == rev.begin()) return nullptr;
    --it;
    return c > it->first && c < it->second ? &*it : nullptr;
  }
  std::vector<Link>::const_iterator link_at(int c) const {
    return std::lower_bound(links.begin(), links.end(), c, [](const Link& l, int x) { return l.cell < x; });
  }
  int next(int c) const {
    if (c >= nin) return cnx[(size_t)(c - nin)];
    const auto it = link_at(c);
    if (it != links.end() && it->cell == c) return it->next;
    if (rev_of(c)) return c - 1;
    return c + 1 < nin ? c + 1 : -1;
  }
  void set_next(int c, int v) {
    if (c >= nin) {
      cnx[(size_t)(c - nin)] = v;
      return;
    }
    auto it = std::lower_bound(links.begin(), links.end(), c, [](const Link& l, int x) { return l.cell < x; });
    if (it != links.end() && it->cell == c) it->next = v;
    else links.insert(it, Link{c, v});
  }
  bool linked_in(int lo, int hi) const {  // a written link among cells lo .. hi
    const auto it = link_at(lo);
    return it != links.end() && it->cell <= hi;
  }
  // the scan's moves of the non-gap input cells at the head of `path` onto
  // `pairs` (Pairpool_pop + List_push_existing each): an untouched run a .. g - 1
  // up to the next gap moves at once (a link for a, the stretch for the rest)
  void move_run(int* path, int* pairs) {
    int x = *path, head = *pairs;
    while (x >= 0 && x < nin) {
      const int g = next_gap(x);
      if (g == x) break;  // a gap pair
      const std::pair<int, int>* r = rev_of(x);
      auto ov = std::upper_bound(rev.begin(), rev.end(), g - 1,
                                 [](int v, const std::pair<int, int>& s) { return v < s.first; });
      const bool rev_clear = ov == rev.begin() || std::prev(ov)->second <= x;
      if (!r && rev_clear && !linked_in(x, g - 1)) {
        set_next(x, head);
        if (g - 1 > x) rev.insert(ov, std::make_pair(x, g));
        head = g - 1;
        x = g < nin ? g : -1;
        continue;
      }
      const int nx = next(x);
      set_next(x, head);
      head = x;
      x = nx;
    }
    *path = x;
    *pairs = head;
  }
  int pairof(int cell) const { return cell < nin ? cell : cp[(size_t)(cell - nin)]; }
  int cell(int pair, int nx) {
    cp.push_back(pair);
    cnx.push_back(nx);
    return nin + (int)cp.size() - 1;
  }
  int pop(int list, int* pair) const {  // Pairpool_pop
    *pair = pairof(list);
    return next(list);
  }
  int push_existing(int list, int c) {  // List_push_existing
    set_next(c, list);
    return c;
  }
  int transfer(int dest, int src) {  // Pairpool_transfer
    for (int p = src, nx; p >= 0; p = nx) {
      nx = next(p);
      set_next(p, dest);
      dest = p;
    }
    return dest;
  }
  int reverse(int list) { return transfer(-1, list); }  // List_reverse (the same cells)
  const gsnapdp_s3_pair& at(int pair) const { return pair < nin ? in[pair] : extra[(size_t)(pair - nin)].p; }
  uint8_t flag(int pair) const { return pair < nin ? in_flags(pair) : extra[(size_t)(pair - nin)].p.flags; }
  const gsnapdp_s3_pair& first(int list) const { return at(pairof(list)); }
  void disallow(int list) {  // pair->disallowedp = true (stage3.c:5873-5880)
    const int p = pairof(list);
    if (p < nin) {
      auto it = std::lower_bound(dis.begin(), dis.end(), p);
      if (it == dis.end() || *it != p) dis.insert(it, p);
    } else {
      extra[(size_t)(p - nin)].p.flags |= GSNAPDP_S3_DISALLOWED;
    }
  }
  int rest(int list) const { return next(list); }
  int push_pair(int list, const gsnapdp_s3_pair& x) {
    extra.emplace_back();
    extra.back().p = x;
    return cell(nin + (int)extra.size() - 1, list);
  }
  // the returned cell as the ABI reports it: an input pair with its flags and
  // src = its index, or a pair the pass made (src -1)
  gsnapdp_s3_pair out(int list) const {
    const int p = pairof(list);
    if (p >= nin) return extra[(size_t)(p - nin)].p;
    gsnapdp_s3_pair x = in[p];
    x.src = p;
    x.flags = in_flags(p);
    return x;
  }
  // the run of input cells from `cell` down: cell, cell - 1, ..., returned as
  // its lowest cell (the scan's reversal of an untouched stretch of the path),
  // in steps of whole stretches between written links
  int run_end(int cell) const {
    if (cell >= nin) return cell;
    int q = cell;
    while (q > 0) {
      const auto it = link_at(q);
      if (it != links.end() && it->cell == q) {
        if (it->next != q - 1) break;
        q--;
        continue;
      }
      const std::pair<int, int>* r = rev_of(q);
      if (!r) break;  // an input link: q + 1
      // cells r->first + 1 .. q link downwards unless written: down to the
      // highest written link below q, or to the stretch's first cell
      const int below = it == links.begin() ? -1 : std::prev(it)->cell;
      q = std::max(r->first, below);
    }
    return q;
  }
};
bool gapp(const gsnapdp_s3_pair& p) { return (p.flags & GSNAPDP_S3_GAPP) != 0; }

// A returned list as segments, in list order: in_run(hi, lo, d) for input
// pairs hi, hi - 1, .., lo (a disallowed pair is a run of its own with d set),
// new_pair(e) for the pass's pair nin + e.  Costs the list's runs, not its pairs.
template <class In, class New>
void walk_list(const Arena& A, int list, In&& in_run, New&& new_pair) {
  for (int p = list; p >= 0;) {
    if (p < A.nin) {
      const int lo = A.run_end(p);
      int hi = p;
      if (!A.dis.empty()) {
        auto it = std::upper_bound(A.dis.begin(), A.dis.end(), hi);
        while (it != A.dis.begin() && *std::prev(it) >= lo) {
          const int d = *--it;
          if (d < hi) in_run(hi, d + 1, false);
          in_run(d, d, true);
          hi = d - 1;
        }
      }
      if (hi >= lo) in_run(hi, lo, false);
      p = A.rest(lo);
    } else {
      const int pr = A.pairof(p);
      if (pr < A.nin) in_run(pr, pr, A.is_dis(pr));
      else new_pair(pr - A.nin);
      p = A.rest(p);
    }
  }
}

// The DP window a path is waiting for, in the batched C-ABI's records.
struct Req {
  int fam = F_NONE;
  std::vector<char> q, qu;  // the window's query bytes; qpos fields are relative to them
  int64_t cap = 0;
  const uint32_t* ops = nullptr;  // the window's op stream in its round's output staging
  gsnapdp_window w;
  gsnapdp_result r;
  gsnapdp_ggap_window gw;
  gsnapdp_ggap_result gr;
  gsnapdp_ggap_trace gt;
  gsnapdp_cgap_window cw;
  gsnapdp_cgap_result cr;
  gsnapdp_micro_window mw;
  gsnapdp_micro_result mr;
};

// where a path resumes when its window has run
enum Stage {
  S_SCAN,         // between gaps
  S_SINGLE,       // traverse_single_gap's Dynprog_single_gap
  S_CDNA_SINGLE,  // traverse_cdna_gap: "really a single gap"
  S_CDNA,         // traverse_cdna_gap's Dynprog_cdna_gap
  S_GG_SINGLE,    // traverse_genome_gap: "really a single gap"
  S_GG_SCORE,     // traverse_genome_gap's score-mode Dynprog_genome_gap
  S_GG_PROB,      // its probability-mode re-run
  S_GG_MICRO,     // its Dynprog_microexon_int
  S_END,          // extend_ending5 / extend_ending3's Dynprog_end5_gap / Dynprog_end3_gap
  S_DUAL_SINGLE,  // traverse_dual_genome_gap: the single-intron Dynprog_genome_gap
  S_DUAL_2,       // its right-of-short-exon window (halfp)
  S_DUAL_1,       // its left-of-short-exon window (halfp)
  S_DUAL_RIGHT,   // single wins, right_end_intron_p: keep the left intron only
  S_DUAL_LEFT,    // single wins, left_end_intron_p: keep the right intron only
  S_DONE
};

struct Path {
  int idx = -1;  // the path's index in the pass (kept by reset)
  gsnapdp_s3_call* c = nullptr;
  const char* q = nullptr;   // queryseq_ptr
  const char* qu = nullptr;  // queryuc_ptr
  Arena A;
  int path = -1, pairs = -1;
  int stage = S_SCAN;
  bool failed = false;
  std::string why;
  // build_pairs_introns' counters (its in/out arguments)
  int minor = 0, major = 0, nintrons = 0, nnonintrons = 0, intronlen = 0, nonintronlen = 0;
  bool shiftp = false, incompletep = false;
  // the gap being traversed (pairptr, leftpair, rightpair) and its peels
  int gapcell = -1, left = -1, right = -1;
  int peeled_pairs = -1, peeled_path = -1;
  int querydp5 = 0, genomedp5 = 0, querydp3 = 0, genomedp3 = 0, queryjump = 0, genomejump = 0;
  // traverse_genome_gap's locals.  new_left/right and introntype keep their
  // values across that function's calls, like the reference's stack slots do
  // when a Dynprog_genome_gap early return leaves them unwritten.
  int finalscore = 0, nmatches = 0, nmismatches = 0, nopens = 0, nindels = 0, exonhead = 0;
  int new_left = 0, new_right = 0, introntype = 0;
  bool newpos_set = false;  // new_left / new_right written in this traverse_genome_gap call
  bool ub = false;          // the outputs took the reference's uninitialised locals
  int ub_bits = 0;          // which (GSNAPDP_S3_UB_*)
  double left_prob = 0.0, right_prob = 0.0;
  int gappairs = -1;
  int undefined = 0;  // probability re-runs with no qualifying candidate
  // build_pairs_dualintrons' midexon_pairs (a function-scope local that keeps
  // its value from one short exon to the next) and traverse_dual_genome_gap's
  // state between its windows
  int midexon = -1;
  struct Dual {
    bool left_end = false, right_end = false;
    int midq = 0, midg = 0;
    int q5 = 0, g5 = 0, q3 = 0, g3 = 0;  // the peeled bounds
    int single = -1, dual2 = -1, dual1 = -1;
    int single_goodness = 0, dual_goodness = 0;
    bool single_typed = false;  // single_introntype written by its Dynprog_genome_gap
    int single_introntype = 0, introntype2 = 0, introntype1 = 0;
    int right_exonhead = 0, left_exonhead = 0;
  } d;
  Req req;
};

// Paths are kept between passes (their vectors keep their capacity), so a
// pass does not fault fresh pages in for every arena; concurrent passes each
// take their own set.
struct PathStore {
  std::vector<Path> paths;
};
std::mutex g_store_mu;
std::vector<PathStore*> g_store;
PathStore* store_acquire() {
  std::lock_guard<std::mutex> l(g_store_mu);
  if (g_store.empty()) return new PathStore;
  PathStore* s = g_store.back();
  g_store.pop_back();
  return s;
}
void store_release(PathStore* s) {
  std::lock_guard<std::mutex> l(g_store_mu);
  g_store.push_back(s);
}
// a path as a fresh Path, keeping its vectors' storage
void reset(Path& k) {
  Arena A = std::move(k.A);
  Req R = std::move(k.req);
  std::string why = std::move(k.why);
  const int idx = k.idx;
  k = Path();
  k.idx = idx;
  k.A = std::move(A);
  k.req = std::move(R);
  k.req.fam = F_NONE;
  k.why = std::move(why);
  k.why.clear();
}

struct Pass {
  gsnapdp_ctx* ctx;
  const uint32_t* blocks;
  size_t nwords;
  const gsnapdp_iit* iit;  // Dynprog_setup's splicing IIT, or nullptr
  gsnapdp_s3_stats st;
  const char* query = nullptr;
  const char* query_uc = nullptr;
  gsnapdp::S3Driver* driver = nullptr;  // driven passes: a path's next pass when one ends
  const int32_t* gaps = nullptr;        // the callers' gap-pair lists (gsnapdp_stage3_pass_runs), or nullptr
  const int64_t* gap_off = nullptr;
};

}  // namespace

// ---- genome characters (stage3.c get_genomic_nt, with no genomic segment)
char gsnapdp::s3_genomic_nt(const uint32_t* blocks, size_t nwords, const gsnapdp_s3_call& c, int gpos) {
  if (gpos < 0 || gpos >= c.genomiclength) return '*';
  const uint32_t base = c.chroffset + c.chrpos;
  if (base < c.chroffset || base >= c.chrhigh) return '*';
  const uint32_t pos = c.watsonp ? base + (uint32_t)gpos : base + (uint32_t)(c.genomiclength - 1) - (uint32_t)gpos;
  const size_t ptr = (size_t)(pos >> 5) * 3;
  if (ptr + 2 >= nwords) return 'N';
  const uint32_t bit = pos & 31u;
  char ch = 'N';
  if (!((blocks[ptr + 2] >> bit) & 1u))
    ch = "ACGT"[((bit < 16 ? blocks[ptr + 1] : blocks[ptr]) >> ((bit & 15u) * 2u)) & 3u];
  if (c.watsonp) return ch;
  switch (ch) {  // complCode
    case 'A': return 'T';
    case 'C': return 'G';
    case 'G': return 'C';
    case 'T': return 'A';
    default: return 'N';
  }
}

namespace {

char genomic_nt(const Pass& P, const Path& k, int gpos) {
  return gsnapdp::s3_genomic_nt(P.blocks, P.nwords, *k.c, gpos);
}
int nt_class(char ch) {
  switch (ch) {
    case 'A': return 0;
    case 'C': return 1;
    case 'G': return 2;
    case 'T': return 3;
    case '*': return 5;
    default: return 4;
  }
}

// ---- Pair_fracidentity (pair.c:5426) and Dynprog_score (dynprog.c:381-394):
// the score of a peeled stretch, for traverse_single_gap's accept test
int peeled_score(Arena& A, int list, int cdna_direction, double defect_rate, std::string* err) {
  (void)cdna_direction;  // only the canonical-intron counts depend on it
  int matches = 0, mismatches = 0, qopens = 0, qindels = 0, topens = 0, tindels = 0;
  int prev = -1;
  for (int p = list; p >= 0; p = A.rest(p)) {
    const gsnapdp_s3_pair& x = A.first(p);
    if (!gapp(x)) {
      if (x.comp == '-' || x.comp == '~') {
        if (x.cdna == ' ') {
          tindels++;
          if (prev >= 0 && A.at(prev).cdna != ' ') topens++;
        } else if (x.genome == ' ') {
          qindels++;
          if (prev >= 0 && A.at(prev).genome != ' ') qopens++;
        } else {
          *err = "Pair_fracidentity: cannot parse comp";  // the reference aborts
          return 0;
        }
      } else if (unknown_base(x.cdna) || unknown_base(x.genome) || x.comp == ':') {
        // unknowns
      } else if (x.comp == '|' || x.comp == '*' || x.comp == ':') {
        matches++;
      } else if (x.comp == ' ') {
        mismatches++;
      } else {
        *err = "Pair_fracidentity: cannot parse comp";
        return 0;
      }
    }
    prev = A.pairof(p);
  }
  const int mism = defect_rate < DEFECT_HIGHQ ? -3 : (defect_rate < DEFECT_MEDQ ? -2 : -1);
  return 3 * matches + mism * mismatches - 10 * qopens - 3 * qindels - 10 * topens - 3 * tindels;
}
int dynprog_score(int qopens, int qindels, int topens, int tindels) {
  return -10 * qopens - 3 * qindels - 10 * topens - 3 * tindels;  // every bin: open -10, extend -3
}

// ---- peel_rightward / peel_leftward (stage3.c:5126-5378, :4887-5122) without
// end-gap pairs (every caller here passes endgappairs = NULL)
int peel_rightward(Arena& A, bool* mismatchp, int* peeled_pairs, int pairs, int* querydp3,
                   int* genomedp3, int maxpeelback, bool throughmismatchp) {
  int peeled = -1, rest = -1, pair = -1, nextpair = -1, npeelback = 0, nconsecutive = 0;
  *mismatchp = false;
  if (pairs >= 0) {
    if (gapp(A.first(pairs))) {  // throw away known gap
      const int ptr = pairs;
      pairs = A.pop(pairs, &pair);
      peeled = A.push_existing(peeled, ptr);
    }
    rest = A.rest(pairs);
    bool stopp = false;
    while (rest >= 0 && !stopp) {
      nextpair = A.pairof(rest);
      const gsnapdp_s3_pair& nx = A.at(nextpair);
      if (gapp(nx) || nx.cdna == ' ' || nx.genome == ' ') stopp = true;
      const int ptr = pairs;
      pairs = A.pop(pairs, &pair);
      peeled = A.push_existing(peeled, ptr);
      if (upper_u2t(A.at(pair).cdna) != upper_u2t(A.at(pair).genome)) *mismatchp = true;
      if (++npeelback >= maxpeelback) stopp = true;
      rest = A.rest(pairs);
    }
    if (throughmismatchp && rest >= 0 && !gapp(A.at(nextpair))) {
      stopp = false;
      while (rest >= 0 && !stopp) {
        nextpair = A.pairof(rest);
        if (gapp(A.at(nextpair))) stopp = true;
        const int ptr = pairs;
        pairs = A.pop(pairs, &pair);
        peeled = A.push_existing(peeled, ptr);
        const gsnapdp_s3_pair& x = A.at(pair);
        if (upper_u2t(x.cdna) != upper_u2t(x.genome)) *mismatchp = true;
        if (x.comp == '-' || x.comp == ' ') nconsecutive = 0;
        else if (++nconsecutive >= SUFFCONSECUTIVE) stopp = true;
        rest = A.rest(pairs);
      }
    }
  }
  if (peeled >= 0) {
    const gsnapdp_s3_pair& lp = A.first(peeled);
    if (gapp(lp)) {  // ran into a gap: undo the peel
      pairs = A.transfer(pairs, peeled);
      *peeled_pairs = -1;
      return pairs;
    }
    *querydp3 = lp.cdna == ' ' ? lp.querypos - 1 : lp.querypos;
    *genomedp3 = lp.genome == ' ' ? lp.genomepos - 1 : lp.genomepos;
  }
  *peeled_pairs = peeled;
  return pairs;
}

int peel_leftward(Arena& A, bool* mismatchp, int* peeled_path, int path, int* querydp5, int* genomedp5,
                  int maxpeelback, bool throughmismatchp) {
  int peeled = -1, rest = -1, pair = -1, nextpair = -1, npeelback = 0, nconsecutive = 0;
  *mismatchp = false;
  if (path >= 0) {
    if (gapp(A.first(path))) {
      const int ptr = path;
      path = A.pop(path, &pair);
      peeled = A.push_existing(peeled, ptr);
    }
    rest = A.rest(path);
    bool stopp = false;
    while (rest >= 0 && !stopp) {
      nextpair = A.pairof(rest);
      const gsnapdp_s3_pair& nx = A.at(nextpair);
      if (gapp(nx) || nx.cdna == ' ' || nx.genome == ' ') stopp = true;
      const int ptr = path;
      path = A.pop(path, &pair);
      peeled = A.push_existing(peeled, ptr);
      if (upper_u2t(A.at(pair).cdna) != upper_u2t(A.at(pair).genome)) *mismatchp = true;
      if (++npeelback >= maxpeelback) stopp = true;
      rest = A.rest(path);
    }
    if (throughmismatchp && rest >= 0 && !gapp(A.at(nextpair))) {
      stopp = false;
      while (rest >= 0 && !stopp) {
        nextpair = A.pairof(rest);
        if (gapp(A.at(nextpair))) stopp = true;
        const int ptr = path;
        path = A.pop(path, &pair);
        peeled = A.push_existing(peeled, ptr);
        const gsnapdp_s3_pair& x = A.at(pair);
        if (upper_u2t(x.cdna) != upper_u2t(x.genome)) *mismatchp = true;
        if (x.comp == '-' || x.comp == ' ') nconsecutive = 0;
        else if (++nconsecutive >= SUFFCONSECUTIVE) stopp = true;
        rest = A.rest(path);
      }
    }
  }
  if (peeled >= 0) {
    const gsnapdp_s3_pair& rp = A.first(peeled);
    if (gapp(rp)) {
      path = A.transfer(path, peeled);
      *peeled_path = -1;
      return path;
    }
    *querydp5 = rp.querypos;
    *genomedp5 = rp.genomepos;
  }
  *peeled_path = peeled;
  return path;
}

// ---- the DP windows, built exactly as the drop-in's Dynprog_* entry points
// build them (gsnapdp_dropin.cpp), from the arguments stage 3 passes

// query bytes [from, from + n) of the path, zero past its end, dword padded
void stage_query(const Path& k, Req& R, int from, int n, size_t extra = 0) {
  const size_t sz = (((size_t)(n > 0 ? n : 0) + 8 + 3) & ~(size_t)3) + extra;
  R.q.assign(sz, 0);
  R.qu.assign(sz, 0);
  for (int i = 0; i < n; i++) {
    const int p = from + i;
    if (p >= 0 && p < k.c->querylength) {
      R.q[(size_t)i] = k.q[p];
      R.qu[(size_t)i] = k.qu[p];
    }
  }
}

// Dynprog_single_gap (dynprog.c:4450-4572), widebandp = true, on dynprogM
void req_single(Path& k) {
  const gsnapdp_s3_call& c = *k.c;
  Req& R = k.req;
  R.fam = F_GAP;
  gsnapdp_window& w = R.w;
  memset(&w, 0, sizeof(w));
  w.kind = GSNAPDP_SINGLE_GAP;
  w.length1 = k.queryjump;
  w.length2 = k.genomejump;
  w.offset1 = k.querydp5;
  w.offset2 = k.genomedp5;
  w.chroffset = c.chroffset;
  w.chrhigh = c.chrhigh;
  w.chrpos = c.chrpos;
  w.genomiclength = (uint32_t)c.genomiclength;
  w.cdna_direction = c.cdna_direction;
  w.extraband = c.extraband_single;
  w.dynprogindex = k.minor;
  w.maxlength1 = c.maxlength1[1];
  w.maxlength2 = c.maxlength2[1];
  w.defect_rate = bin(c.defect_rate);
  w.watsonp = c.watsonp ? 1 : 0;
  w.jump_late_p = c.jump_late_p ? 1 : 0;
  w.widebandp = 1;
  stage_query(k, R, k.querydp5, k.queryjump);
  w.qpos = 0;
  R.cap = (int64_t)(k.queryjump > 0 ? k.queryjump : 0) + (k.genomejump > 0 ? k.genomejump : 0) + 2;
}

// Dynprog_genome_gap (dynprog.c:4798-5061); with a splicing IIT
// the window's known-site record follows its query rows, as the drop-in's
// Dynprog_genome_gap places it
bool req_genome(const Pass& P, Path& k, bool prob, int score_threshold, bool halfp = false, int finalp = -1) {
  const gsnapdp_s3_call& c = *k.c;
  Req& R = k.req;
  R.fam = F_GGAP;
  gsnapdp_ggap_window& w = R.gw;
  memset(&w, 0, sizeof(w));
  w.length1 = k.queryjump;
  w.length2L = k.genomejump;
  w.length2R = k.genomejump;
  w.offset1 = k.querydp5;
  w.offset2L = k.genomedp5;
  w.revoffset2R = k.genomedp3;
  w.chroffset = c.chroffset;
  w.chrhigh = c.chrhigh;
  w.chrpos = c.chrpos;
  w.genomiclength = (uint32_t)c.genomiclength;
  w.qpos = 0;
  w.cdna_direction = c.cdna_direction;
  w.extraband_paired = c.extraband_paired;
  w.maxpeelback = c.maxpeelback;
  w.score_threshold = score_threshold;
  w.dynprogindex = k.major;
  // the two workspaces' limits (:4898-4927), folded into one exact test
  const bool too_long = k.queryjump > c.maxlength1[0] || k.genomejump > c.maxlength2[0] ||
                        k.queryjump > c.maxlength1[2] || k.genomejump > c.maxlength2[2];
  w.maxlength1 = too_long ? -1 : BIG;
  w.maxlength2 = BIG;
  w.defect_rate = bin(c.defect_rate);
  w.watsonp = c.watsonp ? 1 : 0;
  w.jump_late_p = c.jump_late_p ? 1 : 0;
  w.halfp = halfp ? 1 : 0;
  w.finalp = (prob || (finalp < 0 ? c.finalp != 0 : finalp != 0)) ? 1 : 0;
  w.use_probabilities_p = prob ? 1 : 0;
  w.splicingp = c.splicingp ? 1 : 0;
  w.known_mode = GSNAPDP_KNOWN_NONE;
  stage_query(k, R, k.querydp5, k.queryjump);
  const int L1 = k.queryjump > 0 ? k.queryjump : 0;
  R.cap = 2 * (int64_t)L1 + 2 * (int64_t)(k.genomejump > 0 ? k.genomejump : 0) + 4;
  if (P.iit && L1 > 1 && k.genomejump > 0 && !too_long) {
    // the two site arrays and room for a few known introns; a longer intron list
    // (KNOWN_INTRONS mode) asks again with the length the first call reported
    int rcap = (int)std::min<size_t>(2 * (size_t)k.genomejump + 2 + 4 * 64, 0x7fffffff);
    int len = 0, mode = -1;
    for (int tries = 0; tries < 2 && mode < 0; tries++) {
      R.q.resize((size_t)L1 + (size_t)rcap);
      mode = gsnapdp_known_site_record(P.iit, c.novelsplicingp, c.chrnum, c.chrpos, (uint32_t)c.genomiclength,
                                       k.genomedp5, k.genomedp3, k.genomejump, k.genomejump, c.cdna_direction,
                                       c.watsonp, R.q.data() + L1, rcap, &len);
      if (mode < 0 && len > rcap) rcap = len;
      else break;
    }
    if (mode < 0) return false;
    w.known_mode = (uint8_t)mode;
    R.q.resize((((size_t)L1 + (size_t)len + 8) + 3) & ~(size_t)3, 0);
    R.qu.resize(R.q.size(), 0);
  }
  return true;
}

// Dynprog_cdna_gap (dynprog.c:4578-4793): length1L = length1R = queryjump
void req_cdna(Path& k) {
  const gsnapdp_s3_call& c = *k.c;
  Req& R = k.req;
  R.fam = F_CGAP;
  gsnapdp_cgap_window& w = R.cw;
  memset(&w, 0, sizeof(w));
  const int length1 = k.queryjump, length2 = k.genomejump;
  w.length1L = length1;
  w.length1R = length1;
  w.length2 = length2;
  w.offset1L = k.querydp5;
  w.revoffset1R = k.querydp3;
  w.offset2 = k.genomedp5;
  w.chroffset = c.chroffset;
  w.chrhigh = c.chrhigh;
  w.chrpos = c.chrpos;
  w.genomiclength = (uint32_t)c.genomiclength;
  w.cdna_direction = c.cdna_direction;
  w.extraband_paired = c.extraband_paired;
  w.dynprogindex = k.major;
  const bool too_long = length2 > c.maxlength1[2] || length1 > c.maxlength2[2] || length2 > c.maxlength1[0] ||
                        length1 > c.maxlength2[0];
  w.maxlength1 = too_long ? -1 : BIG;
  w.maxlength2 = BIG;
  w.defect_rate = bin(c.defect_rate);
  w.watsonp = c.watsonp ? 1 : 0;
  w.jump_late_p = c.jump_late_p ? 1 : 0;
  // sequence1L[0 .. span) forwards, then revsequence1R[-(nR-1) .. 0]
  const int nL = length1 > 0 ? length1 : 0, nR = nL;
  const int span = k.querydp3 - k.querydp5 + 1 > nL ? k.querydp3 - k.querydp5 + 1 : nL;
  R.q.assign(((size_t)span + nR + 8 + 3) & ~(size_t)3, 0);
  R.qu.assign(R.q.size(), 0);
  if (length2 > 1) {
    for (int i = 0; i < span; i++) {
      const int p = k.querydp5 + i;
      if (p >= 0 && p < c.querylength) {
        R.q[(size_t)i] = k.q[p];
        R.qu[(size_t)i] = k.qu[p];
      }
    }
    for (int i = 0; i < nR; i++) {
      const int p = k.querydp3 - (nR - 1) + i;
      if (p >= 0 && p < c.querylength) {
        R.q[(size_t)(span + i)] = k.q[p];
        R.qu[(size_t)(span + i)] = k.qu[p];
      }
    }
  }
  w.qposL = 0;
  w.qposR = (uint32_t)(span + nR - 1);
  R.cap = (int64_t)nL + nR + 2 * (int64_t)(length2 > 0 ? length2 : 0) + 4;
}

// Dynprog_microexon_int (dynprog.c:7128-7432): sequence1 = &queryseq[offset1]
void req_micro(Path& k) {
  const gsnapdp_s3_call& c = *k.c;
  Req& R = k.req;
  R.fam = F_MICRO;
  const int L1 = k.queryjump > 0 ? k.queryjump : 0;
  const size_t pbase = ((size_t)L1 + 8 + 3) & ~(size_t)3;
  stage_query(k, R, k.querydp5, L1, pbase);
  for (int i = 0; i < L1; i++) {
    R.q[pbase + (size_t)i] = R.q[(size_t)i];
    R.qu[pbase + (size_t)i] = R.qu[(size_t)i];
  }
  gsnapdp_micro_window& w = R.mw;
  memset(&w, 0, sizeof(w));
  w.length1 = k.queryjump;
  w.offset1 = k.querydp5;
  w.offset2L = k.genomedp5;
  w.revoffset2R = k.genomedp3;
  w.cdna_direction = c.cdna_direction;
  w.dynprogindex = k.major;
  w.chroffset = c.chroffset;
  w.chrhigh = c.chrhigh;
  w.chrpos = c.chrpos;
  w.genomiclength = (uint32_t)c.genomiclength;
  w.qpos = 0;
  w.ppos = (uint32_t)pbase;
  w.defect_rate = bin(c.defect_rate);
  w.watsonp = c.watsonp ? 1 : 0;
  R.cap = 0;
}

// Dynprog_end5_gap / Dynprog_end3_gap (dynprog.c:5094-5284 / 5290-5406), as
// extend_ending5 / extend_ending3 call them (stage3.c:6665-6676, :6983-6994):
// dynprogR at the 5' end, dynprogL at the 3' end, widebandp
void req_end(Path& k, bool end5) {
  const gsnapdp_s3_call& c = *k.c;
  Req& R = k.req;
  R.fam = F_GAP;
  gsnapdp_window& w = R.w;
  memset(&w, 0, sizeof(w));
  w.kind = end5 ? GSNAPDP_END5_GAP : GSNAPDP_END3_GAP;
  w.length1 = k.queryjump;
  w.length2 = k.genomejump;
  w.offset1 = end5 ? k.querydp3 : k.querydp5;  // revoffset1 / offset1
  w.offset2 = end5 ? k.genomedp3 : k.genomedp5;
  w.chroffset = c.chroffset;
  w.chrhigh = c.chrhigh;
  w.chrpos = c.chrpos;
  w.genomiclength = (uint32_t)c.genomiclength;
  w.cdna_direction = c.cdna_direction;
  w.extraband = c.extraband_end;
  w.dynprogindex = k.minor;
  w.maxlength1 = c.maxlength1[end5 ? 2 : 0];
  w.maxlength2 = c.maxlength2[end5 ? 2 : 0];
  w.defect_rate = bin(c.defect_rate);
  w.watsonp = c.watsonp ? 1 : 0;
  w.jump_late_p = c.jump_late_p ? 1 : 0;
  w.widebandp = 1;
  w.endalign = (uint8_t)c.endalign;
  const int L1 = k.queryjump > 0 ? k.queryjump : 0;
  // revsequence1[-(L1 - 1) .. 0] ends at querydp3; sequence1 starts at querydp5
  stage_query(k, R, end5 ? k.querydp3 - (L1 - 1) : k.querydp5, L1);
  w.qpos = end5 ? (uint32_t)(L1 > 0 ? L1 - 1 : 0) : 0u;
  R.cap = (int64_t)L1 + (k.genomejump > 0 ? k.genomejump : 0) + 2;
}

void fail(Path& k, const std::string& why) {
  if (!k.failed) k.why = why;
  k.failed = true;
  k.stage = S_DONE;
  k.req.fam = F_NONE;
}

// GSNAPDP_S3_PROFILE=1: where a pass's host time goes (stderr at the end of the pass)
struct Prof {
  bool on = getenv("GSNAPDP_S3_PROFILE") != nullptr;
  std::atomic<int64_t> expand_ns[F_N] = {{0}, {0}, {0}, {0}}, resume_ns{0}, driver_ns{0};
  double init = 0, pack = 0, copy = 0, submit = 0, wait = 0, resume = 0, output = 0;
};
Prof& prof() {
  static Prof p;
  return p;
}
struct Tic {  // adds its lifetime to an atomic nanosecond counter when profiling
  std::atomic<int64_t>* acc;
  std::chrono::steady_clock::time_point t0;
  explicit Tic(std::atomic<int64_t>& a) : acc(prof().on ? &a : nullptr) {
    if (acc) t0 = std::chrono::steady_clock::now();
  }
  ~Tic() {
    if (acc)
      acc->fetch_add(
          std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count());
  }
};

// the pairs a family's op stream expands into (one buffer per host thread)
std::vector<gsnapdp_pair>& expand_buf(size_t n) {
  thread_local std::vector<gsnapdp_pair> v;
  if (v.size() < n) v.resize(n);
  return v;
}

// a gap family's expanded pairs as a list in the path's arena (push order as
// the drop-in's push_pairs: the list's head is pairs[0])
int list_of(Arena& A, const std::vector<gsnapdp_pair>& v, int n, bool micro) {
  if (n <= 0) return -1;
  // pairs nin + e0 .. e0 + n - 1 in cells c0 .. c0 + n - 1: the list's head is
  // v[0]'s cell, and each cell links to the next (push order from v[n - 1])
  const size_t e0 = A.extra.size(), k0 = A.cp.size();
  A.extra.resize(e0 + (size_t)n);
  A.cp.resize(k0 + (size_t)n);
  A.cnx.resize(k0 + (size_t)n);
  const size_t c0 = (size_t)A.nin + k0;
  for (int i = 0; i < n; i++) {
    const gsnapdp_pair& p = v[(size_t)i];
    gsnapdp_s3_pair& x = A.extra[e0 + (size_t)i].p;
    x.queryjump = x.genomejump = 0;
    x.src = -1;
    x.flags = 0;
    if (p.gapp) {  // Pairpool_push_gapholder (pairpool.c:352-410)
      x.querypos = -1;
      x.genomepos = -1;
      x.queryjump = p.queryjump;
      x.genomejump = p.genomejump;
      x.dynprogindex = 0;
      x.cdna = ' ';
      x.comp = micro ? p.comp : ' ';  // gappair->comp = gapchar (dynprog.c:6991)
      x.genome = ' ';
      x.flags = (uint8_t)(GSNAPDP_S3_GAPP | ((p.gapp & 2) ? GSNAPDP_S3_KNOWNGAPP : 0));
    } else {  // Pairpool_push (pairpool.c:169-240)
      x.querypos = p.querypos;
      x.genomepos = p.genomepos;
      x.dynprogindex = p.dynprogindex;
      x.cdna = p.cdna;
      x.comp = p.comp;
      x.genome = p.genome;
    }
    A.cp[k0 + (size_t)i] = A.nin + (int)(e0 + (size_t)i);
    A.cnx[k0 + (size_t)i] = i + 1 < n ? (int)(c0 + (size_t)i + 1) : -1;
  }
  return (int)c0;
}

// ---- results, read back exactly as the drop-in reads them
bool done_single(Pass& P, Path& k, int* list) {
  Req& R = k.req;
  const gsnapdp_result& r = R.r;
  if (r.status == ST_UNSUPPORTED) {
    fail(k, "single-gap window outside the reference's domain (the reference aborts)");
    return false;
  }
  if (r.status == ST_OPS_OVERFLOW) {
    fail(k, "op stream overflow");
    return false;
  }
  std::vector<gsnapdp_pair>& v = expand_buf((size_t)R.cap + 8);
  int fs = 0;
  Tic tic(prof().expand_ns[F_GAP]);
  const int n = gsnapdp_expand(P.ctx, &R.w, &r, R.ops, R.q.data(), R.qu.data(), v.data(), (int)v.size(), &fs);
  if (n < 0 || n > (int)v.size()) {
    fail(k, "gsnapdp_expand failed");
    return false;
  }
  k.minor = r.reserved;
  k.finalscore = r.finalscore;
  k.nmatches = r.nmatches;
  k.nmismatches = r.nmismatches;
  k.nopens = r.nopens;
  k.nindels = r.nindels;
  *list = list_of(k.A, v, n, false);
  return true;
}

// Dynprog_genome_gap's out-parameters into the traversal's variables
// (finalscore, nmismatches, left/right probs: the score call's or the re-run's)
bool done_genome(Pass& P, Path& k, int* finalscore, int* nmismatches, double* lp, double* rp, int* list) {
  Req& R = k.req;
  const gsnapdp_ggap_window& w = R.gw;
  const gsnapdp_ggap_result& r = R.gr;
  const gsnapdp_ggap_trace& t = R.gt;
  *list = -1;
  if (t.status == ST_UNSUPPORTED) {
    fail(k, "genome-gap window outside the reference's domain");
    return false;
  }
  if (t.status == ST_OPS_OVERFLOW || t.status == ST_INTERNAL) {
    fail(k, t.status == ST_INTERNAL ? "genome-gap kernel invariant failed" : "op stream overflow");
    return false;
  }
  k.nmatches = *nmismatches = k.nopens = k.nindels = 0;  // :4853-4854
  *lp = *rp = 0.0;
  *finalscore = r.finalscore;
  k.major = r.dynprogindex;
  if (t.status == ST_EARLY) {
    if (w.maxlength1 == -1) {  // too long (:4898-4927)
      k.new_left = r.new_leftgenomepos;
      k.new_right = r.new_rightgenomepos;
      k.newpos_set = true;
      k.exonhead = r.exonhead;
    }
    return true;
  }
  if (r.bridge_ok == 0) {
    k.undefined++;
    return true;
  }
  // *introntype: always NONINTRON in the constrained known-intron mode (:3695),
  // else written only when a score-mode candidate was taken
  if (w.known_mode == GSNAPDP_KNOWN_INTRONS) k.introntype = NONINTRON;
  else if (!w.use_probabilities_p && r.finalscore != (w.halfp ? -50000 : -100000)) k.introntype = r.introntype;
  if (!t.bridge_accepted) return true;
  k.new_left = r.new_leftgenomepos;
  k.new_right = r.new_rightgenomepos;
  k.newpos_set = true;
  k.exonhead = r.exonhead;
  *lp = r.left_prob;
  *rp = r.right_prob;
  k.nmatches = r.nmatches;
  *nmismatches = r.nmismatches;
  k.nopens = r.nopens;
  k.nindels = r.nindels;
  if (r.returned_null) return true;
  std::vector<gsnapdp_pair>& v = expand_buf((size_t)R.cap + 8);
  Tic tic(prof().expand_ns[F_GGAP]);
  const int n = gsnapdp_ggap_expand(P.ctx, &w, &r, &t, R.ops, R.q.data(), R.qu.data(), v.data(), (int)v.size());
  if (n < 0 || n > (int)v.size()) {
    fail(k, "gsnapdp_ggap_expand failed");
    return false;
  }
  *list = list_of(k.A, v, n, false);
  return true;
}

bool done_cdna(Pass& P, Path& k, int* list) {
  Req& R = k.req;
  const gsnapdp_cgap_result& r = R.cr;
  *list = -1;
  if (r.status == ST_UNSUPPORTED) {
    fail(k, "cDNA-gap window outside the reference's domain (the reference aborts)");
    return false;
  }
  if (r.status == ST_OPS_OVERFLOW) {
    fail(k, "op stream overflow");
    return false;
  }
  k.major = r.dynprogindex;
  if (r.finalscore_set) k.finalscore = r.finalscore;
  if (r.status != ST_OK) return true;
  if (r.incompletep) k.incompletep = true;  // only ever set to true (:4756)
  if (r.returned_null) return true;
  std::vector<gsnapdp_pair>& v = expand_buf((size_t)R.cap + 32);
  Tic tic(prof().expand_ns[F_CGAP]);
  const int n = gsnapdp_cgap_expand(P.ctx, &R.cw, &r, R.ops, R.q.data(), R.qu.data(), nullptr, v.data(),
                                    (int)v.size());
  if (n < 0 || n > (int)v.size()) {
    fail(k, "gsnapdp_cgap_expand failed");
    return false;
  }
  *list = list_of(k.A, v, n, false);
  return true;
}

bool done_micro(Pass& P, Path& k, double* prob2, double* prob3, int* microintrontype, int* list) {
  Req& R = k.req;
  const gsnapdp_micro_result& r = R.mr;
  *list = -1;
  if (r.status != 0) {
    fail(k, "microexon window outside the reference's domain");
    return false;
  }
  *prob2 = r.bestprob2;
  *prob3 = r.bestprob3;
  *microintrontype = r.microintrontype;
  k.major = r.dynprogindex;
  if (!r.found) return true;
  const int L1 = R.mw.length1 > 0 ? R.mw.length1 : 0;
  std::vector<gsnapdp_pair>& v = expand_buf((size_t)L1 + 4);
  Tic tic(prof().expand_ns[F_MICRO]);
  const int n = gsnapdp_micro_expand(P.ctx, &R.mw, &r, R.q.data(), R.qu.data(), v.data(), (int)v.size());
  if (n <= 0 || n > (int)v.size()) {
    fail(k, "gsnapdp_micro_expand failed");
    return false;
  }
  *list = list_of(k.A, v, n, true);
  return true;
}

// ---- the traversals, split where they wait for a window

// the dp5 / dp3 start of every traverse_* (stage3.c:5404-5409)
void gap_bounds(Path& k) {
  const gsnapdp_s3_pair& lp = k.A.at(k.left);
  const gsnapdp_s3_pair& rp = k.A.at(k.right);
  k.querydp5 = lp.querypos + 1;
  k.genomedp5 = lp.genomepos + 1;
  if (lp.cdna == ' ') k.querydp5--;
  if (lp.genome == ' ') k.genomedp5--;
  k.querydp3 = rp.querypos - 1;
  k.genomedp3 = rp.genomepos - 1;
}
bool repeel_prior(Path& k) {  // "Re-peeling prior solution" (:5546, :5677)
  const gsnapdp_s3_pair& lp = k.A.at(k.left);
  const gsnapdp_s3_pair& rp = k.A.at(k.right);
  return lp.dynprogindex < 0 && lp.dynprogindex == rp.dynprogindex;
}
void put_back(Path& k) {
  k.pairs = k.A.transfer(k.pairs, k.peeled_pairs);
  k.path = k.A.transfer(k.path, k.peeled_path);
}
void end_gap(Path& k, bool filledp) {  // build_pairs_introns after a traverse_*
  // replace the gap; build_dual_breaks never does (:7196-7224)
  if (!filledp && k.c->pass != GSNAPDP_S3_DUALBREAKS) k.pairs = k.A.push_existing(k.pairs, k.gapcell);
  k.stage = S_SCAN;
}

// traverse_single_gap (:5381-5515): forcep = false, or true in build_dual_breaks.
// Returns true when it waits.
bool single_start(Path& k) {
  const gsnapdp_s3_call& c = *k.c;
  bool mm = false;
  gap_bounds(k);
  k.pairs = peel_rightward(k.A, &mm, &k.peeled_pairs, k.pairs, &k.querydp3, &k.genomedp3, c.maxpeelback, false);
  k.path = peel_leftward(k.A, &mm, &k.peeled_path, k.path, &k.querydp5, &k.genomedp5, c.maxpeelback, false);
  k.queryjump = k.querydp3 - k.querydp5 + 1;
  k.genomejump = k.genomedp3 - k.genomedp5 + 1;
  if (k.queryjump <= 0 || k.genomejump <= 0) {
    put_back(k);
    end_gap(k, false);
    return false;
  }
  req_single(k);
  k.stage = S_SINGLE;
  return true;
}
void single_done(Pass& P, Path& k) {
  const gsnapdp_s3_call& c = *k.c;
  int gappairs = -1;
  if (!done_single(P, k, &gappairs)) return;
  if (c.pass == GSNAPDP_S3_DUALBREAKS) {  // forcep: "Intended for build_dual_breaks" (:5475-5479)
    k.pairs = k.A.transfer(k.pairs, gappairs);
    return end_gap(k, true);
  }
  std::string err;
  int origscore = peeled_score(k.A, k.peeled_pairs, c.cdna_direction, c.defect_rate, &err);
  origscore += peeled_score(k.A, k.peeled_path, c.cdna_direction, c.defect_rate, &err);
  if (!err.empty()) return fail(k, err);
  const gsnapdp_s3_pair& lp = k.A.at(k.left);
  const gsnapdp_s3_pair& rp = k.A.at(k.right);
  const int queryjump = rp.querypos - lp.querypos - 1;
  if (queryjump > 0) origscore += dynprog_score(1, queryjump, 0, 0);
  const int genomejump = (int)((uint32_t)rp.genomepos - (uint32_t)lp.genomepos - 1u);
  if (genomejump > 0) origscore += dynprog_score(0, 0, 1, genomejump);
  if (origscore > k.finalscore) {
    put_back(k);
    end_gap(k, false);
  } else {
    k.pairs = k.A.transfer(k.pairs, gappairs);
    end_gap(k, true);
  }
}

// traverse_cdna_gap (:5518-5627)
bool cdna_start(Path& k) {
  const gsnapdp_s3_call& c = *k.c;
  bool mm = false;
  gap_bounds(k);
  const bool through = !repeel_prior(k);
  k.pairs = peel_rightward(k.A, &mm, &k.peeled_pairs, k.pairs, &k.querydp3, &k.genomedp3, c.maxpeelback, through);
  k.path = peel_leftward(k.A, &mm, &k.peeled_path, k.path, &k.querydp5, &k.genomedp5, c.maxpeelback, through);
  k.queryjump = k.querydp3 - k.querydp5 + 1;
  k.genomejump = k.genomedp3 - k.genomedp5 + 1;
  if (k.queryjump <= k.genomejump + MININTRONLEN) {  // really a single gap
    req_single(k);
    k.stage = S_CDNA_SINGLE;
  } else {  // square matrices
    k.queryjump = k.genomejump + c.extramaterial_paired;
    req_cdna(k);
    k.stage = S_CDNA;
  }
  return true;
}
void cdna_done(Pass& P, Path& k) {
  int gappairs = -1;
  if (k.stage == S_CDNA_SINGLE) {
    if (!done_single(P, k, &gappairs)) return;
    k.pairs = k.A.transfer(k.pairs, gappairs);
    return end_gap(k, true);
  }
  if (!done_cdna(P, k, &gappairs)) return;
  if (gappairs < 0) {
    put_back(k);
    gsnapdp_s3_pair g;
    memset(&g, 0, sizeof(g));
    g.querypos = -1;
    g.genomepos = -1;
    g.queryjump = UNKNOWNJUMP;
    g.genomejump = UNKNOWNJUMP;
    g.src = -1;
    g.cdna = g.comp = g.genome = ' ';
    g.flags = GSNAPDP_S3_GAPP;
    k.pairs = k.A.push_pair(k.pairs, g);
  } else {
    k.pairs = k.A.transfer(k.pairs, gappairs);
  }
  end_gap(k, true);
}

// traverse_genome_gap (:5633-5976), SHORTCUT on (stage3.c:142)
bool genome_start(Pass& P, Path& k) {
  const gsnapdp_s3_call& c = *k.c;
  bool mr = false, ml = false;
  k.newpos_set = false;  // a new traverse_genome_gap frame
  gap_bounds(k);
  const bool through = !repeel_prior(k);
  if (k.querydp5 != k.querydp3 + 1) {
    k.pairs = peel_rightward(k.A, &mr, &k.peeled_pairs, k.pairs, &k.querydp3, &k.genomedp3, c.maxpeelback, through);
    k.path = peel_leftward(k.A, &ml, &k.peeled_path, k.path, &k.querydp5, &k.genomedp5, c.maxpeelback, through);
  } else {
    const int l1 = nt_class(genomic_nt(P, k, k.genomedp5)), l2 = nt_class(genomic_nt(P, k, k.genomedp5 + 1));
    const int r2 = nt_class(genomic_nt(P, k, k.genomedp3 - 1)), r1 = nt_class(genomic_nt(P, k, k.genomedp3));
    k.introntype = gsnapdp::intron_type_codes(l1, l2, r2, r1, c.cdna_direction);
    k.pairs = peel_rightward(k.A, &mr, &k.peeled_pairs, k.pairs, &k.querydp3, &k.genomedp3, c.maxpeelback, through);
    k.path = peel_leftward(k.A, &ml, &k.peeled_path, k.path, &k.querydp5, &k.genomedp5, c.maxpeelback, through);
    if (c.novelsplicingp && !mr && !ml &&
        ((c.cdna_direction > 0 && k.introntype == GTAG_FWD) || (c.cdna_direction < 0 && k.introntype == GTAG_REV))) {
      put_back(k);  // already canonical
      end_gap(k, false);
      return false;
    }
  }
  k.queryjump = k.querydp3 - k.querydp5 + 1;
  k.genomejump = k.genomedp3 - k.genomedp5 + 1;
  if (k.genomejump <= k.queryjump + MININTRONLEN) {  // really a single gap
    req_single(k);
    k.stage = S_GG_SINGLE;
    return true;
  }
  k.genomejump = k.queryjump + c.extramaterial_paired;  // square matrices
  if (!req_genome(P, k, false, 0)) {
    fail(k, "known-site record");
    return false;
  }
  k.stage = S_GG_SCORE;
  return true;
}

void genome_account(Path& k) {
  // traverse_genome_gap's new_left/rightgenomepos are plain locals: when no
  // Dynprog_genome_gap of this traverse_genome_gap call has written them, the
  // reference adds whatever its stack slots hold (a previous call's value, or
  // garbage that differs between runs of the same input); the pass keeps the
  // path's previous values there and reports the counters as undefined
  if (!k.newpos_set) k.ub = true, k.ub_bits |= GSNAPDP_S3_UB_INTRONLEN;
  if (k.introntype == NONINTRON) {
    k.nnonintrons += 1;
    k.nonintronlen += k.new_right - k.new_left - 1;
  } else {
    k.nintrons += 1;
    k.intronlen += k.new_right - k.new_left - 1;
  }
}

// after the score call and the optional probability re-run (:5858-5964)
void genome_decide(Path& k) {
  const gsnapdp_s3_call& c = *k.c;
  const int acceptable = c.defect_rate < DEFECT_HIGHQ ? 2 : (c.defect_rate < DEFECT_MEDQ ? 2 : 3);
  if (k.gappairs < 0) {
    for (int p = k.peeled_pairs; p >= 0; p = k.A.rest(p)) k.A.disallow(p);
    for (int p = k.peeled_path; p >= 0; p = k.A.rest(p)) k.A.disallow(p);
    put_back(k);
    k.introntype = NONINTRON;
    genome_account(k);
    return end_gap(k, false);
  }
  if (!c.finalp && k.finalscore < 0) {
    put_back(k);
    k.introntype = NONINTRON;
    genome_account(k);
    return end_gap(k, false);
  }
  if (k.introntype != NONINTRON && k.nmismatches <= acceptable && k.nopens <= 1 && k.nindels <= 3) {
    k.pairs = k.A.transfer(k.pairs, k.gappairs);
    genome_account(k);
    return end_gap(k, true);
  }
  if (c.cdna_direction == 0) return fail(k, "cdna_direction is 0 in Dynprog_microexon_int");  // :7203
  if (k.genomedp3 - k.genomedp5 <= 0) return fail(k, "Dynprog_microexon_int: span <= 0");      // :7222
  req_micro(k);
  k.stage = S_GG_MICRO;
}

void genome_done(Pass& P, Path& k) {
  const gsnapdp_s3_call& c = *k.c;
  int list = -1;
  if (k.stage == S_GG_SINGLE) {
    if (!done_single(P, k, &list)) return;
    k.pairs = k.A.transfer(k.pairs, list);
    return end_gap(k, true);
  }
  if (k.stage == S_GG_SCORE) {
    if (!done_genome(P, k, &k.finalscore, &k.nmismatches, &k.left_prob, &k.right_prob, &list)) return;
    k.gappairs = list;
    if (list >= 0 && (k.new_left != k.A.at(k.left).genomepos || k.new_right != k.A.at(k.right).genomepos))
      k.shiftp = true;
    if (c.finalp && c.novelsplicingp && (k.left_prob < 0.90 || k.right_prob < 0.90)) {
      if (!req_genome(P, k, true, k.finalscore + QOPEN + 3 * QINDEL)) return fail(k, "known-site record");
      k.stage = S_GG_PROB;
      return;
    }
    return genome_decide(k);
  }
  if (k.stage == S_GG_PROB) {
    int finalscore_alt = 0, nmismatches_alt = 0;
    double lp = 0.0, rp = 0.0;
    if (!done_genome(P, k, &finalscore_alt, &nmismatches_alt, &lp, &rp, &list)) return;
    if (list >= 0 && lp > k.left_prob && rp > k.right_prob) k.gappairs = list;
    return genome_decide(k);
  }
  // S_GG_MICRO
  double prob2 = 0.0, prob3 = 0.0;
  int microintrontype = 0;
  if (!done_micro(P, k, &prob2, &prob3, &microintrontype, &list)) return;
  bool take = false;
  if (list >= 0) {
    if (k.nindels == 0 && k.nmismatches < 4) take = prob2 >= 0.95 && prob3 >= 0.95;  // a higher standard
    else take = prob2 >= 0.90 || prob3 >= 0.90;
  }
  if (take) {
    k.pairs = k.A.transfer(k.pairs, list);
    k.introntype = microintrontype;
    k.shiftp = true;
  } else {
    k.pairs = k.A.transfer(k.pairs, k.gappairs);
  }
  genome_account(k);
  end_gap(k, true);
}

// ---- build_pairs_end5 (:7351-7450) / build_path_end3 (:7236-7347) with
// extendp: extend_ending5 / extend_ending3 (:6587-6719 / :6906-7041) without
// splice sites.  The list is `pairs` (END5) or `path` (END3); the peeled
// stretch is dropped whatever the window returns, as the reference drops it.
void end_start(Path& k) {
  const gsnapdp_s3_call& c = *k.c;
  const bool end5 = c.pass == GSNAPDP_S3_END5;
  const bool peel = c.endalign != GSNAPDP_QUERYEND_NOGAPS && c.maxpeelback != 0;
  bool mm = false;
  k.stage = S_DONE;
  if (end5) {
    if (k.pairs < 0) return;  // NULL in, NULL out
    const gsnapdp_s3_pair& rp = k.A.first(k.pairs);
    if (rp.querypos < 0) {  // :7386-7390: the whole list is dropped
      k.pairs = -1;
      return;
    }
    const int leftquerypos = rp.querypos > c.nullgap ? rp.querypos - c.nullgap - 1 : -1;
    k.querydp5 = leftquerypos + 1;
    k.querydp3 = rp.querypos - 1;
    k.genomedp3 = rp.genomepos - 1;
    if (peel)
      k.pairs = peel_rightward(k.A, &mm, &k.peeled_pairs, k.pairs, &k.querydp3, &k.genomedp3, c.maxpeelback, true);
    k.queryjump = k.querydp3 - k.querydp5 + 1;
    k.genomejump = k.queryjump + c.extramaterial_end;
    k.genomedp5 = k.genomedp3 - k.genomejump + 1;
  } else {
    if (k.path < 0) return;
    const gsnapdp_s3_pair& lp = k.A.first(k.path);
    if (lp.querypos < 0) {  // :7270-7274
      k.path = -1;
      return;
    }
    int queryjump = c.querylength - lp.querypos - 1;
    if (lp.cdna == ' ') queryjump++;
    const int rightquerypos = queryjump + 1 > c.nullgap ? lp.querypos + c.nullgap + 1 : c.querylength;
    k.querydp5 = lp.cdna == ' ' ? lp.querypos : lp.querypos + 1;
    k.genomedp5 = lp.genome == ' ' ? lp.genomepos : lp.genomepos + 1;
    k.querydp3 = rightquerypos - 1;
    k.genomedp3 = c.genomiclength - 1;
    if (peel)
      k.path = peel_leftward(k.A, &mm, &k.peeled_path, k.path, &k.querydp5, &k.genomedp5, c.maxpeelback, true);
    k.queryjump = k.querydp3 - k.querydp5 + 1;
    k.genomejump = k.queryjump + c.extramaterial_end;
    k.genomedp3 = k.genomedp5 + k.genomejump - 1;
  }
  req_end(k, end5);
  k.stage = S_END;
}
void end_done(Pass& P, Path& k) {
  const bool end5 = k.c->pass == GSNAPDP_S3_END5;
  int list = -1;
  if (!done_single(P, k, &list)) return;
  if (!end5) list = k.A.reverse(list);
  // an indel between the extension and the rest of the read (:6707, :7029)
  if (list >= 0 && k.A.first(list).querypos != (end5 ? k.querydp3 : k.querydp5)) list = -1;
  if (end5) k.pairs = k.A.transfer(k.pairs, list);
  else k.path = k.A.transfer(k.path, list);
  k.stage = S_DONE;
}

// ---- traverse_dual_genome_gap (:5980-6364): one intron or two around a short
// exon.  Its windows run one per round, in the reference's order (the
// dynprogindex each takes is the reference's).
int dual_goodness(const Path& k, int nmismatches) {
  return k.nmatches + MISMATCH * nmismatches + QOPEN * k.nopens + QINDEL * k.nindels;
}
// a Dynprog_genome_gap of the traversal over [q5, q3] x [g5, g3], square
// (genomejump = queryjump + extramaterial_paired), score mode, not final
bool dual_window(Pass& P, Path& k, int q5, int g5, int q3, int g3, bool halfp, int stage) {
  const gsnapdp_s3_call& c = *k.c;
  k.querydp5 = q5;
  k.genomedp5 = g5;
  k.querydp3 = q3;
  k.genomedp3 = g3;
  k.queryjump = q3 - q5 + 1;
  k.genomejump = k.queryjump + c.extramaterial_paired;
  if (!req_genome(P, k, false, 0, halfp, 0)) {
    fail(k, "known-site record");
    return false;
  }
  k.stage = stage;
  return true;
}
// whether [q5, q3] fits the genome stretch: the "bounds don't make sense"
// tests of the half windows (:6128, :6166, :6279, :6325)
bool dual_fits(const Path& k, int q5, int g5, int q3, int g3) {
  return g5 + (q3 - q5 + 1 + k.c->extramaterial_paired) - 1 < g3;
}
void dual_unknown_gap(Path& k) {  // put back, Pairpool_push_gapholder(UNKNOWNJUMP) (:6066-6072)
  put_back(k);
  gsnapdp_s3_pair g;
  memset(&g, 0, sizeof(g));
  g.querypos = -1;
  g.genomepos = -1;
  g.queryjump = UNKNOWNJUMP;
  g.genomejump = UNKNOWNJUMP;
  g.src = -1;
  g.cdna = g.comp = g.genome = ' ';
  g.flags = GSNAPDP_S3_GAPP;
  k.pairs = k.A.push_pair(k.pairs, g);
  k.stage = S_SCAN;
}
bool dual_start(Pass& P, Path& k) {
  const gsnapdp_s3_call& c = *k.c;
  bool mr = false, ml = false;
  gap_bounds(k);
  k.pairs = peel_rightward(k.A, &mr, &k.peeled_pairs, k.pairs, &k.querydp3, &k.genomedp3, c.maxpeelback, true);
  k.path = peel_leftward(k.A, &ml, &k.peeled_path, k.path, &k.querydp5, &k.genomedp5, c.maxpeelback, true);
  Path::Dual& d = k.d;
  d.q5 = k.querydp5, d.g5 = k.genomedp5, d.q3 = k.querydp3, d.g3 = k.genomedp3;
  const int queryjump = d.q3 - d.q5 + 1, genomejump = queryjump + c.extramaterial_paired;
  if (queryjump > c.nullgap || d.g5 + genomejump - 1 >= d.g3 - genomejump + 1) {
    dual_unknown_gap(k);
    return false;
  }
  d.single = d.dual2 = d.dual1 = -1;
  return dual_window(P, k, d.q5, d.g5, d.q3, d.g3, false, S_DUAL_SINGLE);
}
// the single result (or a better one-intron alternative) wins (:6264-6360)
void dual_single_wins(Pass& P, Path& k, int from) {
  Path::Dual& d = k.d;
  if (from < S_DUAL_RIGHT && d.right_end && dual_fits(k, d.q5, d.g5, d.midq, d.midg)) {
    dual_window(P, k, d.q5, d.g5, d.midq, d.midg, false, S_DUAL_RIGHT);
    return;
  }
  if (from < S_DUAL_LEFT && d.left_end && dual_fits(k, d.midq, d.midg, d.q3, d.g3)) {
    dual_window(P, k, d.midq, d.midg, d.q3, d.g3, false, S_DUAL_LEFT);
    return;
  }
  k.pairs = k.A.transfer(k.pairs, d.single);
  k.stage = S_SCAN;
}
void dual_decide(Pass& P, Path& k) {  // :6195-6262
  const gsnapdp_s3_call& c = *k.c;
  Path::Dual& d = k.d;
  if (d.dual2 < 0 || d.dual1 < 0) return dual_single_wins(P, k, S_DUAL_1);
  const int canonical = c.cdna_direction > 0 ? GTAG_FWD : GTAG_REV;
  const bool dual_canonical = d.introntype1 == canonical && d.introntype2 == canonical;
  int middle_exonlength = d.right_exonhead - d.left_exonhead;
  double middle_exonprob;
  if (middle_exonlength <= 0) {
    middle_exonprob = 0.0;
  } else {
    const int interexon_region = k.new_right - k.new_left;
    if (d.introntype2 == canonical) middle_exonlength += DUAL_HALFCANONICAL_POINTS;
    if (d.introntype1 == canonical) middle_exonlength += DUAL_HALFCANONICAL_POINTS;
    middle_exonprob = 1.0 - pow(1.0 - pow(4.0, -(double)middle_exonlength), (double)interexon_region);
  }
  if (dual_canonical && middle_exonprob < 0.001 && d.single_goodness > d.dual_goodness && !d.single_typed)
    k.ub = true, k.ub_bits |= GSNAPDP_S3_UB_DUAL;  // single_canonical_p read an uninitialised introntype
  const bool single_canonical = d.single_typed && d.single_introntype == canonical;
  if (dual_canonical && middle_exonprob < 0.001 && (!single_canonical || d.single_goodness <= d.dual_goodness)) {
    k.pairs = k.A.transfer(k.pairs, d.dual2);
    k.pairs = k.A.transfer(k.pairs, d.dual1);
    k.stage = S_SCAN;
    return;
  }
  dual_single_wins(P, k, S_DUAL_1);
}
void dual_done(Pass& P, Path& k) {
  Path::Dual& d = k.d;
  int fs = 0, nmm = 0, list = -1;
  double lp = 0.0, rp = 0.0;
  const int stage = k.stage;
  const int before = k.introntype;
  k.introntype = INT32_MIN;  // written or not, by this window
  if (!done_genome(P, k, &fs, &nmm, &lp, &rp, &list)) return;
  const bool typed = k.introntype != INT32_MIN;
  const int introntype = k.introntype;
  k.introntype = before;
  switch (stage) {
    case S_DUAL_SINGLE:
      d.single = list;
      d.single_goodness = k.nopens <= 1 ? (k.nmatches + k.nindels) + MISMATCH * nmm
                                        : k.nmatches + MISMATCH * nmm + QOPEN * (k.nopens - 1) + QINDEL * k.nindels;
      d.single_typed = typed;
      d.single_introntype = introntype;
      if (!dual_fits(k, d.midq, d.midg, d.q3, d.g3)) return dual_single_wins(P, k, S_DUAL_1);
      dual_window(P, k, d.midq, d.midg, d.q3, d.g3, true, S_DUAL_2);
      return;
    case S_DUAL_2:
      d.dual2 = list;
      d.dual_goodness = dual_goodness(k, nmm);
      d.right_exonhead = k.exonhead;
      d.introntype2 = typed ? introntype : INT32_MIN;
      if (!dual_fits(k, d.q5, d.g5, d.midq - 1, d.midg - 1)) return dual_single_wins(P, k, S_DUAL_1);
      dual_window(P, k, d.q5, d.g5, d.midq - 1, d.midg - 1, true, S_DUAL_1);
      return;
    case S_DUAL_1:
      d.dual1 = list;
      d.dual_goodness += dual_goodness(k, nmm);
      d.left_exonhead = k.exonhead;
      d.introntype1 = typed ? introntype : INT32_MIN;
      return dual_decide(P, k);
    default: {  // S_DUAL_RIGHT / S_DUAL_LEFT
      const int goodness = dual_goodness(k, nmm);
      if (goodness > d.single_goodness) {
        d.single = list;
        d.single_goodness = goodness;
      }
      return dual_single_wins(P, k, stage);
    }
  }
}

// build_pairs_dualintrons past a gap it may take (:7645-7726): cross the short
// exon after it and run traverse_dual_genome_gap.  Returns true when it waits.
bool dual_gap(Pass& P, Path& k, int gapcell, int gap) {
  Arena& A = k.A;
  Path::Dual& d = k.d;
  d.right_end = (A.flag(gap) & GSNAPDP_S3_END_INTRON) != 0;
  const int midrightpair = A.pairof(k.path);
  // List_transfer_one: the cell moves to midexon_pairs, whose first tail is
  // the local's uninitialised value (see below)
  auto transfer_one = [&]() {
    const int cell = k.path;
    k.path = A.rest(cell);
    A.set_next(cell, k.midexon);
    k.midexon = cell;
  };
  transfer_one();
  bool exonp = true;
  while (k.path >= 0 && exonp) {
    const int mp = A.pairof(k.path);
    if (A.flag(mp) & GSNAPDP_S3_GAPP) {
      d.left_end = (A.flag(mp) & GSNAPDP_S3_END_INTRON) != 0;
      exonp = false;
      k.path = A.rest(k.path);
    } else {
      transfer_one();
    }
  }
  if (k.path < 0) {
    // "Short exon is the first one": Pairpool_push_existing (a new cell) and
    // List_reverse(midexon_pairs), whose last cell links to the value
    // midexon_pairs held before the first short exon of the call: garbage in
    // the reference, taken as NULL here and reported
    k.ub = true, k.ub_bits |= GSNAPDP_S3_UB_DUAL;
    k.pairs = A.cell(gap, k.pairs);
    k.pairs = A.transfer(k.pairs, A.reverse(k.midexon));
    k.midexon = -1;
    return false;
  }
  (void)gapcell;
  const gsnapdp_s3_pair& ml = A.first(k.midexon);
  const gsnapdp_s3_pair& mr = A.at(midrightpair);
  const uint32_t midgenomepos = ((uint32_t)ml.genomepos + (uint32_t)mr.genomepos) / 2u;  // Genomicpos_T
  d.midg = (int)midgenomepos;
  d.midq = mr.querypos - (int)((uint32_t)mr.genomepos - midgenomepos);
  if (k.pairs < 0) {
    fail(k, "dual intron at the end of the path (the reference dereferences NULL)");
    return false;
  }
  k.left = A.pairof(k.path);
  k.right = A.pairof(k.pairs);
  if (d.midq <= A.at(k.left).querypos || d.midq >= A.at(k.right).querypos) return false;  // skip
  k.peeled_pairs = k.peeled_path = -1;
  return dual_start(P, k);
}

// traverse_dual_break (:7044-7142): peel one pair each side, ask the caller's
// stage 2 for the stretch, keep its list if it bridges the whole stretch,
// otherwise put the peels back under an unknown gap
void dual_break(Pass& P, Path& k) {
  const gsnapdp_s3_call& c = *k.c;
  const gsnapdp_s3_stage2 s2 = gsnapdp::s3_stage2(P.ctx);
  if (!s2.compute_one) return fail(k, "a dual break needs stage 2 (Stage2_compute_one) and no stage-2 callback is set");
  bool mm = false;
  gap_bounds(k);
  k.pairs = peel_rightward(k.A, &mm, &k.peeled_pairs, k.pairs, &k.querydp3, &k.genomedp3, 1, true);
  k.path = peel_leftward(k.A, &mm, &k.peeled_path, k.path, &k.querydp5, &k.genomedp5, 1, true);
  const uint32_t genomicstart = c.chroffset + c.chrpos, genomicend = genomicstart + (uint32_t)c.genomiclength;
  const uint32_t mappingstart = c.watsonp ? genomicstart + (uint32_t)k.genomedp5 : genomicend - (uint32_t)k.genomedp3;
  const uint32_t mappingend = c.watsonp ? genomicstart + (uint32_t)k.genomedp3 : genomicend - (uint32_t)k.genomedp5;
  thread_local std::vector<gsnapdp_s3_pair> v;
  int cap = 2 * ((k.querydp3 - k.querydp5 + 1) + (k.genomedp3 - k.genomedp5 + 1)) + 64, n;
  for (;;) {
    if (cap < 64) cap = 64;
    v.resize((size_t)cap);
    n = s2.compute_one(s2.user, &c, k.querydp5, k.querydp3, k.genomedp5, k.genomedp3, mappingstart, mappingend,
                       v.data(), cap);
    if (n <= cap) break;
    cap = n;
  }
  if (n < 0) return fail(k, "the stage-2 callback failed");
  int list = -1;
  for (int i = n - 1; i >= 0; i--) {  // the caller's list, head first
    gsnapdp_s3_pair x = v[(size_t)i];
    x.src = -1;
    list = k.A.push_pair(list, x);
  }
  // lastpair = gappairs->first, firstpair = its last cell (:7121-7122)
  if (n > 0 && v[(size_t)n - 1].querypos == k.querydp5 && v[0].querypos == k.querydp3) {
    k.pairs = k.A.transfer(k.pairs, list);
  } else {
    dual_unknown_gap(k);
  }
  k.stage = S_SCAN;
}

// build_pairs_introns' loop (:7763-7898) until the path waits or ends
void scan(Pass& P, Path& k) {
  const gsnapdp_s3_call& c = *k.c;
  const int minintronlen = c.finalp ? MININTRONLEN_FINAL : MININTRONLEN;
  while (!k.failed && k.stage == S_SCAN) {
    // the non-gap input cells at the head of the path, each pushed onto pairs
    // (Pairpool_pop + List_push_existing, the loop below), a run at a time
    if (k.path >= 0 && k.path < k.A.nin) k.A.move_run(&k.path, &k.pairs);
    if (k.path < 0) {
      k.stage = S_DONE;
      return;
    }
    int pair = -1;
    const int ptr = k.path;
    k.path = k.A.pop(k.path, &pair);
    if (!(k.A.flag(pair) & GSNAPDP_S3_GAPP)) {  // not a gap: keep it
      k.pairs = k.A.push_existing(k.pairs, ptr);
      continue;
    }
    const gsnapdp_s3_pair& g = k.A.at(pair);
    if (c.pass == GSNAPDP_S3_DUALBREAKS) {  // build_dual_breaks (:7168-7226)
      if (g.comp != '#') {  // not DUALBREAK_COMP
        k.pairs = k.A.push_existing(k.pairs, ptr);
        continue;
      }
      // a dual break at an end of the alignment: the gap is dropped (:7179-7187)
      if (k.path < 0 || k.pairs < 0) continue;
      k.left = k.A.pairof(k.path);
      k.right = k.A.pairof(k.pairs);
      if (k.A.at(k.left).querypos < 0 || k.A.at(k.right).querypos < 0) continue;
      k.gapcell = ptr;
      k.peeled_pairs = k.peeled_path = -1;
      if (g.queryjump != 1 && g.genomejump != 1 && g.genomejump - g.queryjump < SINGLESLEN &&
          g.queryjump - g.genomejump < SINGLESLEN) {
        if (single_start(k)) return;  // solved as a single gap, forcep
        continue;
      }
      k.shiftp = true;  // *dual_break_p
      dual_break(P, k);
      continue;
    }
    if (c.pass == GSNAPDP_S3_DUALINTRONS) {  // build_pairs_dualintrons (:7613-7730)
      if (g.queryjump > c.nullgap || g.queryjump > g.genomejump + EXTRAQUERYGAP ||
          g.genomejump <= g.queryjump + MININTRONLEN) {
        k.pairs = k.A.push_existing(k.pairs, ptr);
        continue;
      }
      if (k.path < 0) return fail(k, "dual-intron gap at the end of the path (the reference dereferences NULL)");
      if (!(k.A.flag(k.A.pairof(k.path)) & GSNAPDP_S3_SHORTEXON)) {  // a long exon
        k.pairs = k.A.push_existing(k.pairs, ptr);
        continue;
      }
      if (dual_gap(P, k, ptr, pair)) return;
      continue;
    }
    int kind;  // 0 keep it, 1 cDNA gap, 2 genome gap, 3 single gap
    if (c.pass == GSNAPDP_S3_SINGLES) {  // build_pairs_singles (stage3.c:7469-7583)
      kind = (g.queryjump > c.nullgap || g.queryjump > g.genomejump + EXTRAQUERYGAP ||
              g.genomejump > g.queryjump + SINGLESLEN) ? 0 : 3;
    } else if (g.queryjump > c.nullgap) kind = 0;  // a large gap
    else if (g.queryjump > g.genomejump + EXTRAQUERYGAP) kind = 1;
    else if (g.genomejump > g.queryjump + minintronlen) kind = 2;
    else if (g.genomejump > g.queryjump + SINGLESLEN) kind = 0;  // a short intron
    else kind = 3;
    if (kind == 0) {
      k.pairs = k.A.push_existing(k.pairs, ptr);
      continue;
    }
    if (k.path < 0 || k.pairs < 0)  // build_pairs_introns dereferences NULL; build_pairs_singles aborts (:7543)
      return fail(k, "gap at the end of the path (the reference dereferences NULL or aborts)");
    k.gapcell = ptr;
    k.left = k.A.pairof(k.path);    // leftpair = path->first
    k.right = k.A.pairof(k.pairs);  // rightpair = pairs->first
    k.peeled_pairs = k.peeled_path = -1;
    const bool waits = kind == 1 ? cdna_start(k) : (kind == 2 ? genome_start(P, k) : single_start(k));
    if (waits) return;
  }
}

void resume(Pass& P, Path& k) {
  switch (k.stage) {
    case S_SINGLE: single_done(P, k); break;
    case S_CDNA_SINGLE:
    case S_CDNA: cdna_done(P, k); break;
    case S_GG_SINGLE:
    case S_GG_SCORE:
    case S_GG_PROB:
    case S_GG_MICRO: genome_done(P, k); break;
    case S_END: end_done(P, k); break;
    case S_DUAL_SINGLE:
    case S_DUAL_2:
    case S_DUAL_1:
    case S_DUAL_RIGHT:
    case S_DUAL_LEFT: dual_done(P, k); break;
    default: break;
  }
  if (k.stage == S_SCAN) scan(P, k);
}


// a path at the start of its pass: call c over the list pairs[0 .. npairs)
// (gaps: its gap pairs, ascending, or nullptr to find them from the flags)
void start_path(Pass& P, Path& k, gsnapdp_s3_call* cp, const gsnapdp_s3_pair* pairs, int npairs,
                const int32_t* gaps = nullptr, int ngaps = 0) {
  reset(k);
  gsnapdp_s3_call& c = *cp;
  k.c = cp;
  k.q = P.query + c.qpos;
  k.qu = P.query_uc + c.qpos;
  k.minor = c.in_minor;
  k.major = c.in_major;
  k.nintrons = c.in_nintrons;
  k.nnonintrons = c.in_nnonintrons;
  k.intronlen = c.in_intronlen;
  k.nonintronlen = c.in_nonintronlen;
  k.A.init(pairs, npairs, gaps, ngaps);  // path->first is pairs[0] (cell 0)
  const int list = npairs > 0 ? 0 : -1;
  if (c.use_genomicseg_p) {
    fail(k, "use_genomicseg_p passes are not served (the genome is the context's)");
  } else if (c.pass == GSNAPDP_S3_END5 || c.pass == GSNAPDP_S3_END3) {
    if (c.splicesitesp && c.endalign == GSNAPDP_QUERYEND_GAP)
      fail(k, "an end extension with splice sites (Dynprog_end5/3_known) is not served");
    else if (c.pass == GSNAPDP_S3_END5) k.pairs = list, end_start(k);
    else k.path = list, end_start(k);
  } else {
    k.path = list;
    scan(P, k);
  }
}

// a finished path's counters into its call record
void write_call(const Path& k, gsnapdp_s3_call& c) {
  c.status = k.failed ? -1 : 0;
  c.out_minor = k.minor;
  c.out_major = k.major;
  c.out_nintrons = k.nintrons;
  c.out_nnonintrons = k.nnonintrons;
  c.out_intronlen = k.intronlen;
  c.out_nonintronlen = k.nonintronlen;
  c.shiftp = k.shiftp ? 1 : 0;
  c.incompletep = k.incompletep ? 1 : 0;
  c.ub = k.ub_bits;
}

// driven passes: when a path's pass ends, its list goes to the driver, which
// names the path's next pass (started at once, in this round) or ends it
void finish_path(Pass& P, Path& k) {
  thread_local std::vector<gsnapdp_s3_pair> list;
  while (k.stage == S_DONE || k.failed) {
    list.clear();
    if (!k.failed) {
      if (k.c->pass == GSNAPDP_S3_END3) k.pairs = k.path;  // build_path_end3 returns its path
      const Arena& A = k.A;
      list.reserve((size_t)A.nin + A.extra.size());  // every cell at most once
      // a reversed block copy of each input run; src stays the input pair's own
      // (the driver's numbering, not the pass's position)
      walk_list(
          A, k.pairs,
          [&](int hi, int lo, bool d) {
            list.insert(list.end(), std::make_reverse_iterator(A.in + hi + 1), std::make_reverse_iterator(A.in + lo));
            if (d) list.back().flags |= GSNAPDP_S3_DISALLOWED;  // (a disallowed pair is a run of its own)
          },
          [&](int e) { list.push_back(A.extra[(size_t)e].p); });
    }
    write_call(k, *k.c);
    const gsnapdp_s3_pair* pairs = nullptr;
    int n = 0;
    gsnapdp_s3_call* next;
    {
      Tic tic(prof().driver_ns);
      next = P.driver->next(k.idx, k.c, list, &pairs, &n);
    }
    if (!next) {
      k.stage = S_DONE;
      k.failed = false;  // reported through the call; the path is out of the pass
      k.c = nullptr;
      return;
    }
    start_path(P, k, next, pairs, n);
  }
}

// ---- host threads: one persistent pool per process.  A round's host work is
// a few hundred microseconds, so the workers spin briefly for the next job
// before they sleep, and nothing is spawned per round.
int pass_threads() {
  if (const char* e = getenv("GSNAPDP_S3_THREADS")) return std::max(1, atoi(e));
  const int hw = (int)std::thread::hardware_concurrency();
  return std::max(1, std::min(16, hw));  // a GPU box's CPU share is 16 (nproc shows the whole machine)
}

class Workers {
 public:
  static Workers& get() {
    static Workers* w = new Workers(pass_threads());  // never joined: the workers outlive every pass
    return *w;
  }
  // fn(i) for every i in [0, n), `grain` indices at a time, on the pool and the caller
  void run(int n, int grain, const std::function<void(int)>& fn) {
    if (n <= 0) return;
    if (nthreads_ <= 1 || n <= grain) {
      for (int i = 0; i < n; i++) fn(i);
      return;
    }
    std::lock_guard<std::mutex> one(run_m_);  // concurrent passes take turns
    {
      std::lock_guard<std::mutex> l(m_);
      fn_ = &fn;
      n_ = n;
      grain_ = grain;
      next_.store(0);
      active_.store(nthreads_ - 1);
      gen_.fetch_add(1, std::memory_order_release);
    }
    cv_.notify_all();
    work();
    // the workers are spinning or waking; a run is a few hundred microseconds,
    // so the caller spins for them too rather than sleeping on a condition
    while (active_.load(std::memory_order_acquire) != 0) __builtin_ia32_pause();
    fn_ = nullptr;
  }

 private:
  explicit Workers(int n) : nthreads_(n) {
    for (int t = 1; t < n; t++) std::thread([this] { loop(); }).detach();
  }
  void work() {
    for (int i; (i = next_.fetch_add(grain_)) < n_;)
      for (int j = i; j < std::min(n_, i + grain_); j++) (*fn_)(j);
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      const auto t0 = std::chrono::steady_clock::now();
      while (gen_.load(std::memory_order_acquire) == seen) {
        __builtin_ia32_pause();
        if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(200)) {
          std::unique_lock<std::mutex> l(m_);
          cv_.wait(l, [&] { return gen_.load() != seen; });
          break;
        }
      }
      seen = gen_.load(std::memory_order_acquire);
      work();
      active_.fetch_sub(1, std::memory_order_acq_rel);
    }
  }
  const int nthreads_;
  std::mutex m_, run_m_;
  std::condition_variable cv_;
  const std::function<void(int)>* fn_ = nullptr;
  std::atomic<int> next_{0}, active_{0};
  std::atomic<uint64_t> gen_{0};
  int n_ = 0, grain_ = 1;
};

// ---- a cohort of paths and its round in flight
constexpr size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

struct Cohort {
  std::vector<Path*> paths;     // the paths that may still wait: a path waits in a round only if
                                // it was resumed in the previous one, so after each round this
                                // is that round's `all`
  std::vector<Path*> fam[F_N];  // the round's waiting paths, in batch order
  std::vector<Path*> all;       // the same, concatenated
  std::vector<size_t> qoff;     // each waiting path's query bytes in the packed round (all's order)
  gsnapdp::S3Layout L;
  int slot = 0;
  bool inflight = false;
};

// Packs the cohort's waiting windows into its slot's input staging and
// submits them.  Returns 1 when a round was submitted, 0 when no path waits,
// -1 on an error.
int pack_submit(Pass& P, gsnapdp::S3Exec& X, Cohort& C) {
  using clock = std::chrono::steady_clock;
  const auto t0 = clock::now();
  size_t nwait = 0;
  for (int f = 0; f < F_N; f++) C.fam[f].clear();
  for (Path* k : C.paths)
    if (!k->failed && k->stage != S_DONE && k->req.fam != F_NONE) C.fam[k->req.fam].push_back(k), nwait++;
  C.paths.clear();
  if (!nwait) return 0;
  for (int f = 0; f < F_N; f++) std::sort(C.fam[f].begin(), C.fam[f].end());  // batches in path order
  gsnapdp::S3Layout& L = C.L;
  L = gsnapdp::S3Layout();
  C.all.clear();
  C.qoff.clear();
  size_t q = 0;
  int64_t ncap[F_N] = {0, 0, 0, 0};
  for (int f = 0; f < F_N; f++) {
    L.n[f] = (int)C.fam[f].size();
    for (Path* k : C.fam[f]) {
      C.all.push_back(k);
      C.qoff.push_back(q);
      q += (k->req.q.size() + 3) & ~(size_t)3;
      ncap[f] += k->req.cap;
    }
  }
  L.q = 0;
  L.qbytes = q + 8;
  L.qu = al256(L.qbytes);
  size_t at = L.qu + al256(L.qbytes);
  const size_t wsz[F_N] = {sizeof(gsnapdp_window), sizeof(gsnapdp_ggap_window), sizeof(gsnapdp_cgap_window),
                           sizeof(gsnapdp_micro_window)};
  const size_t rsz[F_N] = {sizeof(gsnapdp_result), sizeof(gsnapdp_ggap_result), sizeof(gsnapdp_cgap_result),
                           sizeof(gsnapdp_micro_result)};
  for (int f = 0; f < F_N; f++) {
    L.w[f] = at;
    at += al256((size_t)L.n[f] * wsz[f]);
    if (f != F_MICRO) {
      L.off[f] = at;
      at += al256((size_t)(L.n[f] + 1) * 8);
    }
  }
  L.in_bytes = at;
  at = 0;
  for (int f = 0; f < F_N; f++) {
    L.r[f] = at;
    at += al256((size_t)L.n[f] * rsz[f]);
    if (f == F_GGAP) {
      L.t = at;
      at += al256((size_t)L.n[f] * sizeof(gsnapdp_ggap_trace));
    }
    if (f != F_MICRO) {
      L.ops[f] = at;
      at += al256((size_t)ncap[f] * 4 + 4);
    }
  }
  L.out_bytes = at;
  char* in = X.in_buf(C.slot, L.in_bytes);
  if (!in || !X.out_buf(C.slot, L.out_bytes)) return -1;
  for (int f = 0; f < F_N; f++) {  // op offsets: each family's capacity layout
    if (f == F_MICRO) continue;
    int64_t* off = (int64_t*)(in + L.off[f]);
    off[0] = 0;
    for (int i = 0; i < L.n[f]; i++) off[i + 1] = off[i] + C.fam[f][(size_t)i]->req.cap;
  }
  memset(in + L.q + q, 0, 8);
  memset(in + L.qu + q, 0, 8);
  int base[F_N + 1] = {0};
  for (int f = 0; f < F_N; f++) base[f + 1] = base[f] + L.n[f];
  const auto t1 = clock::now();
  Workers::get().run((int)C.all.size(), 64, [&](int j) {
    Path& k = *C.all[(size_t)j];
    const Req& R = k.req;
    const size_t qo = C.qoff[(size_t)j];
    const size_t qn = R.q.size();
    memcpy(in + L.q + qo, R.q.data(), qn);
    memcpy(in + L.qu + qo, R.qu.data(), qn);
    const size_t pad = ((qn + 3) & ~(size_t)3) - qn;
    if (pad) memset(in + L.q + qo + qn, 0, pad), memset(in + L.qu + qo + qn, 0, pad);
    const int f = R.fam, i = j - base[f];
    const uint32_t o = (uint32_t)qo;
    if (f == F_GAP) {
      gsnapdp_window w = R.w;
      w.qpos += o;
      memcpy(in + L.w[f] + (size_t)i * sizeof(w), &w, sizeof(w));
    } else if (f == F_GGAP) {
      gsnapdp_ggap_window w = R.gw;
      w.qpos += o;
      memcpy(in + L.w[f] + (size_t)i * sizeof(w), &w, sizeof(w));
    } else if (f == F_CGAP) {
      gsnapdp_cgap_window w = R.cw;
      w.qposL += o;
      w.qposR += o;
      memcpy(in + L.w[f] + (size_t)i * sizeof(w), &w, sizeof(w));
    } else {
      gsnapdp_micro_window w = R.mw;
      w.qpos += o;
      w.ppos += o;
      memcpy(in + L.w[f] + (size_t)i * sizeof(w), &w, sizeof(w));
    }
  });
  const auto t2 = clock::now();
  if (X.submit(C.slot, L)) return -1;
  if (prof().on) {
    const auto t3 = clock::now();
    prof().pack += std::chrono::duration<double>(t1 - t0).count();
    prof().copy += std::chrono::duration<double>(t2 - t1).count();
    prof().submit += std::chrono::duration<double>(t3 - t2).count();
  }
  for (int f = 0; f < F_N; f++)
    if (L.n[f]) {
      P.st.windows[f] += L.n[f];
      P.st.batches[f]++;
    }
  P.st.rounds++;
  return 1;
}

// Hands the round's results to its paths and resumes them (the slot's staging
// stays untouched until the cohort packs its next round).
void unpack_resume(Pass& P, gsnapdp::S3Exec& X, Cohort& C) {
  const gsnapdp::S3Layout& L = C.L;
  const char* in = X.in_buf(C.slot, 0);
  const char* out = X.out_buf(C.slot, 0);
  int base[F_N + 1] = {0};
  for (int f = 0; f < F_N; f++) base[f + 1] = base[f] + L.n[f];
  // small grains when driven: a path's resume can then run a whole host step of its query
  Workers::get().run((int)C.all.size(), P.driver ? 4 : 16, [&](int j) {
    Path& k = *C.all[(size_t)j];
    Req& R = k.req;
    const int f = R.fam, i = j - base[f];
    const int64_t* off = f == F_MICRO ? nullptr : (const int64_t*)(in + L.off[f]);
    if (f == F_GAP) {
      memcpy(&R.r, out + L.r[f] + (size_t)i * sizeof(R.r), sizeof(R.r));
    } else if (f == F_GGAP) {
      memcpy(&R.gr, out + L.r[f] + (size_t)i * sizeof(R.gr), sizeof(R.gr));
      memcpy(&R.gt, out + L.t + (size_t)i * sizeof(R.gt), sizeof(R.gt));
    } else if (f == F_CGAP) {
      memcpy(&R.cr, out + L.r[f] + (size_t)i * sizeof(R.cr), sizeof(R.cr));
    } else {
      memcpy(&R.mr, out + L.r[f] + (size_t)i * sizeof(R.mr), sizeof(R.mr));
    }
    R.ops = off ? (const uint32_t*)(out + L.ops[f]) + off[i] : nullptr;
    R.fam = F_NONE;
    Tic tic(prof().resume_ns);
    resume(P, k);
    if (P.driver && (k.stage == S_DONE || k.failed)) finish_path(P, k);
  });
  C.paths.swap(C.all);  // the candidates for the next round
}

bool call_in_range(const gsnapdp_s3_call& c, int64_t npairs_in, size_t query_bytes) {
  return c.pass >= GSNAPDP_S3_INTRONS && c.pass <= GSNAPDP_S3_DUALBREAKS && c.first_pair >= 0 && c.npairs >= 0 && (int64_t)c.first_pair + c.npairs <= npairs_in && c.qpos >= 0 &&
         c.querylength >= 0 && (uint64_t)c.qpos + (uint64_t)c.querylength <= (uint64_t)query_bytes;
}

}  // namespace

void gsnapdp::s3_parallel_for(int n, int grain, const std::function<void(int)>& fn) { Workers::get().run(n, grain, fn); }

extern "C" int gsnapdp_stage3_set_stage2(gsnapdp_ctx* ctx, const gsnapdp_s3_stage2* stage2) {
  if (!ctx) {
    gsnapdp__set_err("gsnapdp_stage3_set_stage2: no context");
    return -1;
  }
  gsnapdp::s3_set_stage2(ctx, stage2 ? *stage2 : gsnapdp_s3_stage2{nullptr, nullptr});
  return 0;
}

namespace {

// Where a pass writes the returned lists: every cell as a full pair record
// (pairs_out), or compactly (cells_out: the input pair's index, or a new pair
// in new_out; include/gsnapdp.h gsnapdp_stage3_pass_compact).
struct Out {
  gsnapdp_s3_pair* pairs = nullptr;
  int64_t cap = 0;  // pairs, cells or runs
  int32_t* cells = nullptr;
  gsnapdp_s3_run* runs = nullptr;
  gsnapdp_s3_pair* news = nullptr;
  int64_t new_cap = 0;
};

// a returned list's segments as gsnapdp_s3_run records: a run of input pairs
// continued by the next segment's (one below it), and consecutive new pairs,
// merge; o = nullptr counts them
struct RunWriter {
  gsnapdp_s3_run* o = nullptr;
  int64_t n = 0;
  gsnapdp_s3_run cur{0, 0};
  bool open = false;
  void flush() {
    if (open) {
      if (o) o[n] = cur;
      n++;
      open = false;
    }
  }
  void in(int hi, int lo, bool d) {
    const int cnt = hi - lo + 1;
    if (!d && open && cur.start >= 0 && !(cur.count & GSNAPDP_S3_CELL_DISALLOWED) && cur.start - cur.count == hi) {
      cur.count += cnt;
      return;
    }
    flush();
    cur = gsnapdp_s3_run{hi, cnt | (d ? (int32_t)GSNAPDP_S3_CELL_DISALLOWED : 0)};
    open = true;
  }
  void nw(int64_t e) {  // new_out[e]
    if (open && cur.start < 0 && (int64_t)(-1 - cur.start) + cur.count == e) {
      cur.count++;
      return;
    }
    flush();
    cur = gsnapdp_s3_run{(int32_t)(-1 - e), 1};
    open = true;
  }
};

int run_pass(gsnapdp_ctx* ctx, gsnapdp_s3_call* calls, int ncalls, const gsnapdp_s3_pair* pairs_in,
             int64_t npairs_in, const char* query, const char* query_uc, size_t query_bytes, const gsnapdp_iit* iit,
             const Out& out, gsnapdp_s3_stats* stats, gsnapdp::S3Driver* driver = nullptr,
             const int32_t* gaps = nullptr, const int64_t* gap_off = nullptr) {
  if (!ctx || ncalls < 0 || npairs_in < 0 ||
      (ncalls > 0 && (!calls || (npairs_in > 0 && !pairs_in) || !query || !query_uc ||
                      !(driver || out.pairs || ((out.cells || out.runs) && out.news))))) {
    gsnapdp__set_err("gsnapdp_stage3_pass: bad arguments");
    return -1;
  }
  for (int i = 0; i < ncalls; i++)
    if (!call_in_range(calls[i], npairs_in, query_bytes)) {
      gsnapdp__set_err("gsnapdp_stage3_pass: call " + std::to_string(i) +
                       " names pairs or query bytes outside the buffers");
      return -1;
    }
  if ((gaps != nullptr) != (gap_off != nullptr) || (gap_off && ncalls > 0 && gap_off[0] < 0)) {
    gsnapdp__set_err("gsnapdp_stage3_pass_runs: gaps and gap_off go together");
    return -1;
  }
  for (int i = 0; gaps && i < ncalls; i++) {  // ascending pair indices inside each path
    bool ok = gap_off[i + 1] >= gap_off[i];
    for (int64_t j = gap_off[i]; ok && j < gap_off[i + 1]; j++)
      ok = gaps[j] >= 0 && gaps[j] < calls[i].npairs && (j == gap_off[i] || gaps[j] > gaps[j - 1]);
    if (!ok) {
      gsnapdp__set_err("gsnapdp_stage3_pass_runs: call " + std::to_string(i) +
                       "'s gap list is not ascending pair indices of its path");
      return -1;
    }
  }
  Pass P;
  P.ctx = ctx;
  P.blocks = gsnapdp__host_blocks(ctx);
  P.nwords = gsnapdp__host_nwords(ctx);
  P.iit = iit;
  P.query = query;
  P.query_uc = query_uc;
  P.driver = driver;
  P.gaps = gaps;
  P.gap_off = gap_off;
  memset(&P.st, 0, sizeof(P.st));
  using clock = std::chrono::steady_clock;
  const auto t_start = clock::now();
  double wait_s = 0.0;
  Workers& pool = Workers::get();
  PathStore* store = store_acquire();
  if (store->paths.size() < (size_t)ncalls) store->paths.resize((size_t)ncalls);
  Path* paths = store->paths.data();
  for (int i = 0; i < ncalls; i++) paths[(size_t)i].idx = i;
  Prof& pf = prof();
  if (pf.on) {
    for (int f = 0; f < F_N; f++) pf.expand_ns[f] = 0;
    pf.resume_ns = 0;
    pf.driver_ns = 0;
    pf.init = pf.pack = pf.copy = pf.submit = pf.wait = pf.resume = pf.output = 0;
  }
  pool.run(ncalls, 16, [&](int i) {
    Path& k = paths[(size_t)i];
    gsnapdp_s3_call& c = calls[i];
    if (P.gaps) {
      const int64_t g0 = P.gap_off[i], g1 = P.gap_off[i + 1];
      start_path(P, k, &c, pairs_in + c.first_pair, c.npairs, P.gaps + g0, (int)(g1 - g0));
    } else {
      start_path(P, k, &c, pairs_in + c.first_pair, c.npairs);
    }
    if (driver && (k.stage == S_DONE || k.failed)) finish_path(P, k);
  });
  // two cohorts (alternate paths, so both get a similar mix) when there are
  // enough paths for each round to be worth a batch of its own
  const auto t_init = clock::now();
  pf.init = std::chrono::duration<double>(t_init - t_start).count();
  const int ncoh = ncalls >= 256 ? 2 : 1;
  Cohort coh[2];
  for (int i = 0; i < ncalls; i++) coh[i % ncoh].paths.push_back(&paths[(size_t)i]);
  gsnapdp::S3Exec* X = gsnapdp::s3_exec_acquire(ctx);
  int rc = 0;
  for (int h = 0; h < ncoh && !rc; h++) {
    coh[h].slot = h;
    const int s = pack_submit(P, *X, coh[h]);
    if (s < 0) rc = -1;
    coh[h].inflight = s == 1;
  }
  while (!rc && (coh[0].inflight || coh[1].inflight)) {
    for (int h = 0; h < ncoh && !rc; h++) {
      Cohort& C = coh[h];
      if (!C.inflight) continue;
      const auto t0 = clock::now();
      if (X->wait(C.slot)) {
        rc = -1;
        break;
      }
      const auto t1 = clock::now();
      wait_s += std::chrono::duration<double>(t1 - t0).count();
      unpack_resume(P, *X, C);
      pf.resume += std::chrono::duration<double>(clock::now() - t1).count();
      const int s = pack_submit(P, *X, C);
      if (s < 0) rc = -1;
      C.inflight = s == 1;
    }
  }
  if (rc) {
    for (int h = 0; h < ncoh; h++)
      if (coh[h].inflight) (void)X->wait(coh[h].slot);  // drain before the staging is reused
    gsnapdp::s3_exec_release(ctx, X);
    store_release(store);
    return -1;
  }
  gsnapdp::s3_exec_release(ctx, X);
  if (driver) {  // the driver holds every path's lists and calls
    store_release(store);
    P.st.seconds[1] = wait_s;
    P.st.seconds[2] = std::chrono::duration<double>(clock::now() - t_start).count();
    if (pf.on)
      fprintf(stderr,
              "gsnapdp_stage3_pass profile (driven): %d paths, %d rounds, total %.4f s: init %.4f, pack %.4f, "
              "copy %.4f, submit %.4f, wait %.4f, resume %.4f (thread-s: resume %.4f, of which the driver's host "
              "steps %.4f; expand gap %.4f ggap %.4f)\n",
              ncalls, P.st.rounds, P.st.seconds[2], pf.init, pf.pack, pf.copy, pf.submit, wait_s, pf.resume,
              pf.resume_ns * 1e-9, pf.driver_ns * 1e-9, pf.expand_ns[0] * 1e-9, pf.expand_ns[1] * 1e-9);
    P.st.seconds[0] = P.st.seconds[2] - wait_s;
    if (stats) *stats = P.st;
    return 0;
  }
  const auto t_out = clock::now();
  // the returned lists, each path's at its running offset (lengths -- and
  // the new pairs among them -- by the workers, offsets, then the copies)
  std::vector<int64_t> first((size_t)ncalls + 1, 0), nfirst((size_t)ncalls + 1, 0);
  pool.run(ncalls, 16, [&](int i) {
    Path& k = paths[(size_t)i];
    if (k.c->pass == GSNAPDP_S3_END3) k.pairs = k.path;  // build_path_end3 returns its path
    int64_t n = 0, nn = 0;
    if (!k.failed) {
      if (out.runs) {
        RunWriter w;
        walk_list(k.A, k.pairs, [&](int hi, int lo, bool d) { w.in(hi, lo, d); }, [&](int) { w.nw(nn++); });
        w.flush();
        n = w.n;
      } else {
        walk_list(k.A, k.pairs, [&](int hi, int lo, bool) { n += hi - lo + 1; }, [&](int) { n++, nn++; });
      }
    }
    first[(size_t)i + 1] = n;
    nfirst[(size_t)i + 1] = nn;
  });
  for (int i = 0; i < ncalls; i++) {
    first[(size_t)i + 1] += first[(size_t)i];
    nfirst[(size_t)i + 1] += nfirst[(size_t)i];
  }
  P.st.new_pairs = nfirst[(size_t)ncalls];
  P.st.out_needed = first[(size_t)ncalls];
  if (first[(size_t)ncalls] > out.cap || (!out.pairs && nfirst[(size_t)ncalls] > out.new_cap)) {
    gsnapdp__set_err(std::string("gsnapdp_stage3_pass: ") +
                     (first[(size_t)ncalls] > out.cap ? (out.runs ? "the run" : "the cell") : "the new-pair") +
                     " output is too small (" + std::to_string(first[(size_t)ncalls]) +
                     (out.runs ? " runs, " : " cells, ") + std::to_string(nfirst[(size_t)ncalls]) + " new pairs)");
    if (stats) *stats = P.st;
    store_release(store);
    return -1;
  }
  pool.run(ncalls, 16, [&](int i) {
    Path& k = paths[(size_t)i];
    gsnapdp_s3_call& c = *k.c;
    c.status = k.failed ? -1 : 0;
    c.first_out = (int32_t)first[(size_t)i];
    c.nout = (int32_t)(first[(size_t)i + 1] - first[(size_t)i]);
    if (k.failed) return;
    int64_t at = first[(size_t)i], nat = nfirst[(size_t)i];
    const Arena& A = k.A;
    if (out.pairs) {
      walk_list(
          A, k.pairs,
          [&](int hi, int lo, bool d) {  // a reversed block copy
            gsnapdp_s3_pair* o = out.pairs + at;
            for (int x = hi; x >= lo; x--, o++) {
              *o = A.in[x];
              o->src = x;
              if (d) o->flags |= GSNAPDP_S3_DISALLOWED;
            }
            at += hi - lo + 1;
          },
          [&](int e) { out.pairs[at++] = A.extra[(size_t)e].p; });
    } else if (out.runs) {
      RunWriter w;
      w.o = out.runs + at;
      walk_list(
          A, k.pairs, [&](int hi, int lo, bool d) { w.in(hi, lo, d); },
          [&](int e) {
            out.news[nat] = A.extra[(size_t)e].p;
            w.nw(nat++);
          });
      w.flush();
    } else {
      walk_list(
          A, k.pairs,
          [&](int hi, int lo, bool d) {
            int32_t* o = out.cells + at;
            const int32_t f = d ? GSNAPDP_S3_CELL_DISALLOWED : 0;
            for (int x = hi; x >= lo; x--) *o++ = x | f;
            at += hi - lo + 1;
          },
          [&](int e) {
            out.news[nat] = A.extra[(size_t)e].p;
            out.cells[at++] = (int32_t)(-1 - nat++);
          });
    }
    write_call(k, c);
  });
  static const bool debug = getenv("GSNAPDP_S3_DEBUG") != nullptr;
  for (int i = 0; i < ncalls; i++) {
    P.st.undefined += paths[(size_t)i].undefined;
    if (paths[(size_t)i].failed) {
      P.st.failed++;
      if (debug)
        fprintf(stderr, "gsnapdp_stage3_pass: call %d (pass %d, tag %d) failed: %s\n", i, calls[i].pass,
                calls[i].invocation, paths[(size_t)i].why.c_str());
    }
  }
  store_release(store);
  const double total = std::chrono::duration<double>(clock::now() - t_start).count();
  if (pf.on) {
    pf.output = std::chrono::duration<double>(clock::now() - t_out).count();
    fprintf(stderr,
            "gsnapdp_stage3_pass profile: %d paths, %d rounds, total %.4f s: init %.4f, pack %.4f, copy %.4f, "
            "submit %.4f, wait %.4f, resume %.4f (thread-s: resume %.4f; expand gap %.4f ggap %.4f cgap %.4f "
            "micro %.4f), output %.4f\n",
            ncalls, P.st.rounds, total, pf.init, pf.pack, pf.copy, pf.submit, wait_s, pf.resume, pf.resume_ns * 1e-9,
            pf.expand_ns[0] * 1e-9, pf.expand_ns[1] * 1e-9, pf.expand_ns[2] * 1e-9, pf.expand_ns[3] * 1e-9,
            pf.output);
  }
  P.st.seconds[0] = total - wait_s;
  P.st.seconds[1] = wait_s;
  P.st.seconds[2] = total;
  if (stats) *stats = P.st;
  return 0;
}

}  // namespace

extern "C" int gsnapdp_stage3_pass(gsnapdp_ctx* ctx, gsnapdp_s3_call* calls, int ncalls,
                                   const gsnapdp_s3_pair* pairs_in, int64_t npairs_in, const char* query,
                                   const char* query_uc, size_t query_bytes, const gsnapdp_iit* iit,
                                   gsnapdp_s3_pair* pairs_out, int64_t out_cap, gsnapdp_s3_stats* stats) {
  Out o;
  o.pairs = pairs_out;
  o.cap = out_cap;
  return run_pass(ctx, calls, ncalls, pairs_in, npairs_in, query, query_uc, query_bytes, iit, o, stats);
}

extern "C" int gsnapdp_stage3_pass_compact(gsnapdp_ctx* ctx, gsnapdp_s3_call* calls, int ncalls,
                                           const gsnapdp_s3_pair* pairs_in, int64_t npairs_in, const char* query,
                                           const char* query_uc, size_t query_bytes, const gsnapdp_iit* iit,
                                           int32_t* cells_out, int64_t cells_cap, gsnapdp_s3_pair* new_out,
                                           int64_t new_cap, gsnapdp_s3_stats* stats) {
  Out o;
  o.cells = cells_out;
  o.cap = cells_cap;
  o.news = new_out;
  o.new_cap = new_cap;
  return run_pass(ctx, calls, ncalls, pairs_in, npairs_in, query, query_uc, query_bytes, iit, o, stats);
}

extern "C" int gsnapdp_stage3_pass_runs(gsnapdp_ctx* ctx, gsnapdp_s3_call* calls, int ncalls,
                                        const gsnapdp_s3_pair* pairs_in, int64_t npairs_in, const int32_t* gaps,
                                        const int64_t* gap_off, const char* query, const char* query_uc,
                                        size_t query_bytes, const gsnapdp_iit* iit, gsnapdp_s3_run* runs_out,
                                        int64_t runs_cap, gsnapdp_s3_pair* new_out, int64_t new_cap,
                                        gsnapdp_s3_stats* stats) {
  Out o;
  o.runs = runs_out;
  o.cap = runs_cap;
  o.news = new_out;
  o.new_cap = new_cap;
  return run_pass(ctx, calls, ncalls, pairs_in, npairs_in, query, query_uc, query_bytes, iit, o, stats, nullptr, gaps,
                  gap_off);
}

namespace {

constexpr int SI_EXTRAQUERYGAP = 10;       // stage3.h:29
constexpr int SI_MININTRONLEN_FINAL = 50;  // stage3.c:52

// score_introns' test of a gap pair (stage3.c:7971-7987, as gsnapdp_path_introns)
bool si_intron(const gsnapdp_s3_pair& p, int nullgap) {
  return (p.flags & GSNAPDP_S3_GAPP) && p.queryjump <= nullgap && p.queryjump <= p.genomejump + SI_EXTRAQUERYGAP &&
         p.genomejump > p.queryjump + SI_MININTRONLEN_FINAL;
}

// the introns each call's list holds (per[i], path order) -> IIT verdicts and
// one k_introns launch
int score_core(gsnapdp_ctx* ctx, const gsnapdp_s3_call* calls, int ncalls, const gsnapdp_iit* iit,
               std::vector<std::vector<gsnapdp_intron>>& per, std::atomic<int>& bad, const char* who,
               gsnapdp_intron_scores* scores) {
  if (bad.load()) {
    gsnapdp__set_err(std::string(who) + ": call " + std::to_string(bad.load() - 1) +
                     " has an intron at the end of its path (the reference dereferences NULL)");
    return -1;
  }
  if (iit) {
    Workers::get().run(ncalls, 16, [&](int i) {
      const gsnapdp_s3_call& c = calls[i];
      std::vector<gsnapdp_intron>& v = per[(size_t)i];
      if (!v.empty() && gsnapdp_introns_known(iit, c.chrnum, c.chrpos, c.genomiclength, c.cdna_direction,
                                              c.watsonp, v.data(), (int)v.size()))
        bad.store(i + 1);
    });
    if (bad.load()) {
      gsnapdp__set_err(std::string(who) + ": call " + std::to_string(bad.load() - 1) + ": " + gsnapdp_last_error());
      return -1;
    }
  }
  std::vector<gsnapdp_intron_path> ip((size_t)ncalls);
  size_t total = 0;
  for (int i = 0; i < ncalls; i++) total += per[(size_t)i].size();
  std::vector<gsnapdp_intron> all;
  all.reserve(total);
  for (int i = 0; i < ncalls; i++) {
    const gsnapdp_s3_call& c = calls[i];
    gsnapdp_intron_path& p = ip[(size_t)i];
    p.chroffset = c.chroffset;
    p.chrpos = c.chrpos;
    p.genomiclength = c.genomiclength;
    p.cdna_direction = c.cdna_direction;
    p.watsonp = c.watsonp;
    p.first_intron = (int32_t)all.size();
    p.nintrons = (int32_t)per[(size_t)i].size();
    p.pad = 0;
    all.insert(all.end(), per[(size_t)i].begin(), per[(size_t)i].end());
  }
  if (ncalls == 0) return 0;
  if (gsnapdp_score_introns_host(ctx, ip.data(), ncalls, all.empty() ? nullptr : all.data(), (int)all.size(),
                                 scores))
    return -1;
  for (int i = 0; i < ncalls; i++)
    if (calls[i].status != 0) memset(&scores[i], 0, sizeof(scores[i]));
  return 0;
}

}  // namespace

// score_introns on the lists a pass returned (include/gsnapdp.h)
extern "C" int gsnapdp_stage3_score_introns(gsnapdp_ctx* ctx, const gsnapdp_s3_call* calls, int ncalls,
                                            const gsnapdp_s3_pair* pairs_out, const gsnapdp_iit* iit,
                                            gsnapdp_intron_scores* scores) {
  if (!ctx || ncalls < 0 || (ncalls > 0 && (!calls || !scores))) {
    gsnapdp__set_err("gsnapdp_stage3_score_introns: bad arguments");
    return -1;
  }
  std::vector<std::vector<gsnapdp_intron>> per((size_t)ncalls);
  std::atomic<int> bad(0);
  Workers::get().run(ncalls, 16, [&](int i) {
    const gsnapdp_s3_call& c = calls[i];
    if (c.status != 0 || c.nout <= 0) return;
    thread_local std::vector<gsnapdp_path_pair> pp;
    pp.resize((size_t)c.nout);
    for (int j = 0; j < c.nout; j++) {  // List_reverse(pairs): path order
      const gsnapdp_s3_pair& x = pairs_out[(size_t)c.first_out + (size_t)(c.nout - 1 - j)];
      gsnapdp_path_pair& y = pp[(size_t)j];
      y.genomepos = (uint32_t)x.genomepos;
      y.queryjump = x.queryjump;
      y.genomejump = x.genomejump;
      y.gapp = (x.flags & GSNAPDP_S3_GAPP) ? 1 : 0;
      y.knowngapp = (x.flags & GSNAPDP_S3_KNOWNGAPP) ? 1 : 0;
      y.comp = (uint8_t)x.comp;
      y.pad = 0;
    }
    const int n = gsnapdp_path_introns(pp.data(), c.nout, c.nullgap, i, nullptr, 0);
    if (n < 0) {
      bad.store(i + 1);
      return;
    }
    std::vector<gsnapdp_intron>& v = per[(size_t)i];
    v.resize((size_t)n);
    gsnapdp_path_introns(pp.data(), c.nout, c.nullgap, i, v.data(), n);
  });
  return score_core(ctx, calls, ncalls, iit, per, bad, "gsnapdp_stage3_score_introns", scores);
}

// The same on gsnapdp_stage3_pass_runs' output: only the gap pairs of each
// list are visited (an input run's through the gap lists, a new pair run's
// one by one), with their list neighbours for the intron's ends.
extern "C" int gsnapdp_stage3_score_introns_runs(gsnapdp_ctx* ctx, const gsnapdp_s3_call* calls, int ncalls,
                                                 const gsnapdp_s3_pair* pairs_in, const int32_t* gaps,
                                                 const int64_t* gap_off, const gsnapdp_s3_run* runs,
                                                 const gsnapdp_s3_pair* new_pairs, const gsnapdp_iit* iit,
                                                 gsnapdp_intron_scores* scores) {
  if (!ctx || ncalls < 0 || (ncalls > 0 && (!calls || !scores || !pairs_in || !runs)) ||
      (gaps != nullptr) != (gap_off != nullptr)) {
    gsnapdp__set_err("gsnapdp_stage3_score_introns_runs: bad arguments");
    return -1;
  }
  std::vector<std::vector<gsnapdp_intron>> per((size_t)ncalls);
  std::atomic<int> bad(0);
  Workers::get().run(ncalls, 16, [&](int i) {
    const gsnapdp_s3_call& c = calls[i];
    if (c.status != 0 || c.nout <= 0) return;
    const gsnapdp_s3_pair* in = pairs_in + c.first_pair;
    const gsnapdp_s3_run* R = runs + c.first_out;
    const int nr = c.nout;
    auto count = [&](int r) { return (int)(R[r].count & ~GSNAPDP_S3_CELL_DISALLOWED); };
    auto elem = [&](int r, int off) -> const gsnapdp_s3_pair& {
      return R[r].start >= 0 ? in[R[r].start - off] : new_pairs[(int64_t)(-1 - R[r].start) + off];
    };
    thread_local std::vector<int32_t> own;
    const int32_t *g0 = nullptr, *g1 = nullptr;
    if (gaps) {
      g0 = gaps + gap_off[i];
      g1 = gaps + gap_off[i + 1];
    } else {
      own.clear();
      for (int j = 0; j < c.npairs; j++)
        if (in[j].flags & GSNAPDP_S3_GAPP) own.push_back(j);
      g0 = own.data();
      g1 = own.data() + own.size();
    }
    std::vector<gsnapdp_intron>& v = per[(size_t)i];
    v.clear();
    // an intron at (run r, offset off): leftpair is the list's previous pair,
    // rightpair its next (path order reversed, gsnapdp_path_introns)
    auto take = [&](int r, int off) {
      const gsnapdp_s3_pair& p = elem(r, off);
      if (!si_intron(p, c.nullgap)) return;
      const gsnapdp_s3_pair* prev = off > 0 ? &elem(r, off - 1) : (r > 0 ? &elem(r - 1, count(r - 1) - 1) : nullptr);
      const gsnapdp_s3_pair* next = off + 1 < count(r) ? &elem(r, off + 1) : (r + 1 < nr ? &elem(r + 1, 0) : nullptr);
      if (!prev || !next) {
        bad.store(i + 1);
        return;
      }
      gsnapdp_intron x;
      x.left_genomepos = (uint32_t)prev->genomepos;
      x.right_genomepos = (uint32_t)next->genomepos;
      x.path = i;
      x.comp = (uint8_t)p.comp;
      x.knowngapp = (p.flags & GSNAPDP_S3_KNOWNGAPP) ? 1 : 0;
      x.known_donor = x.known_acceptor = 0;
      v.push_back(x);
    };
    for (int r = 0; r < nr; r++) {
      const int n = count(r);
      if (R[r].start >= 0) {  // input pairs start .. start - n + 1: their gaps, descending
        const int hi = R[r].start, lo = hi - n + 1;
        const int32_t* g = std::upper_bound(g0, g1, hi);
        while (g != g0 && *(g - 1) >= lo) {
          --g;
          take(r, hi - *g);
        }
      } else {
        for (int off = 0; off < n; off++)
          if (elem(r, off).flags & GSNAPDP_S3_GAPP) take(r, off);
      }
    }
    std::reverse(v.begin(), v.end());  // path order
  });
  return score_core(ctx, calls, ncalls, iit, per, bad, "gsnapdp_stage3_score_introns_runs", scores);
}

int gsnapdp::s3_run_driven(gsnapdp_ctx* ctx, gsnapdp_s3_call* calls, int ncalls, const gsnapdp_s3_pair* pairs_in,
                           int64_t npairs_in, const char* query, const char* query_uc, size_t query_bytes,
                           const gsnapdp_iit* iit, S3Driver* driver, gsnapdp_s3_stats* stats) {
  return run_pass(ctx, calls, ncalls, pairs_in, npairs_in, query, query_uc, query_bytes, iit, Out(), stats, driver);
}
