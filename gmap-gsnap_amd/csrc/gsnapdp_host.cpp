// gsnapdp_host.cpp -- host half of the product library: substitution tables
// (the profile words the kernels read) and the op-stream -> pair-list
// expansion that reproduces the reference's Pairpool_push sequence.
#include <ctype.h>
#include <stdint.h>
#include <string.h>

#include <vector>

#include "gsnapdp_internal.h"

extern "C" const uint32_t* gsnapdp__host_blocks(gsnapdp_ctx* ctx);
extern "C" size_t gsnapdp__host_nwords(gsnapdp_ctx* ctx);
extern "C" const uint32_t* gsnapdp__host_prof(gsnapdp_ctx* ctx);

namespace gsnapdp {

namespace {
int pd_tab[4][128][128];
unsigned char cons_tab[128][128];
int tab_mode = -1;

void set_all_cases(int a, int b, int score, bool symmetric) {
  // every upper/lower-case combination (permute_cases / _oneway, dynprog.c:1053-1124)
  const int as[2] = {a, tolower(a)}, bs[2] = {b, tolower(b)};
  for (int i = 0; i < 2; i++)
    for (int j = 0; j < 2; j++) {
      cons_tab[as[i]][bs[j]] = 1;
      for (int t = 0; t < 4; t++) pd_tab[t][as[i]][bs[j]] = score;
      if (symmetric) {
        cons_tab[bs[j]][as[i]] = 1;
        for (int t = 0; t < 4; t++) pd_tab[t][bs[j]][as[i]] = score;
      }
    }
}

void init_tables(int mode) {
  // pairdistance_init (dynprog.c:1127-1226)
  static const int mism[4] = {-3, -2, -1, -5};
  memset(pd_tab, 0, sizeof(pd_tab));
  memset(cons_tab, 0, sizeof(cons_tab));
  for (int c1 = 'A'; c1 <= 'z'; c1++)
    for (int c2 = 'A'; c2 < 'z'; c2++)
      for (int t = 0; t < 4; t++) pd_tab[t][c1][c2] = mism[t];
  set_all_cases('U', 'T', 3, true);
  struct Amb { char code; const char* bases; int score; };
  static const Amb amb[] = {{'R', "AG", 1},  {'Y', "TC", 1},  {'W', "AT", 1},  {'S', "GC", 1},
                            {'M', "AC", 1},  {'K', "GT", 1},  {'H', "ATC", -1}, {'B', "GCT", -1},
                            {'V', "GAC", -1}, {'D', "GAT", -1}, {'N', "TCAG", -1}, {'X', "TCAG", -1}};
  for (const Amb& a : amb)
    for (const char* p = a.bases; *p; p++) set_all_cases(a.code, *p, a.score, true);
  if (mode == GSNAPDP_MODE_CMET_STRANDED || mode == GSNAPDP_MODE_CMET_NONSTRANDED) {
    set_all_cases('T', 'C', 3, false);
    set_all_cases('A', 'G', 3, false);
  }
  for (int c = 'A'; c < 'Z'; c++) set_all_cases(c, c, 3, true);
  tab_mode = mode;
}
}  // namespace

void build_profile_table(int mode, uint32_t prof[PROF_WORDS]) {
  init_tables(mode);
  static const char cls[6] = {'A', 'C', 'G', 'T', 'N', '*'};
  for (int t = 0; t < 4; t++)
    for (int c = 0; c < 128; c++) {
      uint32_t w = 0;
      for (int g = 0; g < 6; g++) w |= ((uint32_t)pd_tab[t][c][(int)cls[g]] & 0xFu) << (4 * g);
      for (int g = 0; g < 5; g++) w |= (uint32_t)cons_tab[c][(int)cls[g]] << (24 + g);
      prof[t * 128 + c] = w;
    }
  for (int u = 0; u < 128; u++) {
    uint32_t w = 0;
    for (int g = 0; g < 5; g++)
      if (u == cls[g]) w |= 1u << (24 + g);
    prof[4 * 128 + u] = w;
  }
  for (int c = 0; c < 128; c++) {
    uint32_t w = 0;
    for (int g = 0; g < 5; g++) w |= (uint32_t)cons_tab[(int)cls[g]][c] << (24 + g);
    prof[PROF_CONS_SWAPPED + c] = w;
  }
}

int host_pairdistance(int mt, int c1, int c2) { return pd_tab[mt][c1 & 127][c2 & 127]; }
int host_consistent(int c1, int c2) { return cons_tab[c1 & 127][c2 & 127]; }

}  // namespace gsnapdp

using namespace gsnapdp;

namespace {

struct HostGenome {
  const uint32_t* blocks;
  size_t nwords;
  uint32_t chroffset, chrhigh, chrpos;
  int glen, watson;
  // get_genomic_nt (dynprog.c:403-441)
  char nt(int gpos) const {
    if (gpos < 0 || gpos >= glen) return '*';
    const uint32_t base = chroffset + chrpos;
    if (base < chroffset || base >= chrhigh) return '*';
    const uint32_t pos = watson ? base + (uint32_t)gpos : base + (uint32_t)(glen - 1) - (uint32_t)gpos;
    const size_t ptr = (size_t)(pos >> 5) * 3;
    if (ptr + 2 >= nwords) return 'N';
    const uint32_t bit = pos & 31u;
    char c;
    if ((blocks[ptr + 2] >> bit) & 1u) c = 'N';
    else c = "ACGT"[((bit < 16 ? blocks[ptr + 1] : blocks[ptr]) >> ((bit & 15u) * 2u)) & 3u];
    if (watson) return c;
    switch (c) {
      case 'A': return 'T';
      case 'C': return 'G';
      case 'G': return 'C';
      case 'T': return 'A';
      default: return 'N';
    }
  }
};

}  // namespace

// Replay one traceback's op stream from (r, c) into the pairs the reference
// pushes, in push order (traceback, dynprog.c:2611-2712; add_genomeskip :2416;
// add_queryskip :2372).  q / qu point at the query of row 1 (forward) or at
// sequence1[length1-1] (reversed fills, indexed with negative offsets).
static void replay(const uint32_t* ops, int nops, int r, int c, const char* q, const char* qu,
                   int qoff, int goff, bool rev, const HostGenome& G, const uint32_t* prof,
                   int dpi, std::vector<gsnapdp_pair>& p) {
  auto push = [&](int qpos, int gpos, char cdna, char comp, char g) {
    gsnapdp_pair x;
    memset(&x, 0, sizeof(x));
    x.querypos = qpos;
    x.genomepos = gpos;
    x.dynprogindex = dpi;
    x.cdna = cdna;
    x.comp = comp;
    x.genome = g;
    p.push_back(x);
  };
  auto consistent = [&](unsigned char c1, char g) -> bool {
    int gi = g == 'A' ? 0 : g == 'C' ? 1 : g == 'G' ? 2 : g == 'T' ? 3 : 4;
    return (prof[c1 & 127] >> (24 + gi)) & 1u;  // consistent_array is mode-independent per mt
  };
  for (int k = 0; k < nops; k++) {
    const uint32_t op = ops[k];
    const int cnt = (int)GSNAPDP_OP_COUNT(op);
    switch (GSNAPDP_OP_TYPE(op)) {
      case GSNAPDP_OP_DIAG:
        for (int j = 0; j < cnt; j++, r--, c--) {
          int qc = r - 1, gc = c - 1;
          if (rev) {
            qc = -qc;
            gc = -gc;
          }
          const char c1 = q[qc];
          const char c2 = G.nt(goff + gc);
          if (c2 == '*') continue;  // dynprog.c:2644
          char comp;
          if (qu[qc] == c2) comp = GSNAPDP_DYNPROG_MATCH_COMP;
          else if (consistent((unsigned char)c1, c2)) comp = GSNAPDP_AMBIGUOUS_COMP;
          else comp = GSNAPDP_MISMATCH_COMP;
          push(qoff + qc, goff + gc, c1, comp, c2);
        }
        break;
      case GSNAPDP_OP_HDASH: {  // add_genomeskip dashes (dynprog.c:2478-2499)
        int qc = r - 1, left = c - cnt, right = c - 1, step;
        if (rev) {
          const int t = left;
          qc = -qc;
          left = -right;
          right = -t;
          step = +1;
        } else {
          qc++;
          step = -1;
        }
        int gc = rev ? left : right;
        for (int j = 0; j < cnt; j++, gc += step) push(qoff + qc, goff + gc, ' ', '-', G.nt(goff + gc));
        c -= cnt;
        break;
      }
      case GSNAPDP_OP_HGAP: {  // gapholder (dynprog.c:2507)
        gsnapdp_pair x;
        memset(&x, 0, sizeof(x));
        x.querypos = -1;
        x.genomepos = -1;
        x.queryjump = GSNAPDP_UNKNOWNJUMP;
        x.genomejump = GSNAPDP_UNKNOWNJUMP;
        x.cdna = ' ';
        x.comp = ' ';
        x.genome = ' ';
        x.gapp = 1;
        p.push_back(x);
        c -= cnt;
        break;
      }
      default: {  // GSNAPDP_OP_VSKIP, add_queryskip (dynprog.c:2372-2413)
        int qc = r - 1, gc = c - 1, step;
        if (rev) {
          qc = -qc;
          gc = -gc;
          step = +1;
        } else {
          gc++;
          step = -1;
        }
        for (int j = 0; j < cnt; j++, qc += step) push(qoff + qc, goff + gc, q[qc], '-', ' ');
        r -= cnt;
        break;
      }
    }
  }
}

extern "C" int gsnapdp_expand(gsnapdp_ctx* ctx, const gsnapdp_window* w, const gsnapdp_result* res,
                              const uint32_t* ops, const char* query, const char* query_uc,
                              gsnapdp_pair* pairs, int cap, int* finalscore) {
  if (!ctx || !w || !res) return -1;
  if (finalscore) *finalscore = res->finalscore;
  if (res->status == ST_EARLY || res->status == ST_ZEROED || res->status == ST_UNSUPPORTED) return 0;
  if (res->status == ST_OPS_OVERFLOW) return -1;
  const uint32_t* prof = gsnapdp__host_prof(ctx);
  HostGenome G = {gsnapdp__host_blocks(ctx), gsnapdp__host_nwords(ctx), w->chroffset, w->chrhigh,
                  w->chrpos, (int)w->genomiclength, w->watsonp ? 1 : 0};
  const bool rev = w->kind == GSNAPDP_END5_GAP;
  const char* q = query + w->qpos;
  const char* qu = query_uc + w->qpos;
  const int qoff = w->offset1, goff = w->offset2, dpi = w->dynprogindex;
  int r = res->bestr, c = res->bestc;
  thread_local std::vector<gsnapdp_pair> p;  // push order (a buffer per host thread)
  p.clear();
  replay(ops, res->nops, r, c, q, qu, qoff, goff, rev, G, prof, dpi, p);
  // final list orientation (dynprog.c:4571, 5264-5283, 5721-5740)
  const int m = (int)p.size();
  int n = 0;
  if (w->kind == GSNAPDP_SINGLE_GAP) {
    for (int i = 0; i < m; i++, n++)
      if (n < cap) pairs[n] = p[i];
  } else {
    int j = 0;
    while (j < m && p[j].comp == '-') j++;
    if (w->kind == GSNAPDP_END3_GAP) {
      for (int i = j; i < m; i++, n++)
        if (n < cap) pairs[n] = p[i];
    } else {
      for (int i = m - 1; i >= j; i--, n++)
        if (n < cap) pairs[n] = p[i];
    }
  }
  return n;
}

// traceback_local's pushes (dynprog.c:2874-2968) for the splice-junction end
// gaps: the op stream of the whole traceback is cut at the first loop top
// whose column is <= endc (part one runs while c > contlength), where the
// known gapholder goes (:5517 / :6021); part one's coordinates use goff_far,
// part two's goff_anchor.  Genome chars come from the segment `g` (indexed
// like q: g[c-1] forwards, g[1-c] reversed), with no '*' test.
static void replay_local(const uint32_t* ops, int nops, int r, int c, int endc, const char* q,
                         const char* qu, const char* g, int qoff, int goff_far, int goff_anchor,
                         int jump, bool rev, const uint32_t* prof, int dpi,
                         std::vector<gsnapdp_pair>& p) {
  auto push = [&](int qpos, int gpos, char cdna, char comp, char gc) {
    gsnapdp_pair x;
    memset(&x, 0, sizeof(x));
    x.querypos = qpos;
    x.genomepos = gpos;
    x.dynprogindex = dpi;
    x.cdna = cdna;
    x.comp = comp;
    x.genome = gc;
    p.push_back(x);
  };
  bool second = false;
  int goff = goff_far;
  auto cut = [&]() {  // Pairpool_push_gapholder(queryjump 0, genomejump, knownp true)
    gsnapdp_pair x;
    memset(&x, 0, sizeof(x));
    x.querypos = -1;
    x.genomepos = -1;
    x.queryjump = 0;
    x.genomejump = jump;
    x.cdna = ' ';
    x.comp = ' ';
    x.genome = ' ';
    x.gapp = 3;
    p.push_back(x);
    second = true;
    goff = goff_anchor;
  };
  auto consistent = [&](unsigned char c1, char gch) -> bool {
    const int gi = gch == 'A' ? 0 : gch == 'C' ? 1 : gch == 'G' ? 2 : gch == 'T' ? 3 : 4;
    return (prof[c1 & 127] >> (24 + gi)) & 1u;
  };
  for (int k = 0; k < nops; k++) {
    const uint32_t op = ops[k];
    const int cnt = (int)GSNAPDP_OP_COUNT(op);
    switch (GSNAPDP_OP_TYPE(op)) {
      case GSNAPDP_OP_DIAG:
        for (int j = 0; j < cnt; j++, r--, c--) {
          if (!second && c <= endc) cut();
          int qc = r - 1, gc = c - 1;
          if (rev) {
            qc = -qc;
            gc = -gc;
          }
          const char c1 = q[qc];
          const char c2 = g[gc];
          char comp;
          if (qu[qc] == c2) comp = GSNAPDP_DYNPROG_MATCH_COMP;
          else if (consistent((unsigned char)c1, c2)) comp = GSNAPDP_AMBIGUOUS_COMP;
          else comp = GSNAPDP_MISMATCH_COMP;
          push(qoff + qc, goff + gc, c1, comp, c2);
        }
        break;
      case GSNAPDP_OP_HDASH: {
        int qc = r - 1, left = c - cnt, right = c - 1, step;
        if (rev) {
          const int t = left;
          qc = -qc;
          left = -right;
          right = -t;
          step = +1;
        } else {
          qc++;
          step = -1;
        }
        int gc = rev ? left : right;
        for (int j = 0; j < cnt; j++, gc += step) push(qoff + qc, goff + gc, ' ', '-', g[gc]);
        c -= cnt;
        break;
      }
      case GSNAPDP_OP_HGAP: {
        gsnapdp_pair x;
        memset(&x, 0, sizeof(x));
        x.querypos = -1;
        x.genomepos = -1;
        x.queryjump = GSNAPDP_UNKNOWNJUMP;
        x.genomejump = GSNAPDP_UNKNOWNJUMP;
        x.cdna = ' ';
        x.comp = ' ';
        x.genome = ' ';
        x.gapp = 1;
        p.push_back(x);
        c -= cnt;
        break;
      }
      default: {
        int qc = r - 1, gc = c - 1, step;
        if (rev) {
          qc = -qc;
          gc = -gc;
          step = +1;
        } else {
          gc++;
          step = -1;
        }
        for (int j = 0; j < cnt; j++, qc += step) push(qoff + qc, goff + gc, q[qc], '-', ' ');
        r -= cnt;
        break;
      }
    }
  }
  if (!second) cut();
}

// Dynprog_end5/3_splicejunction's list (dynprog.c:5543-5553 / :6047-6057)
extern "C" int gsnapdp_sj_expand(gsnapdp_ctx* ctx, const gsnapdp_sj_window* w,
                                 const gsnapdp_result* res, const uint32_t* ops, const char* query,
                                 const char* query_uc, gsnapdp_pair* pairs, int cap) {
  if (!ctx || !w || !res) return -1;
  if (res->status == ST_EARLY || res->status == ST_UNSUPPORTED) return 0;
  if (res->status == ST_OPS_OVERFLOW) return -1;
  const bool rev = w->kind == GSNAPDP_END5_GAP;
  const int jump = rev ? w->offset2_anchor - w->offset2_far : w->offset2_far - w->offset2_anchor;
  thread_local std::vector<gsnapdp_pair> p;
  p.clear();
  replay_local(ops, res->nops, res->bestr, res->bestc, w->contlength, query + w->qpos,
               query_uc + w->qpos, query + w->spos, w->offset1, w->offset2_far,
               w->offset2_anchor, jump, rev, gsnapdp__host_prof(ctx), w->dynprogindex, p);
  const int m = (int)p.size();
  int j = 0, n = 0;
  while (j < m && p[j].comp == '-') j++;
  if (!rev) {
    for (int i = j; i < m; i++, n++)
      if (n < cap) pairs[n] = p[i];
  } else {
    for (int i = m - 1; i >= j; i--, n++)
      if (n < cap) pairs[n] = p[i];
  }
  return n;
}

// Dynprog_microexon_int's list (make_microexon_pairs_double, dynprog.c:6949-7055):
// the left segment, a gapholder with comp = the intron's gapchar, the middle
// from genome column offset2M, a second gapholder, the right segment; the
// returned list starts at the last pair pushed.
extern "C" int gsnapdp_micro_expand(gsnapdp_ctx* ctx, const gsnapdp_micro_window* w,
                                    const gsnapdp_micro_result* res, const char* query,
                                    const char* query_uc, gsnapdp_pair* pairs, int cap) {
  if (!ctx || !w || !res) return -1;
  if (res->status != ST_OK || !res->found) return 0;
  HostGenome G = {gsnapdp__host_blocks(ctx), gsnapdp__host_nwords(ctx), w->chroffset, w->chrhigh,
                  w->chrpos, (int)w->genomiclength, w->watsonp ? 1 : 0};
  const uint32_t* prof = gsnapdp__host_prof(ctx);
  const char gapchar = w->cdna_direction > 0 ? '>' : '<';  // FWD/REV_CANONICAL_INTRON_COMP
  // queryseq[offset1 + k] is the staged byte ppos + k
  const char* qs = query + w->ppos;
  const char* qsu = query_uc + w->ppos;
  const int offs1[3] = {0, res->bestcL, res->bestcL + res->middlelength};
  const int offs2[3] = {w->offset2L, res->offset2M, w->revoffset2R - res->bestcR + 1};
  const int lens[3] = {res->bestcL, res->middlelength, res->bestcR};
  thread_local std::vector<gsnapdp_pair> p;
  p.clear();
  for (int seg = 0; seg < 3; seg++) {
    for (int k = 0; k < lens[seg]; k++) {
      const int qi = offs1[seg] + k;
      const char c1 = qs[qi], c2 = G.nt(offs2[seg] + k);
      const int gi = c2 == 'A' ? 0 : c2 == 'C' ? 1 : c2 == 'G' ? 2 : c2 == 'T' ? 3 : c2 == 'N' ? 4 : -1;
      char comp;
      if (qsu[qi] == c2) comp = GSNAPDP_DYNPROG_MATCH_COMP;
      else if (gi >= 0 && ((prof[(unsigned char)c1 & 127] >> (24 + gi)) & 1u)) comp = GSNAPDP_AMBIGUOUS_COMP;
      else comp = GSNAPDP_MISMATCH_COMP;
      gsnapdp_pair x;
      memset(&x, 0, sizeof(x));
      x.querypos = w->offset1 + qi;
      x.genomepos = offs2[seg] + k;
      x.dynprogindex = w->dynprogindex;
      x.cdna = c1;
      x.comp = comp;
      x.genome = c2;
      p.push_back(x);
    }
    if (seg < 2) {
      gsnapdp_pair x;
      memset(&x, 0, sizeof(x));
      x.querypos = -1;
      x.genomepos = -1;
      x.queryjump = GSNAPDP_UNKNOWNJUMP;
      x.genomejump = GSNAPDP_UNKNOWNJUMP;
      x.cdna = ' ';
      x.comp = gapchar;
      x.genome = ' ';
      x.gapp = 1;
      p.push_back(x);
    }
  }
  int n = 0;
  for (int i = (int)p.size() - 1; i >= 0; i--, n++)
    if (n < cap) pairs[n] = p[(size_t)i];
  return n;
}

// Dynprog_genome_gap's list (dynprog.c:5000-5058): traceback of the right flank
// (reversed), List_reverse, the gapholder, traceback of the left flank, then
// List_reverse of the whole -- i.e. the right flank's pairs last-pushed first,
// the gapholder, the left flank's pairs in push order.
extern "C" int gsnapdp_ggap_expand(gsnapdp_ctx* ctx, const gsnapdp_ggap_window* w,
                                   const gsnapdp_ggap_result* res, const gsnapdp_ggap_trace* tr,
                                   const uint32_t* ops, const char* query, const char* query_uc,
                                   gsnapdp_pair* pairs, int cap) {
  if (!ctx || !w || !res || !tr) return -1;
  if (tr->status == ST_OPS_OVERFLOW || tr->status == ST_INTERNAL) return -1;
  if (res->returned_null || tr->status != ST_OK) return 0;
  const uint32_t* prof = gsnapdp__host_prof(ctx);
  HostGenome G = {gsnapdp__host_blocks(ctx), gsnapdp__host_nwords(ctx), w->chroffset, w->chrhigh,
                  w->chrpos, (int)w->genomiclength, w->watsonp ? 1 : 0};
  const int L1 = w->length1, dpi = w->dynprogindex;
  thread_local std::vector<gsnapdp_pair> pr, pl;  // buffers per host thread
  pr.clear();
  pl.clear();
  replay(ops, tr->nops_right, tr->brR, tr->bcR, query + w->qpos + L1 - 1,
         query_uc + w->qpos + L1 - 1, w->offset1 + L1 - 1, w->revoffset2R, true, G, prof, dpi, pr);
  replay(ops + tr->nops_right, tr->nops_left, tr->brL, tr->bcL, query + w->qpos,
         query_uc + w->qpos, w->offset1, w->offset2L, false, G, prof, dpi, pl);
  int n = 0;
  for (int i = (int)pr.size() - 1; i >= 0; i--, n++)
    if (n < cap) pairs[n] = pr[i];
  if (n < cap) {
    gsnapdp_pair x;
    memset(&x, 0, sizeof(x));
    x.querypos = -1;
    x.genomepos = -1;
    x.queryjump = GSNAPDP_UNKNOWNJUMP;
    x.genomejump = GSNAPDP_UNKNOWNJUMP;
    x.cdna = ' ';
    x.comp = ' ';
    x.genome = ' ';
    x.gapp = 1;
    pairs[n] = x;
  }
  n++;
  for (size_t i = 0; i < pl.size(); i++, n++)
    if (n < cap) pairs[n] = pl[i];
  return n;
}

// traceback_cdna's pushes (dynprog.c:2716-2812) from an op stream: genome
// rows r, query columns c; add_queryskip with cdna_gap_p (:2372) for VSKIP,
// add_genomeskip_cdna (:2516) for HDASH / HGAP.
static void replay_cdna(const uint32_t* ops, int nops, int r, int c, const char* q, const char* qu,
                        int qoff, int goff, bool rev, const HostGenome& G, int dpi,
                        std::vector<gsnapdp_pair>& p) {
  auto push = [&](int qpos, int gpos, char cdna, char comp, char g) {
    gsnapdp_pair x;
    memset(&x, 0, sizeof(x));
    x.querypos = qpos;
    x.genomepos = gpos;
    x.dynprogindex = dpi;
    x.cdna = cdna;
    x.comp = comp;
    x.genome = g;
    p.push_back(x);
  };
  for (int k = 0; k < nops; k++) {
    const uint32_t op = ops[k];
    const int cnt = (int)GSNAPDP_OP_COUNT(op);
    switch (GSNAPDP_OP_TYPE(op)) {
      case GSNAPDP_OP_DIAG:
        for (int j = 0; j < cnt; j++, r--, c--) {
          int qc = c - 1, gc = r - 1;
          if (rev) {
            qc = -qc;
            gc = -gc;
          }
          const char c1 = q[qc];
          const char c2 = G.nt(goff + gc);
          char comp;
          if (qu[qc] == c2) comp = GSNAPDP_DYNPROG_MATCH_COMP;
          else if (host_consistent(c2, c1)) comp = GSNAPDP_AMBIGUOUS_COMP;  // swapped (:2760)
          else comp = GSNAPDP_MISMATCH_COMP;
          push(qoff + qc, goff + gc, c1, comp, c2);
        }
        break;
      case GSNAPDP_OP_VSKIP: {  // query skip
        int qc = c - 1, gc = r - 1, step;
        if (rev) {
          qc = -qc;
          gc = -gc;
          step = +1;
        } else {
          gc++;
          step = -1;
        }
        for (int j = 0; j < cnt; j++, qc += step) push(qoff + qc, goff + gc, q[qc], '-', ' ');
        c -= cnt;
        break;
      }
      case GSNAPDP_OP_HDASH: {  // genome skip, dashes
        int qc = c - 1, left = r - cnt, right = r - 1, step;
        if (rev) {
          const int t = left;
          qc = -qc;
          left = -right;
          right = -t;
          step = +1;
        } else {
          qc++;
          step = -1;
        }
        int gc = rev ? left : right;
        for (int j = 0; j < cnt; j++, gc += step) push(qoff + qc, goff + gc, ' ', '-', G.nt(goff + gc));
        r -= cnt;
        break;
      }
      default: {  // GSNAPDP_OP_HGAP: genome skip as a gapholder
        gsnapdp_pair x;
        memset(&x, 0, sizeof(x));
        x.querypos = -1;
        x.genomepos = -1;
        x.queryjump = GSNAPDP_UNKNOWNJUMP;
        x.genomejump = GSNAPDP_UNKNOWNJUMP;
        x.cdna = ' ';
        x.comp = ' ';
        x.genome = ' ';
        x.gapp = 1;
        p.push_back(x);
        r -= cnt;
        break;
      }
    }
  }
}

// Dynprog_cdna_gap's list (dynprog.c:4711-4793): the right side's pairs last
// pushed first, then the INSERT_PAIRS pairs (or the gapholder), then the left
// side's pairs.  `sequence2` is the reference's genomic-segment argument (read
// by the INSERT_PAIRS branch); NULL reads the context genome at the same positions.
extern "C" int gsnapdp_cgap_expand(gsnapdp_ctx* ctx, const gsnapdp_cgap_window* w,
                                   const gsnapdp_cgap_result* res, const uint32_t* ops,
                                   const char* query, const char* query_uc, const char* sequence2,
                                   gsnapdp_pair* pairs, int cap) {
  if (!ctx || !w || !res) return -1;
  if (res->status == ST_OPS_OVERFLOW) return -1;
  if (res->returned_null || res->status != ST_OK) return 0;
  HostGenome G = {gsnapdp__host_blocks(ctx), gsnapdp__host_nwords(ctx), w->chroffset, w->chrhigh,
                  w->chrpos, (int)w->genomiclength, w->watsonp ? 1 : 0};
  const int dpi = w->dynprogindex, revoffset2 = w->offset2 + w->length2 - 1;
  thread_local std::vector<gsnapdp_pair> pr, pl, pi;
  pr.clear();
  pl.clear();
  pi.clear();
  replay_cdna(ops, res->nops_right, res->brR, res->bcR, query + w->qposR, query_uc + w->qposR,
              w->revoffset1R, revoffset2, true, G, dpi, pr);
  replay_cdna(ops + res->nops_right, res->nops_left, res->brL, res->bcL, query + w->qposL,
              query_uc + w->qposL, w->offset1L, w->offset2, false, G, dpi, pl);
  if (res->insert_pairs) {  // :4730-4752
    for (int k = w->revoffset1R - res->bcR; k >= w->offset1L + res->bcL; k--) {
      gsnapdp_pair x;
      memset(&x, 0, sizeof(x));
      x.querypos = k;
      x.genomepos = revoffset2 - res->brR + 1;
      x.dynprogindex = dpi;
      x.cdna = query[w->qposL + (k - w->offset1L)];
      x.comp = '~';  // SHORTGAP_COMP
      x.genome = ' ';
      pi.push_back(x);
    }
    for (int k = revoffset2 - res->brR; k >= w->offset2 + res->brL; k--) {
      gsnapdp_pair x;
      memset(&x, 0, sizeof(x));
      x.querypos = w->offset1L + res->bcL;
      x.genomepos = k;
      x.dynprogindex = dpi;
      x.cdna = ' ';
      x.comp = '~';
      x.genome = sequence2 ? sequence2[k - w->offset2] : G.nt(k);
      pi.push_back(x);
    }
  } else {
    gsnapdp_pair x;
    memset(&x, 0, sizeof(x));
    x.querypos = -1;
    x.genomepos = -1;
    x.queryjump = GSNAPDP_UNKNOWNJUMP;
    x.genomejump = GSNAPDP_UNKNOWNJUMP;
    x.cdna = ' ';
    x.comp = ' ';
    x.genome = ' ';
    x.gapp = 1;
    pi.push_back(x);
  }
  int n = 0;
  for (int i = (int)pr.size() - 1; i >= 0; i--, n++)
    if (n < cap) pairs[n] = pr[i];
  for (size_t i = 0; i < pi.size(); i++, n++)
    if (n < cap) pairs[n] = pi[i];
  for (size_t i = 0; i < pl.size(); i++, n++)
    if (n < cap) pairs[n] = pl[i];
  return n;
}

// score_introns' walk over a path (stage3.c:7960-8146): a gap pair is an
// intron when it is neither past nullgap (:7971) nor query-heavy
// (queryjump > genomejump + EXTRAQUERYGAP, :7979) and its genome jump exceeds
// the query jump by more than MININTRONLEN_FINAL (:7987); its leftpair is the
// next pair of the list (path->first after the pop), its rightpair the
// previous one (pairs->first).  The reference dereferences NULL for an intron
// at either end of the list; that is -1 here.
extern "C" int gsnapdp_path_introns(const gsnapdp_path_pair* pairs, int npairs, int nullgap, int path,
                                    gsnapdp_intron* out, int cap) {
  constexpr int EXTRAQUERYGAP = 10;        // stage3.h:29
  constexpr int MININTRONLEN_FINAL = 50;   // stage3.c:52
  if (npairs < 0 || (npairs > 0 && !pairs)) return -1;
  int n = 0;
  for (int i = 0; i < npairs; i++) {
    const gsnapdp_path_pair& p = pairs[i];
    if (!p.gapp || p.queryjump > nullgap || p.queryjump > p.genomejump + EXTRAQUERYGAP) continue;
    if (p.genomejump > p.queryjump + MININTRONLEN_FINAL) {
      if (i == 0 || i + 1 >= npairs) return -1;
      if (n < cap && out) {
        gsnapdp_intron& x = out[n];
        x.left_genomepos = pairs[i + 1].genomepos;
        x.right_genomepos = pairs[i - 1].genomepos;
        x.path = path;
        x.comp = p.comp;
        x.knowngapp = p.knowngapp;
        x.known_donor = x.known_acceptor = 0;
      }
      n++;
    }
  }
  return n;
}

