/*
 * dp_oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).
 *
 * Clean-room C restatement of the stage-3 gap DP of GMAP/GSNAP 2012-07-03.
 * Each function cites the reference lines (src/dynprog.c unless noted) whose
 * behaviour it restates.  The product library never links this file.
 */
#define _GNU_SOURCE
#include "dp_oracle.h"

#include <ctype.h>
#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define NEG_INF (-1000000) /* dynprog.c:119 (non-DEBUG2 build) */

/* Mismatchtype_T, dynprog.c:150 */
enum { MT_HIGHQ = 0, MT_MEDQ = 1, MT_LOWQ = 2, MT_ENDQ = 3 };

/* Direction_T values, dynprog.c:308-312 */
#define D_STOP 0
#define D_DIAG 1
#define D_HORIZ 2
#define D_VERT 4

/* Scoring constants, dynprog.c:142-293 */
#define FULLMATCH 3
#define HALFMATCH 1
#define AMBIGUOUS (-1)
#define MICROINTRON_LENGTH 9
static const int mismatch_score[4] = {-3, -2, -1, -5}; /* :169-179 */
#define SINGLE_OPEN (-10)
#define SINGLE_EXTEND (-3)
#define PAIRED_OPEN (-18)
#define PAIRED_EXTEND (-3)
#define END_OPEN (-12)
#define END_EXTEND (-1)
static const int canonical_reward_tab[3] = {10, 16, 22};       /* :277-279 */
static const int final_canonical_reward_tab[3] = {30, 36, 42}; /* :281-283 */
#define GCAG_INTRON 15
#define ATAC_INTRON 12
#define FINAL_GCAG_INTRON 20
#define FINAL_ATAC_INTRON 12

/* intron.h:10-29 */
#define LEFT_GT 0x21
#define LEFT_GC 0x10
#define LEFT_AT 0x08
#define LEFT_CT 0x06
#define RIGHT_AG 0x30
#define RIGHT_AC 0x0C
#define RIGHT_GC 0x02
#define RIGHT_AT 0x01
#define GTAG_FWD 0x20
#define GCAG_FWD 0x10
#define ATAC_FWD 0x08
#define GTAG_REV 0x04
#define GCAG_REV 0x02
#define ATAC_REV 0x01
#define NONINTRON 0x00

/* ------------------------------------------------------------------ lists */

void orc_list_init(orc_list *l, int cap) {
  if (cap < 16) cap = 16;
  l->buf = (gsnapdp_pair *)malloc(sizeof(gsnapdp_pair) * (size_t)(2 * cap));
  l->cap = 2 * cap;
  l->head = cap;
  l->n = 0;
}

void orc_list_free(orc_list *l) {
  free(l->buf);
  l->buf = NULL;
}

void orc_list_clear(orc_list *l) {
  l->head = l->cap / 2;
  l->n = 0;
}

static void list_grow(orc_list *l) {
  int newcap = l->cap * 2;
  gsnapdp_pair *nb = (gsnapdp_pair *)malloc(sizeof(gsnapdp_pair) * (size_t)newcap);
  int newhead = newcap / 2 - l->n / 2;
  memcpy(nb + newhead, l->buf + l->head, sizeof(gsnapdp_pair) * (size_t)l->n);
  free(l->buf);
  l->buf = nb;
  l->cap = newcap;
  l->head = newhead;
}

/* Pairpool_push (pairpool.c:169-235): new cell becomes the list head. */
static void push_pair(orc_list *l, int querypos, int genomepos, char cdna, char comp, char genome,
                      int dynprogindex) {
  gsnapdp_pair *p;
  if (l->head == 0) list_grow(l);
  p = &l->buf[--l->head];
  l->n++;
  p->querypos = querypos;
  p->genomepos = genomepos;
  p->queryjump = 0;
  p->genomejump = 0;
  p->dynprogindex = dynprogindex;
  p->cdna = cdna;
  p->comp = comp;
  p->genome = genome;
  p->gapp = 0;
}

/* Pairpool_push_gapholder (pairpool.c:352-400); gapp bit 1 = knowngapp (:383). */
static void push_gapholder_k(orc_list *l, int queryjump, int genomejump, int knownp);
static void push_gapholder(orc_list *l, int queryjump, int genomejump) {
  push_gapholder_k(l, queryjump, genomejump, 0);
}
static void push_gapholder_k(orc_list *l, int queryjump, int genomejump, int knownp) {
  gsnapdp_pair *p;
  if (l->head == 0) list_grow(l);
  p = &l->buf[--l->head];
  l->n++;
  p->querypos = -1;
  p->genomepos = -1;
  p->queryjump = queryjump;
  p->genomejump = genomejump;
  p->dynprogindex = 0;
  p->cdna = ' ';
  p->comp = ' ';
  p->genome = ' ';
  p->gapp = knownp ? 3 : 1;
}

/* List_reverse */
static void list_reverse(orc_list *l) {
  int i = l->head, j = l->head + l->n - 1;
  while (i < j) {
    gsnapdp_pair t = l->buf[i];
    l->buf[i] = l->buf[j];
    l->buf[j] = t;
    i++;
    j--;
  }
}

/* ------------------------------------------------------- substitution tables */

static int pd[4][128][128];
static unsigned char cons[128][128];

static void mark(int a, int b, int score, int both_orders) {
  /* permute_cases / permute_cases_oneway (dynprog.c:1053-1124): all
   * upper/lower combinations of (a,b) (and of (b,a) when both_orders). */
  int la = tolower(a), lb = tolower(b);
  int xs[2] = {a, la}, ys[2] = {b, lb};
  int i, j, t;
  for (i = 0; i < 2; i++)
    for (j = 0; j < 2; j++) {
      cons[xs[i]][ys[j]] = 1;
      for (t = 0; t < 4; t++) pd[t][xs[i]][ys[j]] = score;
      if (both_orders) {
        cons[ys[j]][xs[i]] = 1;
        for (t = 0; t < 4; t++) pd[t][ys[j]][xs[i]] = score;
      }
    }
}

void orc_init(int mode) {
  /* pairdistance_init (dynprog.c:1127-1226) */
  static const struct { char code; const char *bases; int score; } amb[] = {
      {'R', "AG", HALFMATCH},  {'Y', "TC", HALFMATCH},  {'W', "AT", HALFMATCH},
      {'S', "GC", HALFMATCH},  {'M', "AC", HALFMATCH},  {'K', "GT", HALFMATCH},
      {'H', "ATC", AMBIGUOUS}, {'B', "GCT", AMBIGUOUS}, {'V', "GAC", AMBIGUOUS},
      {'D', "GAT", AMBIGUOUS}, {'N', "TCAG", AMBIGUOUS}, {'X', "TCAG", AMBIGUOUS}};
  int c1, c2, t, k;
  const char *p;
  memset(pd, 0, sizeof(pd));
  memset(cons, 0, sizeof(cons));
  /* mismatch fill: c1 in [A,z], c2 in [A,z) (dynprog.c:1150-1151) */
  for (c1 = 'A'; c1 <= 'z'; c1++)
    for (c2 = 'A'; c2 < 'z'; c2++)
      for (t = 0; t < 4; t++) pd[t][c1][c2] = mismatch_score[t];
  mark('U', 'T', FULLMATCH, 1);
  for (k = 0; k < (int)(sizeof(amb) / sizeof(amb[0])); k++)
    for (p = amb[k].bases; *p; p++) mark(amb[k].code, *p, amb[k].score, 1);
  if (mode == GSNAPDP_MODE_CMET_STRANDED || mode == GSNAPDP_MODE_CMET_NONSTRANDED) {
    mark('T', 'C', FULLMATCH, 0); /* :1215-1219 */
    mark('A', 'G', FULLMATCH, 0);
  }
  for (c1 = 'A'; c1 < 'Z'; c1++) mark(c1, c1, FULLMATCH, 1); /* :1221-1223 */
}

int orc_pairdistance(int mt, int c1, int c2) { return pd[mt][c1 & 127][c2 & 127]; }
int orc_consistent(int c1, int c2) { return cons[c1 & 127][c2 & 127]; }

int orc_score(int matches, int mismatches, int qopens, int qindels, int topens, int tindels,
              double defect_rate) {
  /* Dynprog_score (dynprog.c:380-394); open/extend are equal for all bins */
  int mm = defect_rate < 0.003 ? -3 : defect_rate < 0.014 ? -2 : -1;
  return FULLMATCH * matches + mm * mismatches + SINGLE_OPEN * qopens + SINGLE_EXTEND * qindels +
         SINGLE_OPEN * topens + SINGLE_EXTEND * tindels;
}

/* ------------------------------------------------------------------ genome */

static const uint32_t *g_blocks;

void orc_set_genome(const uint32_t *blocks) { g_blocks = blocks; }
const uint32_t *orc_genome_blocks(void) { return g_blocks; }

static char block_char(uint32_t pos) {
  /* uncompress_one_char (genome.c:9325-9360) */
  uint32_t base = pos / 32u * 3u;
  int bit = (int)(pos % 32u);
  if (g_blocks[base + 2] & (1u << bit)) return 'N';
  if (bit < 16) return "ACGT"[(g_blocks[base + 1] >> (2 * bit)) & 3u];
  return "ACGT"[(g_blocks[base] >> (2 * bit - 32)) & 3u];
}

static char compl_char(char c) {
  /* complCode (dynprog.c:401, complement.h) restricted to what the packed
   * genome can produce */
  switch (c) {
    case 'A': return 'T';
    case 'C': return 'G';
    case 'G': return 'C';
    case 'T': return 'A';
    default: return 'N';
  }
}

char orc_get_genomic_nt(int genomicpos, uint32_t chroffset, uint32_t chrhigh, uint32_t chrpos,
                        int genomiclength, int watsonp) {
  /* get_genomic_nt (dynprog.c:403-441) */
  uint32_t pos;
  if (genomicpos < 0) return '*';
  if (genomicpos >= genomiclength) return '*';
  pos = chroffset + chrpos;
  if (pos < chroffset) return '*';
  if (pos >= chrhigh) return '*';
  if (watsonp) return block_char(chroffset + chrpos + (uint32_t)genomicpos);
  return compl_char(block_char(chroffset + chrpos + (uint32_t)(genomiclength - 1) - (uint32_t)genomicpos));
}

typedef struct gpar {
  uint32_t chroffset, chrhigh, chrpos;
  int genomiclength;
  int watsonp;
} gpar;

static inline char gnt(const gpar *g, int pos) {
  return orc_get_genomic_nt(pos, g->chroffset, g->chrhigh, g->chrpos, g->genomiclength, g->watsonp);
}

/* --------------------------------------------------------------- workspace */

/* Each thread keeps its last few workspaces: a batch driver makes one per call,
 * and every fill clears the rectangle it uses (:352-357, as Matrix3_alloc's
 * callers do), so a reused allocation behaves as a fresh one; allocating and
 * unmapping ~18 MB per call serialised the threads of a multi-threaded caller. */
#define ORC_DP_CACHE 4
static __thread orc_dp *dp_cache[ORC_DP_CACHE];

orc_dp *orc_dp_new(int maxlookback, int extraquerygap, int maxpeelback, int extramaterial_end,
                   int extramaterial_paired) {
  /* compute_maxlengths + Dynprog_new (dynprog.c:831-873) */
  orc_dp *dp;
  size_t cells;
  int m1 = maxlookback + maxpeelback, m2, i;
  if (m1 < 500) m1 = 500;
  m2 = m1 + extraquerygap + (extramaterial_end > extramaterial_paired ? extramaterial_end : extramaterial_paired);
  if (m2 < 2000) m2 = 2000;
  for (i = 0; i < ORC_DP_CACHE; i++)
    if (dp_cache[i] && dp_cache[i]->alloc1 == m1 && dp_cache[i]->alloc2 == m2) {
      dp = dp_cache[i];
      dp_cache[i] = NULL;
      dp->maxlength1 = m1;
      dp->maxlength2 = m2;
      return dp;
    }
  dp = (orc_dp *)calloc(1, sizeof(orc_dp));
  dp->maxlength1 = dp->alloc1 = m1;
  dp->maxlength2 = dp->alloc2 = m2;
  cells = (size_t)(dp->maxlength1 + 1) * (size_t)(dp->maxlength2 + 1);
  dp->nogap = (int32_t *)calloc(cells, 4);
  dp->gap1 = (int32_t *)calloc(cells, 4);
  dp->gap2 = (int32_t *)calloc(cells, 4);
  dp->dnogap = (uint8_t *)calloc(cells, 1);
  dp->dgap1 = (uint8_t *)calloc(cells, 1);
  dp->dgap2 = (uint8_t *)calloc(cells, 1);
  return dp;
}

void orc_dp_free(orc_dp *dp) {
  int i;
  if (!dp) return;
  for (i = 0; i < ORC_DP_CACHE; i++)
    if (!dp_cache[i]) {
      dp_cache[i] = dp;
      return;
    }
  free(dp->nogap);
  free(dp->gap1);
  free(dp->gap2);
  free(dp->dnogap);
  free(dp->dgap1);
  free(dp->dgap2);
  free(dp);
}

/* A filled matrix view: row stride = length2+1 like Matrix3_alloc (:490). */
typedef struct mview {
  int L1, L2, stride;
  int32_t *H, *E, *F;       /* nogap, gap1, gap2 */
  uint8_t *dH, *dE, *dF;
} mview;

#define IX(m, r, c) ((size_t)(r) * (size_t)(m)->stride + (size_t)(c))

static void band_widths(int L1, int L2, int extraband, int widebandp, int *lband, int *rband) {
  /* dynprog.c:1442-1454 */
  if (!widebandp) {
    *lband = extraband;
    *rband = extraband;
  } else if (L2 >= L1) {
    *rband = L2 - L1 + extraband;
    *lband = extraband;
  } else {
    *lband = L1 - L2 + extraband;
    *rband = extraband;
  }
}

/* compute_scores_lookup_fwd / _rev (dynprog.c:1424-1578 / 1581-1736).
 * rev: query read as seq1[1-r] and genome at offset2+1-c. */
static void fill_seg(mview *m, orc_dp *dp, const char *seq1, int rev, int offset2, int L1, int L2,
                     const gpar *g, const char *seq2, int mt, int open, int extend, int extraband,
                     int widebandp, int jump_late_p);
static void fill(mview *m, orc_dp *dp, const char *seq1, int rev, int offset2, int L1, int L2,
                 const gpar *g, int mt, int open, int extend, int extraband, int widebandp,
                 int jump_late_p) {
  fill_seg(m, dp, seq1, rev, offset2, L1, L2, g, NULL, mt, open, extend, extraband, widebandp,
           jump_late_p);
}

/* seq2 != NULL: use_genomicseg_p, the genome of column c is seq2[c-1] (fwd) or
 * seq2[1-c] (rev) (:1535 / :1690) */
static void fill_seg(mview *m, orc_dp *dp, const char *seq1, int rev, int offset2, int L1, int L2,
                     const gpar *g, const char *seq2, int mt, int open, int extend, int extraband,
                     int widebandp, int jump_late_p) {
  int lband, rband, r, c, rlo, rhigh, penalty;
  size_t cells = (size_t)(L1 + 1) * (size_t)(L2 + 1);
  int32_t *H = dp->nogap, *E = dp->gap1, *F = dp->gap2;
  uint8_t *dH = dp->dnogap, *dE = dp->dgap1, *dF = dp->dgap2;
  int stride = L2 + 1;
  int(*tab)[128] = pd[mt];

  if (L1 <= 0 || L2 <= 0) {
    fprintf(stderr, "dynprog: lengths are negative: %d %d\n", L1, L2);
    abort(); /* Matrix3_alloc :495-498 */
  }
  m->L1 = L1;
  m->L2 = L2;
  m->stride = stride;
  m->H = H;
  m->E = E;
  m->F = F;
  m->dH = dH;
  m->dE = dE;
  m->dF = dF;
  band_widths(L1, L2, extraband, widebandp, &lband, &rband);

  /* the whole rectangle is cleared per call (:518, :669) */
  memset(H, 0, cells * 4);
  memset(E, 0, cells * 4);
  memset(F, 0, cells * 4);
  memset(dH, 0, cells);
  memset(dE, 0, cells);
  memset(dF, 0, cells);

  H[0] = 0;
  dH[0] = D_STOP;
  E[0] = F[0] = NEG_INF;
  penalty = open;
  for (c = 1; c <= rband && c <= L2; c++) { /* row 0 */
    penalty += extend;
    H[c] = NEG_INF;
    E[c] = penalty;
    dE[c] = D_HORIZ;
    F[c] = NEG_INF;
  }
  dE[1] = D_STOP; /* (*directions)[0][1].gap1 = STOP, written even if L2 == 0 */
  penalty = open;
  for (r = 1; r <= lband && r <= L1; r++) { /* column 0 */
    size_t i = (size_t)r * stride;
    penalty += extend;
    H[i] = NEG_INF;
    E[i] = NEG_INF;
    F[i] = penalty;
    dF[i] = D_VERT;
  }
  dF[(size_t)stride] = D_STOP; /* (*directions)[1][0].gap2 = STOP */

  for (c = 1; c <= L2; c++) {
    int na2 = (unsigned char)(seq2 ? (rev ? seq2[1 - c] : seq2[c - 1])
                                   : gnt(g, rev ? offset2 + 1 - c : offset2 + c - 1)) & 127;
    if ((rlo = c - rband) < 1) {
      rlo = 1;
    } else {
      size_t i = (size_t)(rlo - 1) * stride + c;
      F[i] = NEG_INF;
      H[i] = NEG_INF;
    }
    if ((rhigh = c + lband) > L1) {
      rhigh = L1;
    } else {
      size_t i = (size_t)rhigh * stride + (c - 1);
      E[i] = NEG_INF;
      H[i] = NEG_INF;
    }
    for (r = rlo; r <= rhigh; r++) {
      size_t i = (size_t)r * stride + c;
      size_t il = i - 1, iu = i - stride, id = i - stride - 1;
      int na1 = (unsigned char)(rev ? seq1[1 - r] : seq1[r - 1]) & 127;
      int best, s;
      uint8_t dir;

      best = H[il] + open; /* gap1 */
      dir = D_DIAG;
      s = E[il];
      if (s > best || (s == best && jump_late_p)) {
        best = s;
        dir = D_HORIZ;
      }
      E[i] = best + extend;
      dE[i] = dir;

      best = H[iu] + open; /* gap2 */
      dir = D_DIAG;
      s = F[iu];
      if (s > best || (s == best && jump_late_p)) {
        best = s;
        dir = D_VERT;
      }
      F[i] = best + extend;
      dF[i] = dir;

      best = H[id]; /* nogap */
      dir = D_DIAG;
      s = E[id];
      if (s > best || (s == best && jump_late_p)) {
        best = s;
        dir = D_HORIZ;
      }
      s = F[id];
      if (s > best || (s == best && jump_late_p)) {
        best = s;
        dir = D_VERT;
      }
      H[i] = best + tab[na1][na2];
      dH[i] = dir;
    }
  }
}

/* Intron_type (intron.c:18-180, non-PMAP, no INTRON_HELP) */
static int intron_type(char left1, char left2, char right2, char right1, int cdna_direction) {
  int leftdi, rightdi, t;
  if (left1 == 'G' && left2 == 'T') leftdi = LEFT_GT;
  else if (left1 == 'G' && left2 == 'C') leftdi = LEFT_GC;
  else if (left1 == 'A' && left2 == 'T') leftdi = LEFT_AT;
  else if (left1 == 'C' && left2 == 'T') leftdi = LEFT_CT;
  else return NONINTRON;
  if (right2 == 'A' && right1 == 'G') rightdi = RIGHT_AG;
  else if (right2 == 'A' && right1 == 'C') rightdi = RIGHT_AC;
  else if (right2 == 'G' && right1 == 'C') rightdi = RIGHT_GC;
  else if (right2 == 'A' && right1 == 'T') rightdi = RIGHT_AT;
  else return NONINTRON;
  if ((t = leftdi & rightdi) == 0) return NONINTRON;
  if (cdna_direction > 0) return t < 0x08 ? NONINTRON : t;
  if (cdna_direction < 0) return t > 0x04 ? NONINTRON : t;
  return NONINTRON;
}

typedef struct counts {
  int nmatches, nmismatches, nopens, nindels;
} counts;

/* add_queryskip (dynprog.c:2372-2413), cdna_gap_p == false */
static void add_queryskip(orc_list *l, int r, int c, int dist, const char *qseq, int qoff, int goff,
                          int rev, int dpi) {
  int j, qc = r - 1, gc = c - 1, step;
  if (rev) {
    qc = -qc;
    gc = -gc;
    step = +1;
  } else {
    gc++;
    step = -1;
  }
  for (j = 0; j < dist; j++) {
    push_pair(l, qoff + qc, goff + gc, qseq[qc], '-', ' ', dpi);
    qc += step;
  }
}

/* add_genomeskip (dynprog.c:2416-2512), use_genomicseg_p == false.
 * Returns 1 if dashes were added (counted as an indel). */
static int add_genomeskip(orc_list *l, int r, int c, int dist, int qoff, int goff, int rev,
                          const gpar *g, int cdna_direction, int dpi) {
  int j, qc = r - 1, left = c - dist, right = c - 1, gc, step, dashes;
  if (rev) {
    int t = left;
    qc = -qc;
    left = -right;
    right = -t;
    step = +1;
  } else {
    qc++;
    step = -1;
  }
  if (dist < MICROINTRON_LENGTH) {
    dashes = 1;
  } else {
    char l1 = gnt(g, goff + left), l2 = gnt(g, goff + left + 1);
    char r2 = gnt(g, goff + right - 1), r1 = gnt(g, goff + right);
    dashes = intron_type(l1, l2, r2, r1, cdna_direction) == NONINTRON;
  }
  if (dashes) {
    gc = rev ? left : right;
    for (j = 0; j < dist; j++) {
      push_pair(l, qoff + qc, goff + gc, ' ', '-', gnt(g, goff + gc), dpi);
      gc += step;
    }
  } else {
    push_gapholder(l, GSNAPDP_UNKNOWNJUMP, GSNAPDP_UNKNOWNJUMP);
  }
  return dashes;
}

/* traceback (dynprog.c:2611-2712), use_genomicseg_p == false */
static void traceback(orc_list *l, counts *k, const mview *m, int r, int c, const char *qseq,
                      const char *qseq_uc, int qoff, int goff, int rev, const gpar *g,
                      int cdna_direction, int dpi) {
  while (m->dH[IX(m, r, c)] != D_STOP) {
    int qc = r - 1, gc = c - 1, dist;
    char c1, c2;
    uint8_t d;
    if (rev) {
      qc = -qc;
      gc = -gc;
    }
    c1 = qseq[qc];
    c2 = gnt(g, goff + gc);
    if (c2 == '*') {
      /* no pair past the chromosome end */
    } else if (qseq_uc[qc] == c2) {
      k->nmatches++;
      push_pair(l, qoff + qc, goff + gc, c1, '*', c2, dpi);
    } else if (cons[c1 & 127][c2 & 127]) {
      k->nmatches++;
      push_pair(l, qoff + qc, goff + gc, c1, ':', c2, dpi);
    } else {
      k->nmismatches++;
      push_pair(l, qoff + qc, goff + gc, c1, ' ', c2, dpi);
    }
    d = m->dH[IX(m, r, c)];
    if (d == D_DIAG) {
      r--;
      c--;
    } else if (d == D_HORIZ) {
      dist = 1;
      r--;
      c--;
      while (m->dE[IX(m, r, c)] == D_HORIZ) {
        dist++;
        c--;
      }
      c--;
      if (add_genomeskip(l, r, c + dist, dist, qoff, goff, rev, g, cdna_direction, dpi)) {
        k->nopens++;
        k->nindels += dist;
      }
    } else {
      dist = 1;
      r--;
      c--;
      while (m->dF[IX(m, r, c)] == D_VERT) {
        dist++;
        r--;
      }
      r--;
      add_queryskip(l, r + dist, c, dist, qseq, qoff, goff, rev, dpi);
      k->nopens++;
      k->nindels += dist;
    }
  }
}

/* traceback_nogaps (dynprog.c:2815-2872) */
static void traceback_nogaps(orc_list *l, counts *k, int r, int c, const char *qseq,
                             const char *qseq_uc, int qoff, int goff, int rev, const gpar *g,
                             int dpi) {
  while (r > 0 && c > 0) {
    int qc = r - 1, gc = c - 1;
    char c1, c2;
    if (rev) {
      qc = -qc;
      gc = -gc;
    }
    c1 = qseq[qc];
    c2 = gnt(g, goff + gc);
    if (c2 == '*') {
    } else if (qseq_uc[qc] == c2) {
      k->nmatches++;
      push_pair(l, qoff + qc, goff + gc, c1, '*', c2, dpi);
    } else if (cons[c1 & 127][c2 & 127]) {
      k->nmatches++;
      push_pair(l, qoff + qc, goff + gc, c1, ':', c2, dpi);
    } else {
      k->nmismatches++;
      push_pair(l, qoff + qc, goff + gc, c1, ' ', c2, dpi);
    }
    r--;
    c--;
  }
}

/* find_best_endpoint (dynprog.c:2235-2290): unwidened band, row-major scan */
static void best_endpoint(int *score, int *br, int *bc, const mview *m, int L1, int L2, int band,
                          int jump_late_p) {
  int best = 0, r, c;
  *br = *bc = 0;
  for (r = 1; r <= L1; r++) {
    int clo = r - band, chigh = r + band;
    if (clo < 1) clo = 1;
    if (chigh > L2) chigh = L2;
    for (c = clo; c <= chigh; c++) {
      int s = m->H[IX(m, r, c)];
      if (s > best || (jump_late_p && s == best)) {
        *br = r;
        *bc = c;
        best = s;
      }
    }
  }
  *score = best;
}

/* find_best_endpoint_to_queryend_indels (dynprog.c:2293-2355) */
static void best_endpoint_indels(int *score, int *br, int *bc, const mview *m, int L1, int L2,
                                 int band, int jump_late_p) {
  int best = NEG_INF, lband, rband, clo, chigh, c, r = L1;
  if (L2 >= L1) {
    rband = L2 - L1 + band;
    lband = band;
  } else {
    lband = L1 - L2 + band;
    rband = band;
  }
  *br = L1;
  *bc = 0;
  clo = r - lband;
  chigh = r + rband;
  if (clo < 1) clo = 1;
  if (chigh > L2) chigh = L2;
  for (c = clo; c <= chigh; c++) {
    int s = m->H[IX(m, r, c)];
    if (s > best || (jump_late_p && s == best)) {
      *br = r;
      *bc = c;
      best = s;
    }
  }
  *score = best;
}

static void quality(double defect_rate, int *mt) {
  *mt = defect_rate < 0.003 ? MT_HIGHQ : defect_rate < 0.014 ? MT_MEDQ : MT_LOWQ;
}

static inline int step_index(int dpi) { return dpi + (dpi > 0 ? +1 : -1); }

/* Dynprog_single_gap (dynprog.c:4450-4572) */
void orc_single_gap(orc_list *out, int *dynprogindex, int *finalscore, int *nmatches,
                    int *nmismatches, int *nopens, int *nindels, orc_dp *dp,
                    const char *sequence1, const char *sequenceuc1, int length1, int length2,
                    int offset1, int offset2, uint32_t chroffset, uint32_t chrhigh,
                    uint32_t chrpos, uint32_t genomiclength, int cdna_direction, int watsonp,
                    int jump_late_p, int extraband_single, double defect_rate,
                    int close_indels_mode, int widebandp) {
  int mt;
  mview m;
  counts k = {0, 0, 0, 0};
  gpar g = {chroffset, chrhigh, chrpos, (int)genomiclength, watsonp};
  (void)close_indels_mode; /* only feeds onesidegapp, which no fill reads */
  orc_list_clear(out);
  quality(defect_rate, &mt);
  if (length1 > dp->maxlength1 || length2 > dp->maxlength2) { /* :4509-4519 */
    *finalscore = -10000;
    *nmatches = *nmismatches = *nopens = *nindels = 0;
    *dynprogindex = step_index(*dynprogindex);
    return;
  }
  fill(&m, dp, sequence1, 0, offset2, length1, length2, &g, mt, SINGLE_OPEN, SINGLE_EXTEND,
       extraband_single, widebandp, jump_late_p);
  *finalscore = m.H[IX(&m, length1, length2)];
  traceback(out, &k, &m, length1, length2, sequence1, sequenceuc1, offset1, offset2, 0, &g,
            cdna_direction, *dynprogindex);
  *nmatches = k.nmatches;
  *nmismatches = k.nmismatches;
  *nopens = k.nopens;
  *nindels = k.nindels;
  *dynprogindex = step_index(*dynprogindex);
  list_reverse(out);
}

/* shared body of Dynprog_end5_gap (:5094-5284) and Dynprog_end3_gap (:5556-5741) */
static void end_gap(orc_list *out, int rev, int *dynprogindex, int *finalscore, int *nmatches,
                    int *nmismatches, int *nopens, int *nindels, orc_dp *dp, const char *seq1,
                    const char *seq1uc, int length1, int length2, int off1, int off2,
                    uint32_t chroffset, uint32_t chrhigh, uint32_t chrpos, uint32_t genomiclength,
                    int cdna_direction, int watsonp, int jump_late_p, int extraband_end,
                    int endalign) {
  mview m;
  counts k = {0, 0, 0, 0};
  gpar g = {chroffset, chrhigh, chrpos, (int)genomiclength, watsonp};
  int bestr, bestc, jl = rev ? !jump_late_p : jump_late_p;
  orc_list_clear(out);
  if (length1 <= 0) {
    *nmatches = *nmismatches = *nopens = *nindels = 0;
    *finalscore = 0;
    return;
  } else if (endalign != GSNAPDP_QUERYEND_NOGAPS && length1 > dp->maxlength1) {
    length1 = dp->maxlength1;
  }
  if (length2 <= 0) {
    *nmatches = *nmismatches = *nopens = *nindels = 0;
    *finalscore = 0;
    return;
  } else if (endalign != GSNAPDP_QUERYEND_NOGAPS && length2 > dp->maxlength2) {
    length2 = dp->maxlength2;
  }
  if (endalign == GSNAPDP_QUERYEND_GAP || endalign == GSNAPDP_BEST_LOCAL) {
    fill(&m, dp, seq1, rev, off2, length1, length2, &g, MT_ENDQ, END_OPEN, END_EXTEND,
         extraband_end, 1, jl);
    best_endpoint(finalscore, &bestr, &bestc, &m, length1, length2, extraband_end, jl);
  } else if (endalign == GSNAPDP_QUERYEND_INDELS) {
    fill(&m, dp, seq1, rev, off2, length1, length2, &g, MT_ENDQ, END_OPEN, END_EXTEND,
         extraband_end, 1, jl);
    best_endpoint_indels(finalscore, &bestr, &bestc, &m, length1, length2, extraband_end, jl);
  } else if (endalign == GSNAPDP_QUERYEND_NOGAPS) {
    bestr = bestc = length2 < length1 ? length2 : length1; /* :2358-2369 */
  } else {
    fprintf(stderr, "Unexpected endalign value %d\n", endalign);
    abort();
  }
  if (endalign == GSNAPDP_QUERYEND_NOGAPS) {
    traceback_nogaps(out, &k, bestr, bestc, seq1, seq1uc, off1, off2, rev, &g, *dynprogindex);
    *finalscore = k.nmatches * FULLMATCH + k.nmismatches * mismatch_score[MT_ENDQ];
  } else {
    traceback(out, &k, &m, bestr, bestc, seq1, seq1uc, off1, off2, rev, &g, cdna_direction,
              *dynprogindex);
  }
  *nmatches = k.nmatches;
  *nmismatches = k.nmismatches;
  *nopens = k.nopens;
  *nindels = k.nindels;
  if ((endalign == GSNAPDP_QUERYEND_GAP || endalign == GSNAPDP_BEST_LOCAL) &&
      k.nmatches + 1 < k.nmismatches) {
    *finalscore = 0;
    orc_list_clear(out);
  } else {
    list_reverse(out);
    while (out->n > 0 && out->buf[out->head].comp == '-') { /* strip INDEL_COMP */
      out->head++;
      out->n--;
    }
  }
  *dynprogindex = step_index(*dynprogindex);
  if (rev) list_reverse(out); /* end5 returns List_reverse(pairs); end3 does not */
}

void orc_end5_gap(orc_list *out, int *dynprogindex, int *finalscore, int *nmatches,
                  int *nmismatches, int *nopens, int *nindels, orc_dp *dp,
                  const char *revsequence1, const char *revsequenceuc1, int length1, int length2,
                  int revoffset1, int revoffset2, uint32_t chroffset, uint32_t chrhigh,
                  uint32_t chrpos, uint32_t genomiclength, int cdna_direction, int watsonp,
                  int jump_late_p, int extraband_end, double defect_rate, int endalign) {
  (void)defect_rate; /* END open/extend are equal for all bins (:5128-5137) */
  end_gap(out, 1, dynprogindex, finalscore, nmatches, nmismatches, nopens, nindels, dp,
          revsequence1, revsequenceuc1, length1, length2, revoffset1, revoffset2, chroffset,
          chrhigh, chrpos, genomiclength, cdna_direction, watsonp, jump_late_p, extraband_end,
          endalign);
}

void orc_end3_gap(orc_list *out, int *dynprogindex, int *finalscore, int *nmatches,
                  int *nmismatches, int *nopens, int *nindels, orc_dp *dp,
                  const char *sequence1, const char *sequenceuc1, int length1, int length2,
                  int offset1, int offset2, uint32_t chroffset, uint32_t chrhigh,
                  uint32_t chrpos, uint32_t genomiclength, int cdna_direction, int watsonp,
                  int jump_late_p, int extraband_end, double defect_rate, int endalign) {
  (void)defect_rate;
  end_gap(out, 0, dynprogindex, finalscore, nmatches, nmismatches, nopens, nindels, dp,
          sequence1, sequenceuc1, length1, length2, offset1, offset2, chroffset, chrhigh, chrpos,
          genomiclength, cdna_direction, watsonp, jump_late_p, extraband_end, endalign);
}

/* ------------------------------------------------- splice-junction ends */

/* add_genomeskip (dynprog.c:2416-2512) with use_genomicseg_p: the intron test
 * reads gseq_uc, the dashes gseq (window coordinates, rev-indexed like the query). */
static int add_genomeskip_seg(orc_list *l, int r, int c, int dist, int qoff, int goff, int rev,
                              const char *gseq, const char *gseq_uc, int cdna_direction, int dpi) {
  int j, qc = r - 1, left = c - dist, right = c - 1, gc, step, dashes;
  if (rev) {
    int t = left;
    qc = -qc;
    left = -right;
    right = -t;
    step = +1;
  } else {
    qc++;
    step = -1;
  }
  if (dist < MICROINTRON_LENGTH) {
    dashes = 1;
  } else {
    dashes = intron_type(gseq_uc[left], gseq_uc[left + 1], gseq_uc[right - 1], gseq_uc[right],
                         cdna_direction) == NONINTRON;
  }
  if (dashes) {
    gc = rev ? left : right;
    for (j = 0; j < dist; j++) {
      push_pair(l, qoff + qc, goff + gc, ' ', '-', gseq[gc], dpi);
      gc += step;
    }
  } else {
    push_gapholder(l, GSNAPDP_UNKNOWNJUMP, GSNAPDP_UNKNOWNJUMP);
  }
  return dashes;
}

/* traceback_local (dynprog.c:2874-2968): runs while *c > endc, leaves (*r,*c)
 * where it stopped; genome chars from the segment, every diagonal cell pushes. */
static void traceback_local(orc_list *l, counts *k, const mview *m, int *pr, int *pc, int endc,
                            const char *qseq, const char *qseq_uc, const char *gseq,
                            const char *gseq_uc, int qoff, int goff, int rev, int cdna_direction,
                            int dpi) {
  int r = *pr, c = *pc;
  while (c > endc) {
    int qc = r - 1, gc = c - 1, dist;
    char c1, c2;
    uint8_t d;
    if (rev) {
      qc = -qc;
      gc = -gc;
    }
    c1 = qseq[qc];
    c2 = gseq[gc];
    if (qseq_uc[qc] == c2) {
      k->nmatches++;
      push_pair(l, qoff + qc, goff + gc, c1, '*', c2, dpi);
    } else if (cons[c1 & 127][c2 & 127]) {
      k->nmatches++;
      push_pair(l, qoff + qc, goff + gc, c1, ':', c2, dpi);
    } else {
      k->nmismatches++;
      push_pair(l, qoff + qc, goff + gc, c1, ' ', c2, dpi);
    }
    d = m->dH[IX(m, r, c)];
    if (d == D_DIAG) {
      r--;
      c--;
    } else if (d == D_HORIZ) {
      dist = 1;
      r--;
      c--;
      while (m->dE[IX(m, r, c)] == D_HORIZ) {
        dist++;
        c--;
      }
      c--;
      if (add_genomeskip_seg(l, r, c + dist, dist, qoff, goff, rev, gseq, gseq_uc, cdna_direction,
                             dpi)) {
        k->nopens++;
        k->nindels += dist;
      }
    } else {
      dist = 1;
      r--;
      c--;
      while (m->dF[IX(m, r, c)] == D_VERT) {
        dist++;
        r--;
      }
      r--;
      add_queryskip(l, r + dist, c, dist, qseq, qoff, goff, rev, dpi);
      k->nopens++;
      k->nindels += dist;
    }
  }
  *pr = r;
  *pc = c;
}

/* shared body of Dynprog_end5_splicejunction (:5412-5553, rev) and
 * Dynprog_end3_splicejunction (:5869-6057) */
static void end_splicejunction(orc_list *out, int rev, int *dynprogindex, int *finalscore,
                               int *nmatches, int *nmismatches, int *nopens, int *nindels,
                               orc_dp *dp, const char *seq1, const char *seq1uc, const char *seq2,
                               const char *seq2uc, int length1, int length2, int off1,
                               int off2_anchor, int off2_far, int cdna_direction,
                               int jump_late_p, int extraband_end, int contlength) {
  mview m;
  counts k = {0, 0, 0, 0};
  gpar g = {0, 0, 0, 0, 1};  /* never read: use_genomicseg_p */
  int bestr, bestc, jl = rev ? !jump_late_p : jump_late_p;
  orc_list_clear(out);
  if (length1 <= 0 || length1 > dp->maxlength1 || length2 <= 0 || length2 > dp->maxlength2) {
    *nmatches = *nmismatches = *nopens = *nindels = 0; /* :5446-5461 */
    *finalscore = 0;
    return;
  }
  fill_seg(&m, dp, seq1, rev, off2_anchor, length1, length2, &g, seq2, MT_ENDQ, END_OPEN,
           END_EXTEND, extraband_end, 1, jl);
  best_endpoint_indels(finalscore, &bestr, &bestc, &m, length1, length2, extraband_end, jl);
  traceback_local(out, &k, &m, &bestr, &bestc, contlength, seq1, seq1uc, seq2, seq2uc, off1,
                  off2_far, rev, cdna_direction, *dynprogindex);
  push_gapholder_k(out, 0, rev ? off2_anchor - off2_far : off2_far - off2_anchor, 1);
  traceback_local(out, &k, &m, &bestr, &bestc, 0, seq1, seq1uc, seq2, seq2uc, off1, off2_anchor,
                  rev, cdna_direction, *dynprogindex);
  *nmatches = k.nmatches;
  *nmismatches = k.nmismatches;
  *nopens = k.nopens;
  *nindels = k.nindels;
  *finalscore = k.nmatches * FULLMATCH + k.nmismatches * mismatch_score[MT_ENDQ] +
                k.nopens * END_OPEN + k.nindels * END_EXTEND; /* :5541 / :6045 */
  list_reverse(out);
  while (out->n > 0 && out->buf[out->head].comp == '-') { /* strip INDEL_COMP */
    out->head++;
    out->n--;
  }
  *dynprogindex = step_index(*dynprogindex);
  if (rev) list_reverse(out); /* end5 returns List_reverse(pairs); end3 does not */
}

void orc_end5_splicejunction(orc_list *out, int *dynprogindex, int *finalscore, int *nmatches,
                             int *nmismatches, int *nopens, int *nindels, orc_dp *dp,
                             const char *revsequence1, const char *revsequenceuc1,
                             const char *revsequence2, const char *revsequenceuc2, int length1,
                             int length2, int revoffset1, int revoffset2_anchor,
                             int revoffset2_far, int cdna_direction, int jump_late_p,
                             int extraband_end, double defect_rate, int contlength) {
  (void)defect_rate; /* END open/extend are equal for all bins (:5429-5438) */
  end_splicejunction(out, 1, dynprogindex, finalscore, nmatches, nmismatches, nopens, nindels, dp,
                     revsequence1, revsequenceuc1, revsequence2, revsequenceuc2, length1, length2,
                     revoffset1, revoffset2_anchor, revoffset2_far, cdna_direction, jump_late_p,
                     extraband_end, contlength);
}

void orc_end3_splicejunction(orc_list *out, int *dynprogindex, int *finalscore, int *nmatches,
                             int *nmismatches, int *nopens, int *nindels, orc_dp *dp,
                             const char *sequence1, const char *sequenceuc1, const char *sequence2,
                             const char *sequenceuc2, int length1, int length2, int offset1,
                             int offset2_anchor, int offset2_far, int cdna_direction,
                             int jump_late_p, int extraband_end, double defect_rate,
                             int contlength) {
  (void)defect_rate;
  end_splicejunction(out, 0, dynprogindex, finalscore, nmatches, nmismatches, nopens, nindels, dp,
                     sequence1, sequenceuc1, sequence2, sequenceuc2, length1, length2, offset1,
                     offset2_anchor, offset2_far, cdna_direction, jump_late_p, extraband_end,
                     contlength);
}

/* ------------------------------------------------------------- genome gap */

/* intron_score (dynprog.c:3148-3192), non-PMAP */
static int intron_score(int *introntype, int leftdi, int rightdi, int cdna_direction,
                        int canonical_reward, int finalp) {
  int t = leftdi & rightdi;
  int gcag = finalp ? FINAL_GCAG_INTRON : GCAG_INTRON;
  int atac = finalp ? FINAL_ATAC_INTRON : ATAC_INTRON;
  *introntype = t;
  if (t == NONINTRON) return 0;
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
  *introntype = NONINTRON;
  return 0;
}

/* Maxent_hr site probabilities for a left / right splice column
 * (get_splicesite_probs :3195-3287 and the probability precompute
 * :3856-3903, with no known sites). */
static double left_site_prob(int cL, int leftoffset, const gpar *g, int cdna_direction) {
  uint32_t pos;
  if (g->watsonp) {
    pos = g->chrpos + (uint32_t)leftoffset + (uint32_t)cL;
    return cdna_direction > 0 ? orc_maxent_donor(g->chroffset + pos, g->chroffset)
                              : orc_maxent_antiacceptor(g->chroffset + pos, g->chroffset);
  }
  pos = g->chrpos + (uint32_t)(g->genomiclength - 1) - (uint32_t)leftoffset - (uint32_t)cL + 1u;
  return cdna_direction > 0 ? orc_maxent_antidonor(g->chroffset + pos, g->chroffset)
                            : orc_maxent_acceptor(g->chroffset + pos, g->chroffset);
}

static double right_site_prob(int cR, int rightoffset, const gpar *g, int cdna_direction) {
  uint32_t pos;
  if (g->watsonp) {
    pos = g->chrpos + (uint32_t)rightoffset - (uint32_t)cR + 1u;
    return cdna_direction > 0 ? orc_maxent_acceptor(g->chroffset + pos, g->chroffset)
                              : orc_maxent_antidonor(g->chroffset + pos, g->chroffset);
  }
  pos = g->chrpos + (uint32_t)(g->genomiclength - 1) - (uint32_t)rightoffset + (uint32_t)cR;
  return cdna_direction > 0 ? orc_maxent_antiacceptor(g->chroffset + pos, g->chroffset)
                            : orc_maxent_donor(g->chroffset + pos, g->chroffset);
}

static inline int gapdir_penalty(uint8_t d) { return (d == D_HORIZ || d == D_VERT) ? 1 : 0; }

#define KNOWN_SPLICESITE_REWARD 20 /* dynprog.c:285 */

/* Known-site record of a window (include/gsnapdp.h, gsnapdp_ggap_window):
 * left_known[L2L], right_known[L2R] flags, then the KNOWN_INTRONS pair list. */
typedef struct {
  int mode;
  const unsigned char *rec;
  int L2L, L2R;
} known_t;

static int known_left(const known_t *k, int cL) { /* left_known[cL] (:3375-3550) */
  return (k->mode && cL >= 0 && cL < k->L2L && k->rec[cL]) ? KNOWN_SPLICESITE_REWARD : 0;
}
static int known_right(const known_t *k, int cR) {
  return (k->mode && cR >= 0 && cR < k->L2R && k->rec[k->L2L + cR]) ? KNOWN_SPLICESITE_REWARD : 0;
}
/* IIT_exists_with_divno_signed on the intron (cL, cR) (:3598-3612) */
static int known_intron(const known_t *k, int cL, int cR) {
  const unsigned char *p = k->rec + k->L2L + k->L2R;
  int n = p[0] | (p[1] << 8), i;
  for (i = 0; i < n; i++) {
    const unsigned char *e = p + 2 + 4 * i;
    if ((e[0] | (e[1] << 8)) == cL && (e[2] | (e[3] << 8)) == cR) return 1;
  }
  return 0;
}

/* bridge_intron_gap (dynprog.c:3290-4122).  k->mode selects the splicing-IIT
 * behaviour (include/gsnapdp.h GSNAPDP_KNOWN_*).
 * Returns 1 = accepted, 0 = rejected, -1 = probability mode found nothing
 * (the reference then reads uninitialised indices, :4055). */
static int bridge_intron(int *finalscore, int *brL, int *brR, int *bcL, int *bcR, int *best_type,
                         double *left_prob, double *right_prob, const mview *mL, const mview *mR,
                         int offset2L, int revoffset2R, int L1, int L2L, int L2R,
                         int cdna_direction, const gpar *g, int extraband_paired,
                         int canonical_reward, int leftoffset, int rightoffset, int halfp,
                         int finalp, int use_probabilities_p, int score_threshold,
                         const known_t *kn) {
  int bestscore = -100000, bestscoreI = -100000, scoreL, scoreR, scoreI, introntype;
  int rL, rR, cL, cR, cloL, chighL, cloR, chighR;
  int lbandL = extraband_paired, rbandL = L2L - L1 + extraband_paired;
  int lbandR = extraband_paired, rbandR = L2R - L1 + extraband_paired;
  int *leftdi = (int *)calloc((size_t)L2L + 1, sizeof(int));
  int *rightdi = (int *)calloc((size_t)L2R + 1, sizeof(int));
  int found = 0, result;

  for (cL = 0; cL < L2L - 1; cL++) { /* :3331-3351 */
    char a = gnt(g, offset2L + cL), b = gnt(g, offset2L + cL + 1);
    leftdi[cL] = (a == 'G' && b == 'T')   ? LEFT_GT
                 : (a == 'G' && b == 'C') ? LEFT_GC
                 : (a == 'A' && b == 'T') ? LEFT_AT
                 : (a == 'C' && b == 'T') ? LEFT_CT
                                          : 0;
  }
  for (cR = 0; cR < L2R - 1; cR++) { /* :3353-3373 */
    char b = gnt(g, revoffset2R - cR - 1), a = gnt(g, revoffset2R - cR);
    rightdi[cR] = (b == 'A' && a == 'G')   ? RIGHT_AG
                  : (b == 'A' && a == 'C') ? RIGHT_AC
                  : (b == 'G' && a == 'C') ? RIGHT_GC
                  : (b == 'A' && a == 'T') ? RIGHT_AT
                                           : 0;
  }

  if (kn->mode == GSNAPDP_KNOWN_INTRONS) { /* constrain to given introns, :3552-3697 */
    for (rL = 1, rR = L1 - 1; rL < L1; rL++, rR--) {
      cloL = rL - lbandL < 1 ? 1 : rL - lbandL;
      chighL = rL + rbandL > L2L - 1 ? L2L - 1 : rL + rbandL;
      cloR = rR - lbandR < 1 ? 1 : rR - lbandR;
      chighR = rR + rbandR > L2R - 1 ? L2R - 1 : rR + rbandR;
      for (cL = cloL; cL <= chighL; cL++) { /* indel on left */
        if (known_left(kn, cL) > 0) {
          scoreL = mL->H[IX(mL, rL, cL)] - gapdir_penalty(mL->dH[IX(mL, rL, cL)]);
          cR = rR;
          if (cR < rightoffset - leftoffset - cL && known_right(kn, cR) > 0) {
            scoreR = mR->H[IX(mR, rR, cR)];
            if (scoreL + scoreR > bestscore && known_intron(kn, cL, cR)) {
              bestscore = scoreL + scoreR;
              *brL = rL;
              *brR = rR;
              *bcL = cL;
              *bcR = cR;
            }
          }
        }
      }
      for (cR = cloR; cR <= chighR; cR++) { /* indel on right */
        if (known_right(kn, cR) > 0) {
          scoreR = mR->H[IX(mR, rR, cR)] - gapdir_penalty(mR->dH[IX(mR, rR, cR)]);
          cL = rL;
          if (cL < rightoffset - leftoffset - cR && known_left(kn, cL) > 0) {
            scoreL = mL->H[IX(mL, rL, cL)];
            if (scoreL + scoreR > bestscore && known_intron(kn, cL, cR)) {
              bestscore = scoreL + scoreR;
              *brL = rL;
              *brR = rR;
              *bcL = cL;
              *bcR = cR;
            }
          }
        }
      }
    }
    *finalscore = bestscore;
    *best_type = 0; /* NONINTRON */
  } else if (!use_probabilities_p) { /* :3698-3827 */
    for (rL = 1, rR = L1 - 1; rL < L1; rL++, rR--) {
      cloL = rL - lbandL < 1 ? 1 : rL - lbandL;
      chighL = rL + rbandL > L2L - 1 ? L2L - 1 : rL + rbandL;
      cloR = rR - lbandR < 1 ? 1 : rR - lbandR;
      chighR = rR + rbandR > L2R - 1 ? L2R - 1 : rR + rbandR;
      for (cL = cloL; cL <= chighL; cL++) { /* indel on left */
        scoreL = mL->H[IX(mL, rL, cL)] + known_left(kn, cL) - gapdir_penalty(mL->dH[IX(mL, rL, cL)]);
        cR = rR;
        if (cR < rightoffset - leftoffset - cL) {
          scoreR = mR->H[IX(mR, rR, cR)] + known_right(kn, cR);
          scoreI = intron_score(&introntype, leftdi[cL], rightdi[cR], cdna_direction,
                                canonical_reward, finalp);
          if (scoreL + scoreI + scoreR > bestscore) {
            bestscore = scoreL + scoreI + scoreR;
            bestscoreI = scoreI;
            *brL = rL;
            *brR = rR;
            *bcL = cL;
            *bcR = cR;
            *best_type = introntype;
          }
        }
      }
      for (cR = cloR; cR <= chighR; cR++) { /* indel on right */
        scoreR = mR->H[IX(mR, rR, cR)] + known_right(kn, cR) - gapdir_penalty(mR->dH[IX(mR, rR, cR)]);
        cL = rL;
        if (cL < rightoffset - leftoffset - cR) {
          scoreL = mL->H[IX(mL, rL, cL)] + known_left(kn, cL);
          scoreI = intron_score(&introntype, leftdi[cL], rightdi[cR], cdna_direction,
                                canonical_reward, finalp);
          if (scoreL + scoreI + scoreR > bestscore) {
            bestscore = scoreL + scoreI + scoreR;
            bestscoreI = scoreI;
            *brL = rL;
            *brR = rR;
            *bcL = cL;
            *bcR = cR;
            *best_type = introntype;
          }
        }
      }
    }
    *finalscore = halfp ? bestscore - bestscoreI / 2 : bestscore;
  } else { /* :3829-4081 */
    double *lp = (double *)calloc((size_t)L2L + 1, sizeof(double));
    double *rp = (double *)calloc((size_t)L2R + 1, sizeof(double));
    double bestprob = 0.0, probL, probR;
    for (cL = 0; cL < L2L - 1; cL++)
      lp[cL] = known_left(kn, cL) ? 1.0 : left_site_prob(cL, leftoffset, g, cdna_direction);
    for (cR = 0; cR < L2R - 1; cR++)
      rp[cR] = known_right(kn, cR) ? 1.0 : right_site_prob(cR, rightoffset, g, cdna_direction);
    for (rL = 1, rR = L1 - 1; rL < L1; rL++, rR--) {
      cloL = rL - lbandL < 1 ? 1 : rL - lbandL;
      chighL = rL + rbandL > L2L - 1 ? L2L - 1 : rL + rbandL;
      cloR = rR - lbandR < 1 ? 1 : rR - lbandR;
      chighR = rR + rbandR > L2R - 1 ? L2R - 1 : rR + rbandR;
      for (cL = cloL; cL <= chighL; cL++) {
        probL = lp[cL];
        cR = rR;
        if (cR < rightoffset - leftoffset - cL) {
          probR = rp[cR];
          if (!(probL + probR <= bestprob)) {
            scoreL = mL->H[IX(mL, rL, cL)] + known_left(kn, cL) - gapdir_penalty(mL->dH[IX(mL, rL, cL)]);
            scoreR = mR->H[IX(mR, rR, cR)] + known_right(kn, cR);
            scoreI = intron_score(&introntype, leftdi[cL], rightdi[cR], cdna_direction,
                                  canonical_reward, finalp);
            if (scoreL + scoreI + scoreR >= score_threshold) {
              bestprob = probL + probR;
              *brL = rL;
              *brR = rR;
              *bcL = cL;
              *bcR = cR;
              found = 1;
            }
          }
        }
      }
      for (cR = cloR; cR <= chighR; cR++) {
        probR = rp[cR];
        cL = rL;
        if (cL < rightoffset - leftoffset - cR) {
          probL = lp[cL];
          if (!(probL + probR <= bestprob)) {
            scoreL = mL->H[IX(mL, rL, cL)] + known_left(kn, cL);
            scoreR = mR->H[IX(mR, rR, cR)] + known_right(kn, cR) - gapdir_penalty(mR->dH[IX(mR, rR, cR)]);
            scoreI = intron_score(&introntype, leftdi[cL], rightdi[cR], cdna_direction,
                                  canonical_reward, finalp);
            if (scoreL + scoreI + scoreR >= score_threshold) {
              bestprob = probL + probR;
              *brL = rL;
              *brR = rR;
              *bcL = cL;
              *bcR = cR;
              found = 1;
            }
          }
        }
      }
    }
    free(lp);
    free(rp);
    if (!found) {
      free(leftdi);
      free(rightdi);
      return -1;
    }
    scoreL = mL->H[IX(mL, *brL, *bcL)] + known_left(kn, *bcL) - gapdir_penalty(mL->dH[IX(mL, *brL, *bcL)]);
    scoreR = mR->H[IX(mR, *brR, *bcR)] + known_right(kn, *bcR) - gapdir_penalty(mR->dH[IX(mR, *brR, *bcR)]);
    scoreI = intron_score(&introntype, leftdi[*bcL], rightdi[*bcR], cdna_direction,
                          canonical_reward, finalp);
    *finalscore = halfp ? scoreL + scoreI + scoreR - scoreI / 2 : scoreL + scoreI + scoreR;
  }
  result = *finalscore >= 0; /* :4084-4101 */
  if (result && kn->mode == GSNAPDP_KNOWN_SITES)  /* novel splicing off: both sites known */
    result = known_left(kn, *bcL) > 0 && known_right(kn, *bcR) > 0;
  if (finalp && result) {   /* :4104-4108, get_splicesite_probs :3195-3287 */
    *left_prob = known_left(kn, *bcL) ? 1.0 : left_site_prob(*bcL, leftoffset, g, cdna_direction);
    *right_prob = known_right(kn, *bcR) ? 1.0 : right_site_prob(*bcR, rightoffset, g, cdna_direction);
  }
  free(leftdi);
  free(rightdi);
  return result;
}

/* Dynprog_genome_gap (dynprog.c:4798-5061) */
void orc_genome_gap(orc_list *out, orc_genome_gap_out *o, int dpi, orc_dp *dpL, orc_dp *dpR,
                    const char *sequence1, const char *sequenceuc1, int length1, int length2L,
                    int length2R, int offset1, int offset2L, int revoffset2R, uint32_t chroffset,
                    uint32_t chrhigh, uint32_t chrpos, uint32_t genomiclength, int cdna_direction,
                    int watsonp, int jump_late_p, int extraband_paired, double defect_rate,
                    int maxpeelback, int halfp, int finalp, int use_probabilities_p,
                    int score_threshold, int splicingp, int known_mode) {
  int mt, open, extend, canonical_reward, revoffset1, brL = 0, brR = 0, bcL = 0, bcR = 0, rc;
  known_t kn;
  mview mL, mR;
  counts k = {0, 0, 0, 0};
  gpar g = {chroffset, chrhigh, chrpos, (int)genomiclength, watsonp};
  orc_list_clear(out);
  memset(o, 0, sizeof(*o));
  o->dynprogindex = dpi;
  o->left_prob = o->right_prob = 0.0;
  o->bridge_ok = 1;
  if (length1 <= 1) {
    o->finalscore = NEG_INF;
    o->returned_null = 1;
    return;
  }
  quality(defect_rate, &mt);
  if (length1 > maxpeelback * 4) {
    open = SINGLE_OPEN;
    extend = SINGLE_EXTEND;
  } else {
    open = PAIRED_OPEN;
    extend = PAIRED_EXTEND;
  }
  canonical_reward = !splicingp ? 0 : finalp ? final_canonical_reward_tab[mt] : canonical_reward_tab[mt];
  if (length1 > dpL->maxlength1 || length2L > dpL->maxlength2 || length1 > dpR->maxlength1 ||
      length2R > dpR->maxlength2) {
    o->new_leftgenomepos = offset2L - 1;
    o->new_rightgenomepos = revoffset2R + 1;
    o->exonhead = offset1 + length1 - 1;
    o->dynprogindex = step_index(dpi);
    o->finalscore = NEG_INF;
    o->returned_null = 1;
    return;
  }
  revoffset1 = offset1 + length1 - 1;
  fill(&mL, dpL, sequence1, 0, offset2L, length1, length2L, &g, mt, open, extend, extraband_paired,
       1, jump_late_p);
  fill(&mR, dpR, &sequence1[length1 - 1], 1, revoffset2R, length1, length2R, &g, mt, open, extend,
       extraband_paired, 1, !jump_late_p);
  kn.mode = known_mode;
  kn.rec = (const unsigned char *)sequence1 + length1; /* the record follows the query rows */
  kn.L2L = length2L;
  kn.L2R = length2R;
  rc = bridge_intron(&o->finalscore, &brL, &brR, &bcL, &bcR, &o->introntype, &o->left_prob,
                     &o->right_prob, &mL, &mR, offset2L, revoffset2R, length1, length2L, length2R,
                     cdna_direction, &g, extraband_paired, canonical_reward, offset2L,
                     revoffset2R, halfp, finalp, use_probabilities_p, score_threshold, &kn);
  if (rc < 0) {
    o->bridge_ok = 0;
    o->returned_null = 1;
    o->finalscore = NEG_INF;
    return;
  }
  if (rc == 0) {
    o->returned_null = 1;
    return;
  }
  o->new_leftgenomepos = offset2L + (bcL - 1);
  o->new_rightgenomepos = revoffset2R - (bcR - 1);
  o->exonhead = revoffset1 - (brR - 1);
  traceback(out, &k, &mR, brR, bcR, &sequence1[length1 - 1], &sequenceuc1[length1 - 1],
            revoffset1, revoffset2R, 1, &g, cdna_direction, dpi);
  list_reverse(out);
  push_gapholder(out, GSNAPDP_UNKNOWNJUMP, GSNAPDP_UNKNOWNJUMP);
  traceback(out, &k, &mL, brL, bcL, sequence1, sequenceuc1, offset1, offset2L, 0, &g,
            cdna_direction, dpi);
  o->nmatches = k.nmatches;
  o->nmismatches = k.nmismatches;
  o->nopens = k.nopens;
  o->nindels = k.nindels;
  if (out->n == 1) {
    orc_list_clear(out);
    o->returned_null = 1;
  }
  o->dynprogindex = step_index(dpi);
  list_reverse(out);
}


/* ------------------------------------------------------------- cDNA gap */

#define CDNA_OPEN (-10)   /* dynprog.c:230-232, every quality bin */
#define CDNA_EXTEND (-7)
#define INSERT_PAIRS 9    /* :140 */
#define SHORTGAP_COMP '~' /* comp.h:11 */

/* compute_scores_lookup_fwd_12 / _rev_12 (dynprog.c:1742-2044): the genome in
 * the rows (get_genomic_nt at offset1 +/- (r-1)), the query in the columns,
 * pairdistance[query][genome] ("Note swap"), row-major with the row-wise
 * band-edge sentinels. */
static void fill12(mview *m, orc_dp *dp, int rev, int goff, int Lg, int Lq, const char *qseq,
                   const gpar *g, int mt, int open, int extend, int extraband, int jump_late_p) {
  int lband, rband, r, c, clo, chigh, penalty;
  size_t cells = (size_t)(Lg + 1) * (size_t)(Lq + 1);
  int32_t *H = dp->nogap, *E = dp->gap1, *F = dp->gap2;
  uint8_t *dH = dp->dnogap, *dE = dp->dgap1, *dF = dp->dgap2;
  int stride = Lq + 1;
  int(*tab)[128] = pd[mt];
  if (Lg <= 0 || Lq <= 0) {
    fprintf(stderr, "dynprog: lengths are negative: %d %d\n", Lg, Lq);
    abort();
  }
  m->L1 = Lg;
  m->L2 = Lq;
  m->stride = stride;
  m->H = H;
  m->E = E;
  m->F = F;
  m->dH = dH;
  m->dE = dE;
  m->dF = dF;
  band_widths(Lg, Lq, extraband, 1, &lband, &rband);
  memset(H, 0, cells * 4);
  memset(E, 0, cells * 4);
  memset(F, 0, cells * 4);
  memset(dH, 0, cells);
  memset(dE, 0, cells);
  memset(dF, 0, cells);
  H[0] = 0;
  dH[0] = D_STOP;
  E[0] = F[0] = NEG_INF;
  penalty = open;
  for (c = 1; c <= rband && c <= Lq; c++) { /* row 0 */
    penalty += extend;
    H[c] = NEG_INF;
    E[c] = penalty;
    dE[c] = D_HORIZ;
    F[c] = NEG_INF;
  }
  dE[1] = D_STOP;
  penalty = open;
  for (r = 1; r <= lband && r <= Lg; r++) { /* column 0 */
    size_t i = (size_t)r * stride;
    penalty += extend;
    H[i] = NEG_INF;
    E[i] = NEG_INF;
    F[i] = penalty;
    dF[i] = D_VERT;
  }
  dF[(size_t)stride] = D_STOP;
  for (r = 1; r <= Lg; r++) {
    int na1 = (unsigned char)gnt(g, rev ? goff + 1 - r : goff + r - 1) & 127;
    if ((clo = r - lband) < 1) {
      clo = 1;
    } else {
      size_t i = (size_t)r * stride + (clo - 1);
      E[i] = NEG_INF;
      H[i] = NEG_INF;
    }
    if ((chigh = r + rband) > Lq) {
      chigh = Lq;
    } else {
      size_t i = (size_t)(r - 1) * stride + chigh;
      F[i] = NEG_INF;
      H[i] = NEG_INF;
    }
    for (c = clo; c <= chigh; c++) {
      size_t i = (size_t)r * stride + c;
      size_t il = i - 1, iu = i - stride, id = i - stride - 1;
      int na2 = (unsigned char)(rev ? qseq[1 - c] : qseq[c - 1]) & 127;
      int best, s;
      uint8_t dir;
      best = H[il] + open;
      dir = D_DIAG;
      s = E[il];
      if (s > best || (s == best && jump_late_p)) {
        best = s;
        dir = D_HORIZ;
      }
      E[i] = best + extend;
      dE[i] = dir;
      best = H[iu] + open;
      dir = D_DIAG;
      s = F[iu];
      if (s > best || (s == best && jump_late_p)) {
        best = s;
        dir = D_VERT;
      }
      F[i] = best + extend;
      dF[i] = dir;
      best = H[id];
      dir = D_DIAG;
      s = E[id];
      if (s > best || (s == best && jump_late_p)) {
        best = s;
        dir = D_HORIZ;
      }
      s = F[id];
      if (s > best || (s == best && jump_late_p)) {
        best = s;
        dir = D_VERT;
      }
      H[i] = best + tab[na2][na1];
      dH[i] = dir;
    }
  }
}

/* bridge_cdna_gap (dynprog.c:3068-3146).  `pen` is 0 for the first right row
 * and `open` for every later one (the loop resets it to open - extend before
 * its own += extend).  Returns 0 if no candidate beat -100000 (the reference
 * then traces back from uninitialised indices). */
static int bridge_cdna(int *finalscore, int *brL, int *brR, int *bcL, int *bcR, const mview *mL,
                       const mview *mR, int L2, int L1L, int L1R, int eb, int open, int extend,
                       int leftoffset, int rightoffset) {
  int bestscore = -100000, found = 0, rL, rR, cL, cR, pen;
  int lbandL = eb, rbandL = L1L - L2 + eb, lbandR = eb, rbandR = L1R - L2 + eb;
  for (rL = 1; rL < L2; rL++) {
    for (rR = L2 - rL, pen = 0; rR >= 0; rR--, pen += extend) {
      int cloL = rL - lbandL < 1 ? 1 : rL - lbandL;
      int chighL = rL + rbandL > L1L - 1 ? L1L - 1 : rL + rbandL;
      int cloR = rR - lbandR < 1 ? 1 : rR - lbandR;
      int chighR = rR + rbandR > L1R - 1 ? L1R - 1 : rR + rbandR;
      for (cL = cloL; cL <= chighL; cL++) {
        int scoreL = mL->H[IX(mL, rL, cL)];
        for (cR = cloR; cR <= chighR && cR < rightoffset - leftoffset - cL; cR++) {
          int scoreR = mR->H[IX(mR, rR, cR)];
          if (scoreL + scoreR + pen > bestscore) {
            bestscore = scoreL + scoreR + pen;
            *brL = rL;
            *brR = rR;
            *bcL = cL;
            *bcR = cR;
            found = 1;
          }
        }
      }
      pen = open - extend;
    }
  }
  *finalscore = bestscore;
  return found;
}

/* add_queryskip with cdna_gap_p (dynprog.c:2372-2413): query in the columns */
static void add_queryskip_cdna(orc_list *l, int r, int c, int dist, const char *qseq, int qoff,
                               int goff, int rev, int dpi) {
  int j, qc = c - 1, gc = r - 1, step;
  if (rev) {
    qc = -qc;
    gc = -gc;
    step = +1;
  } else {
    gc++;
    step = -1;
  }
  for (j = 0; j < dist; j++) {
    push_pair(l, qoff + qc, goff + gc, qseq[qc], '-', ' ', dpi);
    qc += step;
  }
}

/* add_genomeskip_cdna (dynprog.c:2516-2608) */
static int add_genomeskip_cdna(orc_list *l, int r, int c, int dist, int qoff, int goff, int rev,
                               const gpar *g, int cdna_direction, int dpi) {
  int j, qc = c - 1, left = r - dist, right = r - 1, gc, step, dashes;
  if (rev) {
    int t = left;
    qc = -qc;
    left = -right;
    right = -t;
    step = +1;
  } else {
    qc++;
    step = -1;
  }
  if (dist < MICROINTRON_LENGTH) {
    dashes = 1;
  } else {
    char l1 = gnt(g, goff + left), l2 = gnt(g, goff + left + 1);
    char r2 = gnt(g, goff + right - 1), r1 = gnt(g, goff + right);
    dashes = intron_type(l1, l2, r2, r1, cdna_direction) == NONINTRON;
  }
  if (dashes) {
    gc = rev ? left : right;
    for (j = 0; j < dist; j++) {
      push_pair(l, qoff + qc, goff + gc, ' ', '-', gnt(g, goff + gc), dpi);
      gc += step;
    }
  } else {
    push_gapholder(l, GSNAPDP_UNKNOWNJUMP, GSNAPDP_UNKNOWNJUMP);
  }
  return dashes;
}

/* traceback_cdna (dynprog.c:2716-2812): rows are genome, columns query; no
 * '*' test; consistent_array[genome][query] ("Note swap") */
static void traceback_cdna(orc_list *l, counts *k, const mview *m, int r, int c, const char *qseq,
                           const char *qseq_uc, int qoff, int goff, int rev, const gpar *g,
                           int cdna_direction, int dpi) {
  while (m->dH[IX(m, r, c)] != D_STOP) {
    int qc = c - 1, gc = r - 1, dist;
    char c1, c2;
    uint8_t d;
    if (rev) {
      qc = -qc;
      gc = -gc;
    }
    c1 = qseq[qc];
    c2 = gnt(g, goff + gc);
    if (qseq_uc[qc] == c2) {
      k->nmatches++;
      push_pair(l, qoff + qc, goff + gc, c1, '*', c2, dpi);
    } else if (cons[c2 & 127][c1 & 127]) {
      k->nmatches++;
      push_pair(l, qoff + qc, goff + gc, c1, ':', c2, dpi);
    } else {
      k->nmismatches++;
      push_pair(l, qoff + qc, goff + gc, c1, ' ', c2, dpi);
    }
    d = m->dH[IX(m, r, c)];
    if (d == D_DIAG) {
      r--;
      c--;
    } else if (d == D_HORIZ) {
      dist = 1;
      r--;
      c--;
      while (m->dE[IX(m, r, c)] == D_HORIZ) {
        dist++;
        c--;
      }
      c--;
      add_queryskip_cdna(l, r, c + dist, dist, qseq, qoff, goff, rev, dpi);
      k->nopens++;
      k->nindels += dist;
    } else {
      dist = 1;
      r--;
      c--;
      while (m->dF[IX(m, r, c)] == D_VERT) {
        dist++;
        r--;
      }
      r--;
      if (add_genomeskip_cdna(l, r + dist, c, dist, qoff, goff, rev, g, cdna_direction, dpi)) {
        k->nopens++;
        k->nindels += dist;
      }
    }
  }
}

/* Dynprog_cdna_gap (dynprog.c:4578-4793) */
void orc_cdna_gap(orc_list *out, orc_cdna_gap_out *o, int dpi, orc_dp *dpL, orc_dp *dpR,
                  const char *sequence1L, const char *sequenceuc1L, const char *revsequence1R,
                  const char *revsequenceuc1R, const char *sequence2, int length1L, int length1R,
                  int length2, int offset1L, int revoffset1R, int offset2, uint32_t chroffset,
                  uint32_t chrhigh, uint32_t chrpos, uint32_t genomiclength, int cdna_direction,
                  int watsonp, int jump_late_p, int extraband_paired, double defect_rate) {
  int mt, brL = 0, brR = 0, bcL = 0, bcR = 0, revoffset2, queryjump, genomejump, kk;
  mview mL, mR;
  counts k = {0, 0, 0, 0};
  gpar g = {chroffset, chrhigh, chrpos, (int)genomiclength, watsonp};
  orc_list_clear(out);
  memset(o, 0, sizeof(*o));
  o->dynprogindex = dpi;
  o->bridge_ok = 1;
  if (length2 <= 1) { /* :4605 */
    o->returned_null = 1;
    return;
  }
  quality(defect_rate, &mt);
  if (length2 > dpR->maxlength1 || length1R > dpR->maxlength2 || length2 > dpL->maxlength1 ||
      length1L > dpL->maxlength2) { /* :4651-4675 */
    o->dynprogindex = step_index(dpi);
    o->returned_null = 1;
    return;
  }
  revoffset2 = offset2 + length2 - 1;
  fill12(&mR, dpR, 1, revoffset2, length2, length1R, revsequence1R, &g, mt, CDNA_OPEN, CDNA_EXTEND,
         extraband_paired, !jump_late_p);
  fill12(&mL, dpL, 0, offset2, length2, length1L, sequence1L, &g, mt, CDNA_OPEN, CDNA_EXTEND,
         extraband_paired, jump_late_p);
  o->finalscore_set = 1;
  if (!bridge_cdna(&o->finalscore, &brL, &brR, &bcL, &bcR, &mL, &mR, length2, length1L, length1R,
                   extraband_paired, CDNA_OPEN, CDNA_EXTEND, offset1L, revoffset1R)) {
    o->bridge_ok = 0;
    o->returned_null = 1;
    return;
  }
  o->brL = brL;
  o->bcL = bcL;
  o->brR = brR;
  o->bcR = bcR;
  traceback_cdna(out, &k, &mR, brR, bcR, revsequence1R, revsequenceuc1R, revoffset1R, revoffset2, 1,
                 &g, cdna_direction, dpi);
  list_reverse(out);
  queryjump = (revoffset1R - bcR) - (offset1L + bcL) + 1;
  genomejump = (revoffset2 - brR) - (offset2 + brL) + 1;
  if (queryjump == INSERT_PAIRS && genomejump == INSERT_PAIRS) { /* :4730-4752 */
    o->insert_pairs = 1;
    for (kk = revoffset1R - bcR; kk >= offset1L + bcL; kk--)
      push_pair(out, kk, revoffset2 - brR + 1, sequence1L[kk - offset1L], SHORTGAP_COMP, ' ', dpi);
    for (kk = revoffset2 - brR; kk >= offset2 + brL; kk--)
      push_pair(out, offset1L + bcL, kk, ' ', SHORTGAP_COMP, sequence2[kk - offset2], dpi);
  } else {
    push_gapholder(out, GSNAPDP_UNKNOWNJUMP, GSNAPDP_UNKNOWNJUMP);
    o->incompletep = 1;
  }
  traceback_cdna(out, &k, &mL, brL, bcL, sequence1L, sequenceuc1L, offset1L, offset2, 0, &g,
                 cdna_direction, dpi);
  if (out->n == 1) {
    orc_list_clear(out);
    o->returned_null = 1;
  }
  o->dynprogindex = step_index(dpi);
  list_reverse(out);
}

/* ------------------------------------------------------------------ batch */

typedef struct batch_job {
  const gsnapdp_window *w;
  int lo, hi;
  const char *query, *query_uc;
  gsnapdp_result *results;
  gsnapdp_pair *pairs;
  const int64_t *pair_offsets;
  int32_t *npairs;
  int maxl1, maxl2;
} batch_job;

static void run_one(orc_dp *dp, orc_list *l, const gsnapdp_window *w, const char *query,
                    const char *query_uc, gsnapdp_result *res) {
  int dpi = w->dynprogindex, fs = 0, nm = 0, nmm = 0, no = 0, ni = 0;
  int saved1 = dp->maxlength1, saved2 = dp->maxlength2;
  dp->maxlength1 = w->maxlength1;
  dp->maxlength2 = w->maxlength2;
  memset(res, 0, sizeof(*res));
  if (w->kind == GSNAPDP_SINGLE_GAP) {
    orc_single_gap(l, &dpi, &fs, &nm, &nmm, &no, &ni, dp, query + w->qpos, query_uc + w->qpos,
                   w->length1, w->length2, w->offset1, w->offset2, w->chroffset, w->chrhigh,
                   w->chrpos, w->genomiclength, w->cdna_direction, w->watsonp, w->jump_late_p,
                   w->extraband, (double)w->defect_rate, 0, w->widebandp);
  } else if (w->kind == GSNAPDP_END5_GAP) {
    orc_end5_gap(l, &dpi, &fs, &nm, &nmm, &no, &ni, dp, query + w->qpos, query_uc + w->qpos,
                 w->length1, w->length2, w->offset1, w->offset2, w->chroffset, w->chrhigh,
                 w->chrpos, w->genomiclength, w->cdna_direction, w->watsonp, w->jump_late_p,
                 w->extraband, (double)w->defect_rate, w->endalign);
  } else {
    orc_end3_gap(l, &dpi, &fs, &nm, &nmm, &no, &ni, dp, query + w->qpos, query_uc + w->qpos,
                 w->length1, w->length2, w->offset1, w->offset2, w->chroffset, w->chrhigh,
                 w->chrpos, w->genomiclength, w->cdna_direction, w->watsonp, w->jump_late_p,
                 w->extraband, (double)w->defect_rate, w->endalign);
  }
  dp->maxlength1 = saved1;
  dp->maxlength2 = saved2;
  res->finalscore = fs;
  res->nmatches = nm;
  res->nmismatches = nmm;
  res->nopens = no;
  res->nindels = ni;
  res->reserved = dpi; /* dynprogindex after the call */
}

static void *batch_worker(void *arg) {
  batch_job *j = (batch_job *)arg;
  orc_dp *dp = orc_dp_new(600, 10, 11, 10, 8);
  orc_list l;
  int i;
  if (j->maxl1 > dp->maxlength1 || j->maxl2 > dp->maxlength2) {
    orc_dp_free(dp);
    dp = orc_dp_new(j->maxl1 > 500 ? j->maxl1 : 500, 0, 0, j->maxl2, 0);
  }
  orc_list_init(&l, 1024);
  for (i = j->lo; i < j->hi; i++) {
    int64_t off = j->pair_offsets ? j->pair_offsets[i] : 0;
    int64_t cap = j->pair_offsets ? j->pair_offsets[i + 1] - off : 0;
    int t;
    run_one(dp, &l, &j->w[i], j->query, j->query_uc, &j->results[i]);
    if (j->npairs) j->npairs[i] = l.n;
    for (t = 0; t < l.n && t < cap; t++) j->pairs[off + t] = l.buf[l.head + t];
  }
  orc_list_free(&l);
  orc_dp_free(dp);
  return NULL;
}

int orc_run_batch(const gsnapdp_window *w, int n, const char *query, const char *query_uc,
                  gsnapdp_result *results, gsnapdp_pair *pairs, const int64_t *pair_offsets,
                  int32_t *npairs, int nthreads) {
  int maxl1 = 0, maxl2 = 0, i, t;
  batch_job *jobs;
  pthread_t *th;
  for (i = 0; i < n; i++) {
    if (w[i].maxlength1 > maxl1) maxl1 = w[i].maxlength1;
    if (w[i].maxlength2 > maxl2) maxl2 = w[i].maxlength2;
    if (w[i].endalign == GSNAPDP_QUERYEND_NOGAPS) continue;
  }
  if (nthreads < 1) nthreads = 1;
  if (nthreads > n) nthreads = n > 0 ? n : 1;
  jobs = (batch_job *)calloc((size_t)nthreads, sizeof(batch_job));
  th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
  for (t = 0; t < nthreads; t++) {
    jobs[t].w = w;
    jobs[t].lo = (int)((int64_t)n * t / nthreads);
    jobs[t].hi = (int)((int64_t)n * (t + 1) / nthreads);
    jobs[t].query = query;
    jobs[t].query_uc = query_uc;
    jobs[t].results = results;
    jobs[t].pairs = pairs;
    jobs[t].pair_offsets = pair_offsets;
    jobs[t].npairs = npairs;
    jobs[t].maxl1 = maxl1;
    jobs[t].maxl2 = maxl2;
  }
  if (nthreads == 1) {
    batch_worker(&jobs[0]);
  } else {
    for (t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, batch_worker, &jobs[t]);
    for (t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  }
  free(jobs);
  free(th);
  return 0;
}

int orc_run_ggap_batch(const gsnapdp_ggap_window *w, int n, const char *query, const char *query_uc,
                       gsnapdp_ggap_result *results, gsnapdp_pair *pairs,
                       const int64_t *pair_offsets, int32_t *npairs) {
  orc_dp *dpL = orc_dp_new(600, 10, 11, 10, 8), *dpR = orc_dp_new(600, 10, 11, 10, 8);
  orc_list l;
  int i, t;
  orc_list_init(&l, 1024);
  for (i = 0; i < n; i++) {
    const gsnapdp_ggap_window *x = &w[i];
    orc_genome_gap_out o;
    gsnapdp_ggap_result *r = &results[i];
    int64_t off = pair_offsets ? pair_offsets[i] : 0;
    int64_t cap = pair_offsets ? pair_offsets[i + 1] - off : 0;
    dpL->maxlength1 = dpR->maxlength1 = x->maxlength1;
    dpL->maxlength2 = dpR->maxlength2 = x->maxlength2;
    orc_genome_gap(&l, &o, x->dynprogindex, dpL, dpR, query + x->qpos, query_uc + x->qpos,
                   x->length1, x->length2L, x->length2R, x->offset1, x->offset2L, x->revoffset2R,
                   x->chroffset, x->chrhigh, x->chrpos, x->genomiclength, x->cdna_direction,
                   x->watsonp, x->jump_late_p, x->extraband_paired, (double)x->defect_rate,
                   x->maxpeelback, x->halfp, x->finalp, x->use_probabilities_p,
                   x->score_threshold, x->splicingp, x->known_mode);
    memset(r, 0, sizeof(*r));
    r->finalscore = o.finalscore;
    r->new_leftgenomepos = o.new_leftgenomepos;
    r->new_rightgenomepos = o.new_rightgenomepos;
    r->nmatches = o.nmatches;
    r->nmismatches = o.nmismatches;
    r->nopens = o.nopens;
    r->nindels = o.nindels;
    r->exonhead = o.exonhead;
    r->introntype = o.introntype;
    r->dynprogindex = o.dynprogindex;
    r->returned_null = o.returned_null;
    r->bridge_ok = o.bridge_ok;
    r->left_prob = o.left_prob;
    r->right_prob = o.right_prob;
    if (npairs) npairs[i] = l.n;
    for (t = 0; t < l.n && t < cap; t++) pairs[off + t] = l.buf[l.head + t];
  }
  orc_list_free(&l);
  orc_dp_free(dpL);
  orc_dp_free(dpR);
  return 0;
}

/* Batch driver over gsnapdp_cgap_window records (single thread).  gseg holds
 * each window's genomic segment (the reference's sequence2, read only by the
 * INSERT_PAIRS branch) at gseg_off[i]. */
int orc_run_cgap_batch(const gsnapdp_cgap_window *w, int n, const char *query, const char *query_uc,
                       const char *gseg, const int64_t *gseg_off, gsnapdp_cgap_result *results,
                       gsnapdp_pair *pairs, const int64_t *pair_offsets, int32_t *npairs) {
  orc_dp *dpL = orc_dp_new(600, 10, 11, 10, 8), *dpR = orc_dp_new(600, 10, 11, 10, 8);
  orc_list l;
  int i, t;
  orc_list_init(&l, 1024);
  for (i = 0; i < n; i++) {
    const gsnapdp_cgap_window *x = &w[i];
    orc_cdna_gap_out o;
    gsnapdp_cgap_result *r = &results[i];
    int64_t off = pair_offsets ? pair_offsets[i] : 0;
    int64_t cap = pair_offsets ? pair_offsets[i + 1] - off : 0;
    dpL->maxlength1 = dpR->maxlength1 = x->maxlength1;
    dpL->maxlength2 = dpR->maxlength2 = x->maxlength2;
    orc_cdna_gap(&l, &o, x->dynprogindex, dpL, dpR, query + x->qposL, query_uc + x->qposL,
                 query + x->qposR, query_uc + x->qposR, gseg + gseg_off[i], x->length1L,
                 x->length1R, x->length2, x->offset1L, x->revoffset1R, x->offset2, x->chroffset,
                 x->chrhigh, x->chrpos, x->genomiclength, x->cdna_direction, x->watsonp,
                 x->jump_late_p, x->extraband_paired, (double)x->defect_rate);
    memset(r, 0, sizeof(*r));
    r->finalscore = o.finalscore;
    r->dynprogindex = o.dynprogindex;
    r->incompletep = o.incompletep;
    r->returned_null = o.returned_null;
    r->status = o.bridge_ok ? 0 : 5;
    r->finalscore_set = o.finalscore_set;
    r->insert_pairs = o.insert_pairs;
    r->brL = o.brL;
    r->bcL = o.bcL;
    r->brR = o.brR;
    r->bcR = o.bcR;
    r->npairs = l.n;
    if (npairs) npairs[i] = l.n;
    for (t = 0; t < l.n && t < cap; t++) pairs[off + t] = l.buf[l.head + t];
  }
  orc_list_free(&l);
  orc_dp_free(dpL);
  orc_dp_free(dpR);
  return 0;
}

/* Batch of splice-junction end gaps (gsnapdp_sj_window), single-threaded. */
int orc_run_sj_batch(const gsnapdp_sj_window *w, int n, const char *query, const char *query_uc,
                     gsnapdp_result *results, gsnapdp_pair *pairs, const int64_t *pair_offsets,
                     int32_t *npairs) {
  orc_dp *dp = orc_dp_new(600, 10, 11, 10, 8);
  orc_list l;
  int i, t;
  orc_list_init(&l, 1024);
  for (i = 0; i < n; i++) {
    const gsnapdp_sj_window *x = &w[i];
    gsnapdp_result *res = &results[i];
    int dpi = x->dynprogindex, fs = 0, nm = 0, nmm = 0, no = 0, ni = 0;
    int64_t off = pair_offsets[i], cap = pair_offsets[i + 1] - off;
    if (x->maxlength1 > 611 || x->maxlength2 > 2000) {
      orc_dp_free(dp);
      dp = orc_dp_new(x->maxlength1 > 500 ? x->maxlength1 : 500, 0, 0, x->maxlength2, 0);
    }
    dp->maxlength1 = x->maxlength1;
    dp->maxlength2 = x->maxlength2;
    if (x->kind == GSNAPDP_END5_GAP)
      orc_end5_splicejunction(&l, &dpi, &fs, &nm, &nmm, &no, &ni, dp, query + x->qpos,
                              query_uc + x->qpos, query + x->spos, query_uc + x->spos, x->length1,
                              x->length2, x->offset1, x->offset2_anchor, x->offset2_far,
                              x->cdna_direction, x->jump_late_p, x->extraband_end,
                              (double)x->defect_rate, x->contlength);
    else
      orc_end3_splicejunction(&l, &dpi, &fs, &nm, &nmm, &no, &ni, dp, query + x->qpos,
                              query_uc + x->qpos, query + x->spos, query_uc + x->spos, x->length1,
                              x->length2, x->offset1, x->offset2_anchor, x->offset2_far,
                              x->cdna_direction, x->jump_late_p, x->extraband_end,
                              (double)x->defect_rate, x->contlength);
    memset(res, 0, sizeof(*res));
    res->finalscore = fs;
    res->nmatches = nm;
    res->nmismatches = nmm;
    res->nopens = no;
    res->nindels = ni;
    res->reserved = dpi;
    npairs[i] = l.n;
    for (t = 0; t < l.n && t < cap; t++) pairs[off + t] = l.buf[l.head + t];
  }
  orc_list_free(&l);
  orc_dp_free(dp);
  return 0;
}

/* ------------------------------------------------------------- microexons */

/* get_genomic_nt of boyer-moore.c:361-380: no '*' rules, straight from the blocks */
static char bm_nt(const gpar *g, int pos) {
  if (g->watsonp) return block_char(g->chroffset + g->chrpos + (uint32_t)pos);
  return compl_char(block_char(g->chroffset + g->chrpos + (uint32_t)(g->genomiclength - 1) - (uint32_t)pos));
}

/* BoyerMoore_nt (boyer-moore.c:384-451): every j in [0, textlen-querylen]
 * where the text matches the (A C G T only, else no hits: query_okay :313)
 * query exactly.  Written as the plain scan; the reference's good-suffix /
 * bad-character shifts only skip non-matching j.  hits[] is in the order the
 * reference's Intlist holds them (pushed while j ascends: largest j first). */
static int bm_hits(int *hits, int cap, const char *query, int querylen, int textoffset, int textlen,
                   const gpar *g) {
  int i, j, n = 0;
  for (i = 0; i < querylen; i++)
    if (query[i] != 'A' && query[i] != 'C' && query[i] != 'G' && query[i] != 'T') return 0;
  for (j = 0; j <= textlen - querylen; j++) {
    for (i = querylen - 1; i >= 0 && query[i] == bm_nt(g, textoffset + i + j); i--)
      ;
    if (i < 0) {
      if (n < cap) hits[n] = j;
      n++;
    }
  }
  for (i = 0; i < n / 2 && i < cap; i++) { /* Intlist_push order */
    int t = hits[i];
    hits[i] = hits[n - 1 - i];
    hits[n - 1 - i] = t;
  }
  return n;
}

#define MIN_MICROEXON_LENGTH 3   /* :133 */
#define MAX_MICROEXON_LENGTH 12  /* :137 (non-PMAP) */

/* Dynprog_microexon_int (dynprog.c:7128-7432), non-PMAP, use_genomicseg_p false.
 * Returns 1 and fills *o when a list is returned, with the list itself in out. */
int orc_microexon_int(orc_list *out, orc_micro_out *o, int dynprogindex, const char *sequence1,
                      const char *sequenceuc1, int length1, int offset1, int offset2L,
                      int revoffset2R, int cdna_direction, const char *queryseq,
                      const char *queryuc, uint32_t chroffset, uint32_t chrhigh, uint32_t chrpos,
                      uint32_t genomiclength, int watsonp, double defect_rate) {
  gpar g = {chroffset, chrhigh, chrpos, (int)genomiclength, watsonp};
  int bestcL = -1, bestcR = -1, best_middlelength = 0, candidate = 0, have_candidate = 0;
  int min_len, span, leftbound, rightbound, nmm, i, cL, cR;
  char intron1, intron2, intron3, intron4, gapchar;
  double pvalue, bestprob = 0.0;
  /* the Boyer-Moore hit buffer: one per thread (the batch runs on many) */
  static __thread int *hits;
  enum { NHITS = 1 << 16 };
  if (!hits && !(hits = (int *)malloc(sizeof(int) * NHITS))) {
    o->unsupported = 1;
    return 0;
  }
  orc_list_clear(out);
  memset(o, 0, sizeof(*o));
  o->dynprogindex = dynprogindex;
  pvalue = defect_rate < 0.003 ? 0.01 : defect_rate < 0.014 ? 0.001 : 0.0001; /* :7171-7177 */
  if (cdna_direction > 0) {
    intron1 = 'G'; intron2 = 'T'; intron3 = 'A'; intron4 = 'G';
    gapchar = '>';
    o->microintrontype = GTAG_FWD;
  } else if (cdna_direction < 0) {
    intron1 = 'C'; intron2 = 'T'; intron3 = 'A'; intron4 = 'C';
    gapchar = '<';
    o->microintrontype = GTAG_REV;
  } else {
    o->unsupported = 1; /* the reference aborts (:7203-7206) */
    return 0;
  }
  span = revoffset2R - offset2L;
  if (span <= 0) {
    o->unsupported = 1; /* :7222-7225 */
    return 0;
  }
  min_len = (int)ceil(-log(1.0 - pow(1.0 - pvalue, 1.0 / (double)span)) / log(4));
  min_len -= 8;
  if (min_len > MAX_MICROEXON_LENGTH) {
    o->microintrontype = NONINTRON;
    return 0;
  } else if (min_len < MIN_MICROEXON_LENGTH) {
    min_len = MIN_MICROEXON_LENGTH;
  }
  leftbound = 0; /* :7241-7262 */
  nmm = 0;
  while (leftbound < length1 - 1 && nmm <= 1) {
    if (sequenceuc1[leftbound] != gnt(&g, offset2L + leftbound)) nmm++;
    leftbound++;
  }
  leftbound--;
  rightbound = 0; /* :7264-7286 */
  i = length1 - 1;
  nmm = 0;
  while (i >= 0 && nmm <= 1) {
    if (sequenceuc1[i] != gnt(&g, revoffset2R - rightbound)) nmm++;
    rightbound++;
    i--;
  }
  rightbound--;
  for (cL = 1; cL <= leftbound; cL++) { /* :7292-7396 */
    if (gnt(&g, offset2L + cL) == intron1 && gnt(&g, offset2L + cL + 1) == intron2) {
      int mincR = length1 - MAX_MICROEXON_LENGTH - cL, maxcR = length1 - min_len - cL;
      if (mincR < 1) mincR = 1;
      if (maxcR > rightbound) maxcR = rightbound;
      for (cR = mincR; cR <= maxcR; cR++) {
        if (gnt(&g, revoffset2R - cR - 1) == intron3 && gnt(&g, revoffset2R - cR) == intron4) {
          int middlelength = length1 - cL - cR;
          int textleft = offset2L + cL + MICROINTRON_LENGTH;
          int textright = revoffset2R - cR - MICROINTRON_LENGTH;
          int nh = bm_hits(hits, NHITS, &sequenceuc1[cL],
                           middlelength, textleft, textright - textleft, &g), h;
          for (h = 0; h < nh; h++) {
            candidate = textleft + hits[h];
            have_candidate = 1;
            if (gnt(&g, candidate - 2) == intron3 && gnt(&g, candidate - 1) == intron4 &&
                gnt(&g, candidate + middlelength) == intron1 &&
                gnt(&g, candidate + middlelength + 1) == intron2) {
              double prob2, prob3;
              uint32_t sp;
              if (watsonp) {
                if (cdna_direction > 0) {
                  sp = chrpos + (uint32_t)(candidate - 1) + 1u;
                  prob2 = orc_maxent_acceptor(chroffset + sp, chroffset);
                  sp = chrpos + (uint32_t)candidate + (uint32_t)middlelength;
                  prob3 = orc_maxent_donor(chroffset + sp, chroffset);
                } else {
                  sp = chrpos + (uint32_t)(candidate - 1) + 1u;
                  prob2 = orc_maxent_antidonor(chroffset + sp, chroffset);
                  sp = chrpos + (uint32_t)candidate + (uint32_t)middlelength;
                  prob3 = orc_maxent_antiacceptor(chroffset + sp, chroffset);
                }
              } else {
                if (cdna_direction > 0) {
                  sp = chrpos + (genomiclength - 1u) - (uint32_t)(candidate - 1);
                  prob2 = orc_maxent_antiacceptor(chroffset + sp, chroffset);
                  sp = chrpos + (genomiclength - 1u) - (uint32_t)(candidate + middlelength) + 1u;
                  prob3 = orc_maxent_antidonor(chroffset + sp, chroffset);
                } else {
                  sp = chrpos + (genomiclength - 1u) - (uint32_t)(candidate - 1);
                  prob2 = orc_maxent_donor(chroffset + sp, chroffset);
                  sp = chrpos + (genomiclength - 1u) - (uint32_t)(candidate + middlelength) + 1u;
                  prob3 = orc_maxent_acceptor(chroffset + sp, chroffset);
                }
              }
              if (prob2 + prob3 > bestprob) {
                bestcL = cL;
                bestcR = cR;
                best_middlelength = middlelength;
                o->bestprob2 = prob2;
                o->bestprob3 = prob3;
                bestprob = prob2 + prob3;
              }
            }
          }
        }
      }
    }
  }
  if (bestcL < 0 || bestcR < 0) {
    o->microintrontype = NONINTRON;
    return 0;
  }
  (void)have_candidate;
  o->found = 1;
  o->bestcL = bestcL;
  o->bestcR = bestcR;
  o->middlelength = best_middlelength;
  o->offset2M = candidate; /* the last hit examined (:7412-7413) */
  {
    /* make_microexon_pairs_double (:6949-7055) */
    const int offs1[3] = {offset1, offset1 + bestcL, offset1 + bestcL + best_middlelength};
    const int offs2[3] = {offset2L, candidate, revoffset2R - bestcR + 1};
    const int lens[3] = {bestcL, best_middlelength, bestcR};
    int seg, k;
    for (seg = 0; seg < 3; seg++) {
      for (k = 0; k < lens[seg]; k++) {
        char c1 = queryseq[offs1[seg] + k], c2 = gnt(&g, offs2[seg] + k);
        char comp = queryuc[offs1[seg] + k] == c2 ? '*' : cons[c1 & 127][c2 & 127] ? ':' : ' ';
        push_pair(out, offs1[seg] + k, offs2[seg] + k, c1, comp, c2, dynprogindex);
      }
      if (seg < 2) {
        push_gapholder(out, GSNAPDP_UNKNOWNJUMP, GSNAPDP_UNKNOWNJUMP);
        out->buf[out->head].comp = gapchar; /* gappair->comp = gapchar */
      }
    }
  }
  o->dynprogindex = step_index(dynprogindex);
  return 1;
}

int orc_run_micro_batch(const gsnapdp_micro_window *w, int n, const char *query,
                        const char *query_uc, gsnapdp_micro_result *results, gsnapdp_pair *pairs,
                        const int64_t *pair_offsets, int32_t *npairs) {
  orc_list l;
  int i, t;
  orc_list_init(&l, 256);
  for (i = 0; i < n; i++) {
    const gsnapdp_micro_window *x = &w[i];
    gsnapdp_micro_result *r = &results[i];
    orc_micro_out o;
    int64_t off = pair_offsets[i], cap = pair_offsets[i + 1] - off;
    /* queryseq such that queryseq[offset1 + k] is the staged byte at ppos + k */
    const char *qs = query + (int64_t)x->ppos - x->offset1, *qsu = query_uc + (int64_t)x->ppos - x->offset1;
    orc_microexon_int(&l, &o, x->dynprogindex, query + x->qpos, query_uc + x->qpos, x->length1,
                      x->offset1, x->offset2L, x->revoffset2R, x->cdna_direction, qs, qsu,
                      x->chroffset, x->chrhigh, x->chrpos, x->genomiclength, x->watsonp,
                      (double)x->defect_rate);
    memset(r, 0, sizeof(*r));
    r->bestprob2 = o.bestprob2;
    r->bestprob3 = o.bestprob3;
    r->microintrontype = o.microintrontype;
    r->dynprogindex = o.dynprogindex;
    r->found = o.found;
    r->status = o.unsupported ? 4 : 0;
    r->bestcL = o.bestcL;
    r->bestcR = o.bestcR;
    r->middlelength = o.middlelength;
    r->offset2M = o.offset2M;
    npairs[i] = l.n;
    for (t = 0; t < l.n && t < cap; t++) pairs[off + t] = l.buf[l.head + t];
  }
  orc_list_free(&l);
  return 0;
}
