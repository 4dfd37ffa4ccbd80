/*
 * maxent_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Clean-room restatement of Maxent_hr_{donor,acceptor,antidonor,
 * antiacceptor}_prob (src/maxent_hr.c:27217-27390).  The reference unrolls
 * each model into 32 shift-specialised handlers (:24816-27180); all of them
 * read the k-mer that starts `off` nucleotides after startpos from the
 * 128-bit little-endian window (low, high, nextlow, nexthigh) of two
 * consecutive genome blocks.  This file states that once, generically.
 * Parity with the handlers is pinned per shift in tests/test_oracle_golden.py.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "dp_oracle.h"

/* Table order (= declaration order in maxent_hr.c:25-22606). */
enum {
  T_DONOR_PLUS, T_DONOR_DI_PLUS, T_ACC1_PLUS, T_ACC2_PLUS, T_ACC3_PLUS, T_ACC_DI_PLUS,
  T_ACC467_PLUS, T_ACC589_PLUS, T_DONOR_MINUS, T_DONOR_DI_MINUS, T_ACC1_MINUS, T_ACC2_MINUS,
  T_ACC3_MINUS, T_ACC_DI_MINUS, T_ACC467_MINUS, T_ACC589_MINUS, T_NTABLES
};
static const int table_len[T_NTABLES] = {16384, 16, 16384, 16384, 16384, 16, 16384, 16384,
                                         16384, 16, 16384, 16384, 16384, 16, 16384, 16384};
static const double *tab[T_NTABLES];
static double *tab_store;

extern const uint32_t *orc_genome_blocks(void);

int orc_maxent_load(const double *tables, size_t ndoubles) {
  size_t need = 0, off = 0;
  int t;
  for (t = 0; t < T_NTABLES; t++) need += (size_t)table_len[t];
  if (ndoubles != need) return -1;
  free(tab_store);
  tab_store = (double *)malloc(need * sizeof(double));
  memcpy(tab_store, tables, need * sizeof(double));
  for (t = 0; t < T_NTABLES; t++) {
    tab[t] = tab_store + off;
    off += (size_t)table_len[t];
  }
  return 0;
}

/* k-mer bits starting `off` nt after startpos (2 bits per nt, LSB first). */
static inline uint32_t window_seq(const uint32_t *blocks, uint32_t startpos, int off) {
  uint32_t ptr = startpos / 32u * 3u;
  int bit = 2 * (int)(startpos % 32u) + 2 * off;
  unsigned __int128 v = (unsigned __int128)blocks[ptr + 1] |
                        ((unsigned __int128)blocks[ptr] << 32) |
                        ((unsigned __int128)blocks[ptr + 4] << 64) |
                        ((unsigned __int128)blocks[ptr + 3] << 96);
  return (uint32_t)(v >> bit);
}

static const uint32_t *blocks(void) { return orc_genome_blocks(); }

double orc_maxent_donor(uint32_t splice_pos, uint32_t chroffset) {
  uint32_t s;
  double odds;
  if (splice_pos < chroffset + 3u) return 0.0; /* DONOR_MODEL_LEFT_MARGIN */
  s = window_seq(blocks(), splice_pos - 3u, 0);
  odds = tab[T_DONOR_PLUS][(s & 0x3Fu) | ((s >> 4) & 0x3FC0u)] * tab[T_DONOR_DI_PLUS][(s >> 6) & 0xFu];
  return odds / (1 + odds);
}

double orc_maxent_antidonor(uint32_t splice_pos, uint32_t chroffset) {
  uint32_t s;
  double odds;
  if (splice_pos < chroffset + 6u) return 0.0; /* DONOR_MODEL_RIGHT_MARGIN */
  s = window_seq(blocks(), splice_pos - 6u, 0);
  odds = tab[T_DONOR_MINUS][(s & 0xFFu) | ((s >> 4) & 0x3F00u)] * tab[T_DONOR_DI_MINUS][(s >> 8) & 0xFu];
  return odds / (1 + odds);
}

double orc_maxent_acceptor(uint32_t splice_pos, uint32_t chroffset) {
  uint32_t sp, s;
  double odds;
  const uint32_t *b = blocks();
  if (splice_pos < chroffset + 20u) return 0.0; /* ACCEPTOR_MODEL_LEFT_MARGIN */
  sp = splice_pos - 20u;
  odds = tab[T_ACC1_PLUS][window_seq(b, sp, 0) & 0x3FFFu];
  odds *= tab[T_ACC2_PLUS][window_seq(b, sp, 7) & 0x3FFFu];
  s = window_seq(b, sp, 14);
  odds *= tab[T_ACC3_PLUS][(s & 0xFFu) | ((s >> 4) & 0x3F00u)];
  odds *= tab[T_ACC_DI_PLUS][(s >> 8) & 0xFu];
  odds *= tab[T_ACC467_PLUS][window_seq(b, sp, 4) & 0x3FFFu];
  odds *= tab[T_ACC589_PLUS][window_seq(b, sp, 11) & 0x3FFFu];
  return odds / (1 + odds);
}

double orc_maxent_antiacceptor(uint32_t splice_pos, uint32_t chroffset) {
  uint32_t sp, s;
  double odds;
  const uint32_t *b = blocks();
  if (splice_pos < chroffset + 3u) return 0.0; /* ACCEPTOR_MODEL_RIGHT_MARGIN */
  sp = splice_pos - 3u;
  odds = tab[T_ACC1_MINUS][window_seq(b, sp, 16) & 0x3FFFu];
  odds *= tab[T_ACC2_MINUS][window_seq(b, sp, 9) & 0x3FFFu];
  s = window_seq(b, sp, 0);
  odds *= tab[T_ACC3_MINUS][(s & 0x3Fu) | ((s >> 4) & 0x3FC0u)];
  odds *= tab[T_ACC_DI_MINUS][(s >> 6) & 0xFu];
  odds *= tab[T_ACC467_MINUS][window_seq(b, sp, 12) & 0x3FFFu];
  odds *= tab[T_ACC589_MINUS][window_seq(b, sp, 5) & 0x3FFFu];
  return odds / (1 + odds);
}

void orc_maxent_batch(const uint8_t *model, const uint32_t *pos, const uint32_t *chroffset,
                      double *out, int n) {
  int i;
  for (i = 0; i < n; i++) {
    switch (model[i]) {
      case 0: out[i] = orc_maxent_donor(pos[i], chroffset[i]); break;
      case 1: out[i] = orc_maxent_acceptor(pos[i], chroffset[i]); break;
      case 2: out[i] = orc_maxent_antidonor(pos[i], chroffset[i]); break;
      default: out[i] = orc_maxent_antiacceptor(pos[i], chroffset[i]); break;
    }
  }
}

/* ---- score_introns (stage3.c:7935-8162), TEST INFRASTRUCTURE ONLY.
 * orc_path_introns restates the walk over a path (the pop loop of :7960-8146):
 * a gap pair counts as an intron unless past nullgap (:7971) or query-heavy
 * (:7979), when its genomejump exceeds queryjump + MININTRONLEN_FINAL (50,
 * stage3.c:52, :7987); leftpair = path->first after the pop (the next list
 * element), rightpair = pairs->first (the previous one).  Returns the count,
 * or -1 where the reference would dereference NULL. */
int orc_path_introns(const gsnapdp_path_pair *pairs, int npairs, int nullgap, int path,
                     gsnapdp_intron *out, int cap) {
  int i, n = 0;
  for (i = 0; i < npairs; i++) {
    const gsnapdp_path_pair *pair = &pairs[i];
    if (pair->gapp == 0) continue;                               /* :7964 */
    if (pair->queryjump > nullgap) continue;                     /* :7971 */
    if (pair->queryjump > pair->genomejump + 10) continue;       /* :7979, EXTRAQUERYGAP stage3.h:29 */
    if (pair->genomejump > pair->queryjump + 50) {               /* :7987 */
      if (i == 0 || i == npairs - 1) return -1;                  /* pairs->first / path->first of NULL */
      if (n < cap) {
        out[n].left_genomepos = pairs[i + 1].genomepos;
        out[n].right_genomepos = pairs[i - 1].genomepos;
        out[n].path = path;
        out[n].comp = pair->comp;
        out[n].knowngapp = pair->knowngapp;
        out[n].known_donor = out[n].known_acceptor = 0;
      }
      n++;
    }
  }
  return n;
}

/* The probabilities and their averages, one path at a time in list order
 * (:7992-8129, :8154-8157).  A known site (the splicing IIT) scores 1.0. */
void orc_score_introns(const gsnapdp_intron_path *paths, int npaths, const gsnapdp_intron *introns,
                       gsnapdp_intron_scores *out) {
  int p, k;
  for (p = 0; p < npaths; p++) {
    const gsnapdp_intron_path *x = &paths[p];
    double avg_donor_score = 0.0, avg_acceptor_score = 0.0, donor_score, acceptor_score;
    int nbadintrons = 0, nintrons = 0;
    uint32_t splicesitepos;
    for (k = 0; k < x->nintrons; k++) {
      const gsnapdp_intron *t = &introns[x->first_intron + k];
      if (x->cdna_direction == +1) {
        if (x->watsonp) {
          splicesitepos = x->chrpos + t->left_genomepos + 1;                                   /* :7997 */
          donor_score = t->known_donor ? 1.0 : orc_maxent_donor(x->chroffset + splicesitepos, x->chroffset);
          splicesitepos = x->chrpos + t->right_genomepos;                                      /* :8007 */
          acceptor_score = t->known_acceptor ? 1.0
                                             : orc_maxent_acceptor(x->chroffset + splicesitepos, x->chroffset);
        } else {
          splicesitepos = x->chrpos + (uint32_t)(x->genomiclength - 1) - t->left_genomepos;    /* :8018 */
          donor_score = t->known_donor ? 1.0 : orc_maxent_antidonor(x->chroffset + splicesitepos, x->chroffset);
          splicesitepos = x->chrpos + (uint32_t)(x->genomiclength - 1) - t->right_genomepos + 1; /* :8028 */
          acceptor_score = t->known_acceptor ? 1.0
                                             : orc_maxent_antiacceptor(x->chroffset + splicesitepos, x->chroffset);
        }
        nintrons += 1;
        if (t->knowngapp) {
          /* skip */
        } else if (t->comp == '>' && (donor_score < 0.9 && acceptor_score < 0.9)) {
          nbadintrons = 1;                                                                     /* :8048 (sic) */
        }
        avg_donor_score += donor_score;
        avg_acceptor_score += acceptor_score;
      } else if (x->cdna_direction == -1) {
        if (x->watsonp) {
          splicesitepos = x->chrpos + t->left_genomepos + 1;                                   /* :8069 */
          acceptor_score = t->known_acceptor ? 1.0
                                             : orc_maxent_antiacceptor(x->chroffset + splicesitepos, x->chroffset);
          splicesitepos = x->chrpos + t->right_genomepos;                                      /* :8080 */
          donor_score = t->known_donor ? 1.0 : orc_maxent_antidonor(x->chroffset + splicesitepos, x->chroffset);
        } else {
          splicesitepos = x->chrpos + (uint32_t)(x->genomiclength - 1) - t->left_genomepos;    /* :8091 */
          acceptor_score = t->known_acceptor ? 1.0
                                             : orc_maxent_acceptor(x->chroffset + splicesitepos, x->chroffset);
          splicesitepos = x->chrpos + (uint32_t)(x->genomiclength - 1) - t->right_genomepos + 1; /* :8101 */
          donor_score = t->known_donor ? 1.0 : orc_maxent_donor(x->chroffset + splicesitepos, x->chroffset);
        }
        nintrons += 1;
        if (t->knowngapp) {
          /* skip */
        } else if (t->comp == '<' && (donor_score < 0.9 && acceptor_score < 0.9)) {
          nbadintrons += 1;                                                                    /* :8119 */
        }
        avg_donor_score += donor_score;
        avg_acceptor_score += acceptor_score;
      }
    }
    if (nintrons > 0) {
      avg_donor_score /= (double)nintrons;
      avg_acceptor_score /= (double)nintrons;
    }
    out[p].avg_donor_score = avg_donor_score;
    out[p].avg_acceptor_score = avg_acceptor_score;
    out[p].nbadintrons = nbadintrons;
    out[p].nintrons = nintrons;
  }
}
