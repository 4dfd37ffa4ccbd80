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
