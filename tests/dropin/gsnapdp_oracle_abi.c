/*
 * gsnapdp_oracle_abi.c -- TEST INFRASTRUCTURE ONLY (never shipped, never on a GPU box).
 *
 * The batched C-ABI of include/gsnapdp.h served on the CPU by the oracle's
 * restatement (oracle/dp_oracle.c), for the subset the drop-in's known-site
 * ends and the stage-3 intron pass use: end and single gaps (gsnapdp_run_host /
 * gsnapdp_expand), splice-junction ends (gsnapdp_sj_*), genome gaps, cDNA gaps,
 * microexons (expansion re-runs the window) and MaxEnt.  It exists so that the
 * drop-in's host control flow (gmap-gsnap_amd/csrc/gsnapdp_dropin.cpp) can be
 * linked, without a GPU, against the reference's own splicetrie.o / pairpool.o /
 * list.o and run under AddressSanitizer (oracle/Makefile `asan`,
 * tests/test_dropin_asan_cpu.py): the production configuration of
 * Dynprog_end5/3_known (dynprog.c:6414-6943) with the host program's
 * Splicetrie_solve_end5/3 (splicetrie.c:881, 952).
 *
 * It also serves gsnapdp_stage3_pass (gmap-gsnap_amd/csrc/gsnapdp_stage3.cpp)
 * for tests/test_stage3_cpu.py.  The op stream between run and expand is this
 * file's own: ops[0] of a gap or splice-junction window is an index into a
 * table of pair lists that run_host filled.
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/gsnapdp.h"
#include "../../oracle/dp_oracle.h"

struct gsnapdp_ctx {
  int mode;
  const uint32_t *blocks;
  size_t nwords;
};

typedef struct {
  gsnapdp_pair *p;
  int n;
} stash_t;
static stash_t *stash;
static size_t nstash, capstash;
static pthread_mutex_t stash_mu = PTHREAD_MUTEX_INITIALIZER;

static uint32_t put(const gsnapdp_pair *p, int n) {
  uint32_t id;
  pthread_mutex_lock(&stash_mu);
  if (nstash == capstash) {
    capstash = capstash ? 2 * capstash : 256;
    stash = (stash_t *)realloc(stash, capstash * sizeof(stash_t));
  }
  stash[nstash].p = (gsnapdp_pair *)malloc((size_t)(n > 0 ? n : 1) * sizeof(gsnapdp_pair));
  memcpy(stash[nstash].p, p, (size_t)n * sizeof(gsnapdp_pair));
  stash[nstash].n = n;
  id = (uint32_t)nstash++;
  pthread_mutex_unlock(&stash_mu);
  return id;
}

static int get(uint32_t id, gsnapdp_pair *out, int cap) {
  int n;
  pthread_mutex_lock(&stash_mu);
  if (id >= nstash) {
    pthread_mutex_unlock(&stash_mu);
    fprintf(stderr, "oracle ABI: unknown op stream %u\n", id);
    abort();
  }
  n = stash[id].n;
  if (n > cap) n = -1;
  else memcpy(out, stash[id].p, (size_t)n * sizeof(gsnapdp_pair));
  pthread_mutex_unlock(&stash_mu);
  return n;
}

gsnapdp_ctx *gsnapdp_create(int device, const uint32_t *blocks, size_t nblocks_u32, int mode) {
  gsnapdp_ctx *c = (gsnapdp_ctx *)calloc(1, sizeof(gsnapdp_ctx));
  (void)device;
  c->mode = mode;
  c->blocks = blocks;
  c->nwords = nblocks_u32;
  orc_init(mode);
  orc_set_genome(blocks);
  return c;
}
void gsnapdp_destroy(gsnapdp_ctx *ctx) { free(ctx); }
const char *gsnapdp_last_error(void) { return "oracle ABI"; }
void *gsnapdp_host_alloc(size_t bytes) { return malloc(bytes); }
void gsnapdp_host_free(void *p) { free(p); }
int gsnapdp_load_maxent_tables(gsnapdp_ctx *ctx, const double *tables, size_t ndoubles) {
  (void)ctx;
  return orc_maxent_load(tables, ndoubles);
}
int gsnapdp_maxent_host(gsnapdp_ctx *ctx, const uint8_t *model, const uint32_t *splice_pos,
                        const uint32_t *chroffset, double *out, int n) {
  int i;
  (void)ctx;
  for (i = 0; i < n; i++) {
    switch (model[i]) {
      case 0: out[i] = orc_maxent_donor(splice_pos[i], chroffset[i]); break;
      case 1: out[i] = orc_maxent_acceptor(splice_pos[i], chroffset[i]); break;
      case 2: out[i] = orc_maxent_antidonor(splice_pos[i], chroffset[i]); break;
      default: out[i] = orc_maxent_antiacceptor(splice_pos[i], chroffset[i]); break;
    }
  }
  return 0;
}

/* one window at a time through the oracle's batch drivers; the pairs go to the
 * stash and ops[op_offsets[i]] names them */
int gsnapdp_run_host(gsnapdp_ctx *ctx, const gsnapdp_window *windows, int n, const char *query,
                     const char *query_uc, size_t query_bytes, gsnapdp_result *results,
                     uint32_t *ops, const int64_t *op_offsets) {
  int i;
  (void)ctx;
  (void)query_bytes;
  for (i = 0; i < n; i++) {
    const int64_t cap = 2 * (int64_t)(windows[i].length1 + windows[i].length2) + 16;
    int64_t po[2] = {0, cap};
    int32_t np = 0;
    gsnapdp_pair *p = (gsnapdp_pair *)malloc((size_t)cap * sizeof(gsnapdp_pair));
    orc_run_batch(&windows[i], 1, query, query_uc, &results[i], p, po, &np, 1);
    results[i].status = 0;
    ops[op_offsets[i]] = put(p, np);
    free(p);
  }
  return 0;
}

int gsnapdp_expand(gsnapdp_ctx *ctx, const gsnapdp_window *w, const gsnapdp_result *res,
                   const uint32_t *ops, const char *query, const char *query_uc,
                   gsnapdp_pair *pairs, int cap, int *finalscore) {
  (void)ctx;
  (void)w;
  (void)query;
  (void)query_uc;
  if (finalscore) *finalscore = res->finalscore;
  return get(ops[0], pairs, cap);
}

int gsnapdp_sj_run_host(gsnapdp_ctx *ctx, const gsnapdp_sj_window *windows, int n,
                        const char *query, const char *query_uc, size_t query_bytes,
                        gsnapdp_result *results, uint32_t *ops, const int64_t *op_offsets) {
  int i;
  (void)ctx;
  (void)query_bytes;
  for (i = 0; i < n; i++) {
    const int64_t cap = 2 * (int64_t)(windows[i].length1 + windows[i].length2) + 16;
    int64_t po[2] = {0, cap};
    int32_t np = 0;
    gsnapdp_pair *p = (gsnapdp_pair *)malloc((size_t)cap * sizeof(gsnapdp_pair));
    orc_run_sj_batch(&windows[i], 1, query, query_uc, &results[i], p, po, &np);
    results[i].status = 0;
    ops[op_offsets[i]] = put(p, np);
    free(p);
  }
  return 0;
}

int gsnapdp_sj_expand(gsnapdp_ctx *ctx, const gsnapdp_sj_window *w, const gsnapdp_result *res,
                      const uint32_t *ops, const char *query, const char *query_uc,
                      gsnapdp_pair *pairs, int cap) {
  (void)ctx;
  (void)w;
  (void)res;
  (void)query;
  (void)query_uc;
  return get(ops[0], pairs, cap);
}

/* genome gaps: the oracle's out-parameters, and the trace's status and
 * bridge_accepted read off them (orc_genome_gap returns early for length1 <= 1
 * or a too-long window, and leaves the intron ends unwritten, 0, when the
 * bridge takes no candidate) */
static void ggap_one(const gsnapdp_ggap_window *w, const char *q, const char *u, gsnapdp_ggap_result *r,
                     gsnapdp_ggap_trace *t, gsnapdp_pair *pairs, int cap, int32_t *np) {
  int64_t po[2] = {0, cap};
  orc_run_ggap_batch(w, 1, q, u, r, pairs, pairs ? po : NULL, np);
  if (t) {
    memset(t, 0, sizeof(*t));
    if (w->length1 <= 1 || w->maxlength1 < 0) {
      t->status = 1;
    } else if (r->bridge_ok) {
      t->bridge_accepted = !(r->returned_null && r->new_leftgenomepos == 0 && r->new_rightgenomepos == 0 &&
                             r->exonhead == 0);
    }
  }
}
int gsnapdp_ggap_run_host(gsnapdp_ctx *c, const gsnapdp_ggap_window *w, int n, const char *q,
                          const char *u, size_t b, gsnapdp_ggap_result *r, gsnapdp_ggap_trace *t,
                          uint32_t *o, const int64_t *off) {
  int i;
  (void)c, (void)b, (void)o, (void)off;
  for (i = 0; i < n; i++) ggap_one(&w[i], q, u, &r[i], &t[i], NULL, 0, NULL);
  return 0;
}
/* expansion re-runs the window (its query bytes are the caller's own) */
int gsnapdp_ggap_expand(gsnapdp_ctx *c, const gsnapdp_ggap_window *w, const gsnapdp_ggap_result *r,
                        const gsnapdp_ggap_trace *t, const uint32_t *o, const char *q, const char *u,
                        gsnapdp_pair *p, int cap) {
  gsnapdp_ggap_result rr;
  int32_t np = 0;
  (void)c, (void)r, (void)t, (void)o;
  ggap_one(w, q, u, &rr, NULL, p, cap, &np);
  return np > cap ? -1 : np;
}
/* the reference's sequence2 of a cDNA gap: get_genomic_nt from offset2 on */
static char *cgap_segment(const gsnapdp_cgap_window *w) {
  int k, n = w->length2 > 0 ? w->length2 : 0;
  char *s = (char *)calloc((size_t)n + 8, 1);
  for (k = 0; k < n; k++)
    s[k] = orc_get_genomic_nt(w->offset2 + k, w->chroffset, w->chrhigh, w->chrpos, (int)w->genomiclength,
                              w->watsonp);
  return s;
}
int gsnapdp_cgap_run_host(gsnapdp_ctx *c, const gsnapdp_cgap_window *w, int n, const char *q,
                          const char *u, size_t b, gsnapdp_cgap_result *r, uint32_t *o,
                          const int64_t *off) {
  int i;
  int64_t zero = 0;
  (void)c, (void)b, (void)o, (void)off;
  for (i = 0; i < n; i++) {
    char *s = cgap_segment(&w[i]);
    orc_run_cgap_batch(&w[i], 1, q, u, s, &zero, &r[i], NULL, NULL, NULL);
    free(s);
  }
  return 0;
}
int gsnapdp_cgap_expand(gsnapdp_ctx *c, const gsnapdp_cgap_window *w, const gsnapdp_cgap_result *r,
                        const uint32_t *o, const char *q, const char *u, const char *s2,
                        gsnapdp_pair *p, int cap) {
  gsnapdp_cgap_result rr;
  int64_t zero = 0, po[2] = {0, cap};
  int32_t np = 0;
  char *s = s2 ? NULL : cgap_segment(w);
  (void)c, (void)r, (void)o;
  orc_run_cgap_batch(w, 1, q, u, s2 ? s2 : s, &zero, &rr, p, po, &np);
  free(s);
  return np > cap ? -1 : np;
}
int gsnapdp_micro_run_host(gsnapdp_ctx *c, const gsnapdp_micro_window *w, int n, const char *q,
                           const char *u, size_t b, gsnapdp_micro_result *r) {
  int i;
  (void)c, (void)b;
  for (i = 0; i < n; i++) {
    int64_t po[2] = {0, 0};
    int32_t np = 0;
    orc_run_micro_batch(&w[i], 1, q, u, &r[i], NULL, po, &np);
  }
  return 0;
}
int gsnapdp_micro_expand(gsnapdp_ctx *c, const gsnapdp_micro_window *w, const gsnapdp_micro_result *r,
                         const char *q, const char *u, gsnapdp_pair *p, int cap) {
  gsnapdp_micro_result rr;
  int64_t po[2] = {0, cap};
  int32_t np = 0;
  (void)c, (void)r;
  orc_run_micro_batch(w, 1, q, u, &rr, p, po, &np);
  return np > cap ? -1 : np;
}

/* the product's internal accessors gsnapdp_stage3.cpp reads */
const uint32_t *gsnapdp__host_blocks(gsnapdp_ctx *ctx) { return ctx->blocks; }
size_t gsnapdp__host_nwords(gsnapdp_ctx *ctx) { return ctx->nwords; }

/* score_introns for gsnapdp_stage3_score_introns: the oracle's walk and sums */
int gsnapdp_path_introns(const gsnapdp_path_pair *pairs, int npairs, int nullgap, int path, gsnapdp_intron *out,
                         int cap) {
  return orc_path_introns(pairs, npairs, nullgap, path, out, cap);
}
int gsnapdp_score_introns_host(gsnapdp_ctx *ctx, const gsnapdp_intron_path *paths, int npaths,
                               const gsnapdp_intron *introns, int nintrons, gsnapdp_intron_scores *out) {
  (void)ctx, (void)nintrons;
  orc_score_introns(paths, npaths, introns, out);
  return 0;
}
