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

/* The lists run_host produced, by id: fixed chunks of slots that never move,
 * so a reader needs no lock (an id reaches its reader only after the writer's
 * batch has returned); a new chunk is the only locked step. */
typedef struct {
  gsnapdp_pair *p;
  int n;
} stash_t;
#define STASH_CHUNK 65536
#define STASH_CHUNKS 4096
static stash_t *stash[STASH_CHUNKS];
static unsigned long stash_next;
static pthread_mutex_t stash_mu = PTHREAD_MUTEX_INITIALIZER;

static uint32_t put(const gsnapdp_pair *p, int n) {
  const unsigned long id = __atomic_fetch_add(&stash_next, 1UL, __ATOMIC_RELAXED);
  const unsigned long c = id / STASH_CHUNK;
  stash_t *e;
  if (c >= STASH_CHUNKS) {
    fprintf(stderr, "oracle ABI: op-stream stash full\n");
    abort();
  }
  if (!__atomic_load_n(&stash[c], __ATOMIC_ACQUIRE)) {
    pthread_mutex_lock(&stash_mu);
    if (!stash[c]) __atomic_store_n(&stash[c], (stash_t *)calloc(STASH_CHUNK, sizeof(stash_t)), __ATOMIC_RELEASE);
    pthread_mutex_unlock(&stash_mu);
  }
  e = &stash[c][id % STASH_CHUNK];
  e->p = (gsnapdp_pair *)malloc((size_t)(n > 0 ? n : 1) * sizeof(gsnapdp_pair));
  memcpy(e->p, p, (size_t)n * sizeof(gsnapdp_pair));
  e->n = n;
  return (uint32_t)id;
}

static int get(uint32_t id, gsnapdp_pair *out, int cap) {
  const stash_t *e;
  if (id >= __atomic_load_n(&stash_next, __ATOMIC_RELAXED) || !stash[id / STASH_CHUNK]) {
    fprintf(stderr, "oracle ABI: unknown op stream %u\n", id);
    abort();
  }
  e = &stash[id / STASH_CHUNK][id % STASH_CHUNK];
  if (e->n > cap) return -1;
  memcpy(out, e->p, (size_t)e->n * sizeof(gsnapdp_pair));
  return e->n;
}

/* frees every stashed list (between runs of a long-lived process) */
void gsnapdp_oracle_stash_reset(void) {
  unsigned long c, i, n = __atomic_load_n(&stash_next, __ATOMIC_RELAXED);
  for (c = 0; c < STASH_CHUNKS && stash[c]; c++) {
    for (i = 0; i < STASH_CHUNK && c * STASH_CHUNK + i < n; i++) free(stash[c][i].p);
    free(stash[c]);
    stash[c] = NULL;
  }
  stash_next = 0;
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

/* pair capacities of a batch: cap(i) pairs for window i (at least 16) */
static int64_t *pair_offsets(int n, int64_t (*cap)(const void *, int), const void *w) {
  int64_t *po = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n + 1));
  int i;
  po[0] = 0;
  for (i = 0; i < n; i++) {
    int64_t c = cap(w, i);
    po[i + 1] = po[i] + (c > 16 ? c : 16);
  }
  return po;
}
/* each window's list to the stash; ops[op_offsets[i]] names it */
static void stash_all(int n, const gsnapdp_pair *p, const int64_t *po, const int32_t *np, uint32_t *ops,
                      const int64_t *op_offsets) {
  int i;
  for (i = 0; i < n; i++) {
    const uint32_t id = put(p + po[i], np[i] < po[i + 1] - po[i] ? np[i] : (int)(po[i + 1] - po[i]));
    if (op_offsets[i + 1] > op_offsets[i]) ops[op_offsets[i]] = id;
  }
}

static int64_t gap_cap(const void *w, int i) {
  const gsnapdp_window *x = (const gsnapdp_window *)w + i;
  return 2 * (int64_t)(x->length1 + x->length2) + 16;
}
/* the whole batch through the oracle's batch driver (one workspace); the pairs
 * go to the stash and ops[op_offsets[i]] names them */
int gsnapdp_run_host(gsnapdp_ctx *ctx, const gsnapdp_window *windows, int n, const char *query,
                     const char *query_uc, size_t query_bytes, gsnapdp_result *results,
                     uint32_t *ops, const int64_t *op_offsets) {
  int i;
  int64_t *po;
  gsnapdp_pair *p;
  int32_t *np;
  (void)ctx;
  (void)query_bytes;
  if (n <= 0) return 0;
  po = pair_offsets(n, gap_cap, windows);
  p = (gsnapdp_pair *)malloc((size_t)po[n] * sizeof(gsnapdp_pair));
  np = (int32_t *)calloc((size_t)n, sizeof(int32_t));
  orc_run_batch(windows, n, query, query_uc, results, p, po, np, 1);
  for (i = 0; i < n; i++) results[i].status = 0;
  stash_all(n, p, po, np, ops, op_offsets);
  free(p);
  free(np);
  free(po);
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
static int64_t ggap_cap(const void *w, int i) {
  const gsnapdp_ggap_window *x = (const gsnapdp_ggap_window *)w + i;
  return 2 * (int64_t)x->length1 + x->length2L + x->length2R + 16;
}
/* the whole batch at once; a window with op capacity stashes its list there
 * (the stage-3 pass), the others' expansion re-runs the window */
int gsnapdp_ggap_run_host(gsnapdp_ctx *c, const gsnapdp_ggap_window *w, int n, const char *q,
                          const char *u, size_t b, gsnapdp_ggap_result *r, gsnapdp_ggap_trace *t,
                          uint32_t *o, const int64_t *off) {
  int i;
  int64_t *po;
  gsnapdp_pair *p;
  int32_t *np;
  (void)c, (void)b;
  if (n <= 0) return 0;
  po = pair_offsets(n, ggap_cap, w);
  p = (gsnapdp_pair *)malloc((size_t)po[n] * sizeof(gsnapdp_pair));
  np = (int32_t *)calloc((size_t)n, sizeof(int32_t));
  orc_run_ggap_batch(w, n, q, u, r, p, po, np);
  for (i = 0; i < n; i++) {
    gsnapdp_ggap_trace *x = &t[i];
    memset(x, 0, sizeof(*x));
    if (w[i].length1 <= 1 || w[i].maxlength1 < 0) {
      x->status = 1;
    } else if (r[i].bridge_ok) {
      x->bridge_accepted = !(r[i].returned_null && r[i].new_leftgenomepos == 0 && r[i].new_rightgenomepos == 0 &&
                             r[i].exonhead == 0);
    }
  }
  if (o && off) stash_all(n, p, po, np, o, off);
  free(p);
  free(np);
  free(po);
  return 0;
}
/* expansion fetches the stashed list, or re-runs the window (its query bytes
 * are the caller's own) when the run had no op capacity */
int gsnapdp_ggap_expand(gsnapdp_ctx *c, const gsnapdp_ggap_window *w, const gsnapdp_ggap_result *r,
                        const gsnapdp_ggap_trace *t, const uint32_t *o, const char *q, const char *u,
                        gsnapdp_pair *p, int cap) {
  gsnapdp_ggap_result rr;
  int32_t np = 0;
  (void)c, (void)r, (void)t;
  if (o) return get(o[0], p, cap);
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
static int64_t cgap_cap(const void *w, int i) {
  const gsnapdp_cgap_window *x = (const gsnapdp_cgap_window *)w + i;
  return (int64_t)x->length1L + x->length1R + 2 * (int64_t)x->length2 + 32;
}
int gsnapdp_cgap_run_host(gsnapdp_ctx *c, const gsnapdp_cgap_window *w, int n, const char *q,
                          const char *u, size_t b, gsnapdp_cgap_result *r, uint32_t *o,
                          const int64_t *off) {
  int i;
  int64_t *so, *po;
  char *seg;
  gsnapdp_pair *p;
  int32_t *np;
  (void)c, (void)b;
  if (n <= 0) return 0;
  so = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n + 1));
  so[0] = 0;
  for (i = 0; i < n; i++) so[i + 1] = so[i] + (w[i].length2 > 0 ? w[i].length2 : 0) + 8;
  seg = (char *)calloc((size_t)so[n] + 8, 1);
  for (i = 0; i < n; i++) {
    char *s = cgap_segment(&w[i]);
    memcpy(seg + so[i], s, (size_t)(so[i + 1] - so[i]));
    free(s);
  }
  po = pair_offsets(n, cgap_cap, w);
  p = (gsnapdp_pair *)malloc((size_t)po[n] * sizeof(gsnapdp_pair));
  np = (int32_t *)calloc((size_t)n, sizeof(int32_t));
  orc_run_cgap_batch(w, n, q, u, seg, so, r, p, po, np);
  if (o && off) stash_all(n, p, po, np, o, off);
  free(p);
  free(np);
  free(po);
  free(seg);
  free(so);
  return 0;
}
int gsnapdp_cgap_expand(gsnapdp_ctx *c, const gsnapdp_cgap_window *w, const gsnapdp_cgap_result *r,
                        const uint32_t *o, const char *q, const char *u, const char *s2,
                        gsnapdp_pair *p, int cap) {
  gsnapdp_cgap_result rr;
  int64_t zero = 0, po[2] = {0, cap};
  int32_t np = 0;
  char *s;
  (void)c, (void)r;
  if (o && !s2) return get(o[0], p, cap);
  s = s2 ? NULL : cgap_segment(w);
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
