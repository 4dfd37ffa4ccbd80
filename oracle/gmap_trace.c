/*
 * gmap_trace.c -- TEST INFRASTRUCTURE ONLY (linked into oracle/_ref/gmap_trace,
 * dev container only, never shipped, never sent to the GPU box).
 *
 * Records the DP windows the reference's gmap program issues, as golden-vector
 * inputs in the record layouts of include/gsnapdp.h.  The reference's own gmap
 * objects are linked with -Wl,--wrap for the gap fillers, so each call stage 3
 * makes (stage3.c:5442-7003) lands here, is recorded, and then runs the
 * reference's own function (__real_*), so gmap's output is unchanged.  The
 * reference's result is recorded too, so that gen_golden.py can check that
 * ref_driver's replay of each recorded window reproduces what gmap got.
 *
 * At exit, with $GMAP_TRACE_DIR set, writes
 *   $GMAP_TRACE_DIR/dp/{windows.bin,query.bin,query_uc.bin,genome.u32,gmap_results.bin}
 *   $GMAP_TRACE_DIR/ggap/{ggap_windows.bin,query.bin,query_uc.bin,genome.u32,gmap_results.bin}
 *   $GMAP_TRACE_DIR/si/{paths.bin,pairs.bin}: every score_introns call (stage3.c:7935),
 *     the path it was given (pair by pair, in list order) and its three outputs;
 *   $GMAP_TRACE_DIR/bpi/{calls,pairs_in,pairs_out,query,query_uc}.bin: every
 *     build_pairs_introns call (stage3.c:7735), one stage-3 intron pass over one path.
 * score_introns and build_pairs_introns are static, so they cannot be wrapped
 * at link time: stage3_si.c hands their addresses over and a hook is patched
 * over each entry at start (x86-64 movabs/jmp); the hook restores the entry,
 * runs the reference's function, records and re-patches (gmap is
 * single-threaded here).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include "bool.h"
#include "chrnum.h"
#include "dynprog.h"
#include "list.h"
#include "listdef.h"
#include "pairdef.h"

#include "../include/gsnapdp.h"

typedef struct {
  char *p;
  size_t n, cap;
} Buf;

static void put(Buf *b, const void *src, size_t n) {
  if (b->n + n > b->cap) {
    b->cap = (b->n + n) * 2 + 4096;
    b->p = (char *)realloc(b->p, b->cap);
    if (!b->p) abort();
  }
  memcpy(b->p + b->n, src, n);
  b->n += n;
}

/* per-kind trace: window records, query bytes, reference results */
typedef struct {
  Buf win, q, qu, res;
} Trace;

static Trace dp, gg;
static Buf si_paths, si_pairs;
static const unsigned int *genome_blocks = NULL;
static size_t genome_nwords = 0;

/* result of the real call, as the test compares it */
typedef struct {
  int32_t finalscore, nmatches, nmismatches, nopens, nindels, dynprogindex, npairs, pad;
} Recorded;

/* query bytes the reference may read: [0, L1) forwards, or [-(L1-1), 0] behind a rev pointer;
 * padded to a 4-byte boundary (the batch buffers are read with dword loads) */
static uint32_t put_query(Trace *t, const char *s, const char *su, int L1, int rev) {
  const int n = L1 > 0 ? L1 : 0;
  const uint32_t base = (uint32_t)t->q.n;
  static const char zero[8] = {0};
  if (n) {
    put(&t->q, rev ? s - (n - 1) : s, (size_t)n);
    put(&t->qu, rev ? su - (n - 1) : su, (size_t)n);
  }
  put(&t->q, zero, 8 - (size_t)(n & 3));
  put(&t->qu, zero, 8 - (size_t)(n & 3));
  return rev ? base + (uint32_t)(n ? n - 1 : 0) : base;
}

static float bin(double defect_rate) { /* dynprog.c:4471-4486: only the bin matters */
  return defect_rate < 0.003 ? 0.001f : (defect_rate < 0.014 ? 0.01f : 0.5f);
}

static void record_result(Trace *t, int dpi, int fs, int nm, int nmm, int no, int ni, List_T pairs) {
  Recorded r = {fs, nm, nmm, no, ni, dpi, List_length(pairs), 0};
  put(&t->res, &r, sizeof(r));
}

static void base_window(gsnapdp_window *w, int kind, Dynprog_T dynprog, int dpi, int length1, int length2,
                        int offset1, int offset2, Genomicpos_T chroffset, Genomicpos_T chrhigh,
                        Genomicpos_T chrpos, Genomicpos_T genomiclength, int cdna_direction, bool watsonp,
                        bool jump_late_p, int extraband, double defect_rate) {
  memset(w, 0, sizeof(*w));
  w->kind = kind;
  w->length1 = length1;
  w->length2 = length2;
  w->offset1 = offset1;
  w->offset2 = offset2;
  w->chroffset = chroffset;
  w->chrhigh = chrhigh;
  w->chrpos = chrpos;
  w->genomiclength = genomiclength;
  w->cdna_direction = cdna_direction;
  w->extraband = extraband;
  w->dynprogindex = dpi;
  w->maxlength1 = ((int *)dynprog)[0]; /* struct Dynprog_T starts maxlength1, maxlength2 (dynprog.c:823-825) */
  w->maxlength2 = ((int *)dynprog)[1];
  w->defect_rate = bin(defect_rate);
  w->watsonp = watsonp ? 1 : 0;
  w->jump_late_p = jump_late_p ? 1 : 0;
}


/* the 12-byte entry patch of a static reference function: movabs rax, hook; jmp rax */
typedef struct {
  unsigned char saved[12], patch[12];
  unsigned char *entry;
} Patch;
static void patch_install(Patch *p, void *fn, void *hook) {
  const long pg = sysconf(_SC_PAGESIZE);
  const uint64_t target = (uint64_t)hook;
  uintptr_t lo;
  p->entry = (unsigned char *)fn;
  lo = (uintptr_t)p->entry & ~(uintptr_t)(pg - 1);
  if (mprotect((void *)lo, (size_t)(2 * pg), PROT_READ | PROT_WRITE | PROT_EXEC) != 0) abort();
  memcpy(p->saved, p->entry, sizeof(p->saved));
  p->patch[0] = 0x48; /* movabs rax, imm64 */
  p->patch[1] = 0xB8;
  memcpy(p->patch + 2, &target, 8);
  p->patch[10] = 0xFF; /* jmp rax */
  p->patch[11] = 0xE0;
  memcpy(p->entry, p->patch, sizeof(p->patch));
}
static void patch_off(Patch *p) { memcpy(p->entry, p->saved, sizeof(p->saved)); }
static void patch_on(Patch *p) { memcpy(p->entry, p->patch, sizeof(p->patch)); }

/* ---- score_introns (stage3.c:7935-8162), static: patched at start */
typedef List_T (*si_fn_t)(double *, double *, int *, List_T, int, bool, int, Genomicpos_T, Genomicpos_T,
                          Genomicpos_T, char *, int, int, bool);
extern void *gmap_trace_score_introns_fn(void);
static Patch si_p;

typedef struct { /* one call: the arguments, the outputs, the path's extent in pairs.bin */
  int32_t cdna_direction, watsonp, chrnum, genomiclength, nullgap, use_genomicseg_p;
  uint32_t chroffset, chrhigh, chrpos;
  int32_t first_pair, npairs, nbadintrons;
  double avg_donor_score, avg_acceptor_score;
} SiCall;
typedef struct { /* the Pair_T fields score_introns reads */
  int32_t querypos;
  uint32_t genomepos;
  int32_t queryjump, genomejump;
  uint8_t gapp, knowngapp, comp, pad;
} SiPair;

static List_T si_hook(double *avg_donor_score, double *avg_acceptor_score, int *nbadintrons, List_T path,
                      int cdna_direction, bool watsonp, int chrnum, Genomicpos_T chroffset,
                      Genomicpos_T chrhigh, Genomicpos_T chrpos, char *genomicuc_ptr, int genomiclength,
                      int nullgap, bool use_genomicseg_p) {
  SiCall c;
  List_T p, out;
  memset(&c, 0, sizeof(c));
  c.cdna_direction = cdna_direction;
  c.watsonp = watsonp;
  c.chrnum = chrnum;
  c.genomiclength = genomiclength;
  c.nullgap = nullgap;
  c.use_genomicseg_p = use_genomicseg_p;
  c.chroffset = chroffset;
  c.chrhigh = chrhigh;
  c.chrpos = chrpos;
  c.first_pair = (int32_t)(si_pairs.n / sizeof(SiPair));
  for (p = path; p != NULL; p = p->rest) {
    const struct Pair_T *x = (const struct Pair_T *)p->first;
    SiPair r = {x->querypos, x->genomepos, x->queryjump, x->genomejump, (uint8_t)x->gapp,
                (uint8_t)x->knowngapp, (uint8_t)x->comp, 0};
    put(&si_pairs, &r, sizeof(r));
    c.npairs++;
  }
  patch_off(&si_p);
  out = ((si_fn_t)(void *)si_p.entry)(avg_donor_score, avg_acceptor_score, nbadintrons, path, cdna_direction,
                                    watsonp, chrnum, chroffset, chrhigh, chrpos, genomicuc_ptr, genomiclength,
                                    nullgap, use_genomicseg_p);
  patch_on(&si_p);
  c.avg_donor_score = *avg_donor_score;
  c.avg_acceptor_score = *avg_acceptor_score;
  c.nbadintrons = *nbadintrons;
  put(&si_paths, &c, sizeof(c));
  return out;
}

/* ---- build_pairs_introns (stage3.c:7735-7901), static: patched at start.
 * One record per call: the arguments, the path it was given (pair by pair, in
 * list order), the list it returned (each pair with the index of the input pair
 * it is, or -1 for a pair the call made), the in/out counters, and the wall time
 * of the reference's own call (its DP included). */
typedef List_T (*bpi_fn_t)(bool *, bool *, int *, int *, int *, int *, int *, int *, List_T, int, Genomicpos_T,
                           Genomicpos_T, Genomicpos_T, void *, int, int, char *, char *, char *, char *, bool, int,
                           bool, bool, int, int, int, int, int, double, int, Pairpool_T, Dynprog_T, Dynprog_T,
                           Dynprog_T, bool);
extern void *gmap_trace_build_pairs_introns_fn(void);
extern int gmap_trace_novelsplicingp(void);
extern int gmap_trace_splicingp(void);
static Patch bpi_p;
static Buf bpi_calls, bpi_in, bpi_out, bpi_q, bpi_qu;
static int32_t pc_passes[6]; /* the pass calls of the path_compute call in progress, by GSNAPDP_S3_* */

typedef struct { /* gsnapdp_s3_call (include/gsnapdp.h) */
  int32_t first_pair, npairs, first_out, nout, qpos, querylength;
  uint32_t chroffset, chrhigh, chrpos;
  int32_t chrnum, genomiclength, cdna_direction;
  int32_t watsonp, jump_late_p, finalp, use_genomicseg_p;
  int32_t maxpeelback, nullgap, extramaterial_paired, extraband_single, extraband_paired, close_indels_mode;
  double defect_rate;
  int32_t maxlength1[3], maxlength2[3]; /* dynprogL, dynprogM, dynprogR */
  int32_t in_minor, in_major, in_nintrons, in_nnonintrons, in_intronlen, in_nonintronlen;
  int32_t out_minor, out_major, out_nintrons, out_nnonintrons, out_intronlen, out_nonintronlen;
  int32_t shiftp, incompletep, novelsplicingp, splicingp;
  int32_t status, ub, pass, endalign, extramaterial_end, extraband_end, splicesitesp, invocation;
  double ref_seconds;
} BpiCall;
_Static_assert(sizeof(BpiCall) == sizeof(gsnapdp_s3_call), "BpiCall is gsnapdp_s3_call");
typedef struct { /* gsnapdp_s3_pair */
  int32_t querypos, genomepos, queryjump, genomejump, dynprogindex, src;
  char cdna, comp, genome;
  uint8_t flags; /* 1 gapp, 2 knowngapp, 4 disallowedp, 8 shortexonp, 16 end_intron_p */
} BpiPair;

static BpiPair bpi_pair(const struct Pair_T *x, int src) {
  BpiPair r;
  r.querypos = x->querypos;
  r.genomepos = (int32_t)x->genomepos;
  r.queryjump = x->queryjump;
  r.genomejump = x->genomejump;
  r.dynprogindex = x->dynprogindex;
  r.src = src;
  r.cdna = x->cdna;
  r.comp = x->comp;
  r.genome = x->genome;
  r.flags = (uint8_t)((x->gapp ? 1 : 0) | (x->knowngapp ? 2 : 0) | (x->disallowedp ? 4 : 0) |
                      (x->shortexonp ? 8 : 0) | (x->end_intron_p ? 16 : 0));
  return r;
}
typedef struct {
  const void *p;
  int i;
} PtrIdx;
static int cmp_ptr(const void *a, const void *b) {
  const uintptr_t x = (uintptr_t)((const PtrIdx *)a)->p, y = (uintptr_t)((const PtrIdx *)b)->p;
  return x < y ? -1 : (x > y ? 1 : 0);
}

/* the call's query, its path (pair by pair, list order), the in-counters */
static PtrIdx *bpi_begin(BpiCall *c, List_T path, const char *queryseq_ptr, const char *queryuc_ptr,
                         int querylength, int *n) {
  List_T p;
  PtrIdx *ix;
  int i;
  static const char zero[8] = {0};
  c->first_pair = (int32_t)(bpi_in.n / sizeof(BpiPair));
  c->qpos = (int32_t)bpi_q.n;
  c->querylength = querylength;
  put(&bpi_q, queryseq_ptr, (size_t)querylength);
  put(&bpi_qu, queryuc_ptr, (size_t)querylength);
  put(&bpi_q, zero, 8 - (size_t)(querylength & 3)); /* dword-padded, as the batch buffers */
  put(&bpi_qu, zero, 8 - (size_t)(querylength & 3));
  c->novelsplicingp = gmap_trace_novelsplicingp();
  c->splicingp = gmap_trace_splicingp();
  *n = 0;
  for (p = path; p != NULL; p = p->rest) (*n)++;
  ix = (PtrIdx *)malloc((size_t)(*n > 0 ? *n : 1) * sizeof(PtrIdx));
  for (p = path, i = 0; p != NULL; p = p->rest, i++) {
    BpiPair r = bpi_pair((const struct Pair_T *)p->first, -1);
    put(&bpi_in, &r, sizeof(r));
    ix[i].p = p->first;
    ix[i].i = i;
  }
  c->npairs = *n;
  qsort(ix, (size_t)*n, sizeof(PtrIdx), cmp_ptr);
  return ix;
}
/* the list the call returned (each cell's input index, or -1) and the call */
static void bpi_end(BpiCall *c, List_T out, PtrIdx *ix, int n, const struct timespec *t0) {
  List_T p;
  struct timespec t1;
  clock_gettime(CLOCK_MONOTONIC, &t1);
  c->ref_seconds = (double)(t1.tv_sec - t0->tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0->tv_nsec);
  c->first_out = (int32_t)(bpi_out.n / sizeof(BpiPair));
  for (p = out; p != NULL; p = p->rest) {
    PtrIdx key, *hit;
    BpiPair r;
    key.p = p->first;
    hit = (PtrIdx *)bsearch(&key, ix, (size_t)n, sizeof(PtrIdx), cmp_ptr);
    r = bpi_pair((const struct Pair_T *)p->first, hit ? hit->i : -1);
    put(&bpi_out, &r, sizeof(r));
    c->nout++;
  }
  free(ix);
  put(&bpi_calls, c, sizeof(*c));
  if (c->pass >= 0 && c->pass < 6) pc_passes[c->pass]++;
}
static void bpi_dynprogs(BpiCall *c, Dynprog_T dynprogL, Dynprog_T dynprogM, Dynprog_T dynprogR) {
  c->maxlength1[0] = ((int *)dynprogL)[0];
  c->maxlength2[0] = ((int *)dynprogL)[1];
  c->maxlength1[1] = ((int *)dynprogM)[0];
  c->maxlength2[1] = ((int *)dynprogM)[1];
  c->maxlength1[2] = ((int *)dynprogR)[0];
  c->maxlength2[2] = ((int *)dynprogR)[1];
}

/* path_compute (stage3.c:8586), static: patched so that every pass call below
 * carries the number of the path_compute call it belongs to (`invocation`) */
static int32_t pc_invocation = -1;
static Buf pc_calls, pc_pairs, pc_probs;
typedef struct { /* one path_compute call (gsnapdp/records.py PC_CALL) */
  int32_t invocation, do_final_p, stage3debug, cdna_direction, querylength, genomiclength, watsonp, pad;
  double defect_rate;              /* its output */
  int32_t first_out, nout;         /* the list it returned: pc_pairs.bin (BpiPair, list order, src -1) and
                                    * pc_probs.bin (donor_prob, acceptor_prob per pair) */
  int32_t intronlen, nonintronlen; /* its outputs */
  int32_t maxpeelback, nullgap, extramaterial_end, extraband_end; /* what passes 7-10 read (stage3.c:8885-9212) */
  int32_t maxintronlen_bound, paired_favor_mode, zero_offset, jump_late_p;
  int32_t passes[6];               /* the pass calls it made */
} PcCall;

static List_T bpi_hook(bool *shiftp, bool *incompletep, int *nintrons, int *nnonintrons, int *intronlen,
                       int *nonintronlen, int *dynprogindex_minor, int *dynprogindex_major, List_T path, int chrnum,
                       Genomicpos_T chroffset, Genomicpos_T chrhigh, Genomicpos_T chrpos, void *genome,
                       int querylength, int genomiclength, char *queryseq_ptr, char *queryuc_ptr,
                       char *genomicseg_ptr, char *genomicuc_ptr, bool use_genomicseg_p, int cdna_direction,
                       bool watsonp, bool jump_late_p, int maxpeelback, int nullgap, int extramaterial_paired,
                       int extraband_single, int extraband_paired, double defect_rate, int close_indels_mode,
                       Pairpool_T pairpool, Dynprog_T dynprogL, Dynprog_T dynprogM, Dynprog_T dynprogR,
                       bool finalp) {
  BpiCall c;
  List_T out;
  PtrIdx *ix;
  int n = 0;
  struct timespec t0;
  memset(&c, 0, sizeof(c));
  c.pass = GSNAPDP_S3_INTRONS;
  c.invocation = pc_invocation;
  c.chroffset = chroffset;
  c.chrhigh = chrhigh;
  c.chrpos = chrpos;
  c.chrnum = chrnum;
  c.genomiclength = genomiclength;
  c.cdna_direction = cdna_direction;
  c.watsonp = watsonp;
  c.jump_late_p = jump_late_p;
  c.finalp = finalp;
  c.use_genomicseg_p = use_genomicseg_p;
  c.maxpeelback = maxpeelback;
  c.nullgap = nullgap;
  c.extramaterial_paired = extramaterial_paired;
  c.extraband_single = extraband_single;
  c.extraband_paired = extraband_paired;
  c.close_indels_mode = close_indels_mode;
  c.defect_rate = defect_rate;
  bpi_dynprogs(&c, dynprogL, dynprogM, dynprogR);
  c.in_minor = *dynprogindex_minor;
  c.in_major = *dynprogindex_major;
  c.in_nintrons = *nintrons;
  c.in_nnonintrons = *nnonintrons;
  c.in_intronlen = *intronlen;
  c.in_nonintronlen = *nonintronlen;
  ix = bpi_begin(&c, path, queryseq_ptr, queryuc_ptr, querylength, &n);
  patch_off(&bpi_p);
  clock_gettime(CLOCK_MONOTONIC, &t0);
  out = ((bpi_fn_t)(void *)bpi_p.entry)(shiftp, incompletep, nintrons, nnonintrons, intronlen, nonintronlen,
                                        dynprogindex_minor, dynprogindex_major, path, chrnum, chroffset, chrhigh,
                                        chrpos, genome, querylength, genomiclength, queryseq_ptr, queryuc_ptr,
                                        genomicseg_ptr, genomicuc_ptr, use_genomicseg_p, cdna_direction, watsonp,
                                        jump_late_p, maxpeelback, nullgap, extramaterial_paired, extraband_single,
                                        extraband_paired, defect_rate, close_indels_mode, pairpool, dynprogL,
                                        dynprogM, dynprogR, finalp);
  patch_on(&bpi_p);
  c.out_minor = *dynprogindex_minor;
  c.out_major = *dynprogindex_major;
  c.out_nintrons = *nintrons;
  c.out_nnonintrons = *nnonintrons;
  c.out_intronlen = *intronlen;
  c.out_nonintronlen = *nonintronlen;
  c.shiftp = *shiftp;
  c.incompletep = *incompletep;
  bpi_end(&c, out, ix, n, &t0);
  return out;
}

/* ---- build_pairs_singles (stage3.c:7454-7583), passes 2A / 2C / 7C: the same
 * records, pass GSNAPDP_S3_SINGLES, dynprogindex_minor in in_minor / out_minor */
typedef List_T (*bps_fn_t)(int *, List_T, Genomicpos_T, Genomicpos_T, Genomicpos_T, Genomicpos_T, char *, char *,
                           char *, char *, int, bool, bool, int, int, int, double, int, Pairpool_T, Dynprog_T);
extern void *gmap_trace_build_pairs_singles_fn(void);
static Patch bps_p;
static List_T bps_hook(int *dynprogindex, List_T path, Genomicpos_T chroffset, Genomicpos_T chrhigh,
                       Genomicpos_T chrpos, Genomicpos_T genomiclength, char *queryseq_ptr, char *queryuc_ptr,
                       char *genomicseg_ptr, char *genomicuc_ptr, int cdna_direction, bool watsonp,
                       bool jump_late_p, int maxpeelback, int nullgap, int extraband_single, double defect_rate,
                       int close_indels_mode, Pairpool_T pairpool, Dynprog_T dynprogM) {
  BpiCall c;
  List_T out;
  PtrIdx *ix;
  int n = 0;
  struct timespec t0;
  memset(&c, 0, sizeof(c));
  c.pass = GSNAPDP_S3_SINGLES;
  c.invocation = pc_invocation;
  c.chroffset = chroffset;
  c.chrhigh = chrhigh;
  c.chrpos = chrpos;
  c.genomiclength = (int32_t)genomiclength;
  c.cdna_direction = cdna_direction;
  c.watsonp = watsonp;
  c.jump_late_p = jump_late_p;
  c.maxpeelback = maxpeelback;
  c.nullgap = nullgap;
  c.extraband_single = extraband_single;
  c.close_indels_mode = close_indels_mode;
  c.defect_rate = defect_rate;
  bpi_dynprogs(&c, dynprogM, dynprogM, dynprogM);
  c.in_minor = *dynprogindex;
  /* the query is gmap's whole query (Sequence_fullpointer, NUL-terminated) */
  ix = bpi_begin(&c, path, queryseq_ptr, queryuc_ptr, (int)strlen(queryseq_ptr), &n);
  patch_off(&bps_p);
  clock_gettime(CLOCK_MONOTONIC, &t0);
  out = ((bps_fn_t)(void *)bps_p.entry)(dynprogindex, path, chroffset, chrhigh, chrpos, genomiclength,
                                        queryseq_ptr, queryuc_ptr, genomicseg_ptr, genomicuc_ptr, cdna_direction,
                                        watsonp, jump_late_p, maxpeelback, nullgap, extraband_single, defect_rate,
                                        close_indels_mode, pairpool, dynprogM);
  patch_on(&bps_p);
  c.out_minor = *dynprogindex;
  bpi_end(&c, out, ix, n, &t0);
  return out;
}

/* ---- build_pairs_end5 (stage3.c:7351-7450) and build_path_end3 (:7236-7347),
 * passes 8, 9a / 9b and 10: pass GSNAPDP_S3_END5 / END3, dynprogindex_minor in
 * in_minor / out_minor, the Dynprog_T's limits in all three slots.  Their other
 * outputs are what extend_ending5/3 leave without splice sites (knownsplicep
 * false, ambig_end_length 0, chop_exon_p false): status 1 marks a call where
 * they are not (none is expected). */
typedef List_T (*bpe5_fn_t)(bool *, int *, int *, bool *, int *, List_T, Genomicpos_T, Genomicpos_T, Genomicpos_T,
                            int, Genomicpos_T, Genomicpos_T, char *, char *, char *, char *, int, bool, bool, int,
                            int, int, int, int, double, Pairpool_T, Dynprog_T, bool, int);
typedef List_T (*bpe3_fn_t)(bool *, int *, int *, bool *, int *, List_T, Genomicpos_T, Genomicpos_T, Genomicpos_T,
                            int, int, Genomicpos_T, Genomicpos_T, char *, char *, char *, char *, int, bool, bool,
                            int, int, int, int, int, double, Pairpool_T, Dynprog_T, bool, int);
extern void *gmap_trace_build_pairs_end5_fn(void);
extern void *gmap_trace_build_path_end3_fn(void);
extern int gmap_trace_splicesitesp(void);
static Patch bpe5_p, bpe3_p;
static void bpe_args(BpiCall *c, int pass, Genomicpos_T chroffset, Genomicpos_T chrhigh, Genomicpos_T chrpos,
                     int genomiclength, int cdna_direction, bool watsonp, bool jump_late_p, int maxpeelback,
                     int nullgap, int extramaterial_end, int extraband_end, double defect_rate, Dynprog_T dynprog,
                     int endalign, int minor) {
  memset(c, 0, sizeof(*c));
  c->pass = pass;
  c->invocation = pc_invocation;
  c->chroffset = chroffset;
  c->chrhigh = chrhigh;
  c->chrpos = chrpos;
  c->genomiclength = genomiclength;
  c->cdna_direction = cdna_direction;
  c->watsonp = watsonp;
  c->jump_late_p = jump_late_p;
  c->maxpeelback = maxpeelback;
  c->nullgap = nullgap;
  c->extramaterial_end = extramaterial_end;
  c->extraband_end = extraband_end;
  c->defect_rate = defect_rate;
  c->endalign = endalign;
  c->splicesitesp = gmap_trace_splicesitesp();
  bpi_dynprogs(c, dynprog, dynprog, dynprog);
  c->in_minor = minor;
}
static List_T bpe5_hook(bool *knownsplicep, int *ambig_end_length_5, int *ambig_splicetype_5, bool *chop_exon_p,
                        int *dynprogindex_minor, List_T pairs, Genomicpos_T chroffset, Genomicpos_T chrhigh,
                        Genomicpos_T chrpos, int genomiclength, Genomicpos_T knownsplice_limit_low,
                        Genomicpos_T knownsplice_limit_high, char *queryseq_ptr, char *queryuc_ptr,
                        char *genomicseg_ptr, char *genomicuc_ptr, int cdna_direction, bool watsonp,
                        bool jump_late_p, int maxpeelback, int maxpeelback_distalmedial, int nullgap,
                        int extramaterial_end, int extraband_end, double defect_rate, Pairpool_T pairpool,
                        Dynprog_T dynprogR, bool extendp, int endalign) {
  BpiCall c;
  List_T out;
  PtrIdx *ix;
  int n = 0;
  struct timespec t0;
  bpe_args(&c, GSNAPDP_S3_END5, chroffset, chrhigh, chrpos, genomiclength, cdna_direction, watsonp, jump_late_p,
           maxpeelback, nullgap, extramaterial_end, extraband_end, defect_rate, dynprogR, endalign,
           *dynprogindex_minor);
  ix = bpi_begin(&c, pairs, queryseq_ptr, queryuc_ptr, (int)strlen(queryseq_ptr), &n);
  patch_off(&bpe5_p);
  clock_gettime(CLOCK_MONOTONIC, &t0);
  out = ((bpe5_fn_t)(void *)bpe5_p.entry)(knownsplicep, ambig_end_length_5, ambig_splicetype_5, chop_exon_p,
                                          dynprogindex_minor, pairs, chroffset, chrhigh, chrpos, genomiclength,
                                          knownsplice_limit_low, knownsplice_limit_high, queryseq_ptr, queryuc_ptr,
                                          genomicseg_ptr, genomicuc_ptr, cdna_direction, watsonp, jump_late_p,
                                          maxpeelback, maxpeelback_distalmedial, nullgap, extramaterial_end,
                                          extraband_end, defect_rate, pairpool, dynprogR, extendp, endalign);
  patch_on(&bpe5_p);
  c.out_minor = *dynprogindex_minor;
  c.status = (!extendp || *knownsplicep || *ambig_end_length_5 != 0 || *chop_exon_p) ? 1 : 0;
  bpi_end(&c, out, ix, n, &t0);
  return out;
}
static List_T bpe3_hook(bool *knownsplicep, int *ambig_end_length_3, int *ambig_splicetype_3, bool *chop_exon_p,
                        int *dynprogindex_minor, List_T path, Genomicpos_T chroffset, Genomicpos_T chrhigh,
                        Genomicpos_T chrpos, int querylength, int genomiclength, Genomicpos_T knownsplice_limit_low,
                        Genomicpos_T knownsplice_limit_high, char *queryseq_ptr, char *queryuc_ptr,
                        char *genomicseg_ptr, char *genomicuc_ptr, int cdna_direction, bool watsonp,
                        bool jump_late_p, int maxpeelback, int maxpeelback_distalmedial, int nullgap,
                        int extramaterial_end, int extraband_end, double defect_rate, Pairpool_T pairpool,
                        Dynprog_T dynprogL, bool extendp, int endalign) {
  BpiCall c;
  List_T out;
  PtrIdx *ix;
  int n = 0;
  struct timespec t0;
  bpe_args(&c, GSNAPDP_S3_END3, chroffset, chrhigh, chrpos, genomiclength, cdna_direction, watsonp, jump_late_p,
           maxpeelback, nullgap, extramaterial_end, extraband_end, defect_rate, dynprogL, endalign,
           *dynprogindex_minor);
  ix = bpi_begin(&c, path, queryseq_ptr, queryuc_ptr, querylength, &n);
  patch_off(&bpe3_p);
  clock_gettime(CLOCK_MONOTONIC, &t0);
  out = ((bpe3_fn_t)(void *)bpe3_p.entry)(knownsplicep, ambig_end_length_3, ambig_splicetype_3, chop_exon_p,
                                          dynprogindex_minor, path, chroffset, chrhigh, chrpos, querylength,
                                          genomiclength, knownsplice_limit_low, knownsplice_limit_high, queryseq_ptr,
                                          queryuc_ptr, genomicseg_ptr, genomicuc_ptr, cdna_direction, watsonp,
                                          jump_late_p, maxpeelback, maxpeelback_distalmedial, nullgap,
                                          extramaterial_end, extraband_end, defect_rate, pairpool, dynprogL, extendp,
                                          endalign);
  patch_on(&bpe3_p);
  c.out_minor = *dynprogindex_minor;
  c.status = (!extendp || *knownsplicep || *ambig_end_length_3 != 0 || *chop_exon_p) ? 1 : 0;
  bpi_end(&c, out, ix, n, &t0);
  return out;
}

/* ---- build_pairs_dualintrons (stage3.c:7592-7733), pass 3b: pass
 * GSNAPDP_S3_DUALINTRONS, dynprogindex_major in in_major / out_major */
typedef List_T (*bpd_fn_t)(int *, List_T, Chrnum_T, Genomicpos_T, Genomicpos_T, Genomicpos_T, int, char *, char *,
                           char *, char *, bool, int, bool, bool, int, int, int, int, double, Pairpool_T, Dynprog_T,
                           Dynprog_T);
extern void *gmap_trace_build_pairs_dualintrons_fn(void);
static Patch bpd_p;
static List_T bpd_hook(int *dynprogindex, List_T path, Chrnum_T chrnum, Genomicpos_T chroffset, Genomicpos_T chrhigh,
                       Genomicpos_T chrpos, int genomiclength, char *queryseq_ptr, char *queryuc_ptr,
                       char *genomicseg_ptr, char *genomicuc_ptr, bool use_genomicseg_p, int cdna_direction,
                       bool watsonp, bool jump_late_p, int maxpeelback, int nullgap, int extramaterial_paired,
                       int extraband_paired, double defect_rate, Pairpool_T pairpool, Dynprog_T dynprogL,
                       Dynprog_T dynprogR) {
  BpiCall c;
  List_T out;
  PtrIdx *ix;
  int n = 0;
  struct timespec t0;
  memset(&c, 0, sizeof(c));
  c.pass = GSNAPDP_S3_DUALINTRONS;
  c.invocation = pc_invocation;
  c.chroffset = chroffset;
  c.chrhigh = chrhigh;
  c.chrpos = chrpos;
  c.chrnum = (int32_t)chrnum;
  c.genomiclength = genomiclength;
  c.cdna_direction = cdna_direction;
  c.watsonp = watsonp;
  c.jump_late_p = jump_late_p;
  c.use_genomicseg_p = use_genomicseg_p;
  c.maxpeelback = maxpeelback;
  c.nullgap = nullgap;
  c.extramaterial_paired = extramaterial_paired;
  c.extraband_paired = extraband_paired;
  c.defect_rate = defect_rate;
  bpi_dynprogs(&c, dynprogL, dynprogL, dynprogR);
  c.in_major = *dynprogindex;
  ix = bpi_begin(&c, path, queryseq_ptr, queryuc_ptr, (int)strlen(queryseq_ptr), &n);
  patch_off(&bpd_p);
  clock_gettime(CLOCK_MONOTONIC, &t0);
  out = ((bpd_fn_t)(void *)bpd_p.entry)(dynprogindex, path, chrnum, chroffset, chrhigh, chrpos, genomiclength,
                                        queryseq_ptr, queryuc_ptr, genomicseg_ptr, genomicuc_ptr, use_genomicseg_p,
                                        cdna_direction, watsonp, jump_late_p, maxpeelback, nullgap,
                                        extramaterial_paired, extraband_paired, defect_rate, pairpool, dynprogL,
                                        dynprogR);
  patch_on(&bpd_p);
  c.out_major = *dynprogindex;
  bpi_end(&c, out, ix, n, &t0);
  return out;
}

/* ---- build_dual_breaks (stage3.c:7149-7232), pass 5: pass GSNAPDP_S3_DUALBREAKS,
 * dynprogindex_minor in in_minor / out_minor, *dual_break_p in shiftp */
typedef List_T (*bdb_fn_t)(bool *, int *, List_T, Genomicpos_T, Genomicpos_T, Genomicpos_T, Genomicpos_T, char *,
                           char *, char *, char *, int, bool, int, bool, Pairpool_T, Dynprog_T, int, void *, int,
                           void *, int, int, int, int, double, int);
extern void *gmap_trace_build_dual_breaks_fn(void);
static Patch bdb_p;
static List_T bdb_hook(bool *dual_break_p, int *dynprogindex_minor, List_T path, Genomicpos_T chroffset,
                       Genomicpos_T chrhigh, Genomicpos_T chrpos, Genomicpos_T genomiclength, char *queryseq_ptr,
                       char *queryuc_ptr, char *genomicseg_ptr, char *genomicuc_ptr, int cdna_direction,
                       bool watsonp, int genestrand, bool jump_late_p, Pairpool_T pairpool, Dynprog_T dynprogM,
                       int maxpeelback, void *oligoindices_minor, int noligoindices_minor, void *diagpool,
                       int sufflookback, int nsufflookback, int maxintronlen_bound, int extraband_single,
                       double defect_rate, int close_indels_mode) {
  BpiCall c;
  List_T out;
  PtrIdx *ix;
  int n = 0;
  struct timespec t0;
  memset(&c, 0, sizeof(c));
  c.pass = GSNAPDP_S3_DUALBREAKS;
  c.invocation = pc_invocation;
  c.chroffset = chroffset;
  c.chrhigh = chrhigh;
  c.chrpos = chrpos;
  c.genomiclength = (int32_t)genomiclength;
  c.cdna_direction = cdna_direction;
  c.watsonp = watsonp;
  c.jump_late_p = jump_late_p;
  c.maxpeelback = maxpeelback;
  c.extraband_single = extraband_single;
  c.close_indels_mode = close_indels_mode;
  c.defect_rate = defect_rate;
  bpi_dynprogs(&c, dynprogM, dynprogM, dynprogM);
  c.in_minor = *dynprogindex_minor;
  ix = bpi_begin(&c, path, queryseq_ptr, queryuc_ptr, (int)strlen(queryseq_ptr), &n);
  patch_off(&bdb_p);
  clock_gettime(CLOCK_MONOTONIC, &t0);
  out = ((bdb_fn_t)(void *)bdb_p.entry)(dual_break_p, dynprogindex_minor, path, chroffset, chrhigh, chrpos,
                                        genomiclength, queryseq_ptr, queryuc_ptr, genomicseg_ptr, genomicuc_ptr,
                                        cdna_direction, watsonp, genestrand, jump_late_p, pairpool, dynprogM,
                                        maxpeelback, oligoindices_minor, noligoindices_minor, diagpool, sufflookback,
                                        nsufflookback, maxintronlen_bound, extraband_single, defect_rate,
                                        close_indels_mode);
  patch_on(&bdb_p);
  c.out_minor = *dynprogindex_minor;
  c.shiftp = *dual_break_p;
  bpi_end(&c, out, ix, n, &t0);
  return out;
}

/* Stage2_compute_one (stage2.c:4260), which only traverse_dual_break calls
 * (stage3.c:7104): every call's stretch and the list it returned, so that the
 * pass's stage-2 callback can be served from the recording (stage 2 itself is
 * out of scope).  S2Call per call, its pairs (BpiPair, list order, src -1) in
 * stage2_pairs.bin. */
typedef struct {
  int32_t invocation, query_offset, querylength, genomiclength;
  uint32_t genomicstart, genomicend, mappingstart, mappingend;
  int32_t plusp, first_pair, npairs, pad;
} S2Call;
static Buf s2_calls, s2_pairs;
extern List_T __real_Stage2_compute_one(int *, int *, char *, char *, int, int, char *, char *, Genomicpos_T,
                                        Genomicpos_T, Genomicpos_T, Genomicpos_T, bool, int, int, void *, int, double,
                                        Pairpool_T, void *, int, int, int, bool, bool, bool, bool, bool, bool, void *,
                                        bool);
List_T __wrap_Stage2_compute_one(int *stage2_source, int *stage2_indexsize, char *queryseq_ptr, char *queryuc_ptr,
                                 int querylength, int query_offset, char *genomicseg_ptr, char *genomicuc_ptr,
                                 Genomicpos_T genomicstart, Genomicpos_T genomicend, Genomicpos_T mappingstart,
                                 Genomicpos_T mappingend, bool plusp, int genestrand, int genomiclength,
                                 void *oligoindices, int noligoindices, double proceed_pctcoverage,
                                 Pairpool_T pairpool, void *diagpool, int sufflookback, int nsufflookback,
                                 int maxintronlen, bool localp, bool skip_repetitive_p, bool use_shifted_canonical_p,
                                 bool favor_right_p, bool debug_graphic_p, bool diagnosticp, void *stopwatch,
                                 bool diag_debug) {
  List_T out, p;
  S2Call r;
  out = __real_Stage2_compute_one(stage2_source, stage2_indexsize, queryseq_ptr, queryuc_ptr, querylength,
                                  query_offset, genomicseg_ptr, genomicuc_ptr, genomicstart, genomicend, mappingstart,
                                  mappingend, plusp, genestrand, genomiclength, oligoindices, noligoindices,
                                  proceed_pctcoverage, pairpool, diagpool, sufflookback, nsufflookback, maxintronlen,
                                  localp, skip_repetitive_p, use_shifted_canonical_p, favor_right_p, debug_graphic_p,
                                  diagnosticp, stopwatch, diag_debug);
  memset(&r, 0, sizeof(r));
  r.invocation = pc_invocation;
  r.query_offset = query_offset;
  r.querylength = querylength;
  r.genomiclength = genomiclength;
  r.genomicstart = genomicstart;
  r.genomicend = genomicend;
  r.mappingstart = mappingstart;
  r.mappingend = mappingend;
  r.plusp = plusp;
  r.first_pair = (int32_t)(s2_pairs.n / sizeof(BpiPair));
  for (p = out; p != NULL; p = p->rest) {
    BpiPair x = bpi_pair((const struct Pair_T *)p->first, -1);
    put(&s2_pairs, &x, sizeof(x));
    r.npairs++;
  }
  put(&s2_calls, &r, sizeof(r));
  return out;
}

/* path_compute with the reference's non-GSNAP, non-PMAP prototype */
typedef List_T (*pc_fn_t)(double *, int *, int *, List_T, int, bool, int, bool, int, int, char *, char *, char *,
                          char *, bool, Chrnum_T, Genomicpos_T, Genomicpos_T, Genomicpos_T, Genomicpos_T,
                          Genomicpos_T, void *, int, int, int, int, int, int, int, int, Pairpool_T, Dynprog_T,
                          Dynprog_T, Dynprog_T, int, bool, void *, int, void *, int, int, int, int, int, int);
extern void *gmap_trace_path_compute_fn(void);
static Patch pc_p;
static List_T pc_hook(double *defect_rate, int *intronlen, int *nonintronlen, List_T path, int cdna_direction,
                      bool watsonp, int genestrand, bool jump_late_p, int querylength, int genomiclength,
                      char *queryseq_ptr, char *queryuc_ptr, char *genomicseg_ptr, char *genomicuc_ptr,
                      bool use_genomicseg_p, Chrnum_T chrnum, Genomicpos_T chroffset, Genomicpos_T chrhigh,
                      Genomicpos_T chrpos, Genomicpos_T knownsplice_limit_low, Genomicpos_T knownsplice_limit_high,
                      void *genome, int maxpeelback, int maxpeelback_distalmedial, int nullgap, int extramaterial_end,
                      int extraband_end, int extramaterial_paired, int extraband_single, int extraband_paired,
                      Pairpool_T pairpool, Dynprog_T dynprogL, Dynprog_T dynprogM, Dynprog_T dynprogR,
                      int stage3debug, bool do_final_p, void *oligoindices_minor, int noligoindices_minor,
                      void *diagpool, int sufflookback, int nsufflookback, int maxintronlen_bound,
                      int close_indels_mode, int paired_favor_mode, int zero_offset) {
  PcCall r;
  List_T out, p;
  memset(&r, 0, sizeof(r));
  memset(pc_passes, 0, sizeof(pc_passes));
  r.invocation = ++pc_invocation;
  r.do_final_p = do_final_p;
  r.stage3debug = stage3debug;
  r.cdna_direction = cdna_direction;
  r.querylength = querylength;
  r.genomiclength = genomiclength;
  r.watsonp = watsonp;
  patch_off(&pc_p);
  out = ((pc_fn_t)(void *)pc_p.entry)(defect_rate, intronlen, nonintronlen, path, cdna_direction, watsonp, genestrand,
                                      jump_late_p, querylength, genomiclength, queryseq_ptr, queryuc_ptr,
                                      genomicseg_ptr, genomicuc_ptr, use_genomicseg_p, chrnum, chroffset, chrhigh,
                                      chrpos, knownsplice_limit_low, knownsplice_limit_high, genome, maxpeelback,
                                      maxpeelback_distalmedial, nullgap, extramaterial_end, extraband_end,
                                      extramaterial_paired, extraband_single, extraband_paired, pairpool, dynprogL,
                                      dynprogM, dynprogR, stage3debug, do_final_p, oligoindices_minor,
                                      noligoindices_minor, diagpool, sufflookback, nsufflookback, maxintronlen_bound,
                                      close_indels_mode, paired_favor_mode, zero_offset);
  patch_on(&pc_p);
  r.defect_rate = *defect_rate;
  r.intronlen = *intronlen;
  r.nonintronlen = *nonintronlen;
  r.maxpeelback = maxpeelback;
  r.nullgap = nullgap;
  r.extramaterial_end = extramaterial_end;
  r.extraband_end = extraband_end;
  r.maxintronlen_bound = maxintronlen_bound;
  r.paired_favor_mode = paired_favor_mode;
  r.zero_offset = zero_offset;
  r.jump_late_p = jump_late_p;
  memcpy(r.passes, pc_passes, sizeof(pc_passes));
  r.first_out = (int32_t)(pc_pairs.n / sizeof(BpiPair));
  for (p = out; p != NULL; p = p->rest) {
    const struct Pair_T *x = (const struct Pair_T *)p->first;
    BpiPair b = bpi_pair(x, -1);
    double pr[2];
    pr[0] = x->donor_prob;
    pr[1] = x->acceptor_prob;
    put(&pc_pairs, &b, sizeof(b));
    put(&pc_probs, pr, sizeof(pr));
    r.nout++;
  }
  put(&pc_calls, &r, sizeof(r));
  return out;
}

__attribute__((constructor)) static void install_hooks(void) {
  patch_install(&si_p, gmap_trace_score_introns_fn(), (void *)&si_hook);
  patch_install(&bpi_p, gmap_trace_build_pairs_introns_fn(), (void *)&bpi_hook);
  patch_install(&bps_p, gmap_trace_build_pairs_singles_fn(), (void *)&bps_hook);
  patch_install(&bpe5_p, gmap_trace_build_pairs_end5_fn(), (void *)&bpe5_hook);
  patch_install(&bpe3_p, gmap_trace_build_path_end3_fn(), (void *)&bpe3_hook);
  patch_install(&bpd_p, gmap_trace_build_pairs_dualintrons_fn(), (void *)&bpd_hook);
  patch_install(&bdb_p, gmap_trace_build_dual_breaks_fn(), (void *)&bdb_hook);
  patch_install(&pc_p, gmap_trace_path_compute_fn(), (void *)&pc_hook);
}

extern unsigned int *__real_Genome_create_blocks(char *genomicseg, unsigned int genomelength);
unsigned int *__wrap_Genome_create_blocks(char *genomicseg, unsigned int genomelength) {
  unsigned int *b = __real_Genome_create_blocks(genomicseg, genomelength);
  /* a copy: gmap frees its blocks before exit (gmap.c:4013) */
  genome_nwords = (size_t)((genomelength + 31) / 32U) * 3 + 4; /* genome-write.c:809-810 */
  genome_blocks = (unsigned int *)malloc(genome_nwords * sizeof(unsigned int));
  memcpy((void *)genome_blocks, b, genome_nwords * sizeof(unsigned int));
  return b;
}

extern List_T __real_Dynprog_single_gap(int *, int *, int *, int *, int *, int *, Dynprog_T, char *, char *,
                                        char *, char *, int, int, int, int, Genomicpos_T, Genomicpos_T,
                                        Genomicpos_T, Genomicpos_T, int, bool, bool, Pairpool_T, int, double,
                                        int, bool);
List_T __wrap_Dynprog_single_gap(int *dynprogindex, int *finalscore, int *nmatches, int *nmismatches,
                                 int *nopens, int *nindels, Dynprog_T dynprog, char *sequence1,
                                 char *sequenceuc1, char *sequence2, char *sequenceuc2, int length1,
                                 int length2, int offset1, int offset2, Genomicpos_T chroffset,
                                 Genomicpos_T chrhigh, Genomicpos_T chrpos, Genomicpos_T genomiclength,
                                 int cdna_direction, bool watsonp, bool jump_late_p, Pairpool_T pairpool,
                                 int extraband_single, double defect_rate, int close_indels_mode,
                                 bool widebandp) {
  gsnapdp_window w;
  List_T pairs;
  base_window(&w, GSNAPDP_SINGLE_GAP, dynprog, *dynprogindex, length1, length2, offset1, offset2, chroffset,
              chrhigh, chrpos, genomiclength, cdna_direction, watsonp, jump_late_p, extraband_single,
              defect_rate);
  w.widebandp = widebandp ? 1 : 0;
  w.qpos = put_query(&dp, sequence1, sequenceuc1, length1, 0);
  put(&dp.win, &w, sizeof(w));
  pairs = __real_Dynprog_single_gap(dynprogindex, finalscore, nmatches, nmismatches, nopens, nindels, dynprog,
                                    sequence1, sequenceuc1, sequence2, sequenceuc2, length1, length2, offset1,
                                    offset2, chroffset, chrhigh, chrpos, genomiclength, cdna_direction,
                                    watsonp, jump_late_p, pairpool, extraband_single, defect_rate,
                                    close_indels_mode, widebandp);
  record_result(&dp, *dynprogindex, *finalscore, *nmatches, *nmismatches, *nopens, *nindels, pairs);
  return pairs;
}

#define END_ARGS                                                                                          \
  int *dynprogindex, int *finalscore, int *nmatches, int *nmismatches, int *nopens, int *nindels,         \
      Dynprog_T dynprog, char *sequence1, char *sequenceuc1, char *sequence2, char *sequenceuc2,          \
      int length1, int length2, int offset1, int offset2, Genomicpos_T chroffset, Genomicpos_T chrhigh,   \
      Genomicpos_T chrpos, Genomicpos_T genomiclength, int cdna_direction, bool watsonp,                  \
      bool jump_late_p, Pairpool_T pairpool, int extraband_end, double defect_rate, Endalign_T endalign, \
      bool use_genomicseg_p
#define END_CALL                                                                                         \
  dynprogindex, finalscore, nmatches, nmismatches, nopens, nindels, dynprog, sequence1, sequenceuc1,     \
      sequence2, sequenceuc2, length1, length2, offset1, offset2, chroffset, chrhigh, chrpos,            \
      genomiclength, cdna_direction, watsonp, jump_late_p, pairpool, extraband_end, defect_rate, endalign, \
      use_genomicseg_p

static List_T end_gap(int kind, List_T (*real)(END_ARGS), END_ARGS) {
  gsnapdp_window w;
  List_T pairs;
  if (use_genomicseg_p) {
    fprintf(stderr, "gmap_trace: use_genomicseg_p end gap (never issued by stage 3, stage3.c:9865)\n");
    abort();
  }
  base_window(&w, kind, dynprog, *dynprogindex, length1, length2, offset1, offset2, chroffset, chrhigh, chrpos,
              genomiclength, cdna_direction, watsonp, jump_late_p, extraband_end, defect_rate);
  w.endalign = (uint8_t)endalign;
  w.qpos = put_query(&dp, sequence1, sequenceuc1, length1, kind == GSNAPDP_END5_GAP);
  put(&dp.win, &w, sizeof(w));
  pairs = real(END_CALL);
  record_result(&dp, *dynprogindex, *finalscore, *nmatches, *nmismatches, *nopens, *nindels, pairs);
  return pairs;
}

extern List_T __real_Dynprog_end5_gap(END_ARGS);
extern List_T __real_Dynprog_end3_gap(END_ARGS);
List_T __wrap_Dynprog_end5_gap(END_ARGS) { return end_gap(GSNAPDP_END5_GAP, __real_Dynprog_end5_gap, END_CALL); }
List_T __wrap_Dynprog_end3_gap(END_ARGS) { return end_gap(GSNAPDP_END3_GAP, __real_Dynprog_end3_gap, END_CALL); }

extern List_T __real_Dynprog_genome_gap(int *, int *, int *, int *, double *, double *, int *, int *, int *, int *,
                                        int *, int *, Dynprog_T, Dynprog_T, char *, char *, char *, char *, char *,
                                        char *, int, int, int, int, int, int, Chrnum_T, Genomicpos_T,
                                        Genomicpos_T, Genomicpos_T, Genomicpos_T, char *, bool, int, bool, bool,
                                        Pairpool_T, int, double, int, bool, bool, bool, int, bool);
List_T __wrap_Dynprog_genome_gap(int *dynprogindex, int *finalscore, int *new_leftgenomepos,
                                 int *new_rightgenomepos, double *left_prob, double *right_prob, int *nmatches,
                                 int *nmismatches, int *nopens, int *nindels, int *exonhead, int *introntype,
                                 Dynprog_T dynprogL, Dynprog_T dynprogR, char *sequence1, char *sequenceuc1,
                                 char *sequence2L, char *sequenceuc2L, char *revsequence2R,
                                 char *revsequenceuc2R, int length1, int length2L, int length2R, int offset1,
                                 int offset2L, int revoffset2R, Chrnum_T chrnum, Genomicpos_T chroffset,
                                 Genomicpos_T chrhigh, Genomicpos_T chrpos, Genomicpos_T genomiclength,
                                 char *genomicuc_ptr, bool use_genomicseg_p, int cdna_direction, bool watsonp,
                                 bool jump_late_p, Pairpool_T pairpool, int extraband_paired,
                                 double defect_rate, int maxpeelback, bool halfp, bool finalp,
                                 bool use_probabilities_p, int score_threshold, bool splicingp) {
  gsnapdp_ggap_window w;
  gsnapdp_ggap_result r;
  List_T pairs;
  if (use_genomicseg_p) {
    fprintf(stderr, "gmap_trace: use_genomicseg_p genome gap (never issued by stage 3, stage3.c:9865)\n");
    abort();
  }
  memset(&w, 0, sizeof(w));
  w.length1 = length1;
  w.length2L = length2L;
  w.length2R = length2R;
  w.offset1 = offset1;
  w.offset2L = offset2L;
  w.revoffset2R = revoffset2R;
  w.chroffset = chroffset;
  w.chrhigh = chrhigh;
  w.chrpos = chrpos;
  w.genomiclength = genomiclength;
  w.cdna_direction = cdna_direction;
  w.extraband_paired = extraband_paired;
  w.maxpeelback = maxpeelback;
  w.score_threshold = score_threshold;
  w.dynprogindex = *dynprogindex;
  w.maxlength1 = ((int *)dynprogL)[0];
  w.maxlength2 = ((int *)dynprogL)[1];
  w.defect_rate = bin(defect_rate);
  w.watsonp = watsonp ? 1 : 0;
  w.jump_late_p = jump_late_p ? 1 : 0;
  w.halfp = halfp ? 1 : 0;
  w.finalp = finalp ? 1 : 0;
  w.use_probabilities_p = use_probabilities_p ? 1 : 0;
  w.splicingp = splicingp ? 1 : 0;
  w.qpos = put_query(&gg, sequence1, sequenceuc1, length1, 0);
  put(&gg.win, &w, sizeof(w));
  pairs = __real_Dynprog_genome_gap(dynprogindex, finalscore, new_leftgenomepos, new_rightgenomepos, left_prob,
                                    right_prob, nmatches, nmismatches, nopens, nindels, exonhead, introntype,
                                    dynprogL, dynprogR, sequence1, sequenceuc1, sequence2L, sequenceuc2L,
                                    revsequence2R, revsequenceuc2R, length1, length2L, length2R, offset1,
                                    offset2L, revoffset2R, chrnum, chroffset, chrhigh, chrpos, genomiclength,
                                    genomicuc_ptr, use_genomicseg_p, cdna_direction, watsonp, jump_late_p,
                                    pairpool, extraband_paired, defect_rate, maxpeelback, halfp, finalp,
                                    use_probabilities_p, score_threshold, splicingp);
  memset(&r, 0, sizeof(r));
  r.finalscore = *finalscore;
  r.new_leftgenomepos = *new_leftgenomepos;
  r.new_rightgenomepos = *new_rightgenomepos;
  r.nmatches = *nmatches;
  r.nmismatches = *nmismatches;
  r.nopens = *nopens;
  r.nindels = *nindels;
  r.exonhead = *exonhead;
  r.introntype = *introntype;
  r.dynprogindex = *dynprogindex;
  r.returned_null = pairs == NULL;
  r.bridge_ok = 1;
  r.left_prob = *left_prob;
  r.right_prob = *right_prob;
  put(&gg.res, &r, sizeof(r));
  return pairs;
}

static void spit(const char *dir, const char *name, const void *p, size_t n) {
  char path[4096];
  FILE *f;
  snprintf(path, sizeof(path), "%s/%s", dir, name);
  if (!(f = fopen(path, "wb"))) {
    perror(path);
    exit(3);
  }
  if (n) fwrite(p, 1, n, f);
  fclose(f);
}

static void dump(const char *root, const char *sub, const char *winname, Trace *t) {
  char dir[4096];
  snprintf(dir, sizeof(dir), "%s/%s", root, sub);
  mkdir(dir, 0755);
  spit(dir, winname, t->win.p, t->win.n);
  spit(dir, "query.bin", t->q.p, t->q.n);
  spit(dir, "query_uc.bin", t->qu.p, t->qu.n);
  spit(dir, "gmap_results.bin", t->res.p, t->res.n);
  spit(dir, "genome.u32", genome_blocks, genome_nwords * sizeof(unsigned int));
}

__attribute__((destructor)) static void write_trace(void) {
  const char *root = getenv("GMAP_TRACE_DIR");
  if (!root || !genome_blocks) return;
  mkdir(root, 0755);
  dump(root, "dp", "windows.bin", &dp);
  dump(root, "ggap", "ggap_windows.bin", &gg);
  {
    char dir[4096];
    snprintf(dir, sizeof(dir), "%s/si", root);
    mkdir(dir, 0755);
    spit(dir, "paths.bin", si_paths.p, si_paths.n);
    spit(dir, "pairs.bin", si_pairs.p, si_pairs.n);
    spit(dir, "genome.u32", genome_blocks, genome_nwords * sizeof(unsigned int));
    snprintf(dir, sizeof(dir), "%s/bpi", root);
    mkdir(dir, 0755);
    spit(dir, "calls.bin", bpi_calls.p, bpi_calls.n);
    spit(dir, "pairs_in.bin", bpi_in.p, bpi_in.n);
    spit(dir, "pairs_out.bin", bpi_out.p, bpi_out.n);
    spit(dir, "query.bin", bpi_q.p, bpi_q.n);
    spit(dir, "query_uc.bin", bpi_qu.p, bpi_qu.n);
    spit(dir, "path_compute.bin", pc_calls.p, pc_calls.n);
    spit(dir, "pc_pairs.bin", pc_pairs.p, pc_pairs.n);
    spit(dir, "pc_probs.bin", pc_probs.p, pc_probs.n);
    spit(dir, "stage2_calls.bin", s2_calls.p, s2_calls.n);
    spit(dir, "stage2_pairs.bin", s2_pairs.p, s2_pairs.n);
  }
}
