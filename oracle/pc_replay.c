/*
 * pc_replay.c -- TEST INFRASTRUCTURE ONLY (oracle/_ref/pc_replay_gmap and
 * oracle/_ref/pc_replay_gsnap; dev container only, never shipped, never sent to
 * the GPU box).
 *
 * Runs the reference's own path_compute (stage3.c:8586-9222) over the
 * path_compute invocations a gmap run recorded (gmap_trace: tests/golden
 * gmap_*_stage3 pc_calls, with each invocation's pass-2A call), in two builds
 * of the same stage3.c compiled where it lies (stage3_si.c):
 *   * pc_replay_gmap  -- gmap's objects, as gmap_trace links them.  It must
 *     reproduce every recorded path_compute return value bit for bit: that
 *     validates this harness;
 *   * pc_replay_gsnap -- the objects of the reference's gsnap program
 *     (-DGSNAP=1 -DMAX_READLENGTH=250, oracle/_ref/gsnap): path_compute as GSNAP
 *     builds it (SCORE_SIGDIFF, smooth.c's SHORTEXONPROB_END, passes 9a / 9b
 *     with QUERYEND_NOGAPS, the end-exon trims that always keep a supported
 *     exon).  Its outputs are the golden vectors of the product's gsnap = 1
 *     flavour (gsnapdp_s3_path_opts.gsnap, tests gmap_*_stage3_gsnap).
 *
 * The product's driver starts at pass 2A (gsnapdp_stage3_path_compute), so the
 * replay does too: path_compute is entered normally, and the first
 * build_pairs_singles call of the invocation (pass 2A, stage3.c:8671) is handed
 * the recorded pass-2A path in place of the one passes 0-1 made.  Passes 0-1
 * (insert_gapholders, Smooth_pairs_by_netgap) have no GSNAP-dependent code, so
 * that path is what GSNAP's passes 0-1 make too; everything from pass 2A on
 * (later iterations of the cycle loop included) is the reference's own code.
 * The pass functions are static: their entries are patched (x86-64 movabs/jmp,
 * as gmap_trace.c does) to count each invocation's pass calls.
 * Stage2_compute_one (traverse_dual_break, stage3.c:7104) is served from the
 * recording (-Wl,--wrap); an invocation whose stage-2 request the recording
 * does not hold is flagged (PcCall.pad = number of misses) and left out of the
 * golden set by gen_golden.py.
 *
 * Usage: pc_replay_{gmap,gsnap} <dir>
 *   in:  <dir>/{genome.u32,calls.bin,pc.bin,pairs_in.bin,query.bin,query_uc.bin,
 *               stage2_calls.bin,stage2_pairs.bin}
 *        calls.bin: one gsnapdp_s3_call per invocation (its pass-2A path in
 *        pairs_in.bin, its arguments; workload.stage3_path_pipeline), pc.bin the
 *        recorded PcCall of the same invocation
 *   out: <dir>/{out_pc.bin,out_pairs.bin,out_probs.bin}
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <unistd.h>

#include "bool.h"
#include "chrnum.h"
#include "dynprog.h"
#include "genome.h"
#include "list.h"
#include "listdef.h"
#include "maxent_hr.h"
#include "pairdef.h"
#include "pairpool.h"
#include "stage3.h"

typedef struct { /* gsnapdp_s3_call (include/gsnapdp.h) */
  int32_t first_pair, npairs, first_out, nout, qpos, querylength;
  uint32_t chroffset, chrhigh, chrpos;
  int32_t chrnum, genomiclength, cdna_direction;
  int32_t watsonp, jump_late_p, finalp, use_genomicseg_p;
  int32_t maxpeelback, nullgap, extramaterial_paired, extraband_single, extraband_paired, close_indels_mode;
  double defect_rate;
  int32_t maxlength1[3], maxlength2[3];
  int32_t in_minor, in_major, in_nintrons, in_nnonintrons, in_intronlen, in_nonintronlen;
  int32_t out_minor, out_major, out_nintrons, out_nnonintrons, out_intronlen, out_nonintronlen;
  int32_t shiftp, incompletep, novelsplicingp, splicingp;
  int32_t status, ub, pass, endalign, extramaterial_end, extraband_end, splicesitesp, invocation;
  double ref_seconds;
} S3Call;
typedef struct { /* gsnapdp_s3_pair */
  int32_t querypos, genomepos, queryjump, genomejump, dynprogindex, src;
  char cdna, comp, genome;
  uint8_t flags; /* 1 gapp, 2 knowngapp, 4 disallowedp, 8 shortexonp, 16 end_intron_p */
} S3Pair;
typedef struct { /* gmap_trace.c PcCall (gsnapdp/records.py PC_CALL) */
  int32_t invocation, do_final_p, stage3debug, cdna_direction, querylength, genomiclength, watsonp, pad;
  double defect_rate;
  int32_t first_out, nout;
  int32_t intronlen, nonintronlen;
  int32_t maxpeelback, nullgap, extramaterial_end, extraband_end;
  int32_t maxintronlen_bound, paired_favor_mode, zero_offset, jump_late_p;
  int32_t passes[6];
} PcCall;
typedef struct { /* gmap_trace.c S2Call (records.S2_CALL) */
  int32_t invocation, query_offset, querylength, genomiclength;
  uint32_t genomicstart, genomicend, mappingstart, mappingend;
  int32_t plusp, first_pair, npairs, pad;
} S2Call;

enum { P_INTRONS = 0, P_SINGLES = 1, P_END5 = 2, P_END3 = 3, P_DUALINTRONS = 4, P_DUALBREAKS = 5 };

static void *slurp(const char *dir, const char *name, size_t *n) {
  char path[4096];
  FILE *f;
  void *buf;
  long sz;
  snprintf(path, sizeof(path), "%s/%s", dir, name);
  if (!(f = fopen(path, "rb"))) {
    fprintf(stderr, "pc_replay: cannot open %s\n", path);
    exit(2);
  }
  fseek(f, 0, SEEK_END);
  sz = ftell(f);
  fseek(f, 0, SEEK_SET);
  buf = calloc(1, (size_t)sz + 64);
  if (sz > 0 && fread(buf, 1, (size_t)sz, f) != (size_t)sz) exit(3);
  fclose(f);
  *n = (size_t)sz;
  return buf;
}
static void spit(const char *dir, const char *name, const void *p, size_t n) {
  char path[4096];
  FILE *f;
  snprintf(path, sizeof(path), "%s/%s", dir, name);
  if (!(f = fopen(path, "wb"))) {
    perror(path);
    exit(4);
  }
  if (n) fwrite(p, 1, n, f);
  fclose(f);
}

/* ---- entry patches of the static pass functions (movabs rax, hook; jmp rax) */
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
  p->patch[0] = 0x48;
  p->patch[1] = 0xB8;
  memcpy(p->patch + 2, &target, 8);
  p->patch[10] = 0xFF;
  p->patch[11] = 0xE0;
  memcpy(p->entry, p->patch, sizeof(p->patch));
}
static void patch_off(Patch *p) { memcpy(p->entry, p->saved, sizeof(p->saved)); }
static void patch_on(Patch *p) { memcpy(p->entry, p->patch, sizeof(p->patch)); }

/* the invocation in progress */
static int32_t cur_passes[6];
static int cur_invocation = -1, cur_s2_missed = 0;
static List_T cur_2a_path = NULL; /* handed to the first build_pairs_singles call, then NULL */
static const S2Call *s2c;
static const S3Pair *s2p;
static size_t ns2c;

/* the pass functions as stage3.c defines them (no PMAP; GSNAP's prototypes are
 * the same without END_KNOWNSPLICING_SHORTCUT, which the reference never defines) */
typedef List_T (*bps_fn_t)(int *, List_T, Genomicpos_T, Genomicpos_T, Genomicpos_T, Genomicpos_T, char *, char *,
                           char *, char *, int, bool, bool, int, int, int, double, int, Pairpool_T, Dynprog_T);
typedef List_T (*bpi_fn_t)(bool *, bool *, int *, int *, int *, int *, int *, int *, List_T, int, Genomicpos_T,
                           Genomicpos_T, Genomicpos_T, void *, int, int, char *, char *, char *, char *, bool, int,
                           bool, bool, int, int, int, int, int, double, int, Pairpool_T, Dynprog_T, Dynprog_T,
                           Dynprog_T, bool);
typedef List_T (*bpe5_fn_t)(bool *, int *, int *, bool *, int *, List_T, Genomicpos_T, Genomicpos_T, Genomicpos_T,
                            int, Genomicpos_T, Genomicpos_T, char *, char *, char *, char *, int, bool, bool, int,
                            int, int, int, int, double, Pairpool_T, Dynprog_T, bool, int);
typedef List_T (*bpe3_fn_t)(bool *, int *, int *, bool *, int *, List_T, Genomicpos_T, Genomicpos_T, Genomicpos_T,
                            int, int, Genomicpos_T, Genomicpos_T, char *, char *, char *, char *, int, bool, bool,
                            int, int, int, int, int, double, Pairpool_T, Dynprog_T, bool, int);
typedef List_T (*bpd_fn_t)(int *, List_T, Chrnum_T, Genomicpos_T, Genomicpos_T, Genomicpos_T, int, char *, char *,
                           char *, char *, bool, int, bool, bool, int, int, int, int, double, Pairpool_T, Dynprog_T,
                           Dynprog_T);
typedef List_T (*bdb_fn_t)(bool *, int *, List_T, Genomicpos_T, Genomicpos_T, Genomicpos_T, Genomicpos_T, char *,
                           char *, char *, char *, int, bool, int, bool, Pairpool_T, Dynprog_T, int, void *, int,
                           void *, int, int, int, int, double, int);
typedef List_T (*pc_fn_t)(double *, int *, int *, List_T, int, bool, int, bool, int, int, char *, char *, char *,
                          char *, bool, Chrnum_T, Genomicpos_T, Genomicpos_T, Genomicpos_T, Genomicpos_T,
                          Genomicpos_T, void *, int, int, int, int, int, int, int, int, Pairpool_T, Dynprog_T,
                          Dynprog_T, Dynprog_T, int, bool, void *, int, void *, int, int, int, int, int, int);
extern void *gmap_trace_build_pairs_singles_fn(void);
extern void *gmap_trace_build_pairs_introns_fn(void);
extern void *gmap_trace_build_pairs_end5_fn(void);
extern void *gmap_trace_build_path_end3_fn(void);
extern void *gmap_trace_build_pairs_dualintrons_fn(void);
extern void *gmap_trace_build_dual_breaks_fn(void);
extern void *gmap_trace_path_compute_fn(void);

static Patch bps_p, bpi_p, bpe5_p, bpe3_p, bpd_p, bdb_p;

static List_T bps_hook(int *dpi, List_T path, Genomicpos_T a1, Genomicpos_T a2, Genomicpos_T a3, Genomicpos_T a4,
                       char *s1, char *s2, char *s3, char *s4, int i1, bool b1, bool b2, int i2, int i3, int i4,
                       double d, int i5, Pairpool_T pool, Dynprog_T dm) {
  List_T out;
  if (cur_2a_path != NULL) { /* pass 2A: the recorded path in place of passes 0-1's */
    path = cur_2a_path;
    cur_2a_path = NULL;
  }
  cur_passes[P_SINGLES]++;
  patch_off(&bps_p);
  out = ((bps_fn_t)(void *)bps_p.entry)(dpi, path, a1, a2, a3, a4, s1, s2, s3, s4, i1, b1, b2, i2, i3, i4, d, i5,
                                        pool, dm);
  patch_on(&bps_p);
  return out;
}
static List_T bpi_hook(bool *x1, bool *x2, int *x3, int *x4, int *x5, int *x6, int *x7, int *x8, List_T path, int i1,
                       Genomicpos_T a1, Genomicpos_T a2, Genomicpos_T a3, void *g, int i2, int i3, char *s1, char *s2,
                       char *s3, char *s4, bool b1, int i4, bool b2, bool b3, int i5, int i6, int i7, int i8, int i9,
                       double d, int i10, Pairpool_T pool, Dynprog_T dl, Dynprog_T dm, Dynprog_T dr, bool fin) {
  List_T out;
  cur_passes[P_INTRONS]++;
  patch_off(&bpi_p);
  out = ((bpi_fn_t)(void *)bpi_p.entry)(x1, x2, x3, x4, x5, x6, x7, x8, path, i1, a1, a2, a3, g, i2, i3, s1, s2, s3,
                                        s4, b1, i4, b2, b3, i5, i6, i7, i8, i9, d, i10, pool, dl, dm, dr, fin);
  patch_on(&bpi_p);
  return out;
}
static List_T bpe5_hook(bool *x1, int *x2, int *x3, bool *x4, int *x5, List_T path, Genomicpos_T a1, Genomicpos_T a2,
                        Genomicpos_T a3, int i1, Genomicpos_T a4, Genomicpos_T a5, char *s1, char *s2, char *s3,
                        char *s4, int i2, bool b1, bool b2, int i3, int i4, int i5, int i6, int i7, double d,
                        Pairpool_T pool, Dynprog_T dyn, bool ext, int ea) {
  List_T out;
  cur_passes[P_END5]++;
  patch_off(&bpe5_p);
  out = ((bpe5_fn_t)(void *)bpe5_p.entry)(x1, x2, x3, x4, x5, path, a1, a2, a3, i1, a4, a5, s1, s2, s3, s4, i2, b1,
                                          b2, i3, i4, i5, i6, i7, d, pool, dyn, ext, ea);
  patch_on(&bpe5_p);
  return out;
}
static List_T bpe3_hook(bool *x1, int *x2, int *x3, bool *x4, int *x5, List_T path, Genomicpos_T a1, Genomicpos_T a2,
                        Genomicpos_T a3, int i1, int i2, Genomicpos_T a4, Genomicpos_T a5, char *s1, char *s2,
                        char *s3, char *s4, int i3, bool b1, bool b2, int i4, int i5, int i6, int i7, int i8, double d,
                        Pairpool_T pool, Dynprog_T dyn, bool ext, int ea) {
  List_T out;
  cur_passes[P_END3]++;
  patch_off(&bpe3_p);
  out = ((bpe3_fn_t)(void *)bpe3_p.entry)(x1, x2, x3, x4, x5, path, a1, a2, a3, i1, i2, a4, a5, s1, s2, s3, s4, i3,
                                          b1, b2, i4, i5, i6, i7, i8, d, pool, dyn, ext, ea);
  patch_on(&bpe3_p);
  return out;
}
static List_T bpd_hook(int *x1, List_T path, Chrnum_T cn, Genomicpos_T a1, Genomicpos_T a2, Genomicpos_T a3, int i1,
                       char *s1, char *s2, char *s3, char *s4, bool b1, int i2, bool b2, bool b3, int i3, int i4,
                       int i5, int i6, double d, Pairpool_T pool, Dynprog_T dl, Dynprog_T dr) {
  List_T out;
  cur_passes[P_DUALINTRONS]++;
  patch_off(&bpd_p);
  out = ((bpd_fn_t)(void *)bpd_p.entry)(x1, path, cn, a1, a2, a3, i1, s1, s2, s3, s4, b1, i2, b2, b3, i3, i4, i5, i6,
                                        d, pool, dl, dr);
  patch_on(&bpd_p);
  return out;
}
static List_T bdb_hook(bool *x1, int *x2, List_T path, Genomicpos_T a1, Genomicpos_T a2, Genomicpos_T a3,
                       Genomicpos_T a4, char *s1, char *s2, char *s3, char *s4, int i1, bool b1, int i2, bool b2,
                       Pairpool_T pool, Dynprog_T dm, int i3, void *oi, int i4, void *dp, int i5, int i6, int i7,
                       int i8, double d, int i9) {
  List_T out;
  cur_passes[P_DUALBREAKS]++;
  patch_off(&bdb_p);
  out = ((bdb_fn_t)(void *)bdb_p.entry)(x1, x2, path, a1, a2, a3, a4, s1, s2, s3, s4, i1, b1, i2, b2, pool, dm, i3,
                                        oi, i4, dp, i5, i6, i7, i8, d, i9);
  patch_on(&bdb_p);
  return out;
}

/* the recorded pairs of one list, pushed so that list order is record order */
static List_T build_list(Pairpool_T pool, const S3Pair *x, int n) {
  List_T path = NULL;
  int j;
  for (j = n - 1; j >= 0; j--) {
    struct Pair_T *y;
    path = Pairpool_push(path, pool, x[j].querypos, x[j].genomepos, x[j].cdna, x[j].comp, x[j].genome,
                         x[j].dynprogindex);
    y = (struct Pair_T *)path->first;
    y->queryjump = x[j].queryjump;
    y->genomejump = x[j].genomejump;
    y->gapp = (x[j].flags & 1) ? true : false;
    y->knowngapp = (x[j].flags & 2) ? true : false;
    y->disallowedp = (x[j].flags & 4) ? true : false;
    y->shortexonp = (x[j].flags & 8) ? true : false;
    y->end_intron_p = (x[j].flags & 16) ? true : false;
  }
  return path;
}

/* Stage2_compute_one (stage2.c:4260), called only by traverse_dual_break: the
 * recorded list of the same invocation and stretch, or a miss */
List_T __wrap_Stage2_compute_one(int *stage2_source, int *stage2_indexsize, char *queryseq_ptr, char *queryuc_ptr,
                                 int querylength, int query_offset, char *genomicseg_ptr, char *genomicuc_ptr,
                                 Genomicpos_T genomicstart, Genomicpos_T genomicend, Genomicpos_T mappingstart,
                                 Genomicpos_T mappingend, bool plusp, int genestrand, int genomiclength,
                                 void *oligoindices, int noligoindices, double proceed_pctcoverage,
                                 Pairpool_T pairpool, void *diagpool, int sufflookback, int nsufflookback,
                                 int maxintronlen, bool localp, bool skip_repetitive_p, bool use_shifted_canonical_p,
                                 bool favor_right_p, bool debug_graphic_p, bool diagnosticp, void *stopwatch,
                                 bool diag_debug) {
  size_t i;
  *stage2_source = 0;
  *stage2_indexsize = 0;
  for (i = 0; i < ns2c; i++) {
    const S2Call *r = &s2c[i];
    if (r->invocation == cur_invocation && r->query_offset == query_offset && r->querylength == querylength &&
        r->mappingstart == mappingstart && r->mappingend == mappingend)
      return build_list(pairpool, s2p + r->first_pair, r->npairs);
  }
  cur_s2_missed++;
  return NULL;
}

int main(int argc, char **argv) {
  const char *dir;
  size_t ng, nc, npc, np, nq, nqu, ns2p, i;
  unsigned int *g;
  S3Call *calls;
  PcCall *pc;
  S3Pair *pin;
  char *q, *qu;
  Pairpool_T pool;
  Dynprog_T dynprogL, dynprogM, dynprogR;
  S3Pair *pout;
  double *probs;
  size_t nout = 0, capout;
  pc_fn_t path_compute = (pc_fn_t)gmap_trace_path_compute_fn();

  if (argc < 2) {
    fprintf(stderr, "usage: pc_replay <dir>\n");
    return 1;
  }
  dir = argv[1];
  g = (unsigned int *)slurp(dir, "genome.u32", &ng);
  calls = (S3Call *)slurp(dir, "calls.bin", &nc);
  pc = (PcCall *)slurp(dir, "pc.bin", &npc);
  pin = (S3Pair *)slurp(dir, "pairs_in.bin", &np);
  q = (char *)slurp(dir, "query.bin", &nq);
  qu = (char *)slurp(dir, "query_uc.bin", &nqu);
  s2c = (const S2Call *)slurp(dir, "stage2_calls.bin", &ns2c);
  s2p = (const S3Pair *)slurp(dir, "stage2_pairs.bin", &ns2p);
  nc /= sizeof(S3Call);
  npc /= sizeof(PcCall);
  np /= sizeof(S3Pair);
  ns2c /= sizeof(S2Call);
  if (nc != npc) {
    fprintf(stderr, "pc_replay: %zu calls but %zu path_compute records\n", nc, npc);
    return 5;
  }
  patch_install(&bps_p, gmap_trace_build_pairs_singles_fn(), (void *)&bps_hook);
  patch_install(&bpi_p, gmap_trace_build_pairs_introns_fn(), (void *)&bpi_hook);
  patch_install(&bpe5_p, gmap_trace_build_pairs_end5_fn(), (void *)&bpe5_hook);
  patch_install(&bpe3_p, gmap_trace_build_path_end3_fn(), (void *)&bpe3_hook);
  patch_install(&bpd_p, gmap_trace_build_pairs_dualintrons_fn(), (void *)&bpd_hook);
  patch_install(&bdb_p, gmap_trace_build_dual_breaks_fn(), (void *)&bdb_hook);

  /* gmap's setup for a user segment (gmap.c:3456, 3803-3837), as s3_replay does it */
  Genome_user_setup(g);
  Maxent_hr_setup(g);
  Dynprog_init(600, 10, 11, 10, 8, STANDARD);
  Dynprog_setup(nc ? calls[0].novelsplicingp : 1, NULL, NULL, -1, -1, NULL, NULL, NULL, 0, NULL, NULL, NULL, NULL,
                /*genome*/ NULL);
  dynprogL = Dynprog_new(600, 10, 11, 10, 8);
  dynprogM = Dynprog_new(600, 10, 11, 10, 8);
  dynprogR = Dynprog_new(600, 10, 11, 10, 8);
  pool = Pairpool_new();

  capout = np * 2 + nc * 64 + 1024;
  pout = (S3Pair *)malloc(capout * sizeof(S3Pair));
  probs = (double *)malloc(capout * 2 * sizeof(double));
  for (i = 0; i < nc; i++) {
    const S3Call *c = &calls[i];
    PcCall *r = &pc[i];
    List_T dummy, out, p;
    double defect_rate = 0.0;
    int intronlen = 0, nonintronlen = 0; /* Stage3_compute's (stage3.c:9825, 9834) */
    if (c->first_pair < 0 || c->npairs < 0 || (size_t)c->first_pair + (size_t)c->npairs > np || c->qpos < 0 ||
        (size_t)c->qpos + (size_t)c->querylength > nq || c->invocation != r->invocation) {
      fprintf(stderr, "pc_replay: call %zu out of range\n", i);
      return 5;
    }
    Stage3_setup(c->splicingp, c->novelsplicingp, NULL, NULL, -1, -1, NULL, /*min_intronlength*/ 9,
                 /*max_deletionlength*/ 50, 0, 0, false);
    Pairpool_reset(pool);
    memset(cur_passes, 0, sizeof(cur_passes));
    cur_invocation = c->invocation;
    cur_s2_missed = 0;
    cur_2a_path = build_list(pool, pin + c->first_pair, c->npairs);
    dummy = build_list(pool, pin + c->first_pair, c->npairs); /* what passes 0-1 run on; their result is replaced */
    out = path_compute(&defect_rate, &intronlen, &nonintronlen, dummy, c->cdna_direction, c->watsonp ? true : false,
                       /*genestrand*/ 0, c->jump_late_p ? true : false, c->querylength, c->genomiclength,
                       q + c->qpos, qu + c->qpos, NULL, NULL, c->use_genomicseg_p ? true : false,
                       (Chrnum_T)c->chrnum, c->chroffset, c->chrhigh, c->chrpos, /*knownsplice_limit_low*/ 0U,
                       /*knownsplice_limit_high*/ -1U, /*genome*/ NULL, r->maxpeelback,
                       /*maxpeelback_distalmedial*/ 100, r->nullgap, r->extramaterial_end, r->extraband_end,
                       c->extramaterial_paired, c->extraband_single, c->extraband_paired, pool, dynprogL, dynprogM,
                       dynprogR, r->stage3debug, r->do_final_p ? true : false, NULL, 0, NULL, 60, 5,
                       r->maxintronlen_bound, c->close_indels_mode, r->paired_favor_mode, r->zero_offset);
    if (cur_2a_path != NULL) {
      fprintf(stderr, "pc_replay: invocation %d made no pass-2A call\n", c->invocation);
      return 6;
    }
    r->defect_rate = defect_rate;
    r->intronlen = intronlen;
    r->nonintronlen = nonintronlen;
    memcpy(r->passes, cur_passes, sizeof(cur_passes));
    r->pad = cur_s2_missed;
    r->first_out = (int32_t)nout;
    r->nout = 0;
    for (p = out; p != NULL; p = p->rest) {
      const struct Pair_T *x = (const struct Pair_T *)p->first;
      S3Pair b;
      if (nout >= capout) {
        capout *= 2;
        pout = (S3Pair *)realloc(pout, capout * sizeof(S3Pair));
        probs = (double *)realloc(probs, capout * 2 * sizeof(double));
      }
      b.querypos = x->querypos;
      b.genomepos = (int32_t)x->genomepos;
      b.queryjump = x->queryjump;
      b.genomejump = x->genomejump;
      b.dynprogindex = x->dynprogindex;
      b.src = -1;
      b.cdna = x->cdna;
      b.comp = x->comp;
      b.genome = x->genome;
      b.flags = (uint8_t)((x->gapp ? 1 : 0) | (x->knowngapp ? 2 : 0) | (x->disallowedp ? 4 : 0) |
                          (x->shortexonp ? 8 : 0) | (x->end_intron_p ? 16 : 0));
      pout[nout] = b;
      probs[2 * nout] = x->donor_prob;
      probs[2 * nout + 1] = x->acceptor_prob;
      nout++;
      r->nout++;
    }
  }
  spit(dir, "out_pc.bin", pc, nc * sizeof(PcCall));
  spit(dir, "out_pairs.bin", pout, nout * sizeof(S3Pair));
  spit(dir, "out_probs.bin", probs, nout * 2 * sizeof(double));
  return 0;
}
