/*
 * s3_replay.c -- TEST INFRASTRUCTURE ONLY (oracle/_ref/s3_replay; dev container
 * only, never shipped, never sent to the GPU box).
 *
 * Runs the reference's own build_pairs_introns (stage3.c:7735-7901) -- and, with
 * --si, its score_introns (:7935-8162) on the list that pass returns, as
 * stage3_compute does after path_compute (:9890-9941) -- over stage-3 calls
 * given as records: the gmap_trace recording format (gsnapdp_s3_call /
 * gsnapdp_s3_pair, include/gsnapdp.h).  The reference's stage3.c is compiled
 * where it lies (stage3_si.c), and so are its dynprog.c, maxent_hr.c, pairpool.c
 * and iit-read.c; this file only builds each path as a List_T of Pair_T in a
 * Pairpool, calls the function and records what it returned.
 *
 * It serves two golden sets gmap cannot record here:
 *   * calls under a splicing IIT.  `gmap -s` reads its IIT only for a genome
 *     database (gmap.c:3281-3318 sits in the -d branch), and a gmapindex
 *     database is out of scope, so the calls gmap_trace recorded with `-g` are
 *     replayed with the IIT set up as gmap.c:3283-3302, 3721-3731, 3828-3837 set
 *     it: Dynprog_setup and Stage3_setup get the IIT, its divint crosstable and
 *     the donor / acceptor type ints, and novelsplicingp on or off;
 *   * C4's transcript-derived paths (workload.c4_transcripts), which no gmap run
 *     produces at that size.
 * Replaying gmap_trace's own calls without an IIT reproduces gmap's recorded
 * lists byte for byte (gen_golden.py checks this before it trusts a replay).
 *
 * traverse_genome_gap reads its locals new_leftgenomepos / new_rightgenomepos
 * uninitialised when a Dynprog_genome_gap returns early without writing them
 * (stage3.c:5633-5976; dynprog.c:4855-4858), and adds their difference to
 * *nonintronlen: that counter then depends on stack garbage.  --poison B fills
 * the stack below the call with byte B first, so that two runs with different
 * bytes show which outputs depend on it (gen_golden.py excludes those fields).
 *
 * Usage: s3_replay <dir> [--iit FILE DIV NOVEL] [--si] [--poison B]
 *   in:  <dir>/{genome.u32,calls.bin,pairs_in.bin,query.bin,query_uc.bin}
 *   out: <dir>/{replay_calls.bin,replay_pairs.bin}  (+ --si: si_paths.bin, si_pairs.bin)
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "bool.h"
#include "chrnum.h"
#include "dynprog.h"
#include "genome.h"
#include "iit-read.h"
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
typedef struct { /* gmap_trace.c SiCall */
  int32_t cdna_direction, watsonp, chrnum, genomiclength, nullgap, use_genomicseg_p;
  uint32_t chroffset, chrhigh, chrpos;
  int32_t first_pair, npairs, nbadintrons;
  double avg_donor_score, avg_acceptor_score;
} SiCall;
typedef struct { /* gmap_trace.c SiPair */
  int32_t querypos;
  uint32_t genomepos;
  int32_t queryjump, genomejump;
  uint8_t gapp, knowngapp, comp, pad;
} SiPair;

typedef List_T (*bpi_fn_t)(bool *, bool *, int *, int *, int *, int *, int *, int *, List_T, int, Genomicpos_T,
                           Genomicpos_T, Genomicpos_T, void *, int, int, char *, char *, char *, char *, bool, int,
                           bool, bool, int, int, int, int, int, double, int, Pairpool_T, Dynprog_T, Dynprog_T,
                           Dynprog_T, bool);
typedef List_T (*si_fn_t)(double *, double *, int *, List_T, int, bool, int, Genomicpos_T, Genomicpos_T,
                          Genomicpos_T, char *, int, int, bool);
extern void *gmap_trace_build_pairs_introns_fn(void);
extern void *gmap_trace_build_pairs_singles_fn(void);
typedef List_T (*bps_fn_t)(int *, List_T, Genomicpos_T, Genomicpos_T, Genomicpos_T, Genomicpos_T, char *, char *,
                           char *, char *, int, bool, bool, int, int, int, double, int, Pairpool_T, Dynprog_T);
extern void *gmap_trace_score_introns_fn(void);
typedef List_T (*bpe5_fn_t)(bool *, int *, int *, bool *, int *, List_T, Genomicpos_T, Genomicpos_T, Genomicpos_T,
                            int, Genomicpos_T, Genomicpos_T, char *, char *, char *, char *, int, bool, bool, int,
                            int, int, int, int, double, Pairpool_T, Dynprog_T, bool, int);
typedef List_T (*bpe3_fn_t)(bool *, int *, int *, bool *, int *, List_T, Genomicpos_T, Genomicpos_T, Genomicpos_T,
                            int, int, Genomicpos_T, Genomicpos_T, char *, char *, char *, char *, int, bool, bool,
                            int, int, int, int, int, double, Pairpool_T, Dynprog_T, bool, int);
typedef List_T (*bpd_fn_t)(int *, List_T, Chrnum_T, Genomicpos_T, Genomicpos_T, Genomicpos_T, int, char *, char *,
                           char *, char *, bool, int, bool, bool, int, int, int, int, double, Pairpool_T, Dynprog_T,
                           Dynprog_T);
extern void *gmap_trace_build_pairs_end5_fn(void);
extern void *gmap_trace_build_path_end3_fn(void);
extern void *gmap_trace_build_pairs_dualintrons_fn(void);

static void *slurp(const char *dir, const char *name, size_t *n) {
  char path[4096];
  FILE *f;
  void *buf;
  long sz;
  snprintf(path, sizeof(path), "%s/%s", dir, name);
  if (!(f = fopen(path, "rb"))) {
    fprintf(stderr, "s3_replay: cannot open %s\n", path);
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

typedef struct {
  const void *p;
  int i;
} PtrIdx;
static int cmp_ptr(const void *a, const void *b) {
  const uintptr_t x = (uintptr_t)((const PtrIdx *)a)->p, y = (uintptr_t)((const PtrIdx *)b)->p;
  return x < y ? -1 : (x > y ? 1 : 0);
}

/* the stack the next call's frames will use, filled with one byte */
__attribute__((noinline)) static void poison_stack(int b) {
  volatile unsigned char buf[1 << 17];
  memset((void *)buf, b, sizeof(buf));
  __asm__ volatile("" : : "r"(buf) : "memory");
}

static S3Pair rec(const struct Pair_T *x, int src) {
  S3Pair r;
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

int main(int argc, char **argv) {
  const char *dir, *iitfile = NULL, *div = NULL;
  int novel = 1, do_si = 0, poison = -1, a;
  size_t ng, nc, np, nq, nqu, i;
  unsigned int *g;
  S3Call *calls;
  S3Pair *pin, *pout;
  SiCall *sic;
  SiPair *sip;
  size_t nout = 0, capout, nsip = 0, capsip;
  char *q, *qu;
  static int crosstable[4];
  IIT_T iit = NULL;
  int donor_typeint = -1, acceptor_typeint = -1;
  Pairpool_T pool;
  Dynprog_T dynprogL, dynprogM, dynprogR;
  bpi_fn_t bpi = (bpi_fn_t)gmap_trace_build_pairs_introns_fn();
  bps_fn_t bps = (bps_fn_t)gmap_trace_build_pairs_singles_fn();
  bpe5_fn_t bpe5 = (bpe5_fn_t)gmap_trace_build_pairs_end5_fn();
  bpe3_fn_t bpe3 = (bpe3_fn_t)gmap_trace_build_path_end3_fn();
  bpd_fn_t bpd = (bpd_fn_t)gmap_trace_build_pairs_dualintrons_fn();
  si_fn_t si = (si_fn_t)gmap_trace_score_introns_fn();

  if (argc < 2) {
    fprintf(stderr, "usage: s3_replay <dir> [--iit FILE DIV NOVEL] [--si]\n");
    return 1;
  }
  dir = argv[1];
  for (a = 2; a < argc; a++) {
    if (!strcmp(argv[a], "--iit") && a + 3 < argc) {
      iitfile = argv[a + 1];
      div = argv[a + 2];
      novel = atoi(argv[a + 3]);
      a += 3;
    } else if (!strcmp(argv[a], "--si")) {
      do_si = 1;
    } else if (!strcmp(argv[a], "--poison") && a + 1 < argc) {
      poison = (int)strtol(argv[++a], NULL, 0);
    } else {
      fprintf(stderr, "s3_replay: unknown argument %s\n", argv[a]);
      return 1;
    }
  }
  g = (unsigned int *)slurp(dir, "genome.u32", &ng);
  calls = (S3Call *)slurp(dir, "calls.bin", &nc);
  pin = (S3Pair *)slurp(dir, "pairs_in.bin", &np);
  q = (char *)slurp(dir, "query.bin", &nq);
  qu = (char *)slurp(dir, "query_uc.bin", &nqu);
  nc /= sizeof(S3Call);
  np /= sizeof(S3Pair);

  /* gmap's setup for a user segment (gmap.c:3456, 3803-3837), as ref_driver does it */
  Genome_user_setup(g);
  Maxent_hr_setup(g);
  Dynprog_init(600, 10, 11, 10, 8, STANDARD);
  if (iitfile) {
    if (!(iit = IIT_read((char *)iitfile, NULL, true, READ_ALL, NULL, false, false))) {
      fprintf(stderr, "s3_replay: cannot read %s\n", iitfile);
      return 2;
    }
    /* a user segment's chrnum is 0 or 1: both map to the IIT's division */
    crosstable[0] = crosstable[1] = IIT_divint(iit, (char *)div);
    if ((donor_typeint = IIT_typeint(iit, "donor")) < 0 || (acceptor_typeint = IIT_typeint(iit, "acceptor")) < 0)
      donor_typeint = acceptor_typeint = -1; /* an introns file */
  } else {
    novel = -1; /* each call's recorded flags */
  }
  Dynprog_setup(iit ? novel : (nc ? calls[0].novelsplicingp : 1), iit, iit ? crosstable : NULL, donor_typeint,
                acceptor_typeint, NULL, NULL, NULL, 0, NULL, NULL, NULL, NULL, /*genome*/ NULL);
  dynprogL = Dynprog_new(600, 10, 11, 10, 8);
  dynprogM = Dynprog_new(600, 10, 11, 10, 8);
  dynprogR = Dynprog_new(600, 10, 11, 10, 8);
  pool = Pairpool_new();

  capout = np * 2 + nc * 64 + 1024;
  pout = (S3Pair *)malloc(capout * sizeof(S3Pair));
  capsip = np * 2 + 1024;
  sic = (SiCall *)calloc(nc + 1, sizeof(SiCall));
  sip = (SiPair *)malloc(capsip * sizeof(SiPair));
  for (i = 0; i < nc; i++) {
    S3Call *c = &calls[i];
    List_T path = NULL, out, p;
    PtrIdx *inptr;
    bool shiftp = false, incompletep = false;
    int nintrons = c->in_nintrons, nnonintrons = c->in_nnonintrons, intronlen = c->in_intronlen,
        nonintronlen = c->in_nonintronlen, minor = c->in_minor, major = c->in_major, j;
    struct timespec t0, t1;
    if (c->first_pair < 0 || c->npairs < 0 || (size_t)c->first_pair + (size_t)c->npairs > np ||
        c->qpos < 0 || (size_t)c->qpos + (size_t)c->querylength > nq) {
      fprintf(stderr, "s3_replay: call %zu out of range\n", i);
      return 5;
    }
    if (iit) {
      c->novelsplicingp = novel;
      c->splicingp = 1; /* novelsplicingp || knownsplicingp (gmap.c:3834) */
    }
    Stage3_setup(c->splicingp, c->novelsplicingp, iit, iit ? crosstable : NULL, donor_typeint, acceptor_typeint,
                 NULL, 9, 50, 0, 0, false);
    Pairpool_reset(pool);
    inptr = (PtrIdx *)malloc(sizeof(*inptr) * (size_t)(c->npairs + 1));
    for (j = c->npairs - 1; j >= 0; j--) {
      const S3Pair *x = &pin[c->first_pair + j];
      struct Pair_T *y;
      path = Pairpool_push(path, pool, x->querypos, x->genomepos, x->cdna, x->comp, x->genome, x->dynprogindex);
      y = (struct Pair_T *)path->first;
      y->queryjump = x->queryjump;
      y->genomejump = x->genomejump;
      y->gapp = (x->flags & 1) ? true : false;
      y->knowngapp = (x->flags & 2) ? true : false;
      y->disallowedp = (x->flags & 4) ? true : false;
      y->shortexonp = (x->flags & 8) ? true : false;
      y->end_intron_p = (x->flags & 16) ? true : false;
      inptr[j].p = y;
      inptr[j].i = j;
    }
    qsort(inptr, (size_t)c->npairs, sizeof(PtrIdx), cmp_ptr);
    if (poison >= 0) poison_stack(poison);
    clock_gettime(CLOCK_MONOTONIC, &t0);
    if (c->pass < 0 || c->pass > 4) { /* build_dual_breaks needs stage 2's oligoindices: not replayed */
      fprintf(stderr, "s3_replay: call %zu: pass %d is not replayed\n", i, c->pass);
      return 6;
    }
    if (c->pass == 2 || c->pass == 3) { /* GSNAPDP_S3_END5 / END3 (stage3.c:7351 / 7236), extendp */
      bool knownsplicep = false, chop_exon_p = false;
      int ambig_end_length = 0, ambig_splicetype = 0;
      if (c->pass == 2)
        out = bpe5(&knownsplicep, &ambig_end_length, &ambig_splicetype, &chop_exon_p, &minor, path, c->chroffset,
                   c->chrhigh, c->chrpos, c->genomiclength, 0, 0, q + c->qpos, qu + c->qpos, NULL, NULL,
                   c->cdna_direction, c->watsonp ? true : false, c->jump_late_p ? true : false, c->maxpeelback,
                   c->maxpeelback, c->nullgap, c->extramaterial_end, c->extraband_end, c->defect_rate, pool,
                   dynprogR, true, c->endalign);
      else
        out = bpe3(&knownsplicep, &ambig_end_length, &ambig_splicetype, &chop_exon_p, &minor, path, c->chroffset,
                   c->chrhigh, c->chrpos, c->querylength, c->genomiclength, 0, 0, q + c->qpos, qu + c->qpos, NULL,
                   NULL, c->cdna_direction, c->watsonp ? true : false, c->jump_late_p ? true : false,
                   c->maxpeelback, c->maxpeelback, c->nullgap, c->extramaterial_end, c->extraband_end,
                   c->defect_rate, pool, dynprogL, true, c->endalign);
      c->status = (knownsplicep || ambig_end_length != 0 || chop_exon_p) ? 1 : 0;
    } else if (c->pass == 4) /* GSNAPDP_S3_DUALINTRONS (stage3.c:7592) */
      out = bpd(&major, path, (Chrnum_T)c->chrnum, c->chroffset, c->chrhigh, c->chrpos, c->genomiclength,
                q + c->qpos, qu + c->qpos, NULL, NULL, c->use_genomicseg_p ? true : false, c->cdna_direction,
                c->watsonp ? true : false, c->jump_late_p ? true : false, c->maxpeelback, c->nullgap,
                c->extramaterial_paired, c->extraband_paired, c->defect_rate, pool, dynprogL, dynprogR);
    else if (c->pass == 1) /* GSNAPDP_S3_SINGLES: build_pairs_singles (stage3.c:7454) */
      out = bps(&minor, path, c->chroffset, c->chrhigh, c->chrpos, (Genomicpos_T)c->genomiclength, q + c->qpos,
                qu + c->qpos, NULL, NULL, c->cdna_direction, c->watsonp ? true : false,
                c->jump_late_p ? true : false, c->maxpeelback, c->nullgap, c->extraband_single, c->defect_rate,
                c->close_indels_mode, pool, dynprogM);
    else
      out = bpi(&shiftp, &incompletep, &nintrons, &nnonintrons, &intronlen, &nonintronlen, &minor, &major, path,
                c->chrnum, c->chroffset, c->chrhigh, c->chrpos, NULL, c->querylength, c->genomiclength, q + c->qpos,
                qu + c->qpos, NULL, NULL, c->use_genomicseg_p ? true : false, c->cdna_direction,
                c->watsonp ? true : false, c->jump_late_p ? true : false, c->maxpeelback, c->nullgap,
                c->extramaterial_paired, c->extraband_single, c->extraband_paired, c->defect_rate,
                c->close_indels_mode, pool, dynprogL, dynprogM, dynprogR, c->finalp ? true : false);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    c->ref_seconds = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    c->first_out = (int32_t)nout;
    c->nout = 0;
    for (p = out; p != NULL; p = p->rest) {
      PtrIdx key, *hit;
      int src;
      key.p = p->first;
      hit = (PtrIdx *)bsearch(&key, inptr, (size_t)c->npairs, sizeof(PtrIdx), cmp_ptr);
      src = hit ? hit->i : -1;
      if (nout >= capout) {
        capout *= 2;
        pout = (S3Pair *)realloc(pout, capout * sizeof(S3Pair));
      }
      pout[nout++] = rec((const struct Pair_T *)p->first, src);
      c->nout++;
    }
    free(inptr);
    c->out_minor = minor;
    c->out_major = major;
    c->out_nintrons = nintrons;
    c->out_nnonintrons = nnonintrons;
    c->out_intronlen = intronlen;
    c->out_nonintronlen = nonintronlen;
    c->shiftp = shiftp;
    c->incompletep = incompletep;
    if (c->pass != 2 && c->pass != 3) c->status = 0;
    if (do_si) { /* stage3_compute after path_compute (:9890-9941): score_introns(List_reverse(pairs)) */
      SiCall *s = &sic[i];
      double d = 0.0, acc = 0.0;
      int nb = 0;
      List_T sp = List_reverse(out);
      s->cdna_direction = c->cdna_direction;
      s->watsonp = c->watsonp;
      s->chrnum = c->chrnum;
      s->genomiclength = c->genomiclength;
      s->nullgap = c->nullgap;
      s->chroffset = c->chroffset;
      s->chrhigh = c->chrhigh;
      s->chrpos = c->chrpos;
      s->first_pair = (int32_t)nsip;
      for (p = sp; p != NULL; p = p->rest) {
        const struct Pair_T *x = (const struct Pair_T *)p->first;
        SiPair r = {x->querypos, x->genomepos, x->queryjump, x->genomejump, (uint8_t)x->gapp,
                    (uint8_t)x->knowngapp, (uint8_t)x->comp, 0};
        if (nsip >= capsip) {
          capsip *= 2;
          sip = (SiPair *)realloc(sip, capsip * sizeof(SiPair));
        }
        sip[nsip++] = r;
        s->npairs++;
      }
      si(&d, &acc, &nb, sp, c->cdna_direction, c->watsonp ? true : false, c->chrnum, c->chroffset, c->chrhigh,
         c->chrpos, NULL, c->genomiclength, c->nullgap, false);
      s->avg_donor_score = d;
      s->avg_acceptor_score = acc;
      s->nbadintrons = nb;
    }
  }
  spit(dir, "replay_calls.bin", calls, nc * sizeof(S3Call));
  spit(dir, "replay_pairs.bin", pout, nout * sizeof(S3Pair));
  if (do_si) {
    spit(dir, "si_paths.bin", sic, nc * sizeof(SiCall));
    spit(dir, "si_pairs.bin", sip, nsip * sizeof(SiPair));
  }
  return 0;
}
