/*
 * ref_driver.c -- TEST INFRASTRUCTURE ONLY.  Built only in the survey/dev
 * container, against the reference's own sources under /root/reference/src
 * (see oracle/Makefile).  Output goes to oracle/_ref/ (git-ignored) and is used
 * to generate the golden fixtures in tests/golden/.  Never shipped, never
 * loaded by the product library.
 *
 * Usage:
 *   ref_driver dp     <dir>   windows.bin query.bin query_uc.bin genome.u32 -> results.bin pairs.bin npairs.i32
 *   ref_driver ggap   <dir>   ggap_windows.bin query.bin query_uc.bin genome.u32 -> ggap_results.bin pairs.bin npairs.i32
 *   ref_driver ggapk  <dir> 0 <splicing.iit> <div> <novelsplicingp>
 *                             the same with a splicing IIT given to Dynprog_setup (known-site
 *                             rewards / constrained introns, dynprog.c:3375-3697); chrnum 1 maps to <div>
 *   ref_driver cgap   <dir>   cgap_windows.bin query.bin query_uc.bin gseg.bin gseg_off.i64 genome.u32
 *                             -> cgap_results.bin pairs.bin npairs.i32
 *   ref_driver sj     <dir>   sj_windows.bin query.bin query_uc.bin -> results.bin pairs.bin npairs.i32
 *   ref_driver mksj   <dir>   mksj_in.bin genome.u32 -> mksj_out.bin
 *   ref_driver micro  <dir>   micro_windows.bin query.bin query_uc.bin genome.u32 -> micro_results.bin pairs.bin npairs.i32
 *   ref_driver known  <dir> 0 [amb_closest]  known_windows.bin query*.bin genome.u32 sites.u32 types.i32
 *                             [tobs cobs tmax cmax].u32 -> known_results.bin pairs.bin npairs.i32
 *   ref_driver maxent <dir>   maxent_in.bin genome.u32 -> maxent_out.f64
 *   ref_driver pdist  <dir>   -> pdist.i32 (4 x 128 x 128 via Dynprog_pairdistance for HIGHQ only) + consistent probe
 * All inputs use the record layouts of include/gsnapdp.h.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* reference headers (from -I/root/reference/src) */
#include "bool.h"
#include "dynprog.h"
#include "genome.h"
#include "list.h"
#include "listdef.h"
#include "maxent_hr.h"
#include "pairdef.h"
#include "pairpool.h"
#include "splicetrie_build.h"
#include "splicetrie.h"
#include "iit-read.h"

/* our record layouts */
#include "../include/gsnapdp.h"

static void *slurp(const char *dir, const char *name, size_t *n) {
  char path[4096];
  FILE *f;
  void *buf;
  long sz;
  snprintf(path, sizeof(path), "%s/%s", dir, name);
  f = fopen(path, "rb");
  if (!f) {
    fprintf(stderr, "cannot open %s\n", path);
    exit(2);
  }
  fseek(f, 0, SEEK_END);
  sz = ftell(f);
  fseek(f, 0, SEEK_SET);
  buf = malloc((size_t)sz + 64);
  memset(buf, 0, (size_t)sz + 64);
  if (sz > 0 && fread(buf, 1, (size_t)sz, f) != (size_t)sz) exit(3);
  fclose(f);
  *n = (size_t)sz;
  return buf;
}

static void spit(const char *dir, const char *name, const void *buf, size_t n) {
  char path[4096];
  FILE *f;
  snprintf(path, sizeof(path), "%s/%s", dir, name);
  f = fopen(path, "wb");
  if (!f) exit(4);
  if (n) fwrite(buf, 1, n, f);
  fclose(f);
}

/* Walk a reference List_T of Pair_T into flat records. */
static int flatten(List_T pairs, gsnapdp_pair *out, int cap) {
  int n = 0;
  List_T p;
  for (p = pairs; p != NULL; p = p->rest) {
    Pair_T pair = (Pair_T)p->first;
    if (n < cap) {
      gsnapdp_pair *o = &out[n];
      memset(o, 0, sizeof(*o));
      o->querypos = pair->querypos;
      o->genomepos = (int32_t)pair->genomepos;
      o->queryjump = pair->gapp ? pair->queryjump : 0;
      o->genomejump = pair->gapp ? pair->genomejump : 0;
      o->dynprogindex = pair->dynprogindex;
      o->cdna = pair->cdna;
      o->comp = pair->comp;
      o->genome = pair->genome;
      o->gapp = (pair->gapp ? 1 : 0) | (pair->knowngapp ? 2 : 0);
    }
    n++;
  }
  return n;
}

#define PAIRCAP 8192

static int run_dp(const char *dir) {
  size_t nw, nq, nu, ng;
  gsnapdp_window *w = (gsnapdp_window *)slurp(dir, "windows.bin", &nw);
  char *q = (char *)slurp(dir, "query.bin", &nq);
  char *qu = (char *)slurp(dir, "query_uc.bin", &nu);
  UINT4 *g = (UINT4 *)slurp(dir, "genome.u32", &ng);
  int n = (int)(nw / sizeof(gsnapdp_window)), i;
  gsnapdp_result *res = (gsnapdp_result *)calloc((size_t)n + 1, sizeof(gsnapdp_result));
  int32_t *npairs = (int32_t *)calloc((size_t)n + 1, sizeof(int32_t));
  gsnapdp_pair *tmp = (gsnapdp_pair *)malloc(sizeof(gsnapdp_pair) * PAIRCAP);
  FILE *fp;
  char path[4096];
  Dynprog_T dp = Dynprog_new(600, 10, 11, 10, 8);
  Pairpool_T pool = Pairpool_new();

  Genome_user_setup(g);
  Maxent_hr_setup(g);
  snprintf(path, sizeof(path), "%s/pairs.bin", dir);
  fp = fopen(path, "wb");
  for (i = 0; i < n; i++) {
    gsnapdp_window *x = &w[i];
    int dpi = x->dynprogindex, fs = 0, nm = 0, nmm = 0, no = 0, ni = 0, k;
    List_T pairs = NULL;
    if (x->maxlength1 != 611 || x->maxlength2 != 2000) {
      fprintf(stderr, "window %d: ref driver only supports maxlength 611x2000\n", i);
      return 5;
    }
    Pairpool_reset(pool);
    if (getenv("REF_TRACE")) {
      fprintf(stderr, "w %d kind %d L1 %d L2 %d off2 %d glen %u chrpos %u chrhigh %u chroff %u watson %d band %d end %d\n",
              i, x->kind, x->length1, x->length2, x->offset2, x->genomiclength, x->chrpos, x->chrhigh,
              x->chroffset, x->watsonp, x->extraband, x->endalign);
      fflush(stderr);
    }
    if (x->kind == GSNAPDP_SINGLE_GAP) {
      pairs = Dynprog_single_gap(&dpi, &fs, &nm, &nmm, &no, &ni, dp, q + x->qpos, qu + x->qpos,
                                 NULL, NULL, x->length1, x->length2, x->offset1, x->offset2,
                                 x->chroffset, x->chrhigh, x->chrpos, x->genomiclength,
                                 x->cdna_direction, x->watsonp, x->jump_late_p, pool, x->extraband,
                                 (double)x->defect_rate, 0, x->widebandp);
    } else if (x->kind == GSNAPDP_END5_GAP) {
      pairs = Dynprog_end5_gap(&dpi, &fs, &nm, &nmm, &no, &ni, dp, q + x->qpos, qu + x->qpos, NULL,
                               NULL, x->length1, x->length2, x->offset1, x->offset2, x->chroffset,
                               x->chrhigh, x->chrpos, x->genomiclength, x->cdna_direction,
                               x->watsonp, x->jump_late_p, pool, x->extraband,
                               (double)x->defect_rate, (Endalign_T)x->endalign,
                               /*use_genomicseg_p*/ false);
    } else {
      pairs = Dynprog_end3_gap(&dpi, &fs, &nm, &nmm, &no, &ni, dp, q + x->qpos, qu + x->qpos, NULL,
                               NULL, x->length1, x->length2, x->offset1, x->offset2, x->chroffset,
                               x->chrhigh, x->chrpos, x->genomiclength, x->cdna_direction,
                               x->watsonp, x->jump_late_p, pool, x->extraband,
                               (double)x->defect_rate, (Endalign_T)x->endalign, false);
    }
    res[i].finalscore = fs;
    res[i].nmatches = nm;
    res[i].nmismatches = nmm;
    res[i].nopens = no;
    res[i].nindels = ni;
    res[i].reserved = dpi;
    k = flatten(pairs, tmp, PAIRCAP);
    npairs[i] = k;
    fwrite(tmp, sizeof(gsnapdp_pair), (size_t)(k < PAIRCAP ? k : PAIRCAP), fp);
  }
  fclose(fp);
  spit(dir, "results.bin", res, sizeof(gsnapdp_result) * (size_t)n);
  spit(dir, "npairs.i32", npairs, sizeof(int32_t) * (size_t)n);
  return 0;
}

static int run_ggap(const char *dir) {
  size_t nw, nq, nu, ng;
  gsnapdp_ggap_window *w = (gsnapdp_ggap_window *)slurp(dir, "ggap_windows.bin", &nw);
  char *q = (char *)slurp(dir, "query.bin", &nq);
  char *qu = (char *)slurp(dir, "query_uc.bin", &nu);
  UINT4 *g = (UINT4 *)slurp(dir, "genome.u32", &ng);
  int n = (int)(nw / sizeof(gsnapdp_ggap_window)), i;
  gsnapdp_ggap_result *res = (gsnapdp_ggap_result *)calloc((size_t)n + 1, sizeof(*res));
  int32_t *npairs = (int32_t *)calloc((size_t)n + 1, sizeof(int32_t));
  gsnapdp_pair *tmp = (gsnapdp_pair *)malloc(sizeof(gsnapdp_pair) * PAIRCAP);
  FILE *fp;
  char path[4096];
  Dynprog_T dpL = Dynprog_new(600, 10, 11, 10, 8), dpR = Dynprog_new(600, 10, 11, 10, 8);
  Pairpool_T pool = Pairpool_new();

  Genome_user_setup(g);
  Maxent_hr_setup(g);
  snprintf(path, sizeof(path), "%s/pairs.bin", dir);
  fp = fopen(path, "wb");
  for (i = 0; i < n; i++) {
    gsnapdp_ggap_window *x = &w[i];
    gsnapdp_ggap_result *o = &res[i];
    int dpi = x->dynprogindex, k;
    int fs = 0, nl = 0, nr = 0, nm = 0, nmm = 0, no = 0, ni = 0, eh = 0, it = 0;
    double lp = 0, rp = 0;
    List_T pairs;
    const char *s1 = q + x->qpos, *s1u = qu + x->qpos;
    Pairpool_reset(pool);
    pairs = Dynprog_genome_gap(&dpi, &fs, &nl, &nr, &lp, &rp, &nm, &nmm, &no, &ni, &eh, &it, dpL,
                               dpR, (char *)s1, (char *)s1u, NULL, NULL, NULL, NULL, x->length1,
                               x->length2L, x->length2R, x->offset1, x->offset2L, x->revoffset2R,
                               /*chrnum*/ 1, x->chroffset, x->chrhigh, x->chrpos, x->genomiclength,
                               NULL, false, x->cdna_direction, x->watsonp, x->jump_late_p, pool,
                               x->extraband_paired, (double)x->defect_rate, x->maxpeelback,
                               x->halfp, x->finalp, x->use_probabilities_p, x->score_threshold,
                               x->splicingp);
    o->finalscore = fs;
    o->new_leftgenomepos = nl;
    o->new_rightgenomepos = nr;
    o->nmatches = nm;
    o->nmismatches = nmm;
    o->nopens = no;
    o->nindels = ni;
    o->exonhead = eh;
    o->introntype = it;
    o->dynprogindex = dpi;
    o->returned_null = pairs == NULL;
    o->bridge_ok = 1;
    o->left_prob = lp;
    o->right_prob = rp;
    k = flatten(pairs, tmp, PAIRCAP);
    npairs[i] = k;
    fwrite(tmp, sizeof(gsnapdp_pair), (size_t)(k < PAIRCAP ? k : PAIRCAP), fp);
  }
  fclose(fp);
  spit(dir, "ggap_results.bin", res, sizeof(*res) * (size_t)n);
  spit(dir, "npairs.i32", npairs, sizeof(int32_t) * (size_t)n);
  return 0;
}

static int run_cgap(const char *dir) {
  size_t nw, nq, nu, ng, ns, no;
  gsnapdp_cgap_window *w = (gsnapdp_cgap_window *)slurp(dir, "cgap_windows.bin", &nw);
  char *q = (char *)slurp(dir, "query.bin", &nq);
  char *qu = (char *)slurp(dir, "query_uc.bin", &nu);
  char *gs = (char *)slurp(dir, "gseg.bin", &ns);
  int64_t *goff = (int64_t *)slurp(dir, "gseg_off.i64", &no);
  UINT4 *g = (UINT4 *)slurp(dir, "genome.u32", &ng);
  int n = (int)(nw / sizeof(gsnapdp_cgap_window)), i;
  gsnapdp_cgap_result *res = (gsnapdp_cgap_result *)calloc((size_t)n + 1, sizeof(*res));
  int32_t *npairs = (int32_t *)calloc((size_t)n + 1, sizeof(int32_t));
  gsnapdp_pair *tmp = (gsnapdp_pair *)malloc(sizeof(gsnapdp_pair) * PAIRCAP);
  FILE *fp;
  char path[4096];
  Dynprog_T dpL = Dynprog_new(600, 10, 11, 10, 8), dpR = Dynprog_new(600, 10, 11, 10, 8);
  Pairpool_T pool = Pairpool_new();

  Genome_user_setup(g);
  Maxent_hr_setup(g);
  snprintf(path, sizeof(path), "%s/pairs.bin", dir);
  fp = fopen(path, "wb");
  for (i = 0; i < n; i++) {
    gsnapdp_cgap_window *x = &w[i];
    gsnapdp_cgap_result *o = &res[i];
    int dpi = x->dynprogindex, fs = -777777, k;
    bool incomplete = false;
    List_T pairs;
    char *seg = gs + goff[i];
    if (x->maxlength1 != 611 || x->maxlength2 != 2000) {
      /* the too-long returns: shrink the workspaces' limits like Dynprog_new would */
      ((int *)dpL)[0] = ((int *)dpR)[0] = x->maxlength1;
      ((int *)dpL)[1] = ((int *)dpR)[1] = x->maxlength2;
    }
    Pairpool_reset(pool);
    pairs = Dynprog_cdna_gap(&dpi, &fs, &incomplete, dpL, dpR, q + x->qposL, qu + x->qposL,
                             q + x->qposR, qu + x->qposR, seg, seg, x->length1L, x->length1R,
                             x->length2, x->offset1L, x->revoffset1R, x->offset2, x->chroffset,
                             x->chrhigh, x->chrpos, x->genomiclength, x->cdna_direction, x->watsonp,
                             x->jump_late_p, pool, x->extraband_paired, (double)x->defect_rate);
    ((int *)dpL)[0] = ((int *)dpR)[0] = 611;
    ((int *)dpL)[1] = ((int *)dpR)[1] = 2000;
    o->finalscore = fs == -777777 ? 0 : fs;
    o->finalscore_set = fs != -777777;
    o->dynprogindex = dpi;
    o->incompletep = incomplete ? 1 : 0;
    o->returned_null = pairs == NULL;
    k = flatten(pairs, tmp, PAIRCAP);
    npairs[i] = k;
    o->npairs = k;
    fwrite(tmp, sizeof(gsnapdp_pair), (size_t)(k < PAIRCAP ? k : PAIRCAP), fp);
  }
  fclose(fp);
  spit(dir, "cgap_results.bin", res, sizeof(*res) * (size_t)n);
  spit(dir, "npairs.i32", npairs, sizeof(int32_t) * (size_t)n);
  return 0;
}


static int run_sj(const char *dir) {
  size_t nw, nq, nu;
  gsnapdp_sj_window *w = (gsnapdp_sj_window *)slurp(dir, "sj_windows.bin", &nw);
  char *q = (char *)slurp(dir, "query.bin", &nq);
  char *qu = (char *)slurp(dir, "query_uc.bin", &nu);
  int n = (int)(nw / sizeof(gsnapdp_sj_window)), i;
  gsnapdp_result *res = (gsnapdp_result *)calloc((size_t)n + 1, sizeof(gsnapdp_result));
  int32_t *npairs = (int32_t *)calloc((size_t)n + 1, sizeof(int32_t));
  gsnapdp_pair *tmp = (gsnapdp_pair *)malloc(sizeof(gsnapdp_pair) * PAIRCAP);
  FILE *fp;
  char path[4096];
  Dynprog_T dp = Dynprog_new(600, 10, 11, 10, 8);
  Pairpool_T pool = Pairpool_new();

  snprintf(path, sizeof(path), "%s/pairs.bin", dir);
  fp = fopen(path, "wb");
  for (i = 0; i < n; i++) {
    gsnapdp_sj_window *x = &w[i];
    int dpi = x->dynprogindex, fs = -777, nm = -1, nmm = -1, no = -1, ni = -1, k;
    List_T pairs;
    ((int *)dp)[0] = x->maxlength1 < 611 ? x->maxlength1 : 611;
    ((int *)dp)[1] = x->maxlength2 < 2000 ? x->maxlength2 : 2000;
    Pairpool_reset(pool);
    if (x->kind == GSNAPDP_END5_GAP)
      pairs = Dynprog_end5_splicejunction(
          &dpi, &fs, &nm, &nmm, &no, &ni, dp, q + x->qpos, qu + x->qpos, q + x->spos, qu + x->spos,
          x->length1, x->length2, x->offset1, x->offset2_anchor, x->offset2_far, 0, 0, 0, 0,
          x->cdna_direction, x->watsonp, x->jump_late_p, pool, x->extraband_end,
          (double)x->defect_rate, x->contlength);
    else
      pairs = Dynprog_end3_splicejunction(
          &dpi, &fs, &nm, &nmm, &no, &ni, dp, q + x->qpos, qu + x->qpos, q + x->spos, qu + x->spos,
          x->length1, x->length2, x->offset1, x->offset2_anchor, x->offset2_far, 0, 0, 0, 0,
          x->cdna_direction, x->watsonp, x->jump_late_p, pool, x->extraband_end,
          (double)x->defect_rate, x->contlength);
    ((int *)dp)[0] = 611;
    ((int *)dp)[1] = 2000;
    res[i].finalscore = fs;
    res[i].nmatches = nm;
    res[i].nmismatches = nmm;
    res[i].nopens = no;
    res[i].nindels = ni;
    res[i].reserved = dpi;
    k = flatten(pairs, tmp, PAIRCAP);
    npairs[i] = k;
    fwrite(tmp, sizeof(gsnapdp_pair), (size_t)(k < PAIRCAP ? k : PAIRCAP), fp);
  }
  fclose(fp);
  spit(dir, "results.bin", res, sizeof(gsnapdp_result) * (size_t)n);
  spit(dir, "npairs.i32", npairs, sizeof(int32_t) * (size_t)n);
  return 0;
}

/* Dynprog_make_splicejunction_5/3 (dynprog.c:6061, 6149) on the packed genome:
 * record {end(5|3), splicecoord, splicelength, contlength, far_splicetype,
 * watsonp}; output = the junction buffer (contlength + splicelength bytes,
 * pre-filled with '#') per record. */
typedef struct mksj_in {
  int32_t end, splicecoord, splicelength, contlength, far_splicetype, watsonp;
} mksj_in;

static int run_mksj(const char *dir) {
  size_t ni, ng;
  mksj_in *in = (mksj_in *)slurp(dir, "mksj_in.bin", &ni);
  UINT4 *g = (UINT4 *)slurp(dir, "genome.u32", &ng);
  int n = (int)(ni / sizeof(mksj_in)), i;
  char path[4096];
  FILE *fp;
  Genome_user_setup(g);
  snprintf(path, sizeof(path), "%s/mksj_out.bin", dir);
  fp = fopen(path, "wb");
  for (i = 0; i < n; i++) {
    int len = in[i].contlength + in[i].splicelength;
    char *buf = (char *)malloc((size_t)len + 1);
    memset(buf, '#', (size_t)len + 1);
    if (in[i].end == 5)
      Dynprog_make_splicejunction_5(buf, (Genomicpos_T)in[i].splicecoord, in[i].splicelength,
                                    in[i].contlength, (Splicetype_T)in[i].far_splicetype,
                                    in[i].watsonp);
    else
      Dynprog_make_splicejunction_3(buf, (Genomicpos_T)in[i].splicecoord, in[i].splicelength,
                                    in[i].contlength, (Splicetype_T)in[i].far_splicetype,
                                    in[i].watsonp);
    fwrite(buf, 1, (size_t)len, fp);
    free(buf);
  }
  fclose(fp);
  return 0;
}

static int run_micro(const char *dir) {
  size_t nw, nq, nu, ng;
  gsnapdp_micro_window *w = (gsnapdp_micro_window *)slurp(dir, "micro_windows.bin", &nw);
  char *q = (char *)slurp(dir, "query.bin", &nq);
  char *qu = (char *)slurp(dir, "query_uc.bin", &nu);
  UINT4 *g = (UINT4 *)slurp(dir, "genome.u32", &ng);
  int n = (int)(nw / sizeof(gsnapdp_micro_window)), i;
  gsnapdp_micro_result *res = (gsnapdp_micro_result *)calloc((size_t)n + 1, sizeof(*res));
  int32_t *npairs = (int32_t *)calloc((size_t)n + 1, sizeof(int32_t));
  gsnapdp_pair *tmp = (gsnapdp_pair *)malloc(sizeof(gsnapdp_pair) * PAIRCAP);
  FILE *fp;
  char path[4096];
  Pairpool_T pool = Pairpool_new();

  Genome_user_setup(g);
  Maxent_hr_setup(g);
  snprintf(path, sizeof(path), "%s/pairs.bin", dir);
  fp = fopen(path, "wb");
  for (i = 0; i < n; i++) {
    gsnapdp_micro_window *x = &w[i];
    gsnapdp_micro_result *o = &res[i];
    double p2 = -1, p3 = -1;
    int dpi = x->dynprogindex, it = -77, k;
    List_T pairs;
    char *qs = q + (long)x->ppos - x->offset1, *qsu = qu + (long)x->ppos - x->offset1;
    Pairpool_reset(pool);
    pairs = Dynprog_microexon_int(&p2, &p3, &dpi, &it, q + x->qpos, qu + x->qpos, NULL, NULL, NULL,
                                  NULL, x->length1, 0, 0, x->offset1, x->offset2L, x->revoffset2R,
                                  x->cdna_direction, qs, qsu, NULL, NULL, x->chroffset, x->chrhigh,
                                  x->chrpos, x->genomiclength, x->watsonp, false, pool,
                                  (double)x->defect_rate);
    o->bestprob2 = p2;
    o->bestprob3 = p3;
    o->microintrontype = it;
    o->dynprogindex = dpi;
    o->found = pairs != NULL;
    k = flatten(pairs, tmp, PAIRCAP);
    npairs[i] = k;
    fwrite(tmp, sizeof(gsnapdp_pair), (size_t)(k < PAIRCAP ? k : PAIRCAP), fp);
  }
  fclose(fp);
  spit(dir, "micro_results.bin", res, sizeof(*res) * (size_t)n);
  spit(dir, "npairs.i32", npairs, sizeof(int32_t) * (size_t)n);
  return 0;
}

/* Dynprog_end5_known / Dynprog_end3_known (dynprog.c:6414, 6680) with known
 * splice sites and their tries (Dynprog_setup + Splicetrie_setup). */
typedef struct known_in {
  int32_t end, length1, length2, offset1, offset2, querylength, genomiclength, cdna_direction;
  int32_t watsonp, jump_late_p, extraband_end, dynprogindex;
  uint32_t chroffset, chrhigh, chrpos, limit_low, limit_high, qpos;
  float defect_rate;
  int32_t pad;
} known_in;

typedef struct known_out {
  int32_t knownsplicep, dynprogindex, finalscore, ambig_end_length, ambig_splicetype;
  int32_t nmatches, nmismatches, nopens, nindels, protectedp, returned_null, pad;
} known_out;

static void *slurp_or_null(const char *dir, const char *name, size_t *n) {
  void *p = slurp(dir, name, n);
  return *n ? p : NULL;
}

static int run_known(const char *dir, int amb_closest) {
  size_t nw, nq, nu, ng, ns, nt, n1, n2, n3, n4;
  known_in *w = (known_in *)slurp(dir, "known_windows.bin", &nw);
  char *q = (char *)slurp(dir, "query.bin", &nq);
  char *qu = (char *)slurp(dir, "query_uc.bin", &nu);
  UINT4 *g = (UINT4 *)slurp(dir, "genome.u32", &ng);
  Genomicpos_T *sites = (Genomicpos_T *)slurp(dir, "sites.u32", &ns);
  Splicetype_T *types = (Splicetype_T *)slurp(dir, "types.i32", &nt);
  unsigned int *tobs = (unsigned int *)slurp_or_null(dir, "tobs.u32", &n1);
  unsigned int *cobs = (unsigned int *)slurp_or_null(dir, "cobs.u32", &n2);
  unsigned int *tmax = (unsigned int *)slurp_or_null(dir, "tmax.u32", &n3);
  unsigned int *cmax = (unsigned int *)slurp_or_null(dir, "cmax.u32", &n4);
  int n = (int)(nw / sizeof(known_in)), i;
  known_out *res = (known_out *)calloc((size_t)n + 1, sizeof(known_out));
  int32_t *npairs = (int32_t *)calloc((size_t)n + 1, sizeof(int32_t));
  gsnapdp_pair *tmp = (gsnapdp_pair *)malloc(sizeof(gsnapdp_pair) * PAIRCAP);
  FILE *fp;
  char path[4096];
  Dynprog_T dp = Dynprog_new(600, 10, 11, 10, 8);
  Pairpool_T pool = Pairpool_new();

  Genome_user_setup(g);
  Maxent_hr_setup(g);
  Dynprog_setup(false, NULL, NULL, -1, -1, sites, types, NULL, (int)(ns / 4), tobs, cobs, tmax, cmax,
                NULL);
  Splicetrie_setup(sites, NULL, NULL, tobs, cobs, tmax, cmax, false, amb_closest, false, 0);
  snprintf(path, sizeof(path), "%s/pairs.bin", dir);
  fp = fopen(path, "wb");
  for (i = 0; i < n; i++) {
    known_in *x = &w[i];
    known_out *o = &res[i];
    bool known = 77;
    int dpi = x->dynprogindex, fs = -777, amb = -777, nm = -1, nmm = -1, no = -1, ni = -1, k;
    Splicetype_T at = (Splicetype_T)77;
    List_T pairs, p;
    Pairpool_reset(pool);
    if (x->end == 5)
      pairs = Dynprog_end5_known(&known, &dpi, &fs, &amb, &at, &nm, &nmm, &no, &ni, dp,
                                 q + x->qpos, qu + x->qpos, NULL, NULL, x->length1, x->length2,
                                 x->offset1, x->offset2, x->chroffset, x->chrhigh, x->chrpos,
                                 x->genomiclength, x->limit_low, x->limit_high, x->cdna_direction,
                                 x->watsonp, x->jump_late_p, pool, x->extraband_end,
                                 (double)x->defect_rate);
    else
      pairs = Dynprog_end3_known(&known, &dpi, &fs, &amb, &at, &nm, &nmm, &no, &ni, dp,
                                 q + x->qpos, qu + x->qpos, NULL, NULL, x->length1, x->length2,
                                 x->offset1, x->offset2, x->querylength, x->chroffset, x->chrhigh,
                                 x->chrpos, x->genomiclength, x->limit_low, x->limit_high,
                                 x->cdna_direction, x->watsonp, x->jump_late_p, pool,
                                 x->extraband_end, (double)x->defect_rate);
    o->knownsplicep = known;
    o->dynprogindex = dpi;
    o->finalscore = fs;
    o->ambig_end_length = amb;
    o->ambig_splicetype = (int32_t)at;
    o->nmatches = nm;
    o->nmismatches = nmm;
    o->nopens = no;
    o->nindels = ni;
    o->returned_null = pairs == NULL;
    o->protectedp = pairs != NULL;
    for (p = pairs; p != NULL; p = p->rest)
      if (!((Pair_T)p->first)->protectedp) o->protectedp = 0;
    k = flatten(pairs, tmp, PAIRCAP);
    npairs[i] = k;
    fwrite(tmp, sizeof(gsnapdp_pair), (size_t)(k < PAIRCAP ? k : PAIRCAP), fp);
  }
  fclose(fp);
  spit(dir, "known_results.bin", res, sizeof(known_out) * (size_t)n);
  spit(dir, "npairs.i32", npairs, sizeof(int32_t) * (size_t)n);
  return 0;
}

typedef struct maxent_in {
  uint32_t model, splice_pos, chroffset, pad;
} maxent_in;

static int run_maxent(const char *dir) {
  size_t ni, ng;
  maxent_in *in = (maxent_in *)slurp(dir, "maxent_in.bin", &ni);
  UINT4 *g = (UINT4 *)slurp(dir, "genome.u32", &ng);
  int n = (int)(ni / sizeof(maxent_in)), i;
  double *out = (double *)calloc((size_t)n + 1, sizeof(double));
  Genome_user_setup(g);
  Maxent_hr_setup(g);
  for (i = 0; i < n; i++) {
    switch (in[i].model) {
      case 0: out[i] = Maxent_hr_donor_prob(in[i].splice_pos, in[i].chroffset); break;
      case 1: out[i] = Maxent_hr_acceptor_prob(in[i].splice_pos, in[i].chroffset); break;
      case 2: out[i] = Maxent_hr_antidonor_prob(in[i].splice_pos, in[i].chroffset); break;
      default: out[i] = Maxent_hr_antiacceptor_prob(in[i].splice_pos, in[i].chroffset); break;
    }
  }
  spit(dir, "maxent_out.f64", out, sizeof(double) * (size_t)n);
  return 0;
}

static int run_pdist(const char *dir) {
  /* Only HIGHQ is exported by the reference (Dynprog_pairdistance :1048). */
  int32_t *t = (int32_t *)malloc(sizeof(int32_t) * 128 * 128);
  int a, b;
  for (a = 0; a < 128; a++)
    for (b = 0; b < 128; b++) t[a * 128 + b] = Dynprog_pairdistance(a, b);
  spit(dir, "pdist_highq.i32", t, sizeof(int32_t) * 128 * 128);
  return 0;
}

/* Dynprog_setup with the splicing IIT, as gmap.c:3283-3302 / 3729-3731 set it up */
static int setup_splicing_iit(const char *iitfile, const char *div, int novelsplicingp) {
  static int crosstable[2];
  IIT_T iit = IIT_read((char *)iitfile, NULL, true, READ_ALL, NULL, false, false);
  int donor_typeint, acceptor_typeint;
  if (!iit) {
    fprintf(stderr, "cannot read %s\n", iitfile);
    exit(2);
  }
  crosstable[0] = -1;
  crosstable[1] = IIT_divint(iit, (char *)div);
  if ((donor_typeint = IIT_typeint(iit, "donor")) < 0 || (acceptor_typeint = IIT_typeint(iit, "acceptor")) < 0) {
    donor_typeint = acceptor_typeint = -1;  /* an introns file */
  }
  Dynprog_setup(novelsplicingp, iit, crosstable, donor_typeint, acceptor_typeint, NULL, NULL, NULL, 0,
                NULL, NULL, NULL, NULL, /*genome*/ NULL);
  return 0;
}

int main(int argc, char **argv) {
  int mode = 0; /* STANDARD */
  if (argc < 3) {
    fprintf(stderr, "usage: ref_driver dp|ggap|maxent|pdist <dir> [mode]\n");
    return 1;
  }
  if (argc > 3) mode = atoi(argv[3]);
  Dynprog_init(600, 10, 11, 10, 8, (Mode_T)mode);
  Dynprog_setup(/*novelsplicingp*/ false, NULL, NULL, -1, -1, NULL, NULL, NULL, 0, NULL, NULL,
                NULL, NULL, /*genome*/ NULL);
  if (!strcmp(argv[1], "dp")) return run_dp(argv[2]);
  if (!strcmp(argv[1], "ggap")) return run_ggap(argv[2]);
  if (!strcmp(argv[1], "ggapk") && argc > 6) {
    setup_splicing_iit(argv[4], argv[5], atoi(argv[6]));
    return run_ggap(argv[2]);
  }
  if (!strcmp(argv[1], "cgap")) return run_cgap(argv[2]);
  if (!strcmp(argv[1], "maxent")) return run_maxent(argv[2]);
  if (!strcmp(argv[1], "sj")) return run_sj(argv[2]);
  if (!strcmp(argv[1], "mksj")) return run_mksj(argv[2]);
  if (!strcmp(argv[1], "micro")) return run_micro(argv[2]);
  if (!strcmp(argv[1], "known")) return run_known(argv[2], argc > 4 ? atoi(argv[4]) : 0);
  if (!strcmp(argv[1], "pdist")) return run_pdist(argv[2]);
  return 1;
}
