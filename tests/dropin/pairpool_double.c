/* Test double for the host program's Pairpool_push / Pairpool_push_gapholder
 * (reference pairpool.c:169, 352), Pairpool_pop (pairpool.c) and Pair_protect
 * (pair.c).  Cells use the reference's own List_T / Pair_T layouts (listdef.h,
 * pairdef.h:9-49), as the real host program's would, so the drop-in sees the
 * same memory it sees in a gmap/gsnap link; dbl_list_read flattens a list into
 * gsnapdp_pair records for the tests.  Test infrastructure only; the real host
 * links pairpool.o / pair.o. */
#include <execinfo.h>
#include <signal.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#include <unistd.h>

/* a crash inside the shim or the host-side code prints its C frames */
static void on_segv(int sig) {
  void* frames[64];
  int n = backtrace(frames, 64);
  backtrace_symbols_fd(frames, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}
__attribute__((constructor)) static void install_segv_handler(void) {
  if (getenv("DBL_BACKTRACE")) signal(SIGSEGV, on_segv);
}

typedef struct PairRec { /* pairdef.h:9-49, field for field */
  int querypos;
  unsigned int genomepos;
  int refquerypos;
  int aapos;
  int queryjump;
  int genomejump;
  int aaphase_g;
  int aaphase_e;
  int dynprogindex;
  char cdna, comp, genome, aa_g, aa_e;
  unsigned char gapp, knowngapp, extraexonp, shortexonp;
  int state, vstate_good, vstate_bad;
  unsigned char protectedp, disallowedp;
  double donor_prob, acceptor_prob;
  unsigned char end_intron_p;
} PairRec;

typedef struct Rec { /* gsnapdp_pair */
  int querypos, genomepos, queryjump, genomejump, dynprogindex;
  char cdna, comp, genome;
  unsigned char gapp;
} Rec;

typedef struct List_T { /* listdef.h */
  void* first;
  struct List_T* rest;
} * List_T;

typedef struct Pairpool_T {
  int dummy;
} * Pairpool_T;

static List_T cons(List_T list, PairRec* r) {
  List_T n = (List_T)malloc(sizeof(*n));
  n->first = r;
  n->rest = list;
  return n;
}

List_T Pairpool_push(List_T list, Pairpool_T pool, int querypos, int genomepos, char cdna, char comp,
                     char genome, int dynprogindex) {
  (void)pool;
  PairRec* r = (PairRec*)calloc(1, sizeof(PairRec));
  r->querypos = querypos;
  r->genomepos = (unsigned int)genomepos;
  r->dynprogindex = dynprogindex;
  r->cdna = cdna;
  r->comp = comp;
  r->genome = genome;
  return cons(list, r);
}

List_T Pairpool_push_gapholder(List_T list, Pairpool_T pool, int queryjump, int genomejump,
                               unsigned char knownp) {
  (void)pool;
  PairRec* r = (PairRec*)calloc(1, sizeof(PairRec));
  r->querypos = -1;
  r->genomepos = (unsigned int)-1;
  r->queryjump = queryjump;
  r->genomejump = genomejump;
  r->cdna = ' ';
  r->comp = ' ';
  r->genome = ' ';
  r->gapp = 1;
  r->knowngapp = knownp ? 1 : 0;
  r->donor_prob = r->acceptor_prob = knownp ? 2.0 : 0.0;
  return cons(list, r);
}

/* pairpool.c Pairpool_pop: the head cell's pair and the rest of the list */
List_T Pairpool_pop(List_T list, PairRec** x) {
  List_T rest;
  if (!list) return NULL;
  *x = (PairRec*)list->first;
  rest = list->rest;
  free(list); /* the pair itself stays (pool memory in the reference) */
  return rest;
}

/* list.c List_reverse */
List_T List_reverse(List_T list) {
  List_T head = NULL, next;
  for (; list; list = next) {
    next = list->rest;
    list->rest = head;
    head = list;
  }
  return head;
}

/* pair.c Pair_protect: mark every pair protected, return the list */
List_T Pair_protect(List_T list) {
  List_T p;
  for (p = list; p; p = p->rest) ((PairRec*)p->first)->protectedp = 1;
  return list;
}

/* Copy the list (head first) into out[cap] as gsnapdp_pair records (gapp bit 1
 * = knowngapp); returns its length. */
int dbl_list_read(List_T list, Rec* out, int cap) {
  int n = 0;
  for (; list; list = list->rest, n++) {
    const PairRec* p = (const PairRec*)list->first;
    if (n < cap) {
      Rec* o = &out[n];
      memset(o, 0, sizeof(*o));
      o->querypos = p->querypos;
      o->genomepos = (int)p->genomepos;
      o->queryjump = p->gapp ? p->queryjump : 0;
      o->genomejump = p->gapp ? p->genomejump : 0;
      o->dynprogindex = p->dynprogindex;
      o->cdna = p->cdna;
      o->comp = p->comp;
      o->genome = p->genome;
      o->gapp = (unsigned char)((p->gapp ? 1 : 0) | (p->knowngapp ? 2 : 0));
    }
  }
  return n;
}

/* 1 if every pair of the list is protected (Pair_protect) */
int dbl_list_protected(List_T list) {
  for (; list; list = list->rest)
    if (!((PairRec*)list->first)->protectedp) return 0;
  return 1;
}

void dbl_list_free(List_T list) {
  while (list) {
    List_T next = list->rest;
    free(list->first);
    free(list);
    list = next;
  }
}

/* A path for score_introns tests: records (the golden's SiPair layout:
 * querypos, genomepos, queryjump, genomejump, gapp, knowngapp, comp, pad) ->
 * a list whose head is recs[0]. */
typedef struct PathRec {
  int querypos;
  unsigned int genomepos;
  int queryjump, genomejump;
  unsigned char gapp, knowngapp, comp, pad;
} PathRec;
List_T dbl_list_build(const PathRec* recs, int n) {
  List_T list = NULL;
  int i;
  for (i = n - 1; i >= 0; i--) {
    PairRec* r = (PairRec*)calloc(1, sizeof(PairRec));
    r->querypos = recs[i].querypos;
    r->genomepos = recs[i].genomepos;
    r->queryjump = recs[i].queryjump;
    r->genomejump = recs[i].genomejump;
    r->gapp = recs[i].gapp;
    r->knowngapp = recs[i].knowngapp;
    r->comp = (char)recs[i].comp;
    list = cons(list, r);
  }
  return list;
}

/* A stage-3 path (gsnapdp_s3_pair records, list order) -> a list whose head is
 * recs[0]; refquerypos carries index + 1 so that dbl_s3_read can name the input
 * pair a returned cell holds (0 for a pair the callee pushed). */
typedef struct S3Rec {
  int querypos, genomepos, queryjump, genomejump, dynprogindex, src;
  char cdna, comp, genome;
  unsigned char flags; /* 1 gapp, 2 knowngapp, 4 disallowedp, 8 shortexonp, 16 end_intron_p */
} S3Rec;
List_T dbl_s3_build(const S3Rec* recs, int n) {
  List_T list = NULL;
  int i;
  for (i = n - 1; i >= 0; i--) {
    PairRec* r = (PairRec*)calloc(1, sizeof(PairRec));
    r->querypos = recs[i].querypos;
    r->genomepos = (unsigned int)recs[i].genomepos;
    r->refquerypos = i + 1;
    r->queryjump = recs[i].queryjump;
    r->genomejump = recs[i].genomejump;
    r->dynprogindex = recs[i].dynprogindex;
    r->cdna = recs[i].cdna;
    r->comp = recs[i].comp;
    r->genome = recs[i].genome;
    r->gapp = recs[i].flags & 1;
    r->knowngapp = (recs[i].flags >> 1) & 1;
    r->disallowedp = (recs[i].flags >> 2) & 1;
    r->shortexonp = (recs[i].flags >> 3) & 1;
    r->end_intron_p = (recs[i].flags >> 4) & 1;
    list = cons(list, r);
  }
  return list;
}
int dbl_s3_read(List_T list, S3Rec* out, int cap) {
  int n = 0;
  for (; list; list = list->rest, n++) {
    const PairRec* p = (const PairRec*)list->first;
    if (n < cap) {
      S3Rec* o = &out[n];
      memset(o, 0, sizeof(*o));
      o->querypos = p->querypos;
      o->genomepos = (int)p->genomepos;
      o->queryjump = p->queryjump;
      o->genomejump = p->genomejump;
      o->dynprogindex = p->dynprogindex;
      o->src = p->refquerypos - 1;
      o->cdna = p->cdna;
      o->comp = p->comp;
      o->genome = p->genome;
      o->flags = (unsigned char)((p->gapp ? 1 : 0) | (p->knowngapp ? 2 : 0) | (p->disallowedp ? 4 : 0) |
                                 (p->shortexonp ? 8 : 0) | (p->end_intron_p ? 16 : 0));
    }
  }
  return n;
}

/* Stage2_compute_one (stage2.c:4260) for the drop-in's traverse_dual_break:
 * answers from the stage-2 calls gmap_trace recorded (records.S2_CALL and their
 * lists in S3Rec), matched on the query stretch and the mapping bounds, with a
 * fresh list of fresh PairRec cells (refquerypos 0: pairs the callee made).
 * A request the recording does not hold aborts. */
typedef struct S2Rec {
  int invocation, query_offset, querylength, genomiclength;
  unsigned int genomicstart, genomicend, mappingstart, mappingend;
  int plusp, first_pair, npairs, pad;
} S2Rec;
static const S2Rec* s2_calls;
static const S3Rec* s2_pairs;
static int s2_ncalls, s2_served;
void dbl_stage2_load(const S2Rec* calls, int ncalls, const S3Rec* pairs) {
  s2_calls = calls;
  s2_ncalls = ncalls;
  s2_pairs = pairs;
  s2_served = 0;
}
int dbl_stage2_served(void) { return s2_served; }
List_T Stage2_compute_one(int* stage2_source, int* stage2_indexsize, char* queryseq_ptr, char* queryuc_ptr,
                          int querylength, int query_offset, char* genomicseg_ptr, char* genomicuc_ptr,
                          unsigned int genomicstart, unsigned int genomicend, unsigned int mappingstart,
                          unsigned int mappingend, unsigned char plusp, int genestrand, int genomiclength,
                          void* oligoindices, int noligoindices, double proceed_pctcoverage, void* pairpool,
                          void* diagpool, int sufflookback, int nsufflookback, int maxintronlen, unsigned char localp,
                          unsigned char skip_repetitive_p, unsigned char use_shifted_canonical_p,
                          unsigned char favor_right_p, unsigned char debug_graphic_p, unsigned char diagnosticp,
                          void* stopwatch, unsigned char diag_debug) {
  int i, j;
  (void)stage2_source, (void)stage2_indexsize, (void)queryseq_ptr, (void)queryuc_ptr, (void)genomicseg_ptr;
  (void)genomicuc_ptr, (void)plusp, (void)genestrand, (void)oligoindices, (void)noligoindices;
  (void)proceed_pctcoverage, (void)pairpool, (void)diagpool, (void)sufflookback, (void)nsufflookback;
  (void)maxintronlen, (void)localp, (void)skip_repetitive_p, (void)use_shifted_canonical_p, (void)favor_right_p;
  (void)debug_graphic_p, (void)diagnosticp, (void)stopwatch, (void)diag_debug;
  for (i = 0; i < s2_ncalls; i++) {
    const S2Rec* r = &s2_calls[i];
    if (r->query_offset == query_offset && r->querylength == querylength && r->genomicstart == genomicstart &&
        r->genomicend == genomicend && r->mappingstart == mappingstart && r->mappingend == mappingend &&
        r->genomiclength == genomiclength) {
      List_T list = NULL;
      for (j = r->npairs - 1; j >= 0; j--) {
        const S3Rec* x = &s2_pairs[r->first_pair + j];
        PairRec* p = (PairRec*)calloc(1, sizeof(PairRec));
        p->querypos = x->querypos;
        p->genomepos = (unsigned int)x->genomepos;
        p->queryjump = x->queryjump;
        p->genomejump = x->genomejump;
        p->dynprogindex = x->dynprogindex;
        p->cdna = x->cdna;
        p->comp = x->comp;
        p->genome = x->genome;
        p->gapp = x->flags & 1;
        p->knowngapp = (x->flags >> 1) & 1;
        p->disallowedp = (x->flags >> 2) & 1;
        p->shortexonp = (x->flags >> 3) & 1;
        p->end_intron_p = (x->flags >> 4) & 1;
        list = cons(list, p);
      }
      s2_served++;
      return list;
    }
  }
  fprintf(stderr, "Stage2_compute_one double: no recorded call for query %d+%d, mapping %u..%u\n", query_offset,
          querylength, mappingstart, mappingend);
  abort();
}
