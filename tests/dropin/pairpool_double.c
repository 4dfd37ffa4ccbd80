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
