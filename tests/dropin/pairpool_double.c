/* Test double for the host program's Pairpool_push / Pairpool_push_gapholder
 * (reference pairpool.c:169, 352): a list of records in the field order of
 * gsnapdp_pair, so tests can compare the drop-in's List_T with the golden
 * pair lists.  Test infrastructure only; the real host links pairpool.o. */
#include <stdlib.h>
#include <string.h>

typedef struct Rec {
  int querypos, genomepos, queryjump, genomejump, dynprogindex;
  char cdna, comp, genome;
  unsigned char gapp;
} Rec;

typedef struct List_T {
  Rec* first;
  struct List_T* rest;
} * List_T;

typedef struct Pairpool_T {
  int dummy;
} * Pairpool_T;

static List_T cons(List_T list, Rec* r) {
  List_T n = (List_T)malloc(sizeof(*n));
  n->first = r;
  n->rest = list;
  return n;
}

List_T Pairpool_push(List_T list, Pairpool_T pool, int querypos, int genomepos, char cdna, char comp,
                     char genome, int dynprogindex) {
  (void)pool;
  Rec* r = (Rec*)calloc(1, sizeof(Rec));
  r->querypos = querypos;
  r->genomepos = genomepos;
  r->dynprogindex = dynprogindex;
  r->cdna = cdna;
  r->comp = comp;
  r->genome = genome;
  return cons(list, r);
}

List_T Pairpool_push_gapholder(List_T list, Pairpool_T pool, int queryjump, int genomejump,
                               unsigned char knownp) {
  (void)pool;
  Rec* r = (Rec*)calloc(1, sizeof(Rec));
  r->querypos = -1;
  r->genomepos = -1;
  r->queryjump = queryjump;
  r->genomejump = genomejump;
  r->cdna = ' ';
  r->comp = ' ';
  r->genome = ' ';
  r->gapp = knownp ? 3 : 1; /* gapp | knowngapp << 1, as gsnapdp_pair */
  return cons(list, r);
}

/* Copy the list (head first) into out[cap]; returns its length. */
int dbl_list_read(List_T list, Rec* out, int cap) {
  int n = 0;
  for (; list; list = list->rest, n++)
    if (n < cap) out[n] = *list->first;
  return n;
}

void dbl_list_free(List_T list) {
  while (list) {
    List_T next = list->rest;
    free(list->first);
    free(list);
    list = next;
  }
}
