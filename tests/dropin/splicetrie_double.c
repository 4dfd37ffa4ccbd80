/* Test double for the host program's Splicetrie_setup / Splicetrie_solve_end5 /
 * Splicetrie_solve_end3 (reference splicetrie.c:85, 881, 952), the code the
 * drop-in's Dynprog_end5/3_known calls back through (dynprog.c:6414, 6680).
 * Clean-room restatement of the contract, test infrastructure only: a real
 * gmap/gsnap link supplies its own splicetrie.o.
 *
 * Contract restated (splicetrie.c:307-880):
 *  - A trie node at triestart[0] is a single leaf (value < DUPLICATE_NODE,
 *    the value is a splice-site index), a run of -value leaves at
 *    triestart[1..] (value < INTERNAL_NODE), or an internal node whose four
 *    child offsets (A, C, G, T) sit at triestart[1..4], the child at
 *    triestart - offset, visited in A C G T order when the offset is > 0
 *    (splicetrie_build.h:19-27, no 2-byte offsets).
 *  - Each leaf whose coordinate lies in [limit_low, limit_high] builds the
 *    junction (Dynprog_make_splicejunction_5/3), aligns the end against it
 *    (Dynprog_end5/3_splicejunction, anchor offset = the window's
 *    (rev)offset2, far offset moved by the coordinate difference in the
 *    strand's direction) and scores miss = perfect - score.
 *  - score > 0 and miss < threshold - penalty: new best (out-parameters,
 *    knownsplicep, ambig_end_length = length1 - contlength, threshold = miss
 *    + penalty), the coordinate list restarts with this coordinate, and the
 *    node's shortest intron becomes this intron.
 *  - miss == threshold - penalty: without amb_closest the coordinate is
 *    appended (ambiguity); with amb_closest it becomes the new best unless
 *    its intron is longer than the shortest one seen at this trie node.  The
 *    "shortest" tracker is local to one node visit (it starts at the
 *    largest value for every node, as in the reference).
 *  - At the end, more than one distinct coordinate recorded -> NULL list
 *    (the out-parameters keep their values).
 */
#include <stdlib.h>

typedef unsigned int Genomicpos_T;
typedef unsigned char bool_t;
typedef void* List_T;
typedef void* Dynprog_T;
typedef void* Pairpool_T;
typedef int Splicetype_T;

#define NULL_POINTER 0xFFFFFFFFu
#define DUPLICATE_NODE 0xFFFFFC18u /* -1000U */
#define INTERNAL_NODE 0xFFFFFFFFu

/* provided by the drop-in (libgsnapdp_dropin.so) */
extern void Dynprog_make_splicejunction_5(char* splicejunction, Genomicpos_T splicecoord, int splicelength,
                                          int contlength, Splicetype_T far_splicetype, bool_t watsonp);
extern void Dynprog_make_splicejunction_3(char* splicejunction, Genomicpos_T splicecoord, int splicelength,
                                          int contlength, Splicetype_T far_splicetype, bool_t watsonp);
extern List_T Dynprog_end5_splicejunction(int* dynprogindex, int* finalscore, int* nmatches, int* nmismatches,
                                          int* nopens, int* nindels, Dynprog_T dynprog, char* revsequence1,
                                          char* revsequenceuc1, char* revsequence2, char* revsequenceuc2,
                                          int length1, int length2, int revoffset1, int revoffset2_anchor,
                                          int revoffset2_far, Genomicpos_T chroffset, Genomicpos_T chrhigh,
                                          Genomicpos_T chrpos, int genomiclength, int cdna_direction,
                                          bool_t watsonp, bool_t jump_late_p, Pairpool_T pairpool,
                                          int extraband_end, double defect_rate, int contlength);
extern List_T Dynprog_end3_splicejunction(int* dynprogindex, int* finalscore, int* nmatches, int* nmismatches,
                                          int* nopens, int* nindels, Dynprog_T dynprog, char* sequence1,
                                          char* sequenceuc1, char* sequence2, char* sequenceuc2, int length1,
                                          int length2, int offset1, int offset2_anchor, int offset2_far,
                                          Genomicpos_T chroffset, Genomicpos_T chrhigh, Genomicpos_T chrpos,
                                          int genomiclength, int cdna_direction, bool_t watsonp,
                                          bool_t jump_late_p, Pairpool_T pairpool, int extraband_end,
                                          double defect_rate, int contlength);

static Genomicpos_T* sites;
static int amb_closest;

void Splicetrie_setup(Genomicpos_T* splicesites_in, unsigned* frags_ref, unsigned* frags_alt,
                      unsigned* trieoffsets_obs, unsigned* triecontents_obs, unsigned* trieoffsets_max,
                      unsigned* triecontents_max, bool_t snpp, bool_t amb_closest_p, bool_t amb_clip_p,
                      int min_shortend) {
  (void)frags_ref, (void)frags_alt, (void)trieoffsets_obs, (void)triecontents_obs;
  (void)trieoffsets_max, (void)triecontents_max, (void)snpp, (void)amb_clip_p, (void)min_shortend;
  sites = splicesites_in;
  amb_closest = amb_closest_p ? 1 : 0;
}

/* everything one solve needs, shared by the recursive visit */
typedef struct {
  int end5;
  Genomicpos_T lo, hi, anchor;
  int *finalscore, *nmatches, *nmismatches, *nopens, *nindels, *ambig_end_length, *threshold;
  bool_t* knownsplicep;
  int penalty, perfect;
  char* junction;
  int splicelength, contlength;
  Splicetype_T far_type;
  Genomicpos_T chroffset, chrhigh, chrpos;
  int genomiclength;
  int* dynprogindex;
  Dynprog_T dynprog;
  char *seq, *sequc;
  int length1, length2, off1, off2;
  int cdna_direction;
  bool_t watsonp, jump_late_p;
  Pairpool_T pairpool;
  int extraband_end;
  double defect_rate;
  Genomicpos_T* coords; /* recorded coordinates */
  int ncoords;
  List_T best;
} Solve;

static Genomicpos_T span(Genomicpos_T a, Genomicpos_T b) { return a > b ? a - b : b - a; }

static void try_leaf(Solve* S, unsigned leaf, Genomicpos_T* shortest) {
  const Genomicpos_T coord = sites[leaf];
  int score, nm, nmm, no, ni, far;
  List_T pairs;
  if (coord < S->lo || coord > S->hi) return;
  /* the far part's genome offset moves with the coordinate, against the strand on minus */
  far = S->watsonp ? (int)(S->off2 - S->anchor + coord) : (int)(S->off2 + S->anchor - coord);
  if (S->end5) {
    Dynprog_make_splicejunction_5(S->junction, coord, S->splicelength, S->contlength, S->far_type, S->watsonp);
    pairs = Dynprog_end5_splicejunction(S->dynprogindex, &score, &nm, &nmm, &no, &ni, S->dynprog, S->seq,
                                        S->sequc, &S->junction[S->length2 - 1], &S->junction[S->length2 - 1],
                                        S->length1, S->length2, S->off1, S->off2, far, S->chroffset,
                                        S->chrhigh, S->chrpos, S->genomiclength, S->cdna_direction, S->watsonp,
                                        S->jump_late_p, S->pairpool, S->extraband_end, S->defect_rate,
                                        S->contlength);
  } else {
    Dynprog_make_splicejunction_3(S->junction, coord, S->splicelength, S->contlength, S->far_type, S->watsonp);
    pairs = Dynprog_end3_splicejunction(S->dynprogindex, &score, &nm, &nmm, &no, &ni, S->dynprog, S->seq,
                                        S->sequc, S->junction, S->junction, S->length1, S->length2, S->off1,
                                        S->off2, far, S->chroffset, S->chrhigh, S->chrpos, S->genomiclength,
                                        S->cdna_direction, S->watsonp, S->jump_late_p, S->pairpool,
                                        S->extraband_end, S->defect_rate, S->contlength);
  }
  const int miss = S->perfect - score;
  const int bar = *S->threshold - S->penalty;
  int take = 0;
  if (score > 0 && miss < bar) {
    take = 1;
  } else if (miss == bar) {
    if (!amb_closest) S->coords[S->ncoords++] = coord; /* ambiguity */
    else if (span(coord, S->anchor) <= *shortest) take = 1;
  }
  if (take) {
    S->best = pairs;
    *S->finalscore = score;
    *S->nmatches = nm;
    *S->nmismatches = nmm;
    *S->nopens = no;
    *S->nindels = ni;
    *S->knownsplicep = 1;
    *S->ambig_end_length = S->length1 - S->contlength;
    *S->threshold = miss + S->penalty;
    *shortest = span(coord, S->anchor);
    S->ncoords = 0;
    S->coords[S->ncoords++] = coord;
  }
}

static void visit(Solve* S, const unsigned* node) {
  Genomicpos_T shortest = 0xFFFFFFFFu; /* per node visit */
  const unsigned v = node[0];
  if (v < DUPLICATE_NODE) {
    try_leaf(S, v, &shortest);
  } else if (v < INTERNAL_NODE) {
    const int n = -(int)v;
    for (int i = 1; i <= n; i++) try_leaf(S, node[i], &shortest);
  } else {
    for (int b = 1; b <= 4; b++)
      if ((int)node[b] > 0) visit(S, node - (int)node[b]);
  }
}

static int leaves(const unsigned* node) {
  const unsigned v = node[0];
  if (v < DUPLICATE_NODE) return 1;
  if (v < INTERNAL_NODE) return -(int)v;
  int n = 0;
  for (int b = 1; b <= 4; b++)
    if ((int)node[b] > 0) n += leaves(node - (int)node[b]);
  return n;
}

static List_T solve(int end5, List_T best_pairs, unsigned* triecontents, unsigned* trieoffsets, int j,
                    Genomicpos_T lo, Genomicpos_T hi, int* finalscore, int* nmatches, int* nmismatches,
                    int* nopens, int* nindels, bool_t* knownsplicep, int* ambig_end_length, int* threshold,
                    int penalty, int perfect, Genomicpos_T anchor, char* junction, int splicelength,
                    int contlength, Splicetype_T far_type, Genomicpos_T chroffset, Genomicpos_T chrhigh,
                    Genomicpos_T chrpos, int genomiclength, int* dynprogindex, Dynprog_T dynprog, char* seq,
                    char* sequc, int length1, int length2, int off1, int off2, int cdna_direction,
                    bool_t watsonp, bool_t jump_late_p, Pairpool_T pairpool, int extraband_end,
                    double defect_rate) {
  if (trieoffsets[j] == NULL_POINTER) return best_pairs;
  const unsigned* root = &triecontents[trieoffsets[j]];
  const int size = leaves(root);
  if (size == 0) return best_pairs;
  Solve S = {end5, lo, hi, anchor, finalscore, nmatches, nmismatches, nopens, nindels, ambig_end_length,
             threshold, knownsplicep, penalty, perfect, junction, splicelength, contlength, far_type,
             chroffset, chrhigh, chrpos, genomiclength, dynprogindex, dynprog, seq, sequc, length1, length2,
             off1, off2, cdna_direction, watsonp, jump_late_p, pairpool, extraband_end, defect_rate,
             (Genomicpos_T*)calloc((size_t)size, sizeof(Genomicpos_T)), 0, best_pairs};
  visit(&S, root);
  for (int i = 1; i < S.ncoords; i++)
    if (S.coords[i] != S.coords[0]) {
      S.best = NULL; /* more than one coordinate: ambiguous */
      break;
    }
  free(S.coords);
  return S.best;
}

List_T Splicetrie_solve_end5(List_T best_pairs, unsigned* triecontents, unsigned* trieoffsets, int j,
                             Genomicpos_T lo, Genomicpos_T hi, int* finalscore, int* nmatches, int* nmismatches,
                             int* nopens, int* nindels, bool_t* knownsplicep, int* ambig_end_length,
                             int* threshold_miss_score, int obsmax_penalty, int perfect_score,
                             Genomicpos_T anchor_splicesite, char* splicejunction, int splicelength,
                             int contlength, Splicetype_T far_splicetype, Genomicpos_T chroffset,
                             Genomicpos_T chrhigh, Genomicpos_T chrpos, int genomiclength, int* dynprogindex,
                             Dynprog_T dynprog, char* revsequence1, char* revsequenceuc1, int length1,
                             int length2, int revoffset1, int revoffset2, int cdna_direction, bool_t watsonp,
                             bool_t jump_late_p, Pairpool_T pairpool, int extraband_end, double defect_rate) {
  return solve(1, best_pairs, triecontents, trieoffsets, j, lo, hi, finalscore, nmatches, nmismatches, nopens,
               nindels, knownsplicep, ambig_end_length, threshold_miss_score, obsmax_penalty, perfect_score,
               anchor_splicesite, splicejunction, splicelength, contlength, far_splicetype, chroffset, chrhigh,
               chrpos, genomiclength, dynprogindex, dynprog, revsequence1, revsequenceuc1, length1, length2,
               revoffset1, revoffset2, cdna_direction, watsonp, jump_late_p, pairpool, extraband_end,
               defect_rate);
}

List_T Splicetrie_solve_end3(List_T best_pairs, unsigned* triecontents, unsigned* trieoffsets, int j,
                             Genomicpos_T lo, Genomicpos_T hi, int* finalscore, int* nmatches, int* nmismatches,
                             int* nopens, int* nindels, bool_t* knownsplicep, int* ambig_end_length,
                             int* threshold_miss_score, int obsmax_penalty, int perfect_score,
                             Genomicpos_T anchor_splicesite, char* splicejunction, int splicelength,
                             int contlength, Splicetype_T far_splicetype, Genomicpos_T chroffset,
                             Genomicpos_T chrhigh, Genomicpos_T chrpos, int genomiclength, int* dynprogindex,
                             Dynprog_T dynprog, char* sequence1, char* sequenceuc1, int length1, int length2,
                             int offset1, int offset2, int cdna_direction, bool_t watsonp, bool_t jump_late_p,
                             Pairpool_T pairpool, int extraband_end, double defect_rate) {
  return solve(0, best_pairs, triecontents, trieoffsets, j, lo, hi, finalscore, nmatches, nmismatches, nopens,
               nindels, knownsplicep, ambig_end_length, threshold_miss_score, obsmax_penalty, perfect_score,
               anchor_splicesite, splicejunction, splicelength, contlength, far_splicetype, chroffset, chrhigh,
               chrpos, genomiclength, dynprogindex, dynprog, sequence1, sequenceuc1, length1, length2, offset1,
               offset2, cdna_direction, watsonp, jump_late_p, pairpool, extraband_end, defect_rate);
}
