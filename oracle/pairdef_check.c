/*
 * pairdef_check.c -- TEST INFRASTRUCTURE ONLY (dev container: compiled by
 * `make -C oracle ref` / `asan` against the reference's headers, never shipped).
 *
 * The drop-in reads and writes the host program's Pair_T and List_T cells in
 * place (Gsnapdp_build_pairs_introns, Gsnapdp_score_introns, the microexon
 * gapholder comp).  Its mirror structs are static-asserted against
 * gmap-gsnap_amd/csrc/gsnapdp_pairlayout.h; this file asserts the same constants
 * against the reference's own pairdef.h (:9-49) and listdef.h, so the two
 * cannot drift apart silently.  It only has to compile.
 */
#include <stddef.h>

#include "bool.h"
#include "genomicpos.h"
#include "listdef.h"
#include "pairdef.h"

#include "../gmap-gsnap_amd/csrc/gsnapdp_pairlayout.h"

#define AT(f, k) _Static_assert(offsetof(struct Pair_T, f) == GSNAPDP_PAIR_OFF_##k, "Pair_T." #f)
AT(querypos, QUERYPOS);
AT(genomepos, GENOMEPOS);
AT(queryjump, QUERYJUMP);
AT(genomejump, GENOMEJUMP);
AT(dynprogindex, DYNPROGINDEX);
AT(cdna, CDNA);
AT(comp, COMP);
AT(genome, GENOME);
AT(gapp, GAPP);
AT(knowngapp, KNOWNGAPP);
AT(disallowedp, DISALLOWEDP);
AT(donor_prob, DONOR_PROB);
AT(shortexonp, SHORTEXONP);
AT(end_intron_p, END_INTRON_P);
_Static_assert(sizeof(struct Pair_T) == GSNAPDP_PAIR_SIZE, "sizeof(Pair_T)");
_Static_assert(sizeof(bool) == 1, "bool");
_Static_assert(offsetof(struct List_T, first) == GSNAPDP_LIST_OFF_FIRST, "List_T.first");
_Static_assert(offsetof(struct List_T, rest) == GSNAPDP_LIST_OFF_REST, "List_T.rest");
_Static_assert(sizeof(struct List_T) == GSNAPDP_LIST_SIZE, "sizeof(List_T)");

int gsnapdp_pairdef_check_compiled = 1;
