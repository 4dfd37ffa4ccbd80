/* TEST INFRASTRUCTURE ONLY (linked into oracle/_ref/gmap_cpu and gmap_gpu).
 *
 * The index-reading genome_hr functions (genome_hr.h:23-30: gamma-coded offset
 * pointers of a gmapindex database).  genome_hr.c is a missing blob in the
 * reference and these are not on the DP path: `gmap -g` (a user genomic
 * segment, as in align.test) never calls them, but indexdb.c takes their
 * addresses, so a dynamically linked gmap needs the symbols to exist.
 */
#include <stdio.h>
#include <stdlib.h>

static void out_of_scope(const char *name) {
  fprintf(stderr, "%s: gmapindex databases are out of scope for this build (use -g)\n", name);
  abort();
}

void Genome_read_gamma(void) { out_of_scope("Genome_read_gamma"); }
void Genome_offsetptr_from_gammas(void) { out_of_scope("Genome_offsetptr_from_gammas"); }
void Genome_offsetptr_only_from_gammas(void) { out_of_scope("Genome_offsetptr_only_from_gammas"); }
