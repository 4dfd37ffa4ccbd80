/* TEST INFRASTRUCTURE ONLY (linked into oracle/_ref/gsnap_gpu, never shipped).
 *
 * GSNAP's genome_hr mismatch / splice-site-scan functions (genome_hr.h:44-104).  Their
 * definitions are in genome_hr.c, a missing blob in the reference, so no reference
 * algorithm exists here to restate or pin.  gsnap's objects
 * call them from stage1hr.c / substring.c / stage3hr.c, which run only on a gmapindex
 * database (out of scope), so the link test gets aborting stand-ins: the program links
 * with zero unresolved symbols, every Dynprog_* / Maxent_hr_* symbol comes from
 * libgsnapdp_dropin.so, and it starts (--version).
 */
#include <stdio.h>
#include <stdlib.h>

static void missing_blob(const char *name) {
  fprintf(stderr, "%s: defined in the reference's missing genome_hr.c blob; not built (DESIGN.md 7)\n", name);
  abort();
}

#define STUB(name) void name(void) { missing_blob(#name); }
STUB(Genome_count_mismatches_substring)
STUB(Genome_count_mismatches_substring_ref)
STUB(Genome_count_mismatches_limit)
STUB(Genome_count_mismatches_fragment)
STUB(Genome_query_shift_fragment_left)
STUB(Genome_query_shift_fragment_right)
STUB(Genome_mismatches_left)
STUB(Genome_mismatches_right)
STUB(Genome_mark_mismatches)
STUB(Genome_mark_mismatches_ref)
STUB(Genome_donor_positions)
STUB(Genome_acceptor_positions)
STUB(Genome_antidonor_positions)
STUB(Genome_antiacceptor_positions)
