/*
 * stage3_si.c -- TEST INFRASTRUCTURE ONLY (oracle/_ref/gmap_trace; dev container only).
 *
 * The reference's own stage3.c, compiled where it lies (-I$(REF); nothing is
 * copied), plus one accessor: the address of its static score_introns
 * (stage3.c:7935-8162), so that gmap_trace.c can record every call's path and
 * outputs (golden vectors for gsnapdp_score_introns_*).  Built in place of
 * stage3.o with IPA cloning off, so that both call sites (stage3.c:9892, 9935)
 * call that one function.
 */
#include "stage3.c"

void *gmap_trace_score_introns_fn(void) { return (void *)&score_introns; }
