/*
 * stage3_si.c -- TEST INFRASTRUCTURE ONLY (oracle/_ref/gmap_trace; dev container only).
 *
 * The reference's own stage3.c, compiled where it lies (-I$(REF); nothing is
 * copied), plus accessors: the addresses of its static score_introns
 * (stage3.c:7935-8162), build_pairs_introns (:7735-7901), build_pairs_singles
 * (:7454-7583), build_pairs_end5 (:7351), build_path_end3 (:7236) and
 * build_pairs_dualintrons (:7592), build_dual_breaks (:7149) and path_compute
 * (:8586), so that
 * gmap_trace.c can record every call's inputs and outputs (golden vectors for
 * gsnapdp_score_introns_* and gsnapdp_stage3_pass), and the two module flags
 * Stage3_setup sets (:238-239).  Built in place of stage3.o with IPA cloning
 * off, so that each function's call sites call that one function.
 */
#include "stage3.c"

void *gmap_trace_score_introns_fn(void) { return (void *)&score_introns; }
void *gmap_trace_build_pairs_introns_fn(void) { return (void *)&build_pairs_introns; }
void *gmap_trace_build_pairs_singles_fn(void) { return (void *)&build_pairs_singles; }
void *gmap_trace_build_pairs_end5_fn(void) { return (void *)&build_pairs_end5; }
void *gmap_trace_build_path_end3_fn(void) { return (void *)&build_path_end3; }
void *gmap_trace_build_pairs_dualintrons_fn(void) { return (void *)&build_pairs_dualintrons; }
void *gmap_trace_build_dual_breaks_fn(void) { return (void *)&build_dual_breaks; }
void *gmap_trace_path_compute_fn(void) { return (void *)&path_compute; }
int gmap_trace_splicesitesp(void) { return splicesites != NULL ? 1 : 0; }
int gmap_trace_novelsplicingp(void) { return novelsplicingp ? 1 : 0; }
int gmap_trace_splicingp(void) { return splicingp ? 1 : 0; }
