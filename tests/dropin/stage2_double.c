/*
 * stage2_double.c -- TEST INFRASTRUCTURE ONLY (never shipped).
 *
 * A stage-2 callback for gsnapdp_stage3_set_stage2 served from a recording:
 * every Stage2_compute_one call traverse_dual_break made in the reference's
 * gmap (oracle/gmap_trace.c, golden arrays s2_calls / s2_pairs).  A request is
 * answered with the recorded list of the call with the same path_compute
 * invocation, query stretch and mapping bounds; a request the recording does
 * not hold fails (-1), so a pass that asks for a different stretch than the
 * reference did fails its path instead of passing silently.  Thread-safe
 * (read-only after s2dbl_new).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/gsnapdp.h"

typedef struct { /* records.S2_CALL */
  int32_t invocation, query_offset, querylength, genomiclength;
  uint32_t genomicstart, genomicend, mappingstart, mappingend;
  int32_t plusp, first_pair, npairs, pad;
} S2Rec;

typedef struct {
  S2Rec *calls;
  int ncalls;
  gsnapdp_s3_pair *pairs;
  int npairs;
  int served, missed; /* counters (racy increments are fine for a test) */
} S2Dbl;

void *s2dbl_new(const void *calls, int ncalls, const gsnapdp_s3_pair *pairs, int npairs) {
  S2Dbl *d = (S2Dbl *)calloc(1, sizeof(S2Dbl));
  d->calls = (S2Rec *)malloc(sizeof(S2Rec) * (size_t)(ncalls > 0 ? ncalls : 1));
  d->pairs = (gsnapdp_s3_pair *)malloc(sizeof(gsnapdp_s3_pair) * (size_t)(npairs > 0 ? npairs : 1));
  if (ncalls > 0) memcpy(d->calls, calls, sizeof(S2Rec) * (size_t)ncalls);
  if (npairs > 0) memcpy(d->pairs, pairs, sizeof(gsnapdp_s3_pair) * (size_t)npairs);
  d->ncalls = ncalls;
  d->npairs = npairs;
  return d;
}

void s2dbl_free(void *u) {
  S2Dbl *d = (S2Dbl *)u;
  if (!d) return;
  free(d->calls);
  free(d->pairs);
  free(d);
}

int s2dbl_counts(void *u, int *served, int *missed) {
  S2Dbl *d = (S2Dbl *)u;
  *served = d->served;
  *missed = d->missed;
  return 0;
}

int s2dbl_compute_one(void *u, const gsnapdp_s3_call *call, int querydp5, int querydp3, int genomedp5,
                      int genomedp3, uint32_t mappingstart, uint32_t mappingend, gsnapdp_s3_pair *out, int cap) {
  S2Dbl *d = (S2Dbl *)u;
  int i, j;
  (void)genomedp5;
  (void)genomedp3;
  for (i = 0; i < d->ncalls; i++) {
    const S2Rec *r = &d->calls[i];
    if (r->invocation == call->invocation && r->query_offset == querydp5 &&
        r->querylength == querydp3 - querydp5 + 1 && r->mappingstart == mappingstart &&
        r->mappingend == mappingend) {
      if (r->npairs <= cap)
        for (j = 0; j < r->npairs; j++) out[j] = d->pairs[r->first_pair + j];
      d->served++;
      return r->npairs;
    }
  }
  d->missed++;
  return -1;
}
