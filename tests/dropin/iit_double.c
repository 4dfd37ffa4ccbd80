/* TEST DOUBLE (tests/test_dropin.py): the four splicing-IIT queries
 * bridge_intron_gap makes (iit-read.c:3770 IIT_low_exists_signed_p, :3808
 * IIT_high_exists_signed_p, :3973 IIT_exists_with_divno_signed, :4011
 * IIT_exists_with_divno_typed_signed), answered by a linear scan over one
 * division's intervals.  Same existence semantics: an interval whose low
 * (high) end, both ends, type and sign equal the query.  The interval list
 * is the `intervals` array of the ggap_known_* golden sets, which the
 * reference's own iit_store turned into the IIT its goldens were made with.
 * The shim finds these symbols in the process, as it finds gmap's iit-read.o. */
#include <stdlib.h>

typedef struct {
  int n;
  unsigned *low, *high;
  int *type, *sign;
} iitdbl;

/* start/end as iit_store reads them (start > end: minus sign, interval.c:22-40) */
void *iitdbl_new(int n, const long long *start, const long long *end, const int *type) {
  iitdbl *t = (iitdbl *)calloc(1, sizeof(iitdbl));
  int i;
  t->n = n;
  t->low = (unsigned *)malloc(sizeof(unsigned) * (size_t)(n + 1));
  t->high = (unsigned *)malloc(sizeof(unsigned) * (size_t)(n + 1));
  t->type = (int *)malloc(sizeof(int) * (size_t)(n + 1));
  t->sign = (int *)malloc(sizeof(int) * (size_t)(n + 1));
  for (i = 0; i < n; i++) {
    unsigned a = (unsigned)start[i], b = (unsigned)end[i];
    t->low[i] = a < b ? a : b;
    t->high[i] = a < b ? b : a;
    t->sign[i] = a < b ? 1 : (a > b ? -1 : 0);
    t->type[i] = type[i];
  }
  return t;
}

void iitdbl_free(void *p) {
  iitdbl *t = (iitdbl *)p;
  free(t->low);
  free(t->high);
  free(t->type);
  free(t->sign);
  free(t);
}

unsigned char IIT_low_exists_signed_p(void *p, int divno, unsigned x, int sign) {
  iitdbl *t = (iitdbl *)p;
  int i;
  if (divno < 0) return 0;
  for (i = 0; i < t->n; i++)
    if (t->low[i] == x && t->sign[i] == sign) return 1;
  return 0;
}

unsigned char IIT_high_exists_signed_p(void *p, int divno, unsigned x, int sign) {
  iitdbl *t = (iitdbl *)p;
  int i;
  if (divno < 0) return 0;
  for (i = 0; i < t->n; i++)
    if (t->high[i] == x && t->sign[i] == sign) return 1;
  return 0;
}

unsigned char IIT_exists_with_divno_signed(void *p, int divno, unsigned x, unsigned y, int sign) {
  iitdbl *t = (iitdbl *)p;
  int i;
  if (divno < 0) return 0;
  for (i = 0; i < t->n; i++)
    if (t->low[i] == x && t->high[i] == y && t->sign[i] == sign) return 1;
  return 0;
}

unsigned char IIT_exists_with_divno_typed_signed(void *p, int divno, unsigned x, unsigned y, int type,
                                                 int sign) {
  iitdbl *t = (iitdbl *)p;
  int i;
  if (divno < 0) return 0;
  for (i = 0; i < t->n; i++)
    if (t->low[i] == x && t->high[i] == y && t->type[i] == type && t->sign[i] == sign) return 1;
  return 0;
}
