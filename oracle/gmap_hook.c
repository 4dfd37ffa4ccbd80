/* TEST INFRASTRUCTURE ONLY (linked into oracle/_ref/gmap_gpu, never shipped).
 *
 * The one setup call INTEGRATION.md asks a gmap maintainer to add after the
 * genome blocks exist (gmap.c:3469, user segment; gmap.c:3511 for an index),
 * made here at link time instead of by editing gmap.c: the reference's own
 * objects are linked with -Wl,--wrap=Genome_create_blocks, so gmap.c's call
 * lands here, builds the blocks with the reference's function
 * (genome-write.c:805-827) and hands them to the drop-in.
 */
#include <stddef.h>

extern unsigned int *__real_Genome_create_blocks(char *genomicseg, unsigned int genomelength);
extern int Gsnapdp_dropin_genome(const unsigned int *blocks, size_t nwords, int device);

unsigned int *__wrap_Genome_create_blocks(char *genomicseg, unsigned int genomelength) {
  unsigned int *blocks = __real_Genome_create_blocks(genomicseg, genomelength);
  /* genome-write.c:809-810: 3 words per 32 nt, plus 4 words of padding */
  Gsnapdp_dropin_genome(blocks, (size_t)((genomelength + 31) / 32U) * 3 + 4, 0);
  return blocks;
}
