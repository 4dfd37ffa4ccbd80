/* Clean-room subset of genome_hr (the reference's src/genome_hr.c is a missing
 * blob, /root/reference/.MISSING_LARGE_BLOBS): the setup calls and the
 * splice-site dinucleotide queries GMAP's stage 2 makes, so that a gmap built
 * against the drop-in runs end to end.
 *
 * Prototypes: genome_hr.h:12-20 (setup), genome_hr.h:106-112 (prev positions).
 * Semantics: stage2.c:900-970 (check_canonical_dinucleotides_hr) requires
 * Genome_prev_X_position(pos, ..., pos5=1, plusp) == lastX[pos] wherever the
 * string scan find_canonical_dinucleotides (stage2.c:742-850) found a site,
 * and find_shifted_canonical (stage2.c:1141-1228) reads -1 as "none". So:
 *
 *   s[i]  = genome[genomicstart + i]                   (plusp)
 *         = complement(genome[genomicend - 1 - i])     (minus: the revcomp
 *           segment stage 2 aligns against, genomicend = start + length,
 *           gmap.c:731)
 *   donor        p: s[p+1] s[p+2] == "GT"   -> returns p     (stage2.c:766-768)
 *   antiacceptor p: s[p+1] s[p+2] == "CT"   -> returns p     (:770-771)
 *   acceptor     q: s[q-2] s[q-1] == "AG"   -> returns q     (:786-789)
 *   antidonor    q: s[q-2] s[q-1] == "AC"   -> returns q     (:791-794)
 *
 * and the search runs down from pos over the scan positions k >= pos5 of
 * that string scan (p = k for the GT/CT sites, q = k + 3 for AG/AC), so the
 * answer is the largest site <= pos, or -1.  Characters come from the packed
 * blocks (genome.c:9325: a set flag bit reads as N, which matches nothing);
 * positions before the genome start match nothing.
 *
 * Host code: these are per-call scalar queries inside stage 2's link scoring,
 * not DP work.
 */
#include <stddef.h>

typedef unsigned int UINT4;
typedef unsigned int Genomicpos_T;
typedef unsigned char gbool; /* the reference's bool (bool.h:7) */

static const UINT4 *ref_blocks = NULL;

void Genome_hr_setup(UINT4 *ref_blocks_in, UINT4 *snp_blocks_in, gbool query_unk_mismatch_p_in,
                     gbool genome_unk_mismatch_p_in, int mode_in) {
  (void)snp_blocks_in;
  (void)query_unk_mismatch_p_in;
  (void)genome_unk_mismatch_p_in;
  (void)mode_in;
  ref_blocks = ref_blocks_in;
}

void Genome_hr_user_setup(UINT4 *ref_blocks_in, gbool query_unk_mismatch_p_in,
                          gbool genome_unk_mismatch_p_in, int mode_in) {
  Genome_hr_setup(ref_blocks_in, NULL, query_unk_mismatch_p_in, genome_unk_mismatch_p_in, mode_in);
}

/* 2-bit code of the genome at gpos, or -1 for N/X (flag bit) */
static int code_at(long long gpos) {
  if (gpos < 0) return -1;
  const UINT4 *b = ref_blocks + (size_t)(gpos >> 5) * 3;
  const unsigned bit = (unsigned)(gpos & 31);
  if ((b[2] >> bit) & 1u) return -1;
  const UINT4 word = bit < 16 ? b[1] : b[0];
  return (int)((word >> ((bit & 15u) * 2u)) & 3u);
}

/* code of s[i] in the segment's own orientation (A0 C1 G2 T3) */
static int seg_code(int i, Genomicpos_T genomicstart, Genomicpos_T genomicend, gbool plusp) {
  if (plusp) return code_at((long long)genomicstart + i);
  const int c = code_at((long long)genomicend - 1 - i);
  return c < 0 ? -1 : 3 - c;
}

enum { A = 0, C = 1, G = 2, T = 3 };

/* largest scan position k in [pos5, last_k] with s[k+1] s[k+2] == (c1, c2), or -1 */
static int prev_pair(int last_k, int pos5, int c1, int c2, Genomicpos_T genomicstart,
                     Genomicpos_T genomicend, gbool plusp) {
  if (ref_blocks == NULL) return -1;
  for (int k = last_k; k >= pos5; k--) {
    if (seg_code(k + 2, genomicstart, genomicend, plusp) == c2 &&
        seg_code(k + 1, genomicstart, genomicend, plusp) == c1)
      return k;
  }
  return -1;
}

int Genome_prev_donor_position(int pos, Genomicpos_T genomicstart, Genomicpos_T genomicend, int pos5,
                               gbool plusp) {
  return prev_pair(pos, pos5, G, T, genomicstart, genomicend, plusp);
}

int Genome_prev_antiacceptor_position(int pos, Genomicpos_T genomicstart, Genomicpos_T genomicend,
                                      int pos5, gbool plusp) {
  return prev_pair(pos, pos5, C, T, genomicstart, genomicend, plusp);
}

int Genome_prev_acceptor_position(int pos, Genomicpos_T genomicstart, Genomicpos_T genomicend, int pos5,
                                  gbool plusp) {
  const int k = prev_pair(pos - 3, pos5, A, G, genomicstart, genomicend, plusp);
  return k < 0 ? -1 : k + 3;
}

int Genome_prev_antidonor_position(int pos, Genomicpos_T genomicstart, Genomicpos_T genomicend, int pos5,
                                   gbool plusp) {
  const int k = prev_pair(pos - 3, pos5, A, C, genomicstart, genomicend, plusp);
  return k < 0 ? -1 : k + 3;
}
