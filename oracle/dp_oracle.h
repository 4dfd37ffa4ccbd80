/*
 * dp_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * Clean-room CPU restatement of GMAP/GSNAP's stage-3 gap DP
 * (src/dynprog.c) and MaxEnt splice scoring (src/maxent_hr.c), version
 * 2012-07-03.  It is the parity checker for the HIP path and the
 * "port" CPU baseline in bench.py.  It must never be linked into, loaded
 * by, or called from the product library (gmap-gsnap_amd/).
 *
 * Parity of this restatement is pinned against the reference compiled from
 * its own sources (oracle/Makefile -> oracle/_ref/ref_driver) through the
 * golden vectors in tests/golden/ (see tests/test_oracle_golden.py).
 */
#ifndef DP_ORACLE_H
#define DP_ORACLE_H

#include <stdint.h>
#include "../include/gsnapdp.h"

#ifdef __cplusplus
extern "C" {
#endif

/* A pair list in list order (head first), with O(1) push-front like the
 * reference's List_T of Pairpool cells (pairpool.c:169). */
typedef struct orc_list {
  gsnapdp_pair *buf;
  int cap;    /* capacity of buf */
  int head;   /* index of the list head in buf */
  int n;      /* number of cells */
} orc_list;

void orc_list_init(orc_list *l, int cap);
void orc_list_free(orc_list *l);
void orc_list_clear(orc_list *l);

/* Per-thread workspace, the analogue of struct Dynprog_T (dynprog.c:822). */
typedef struct orc_dp {
  int maxlength1, maxlength2;
  int32_t *nogap, *gap1, *gap2;     /* (maxlength1+1) x (maxlength2+1) */
  uint8_t *dnogap, *dgap1, *dgap2;
  int alloc1, alloc2;               /* the allocation's maxlengths (a reused workspace) */
} orc_dp;

/* Dynprog_init (dynprog.c:1339): builds the substitution tables. */
void orc_init(int mode);
/* Genome_user_setup + Maxent_hr_setup: the packed genome blocks. */
void orc_set_genome(const uint32_t *blocks);
/* Dynprog_new / Dynprog_free (dynprog.c:855-887). */
orc_dp *orc_dp_new(int maxlookback, int extraquerygap, int maxpeelback,
                   int extramaterial_end, int extramaterial_paired);
void orc_dp_free(orc_dp *dp);

int orc_pairdistance(int mismatchtype, int c1, int c2);
int orc_consistent(int c1, int c2);
char orc_get_genomic_nt(int genomicpos, uint32_t chroffset, uint32_t chrhigh,
                        uint32_t chrpos, int genomiclength, int watsonp);

/* Entry points.  Same arguments as the reference (dynprog.h:74-160), minus
 * the unused sequence2/sequenceuc2 (use_genomicseg_p is false on the hot
 * path, stage3.c:9864), with the pair list written to *out (cleared first,
 * in final list order, i.e. what the reference returns). */
void orc_single_gap(orc_list *out, int *dynprogindex, int *finalscore, int *nmatches,
                    int *nmismatches, int *nopens, int *nindels, orc_dp *dp,
                    const char *sequence1, const char *sequenceuc1, int length1, int length2,
                    int offset1, int offset2, uint32_t chroffset, uint32_t chrhigh,
                    uint32_t chrpos, uint32_t genomiclength, int cdna_direction, int watsonp,
                    int jump_late_p, int extraband_single, double defect_rate,
                    int close_indels_mode, int widebandp);

void orc_end5_gap(orc_list *out, int *dynprogindex, int *finalscore, int *nmatches,
                  int *nmismatches, int *nopens, int *nindels, orc_dp *dp,
                  const char *revsequence1, const char *revsequenceuc1, int length1, int length2,
                  int revoffset1, int revoffset2, uint32_t chroffset, uint32_t chrhigh,
                  uint32_t chrpos, uint32_t genomiclength, int cdna_direction, int watsonp,
                  int jump_late_p, int extraband_end, double defect_rate, int endalign);

void orc_end3_gap(orc_list *out, int *dynprogindex, int *finalscore, int *nmatches,
                  int *nmismatches, int *nopens, int *nindels, orc_dp *dp,
                  const char *sequence1, const char *sequenceuc1, int length1, int length2,
                  int offset1, int offset2, uint32_t chroffset, uint32_t chrhigh,
                  uint32_t chrpos, uint32_t genomiclength, int cdna_direction, int watsonp,
                  int jump_late_p, int extraband_end, double defect_rate, int endalign);

/* Dynprog_genome_gap (dynprog.c:4798-5061) with splicing_iit == NULL
 * (no known-site rewards).  Returns 1 if a list was produced (possibly
 * empty), 0 for the reference's NULL returns. */
typedef struct orc_genome_gap_out {
  int finalscore, new_leftgenomepos, new_rightgenomepos;
  double left_prob, right_prob;
  int nmatches, nmismatches, nopens, nindels, exonhead, introntype;
  int dynprogindex;
  int returned_null;
  int bridge_ok;            /* 0 if probability mode found no candidate (reference UB) */
} orc_genome_gap_out;

void orc_genome_gap(orc_list *out, orc_genome_gap_out *o, int dynprogindex_in,
                    orc_dp *dpL, orc_dp *dpR, const char *sequence1, const char *sequenceuc1,
                    int length1, int length2L, int length2R, int offset1, int offset2L,
                    int revoffset2R, uint32_t chroffset, uint32_t chrhigh, uint32_t chrpos,
                    uint32_t genomiclength, int cdna_direction, int watsonp, int jump_late_p,
                    int extraband_paired, double defect_rate, int maxpeelback, int halfp,
                    int finalp, int use_probabilities_p, int score_threshold, int splicingp,
                    int known_mode); /* GSNAPDP_KNOWN_*: record at sequence1[length1] */

/* Dynprog_cdna_gap (dynprog.c:4578-4793). */
typedef struct orc_cdna_gap_out {
  int finalscore, dynprogindex, incompletep, returned_null;
  int finalscore_set;  /* 0 on the early returns (*finalscore untouched) */
  int insert_pairs;    /* the INSERT_PAIRS branch (:4730) was taken */
  int bridge_ok;       /* 0: no bridge candidate (reference UB) */
  int brL, bcL, brR, bcR;
} orc_cdna_gap_out;

void orc_cdna_gap(orc_list *out, orc_cdna_gap_out *o, int dpi, orc_dp *dpL, orc_dp *dpR,
                  const char *sequence1L, const char *sequenceuc1L, const char *revsequence1R,
                  const char *revsequenceuc1R, const char *sequence2, int length1L, int length1R,
                  int length2, int offset1L, int revoffset1R, int offset2, uint32_t chroffset,
                  uint32_t chrhigh, uint32_t chrpos, uint32_t genomiclength, int cdna_direction,
                  int watsonp, int jump_late_p, int extraband_paired, double defect_rate);

int orc_run_cgap_batch(const gsnapdp_cgap_window *w, int n, const char *query, const char *query_uc,
                       const char *gseg, const int64_t *gseg_off, gsnapdp_cgap_result *results,
                       gsnapdp_pair *pairs, const int64_t *pair_offsets, int32_t *npairs);

/* Dynprog_score (dynprog.c:380). */
int orc_score(int matches, int mismatches, int qopens, int qindels, int topens, int tindels,
              double defect_rate);

/* MaxEnt (maxent_hr.c).  Tables: 16 arrays in the order of
 * orc_maxent_table_names(); returns 0 on success. */
int orc_maxent_load(const double *tables, size_t ndoubles);
double orc_maxent_donor(uint32_t splice_pos, uint32_t chroffset);
double orc_maxent_acceptor(uint32_t splice_pos, uint32_t chroffset);
double orc_maxent_antidonor(uint32_t splice_pos, uint32_t chroffset);
double orc_maxent_antiacceptor(uint32_t splice_pos, uint32_t chroffset);
/* score_introns (stage3.c:7935-8162): the intron walk and the sums (maxent_oracle.c) */
int orc_path_introns(const gsnapdp_path_pair *pairs, int npairs, int nullgap, int path, gsnapdp_intron *out,
                     int cap);
void orc_score_introns(const gsnapdp_intron_path *paths, int npaths, const gsnapdp_intron *introns,
                       gsnapdp_intron_scores *out);

/* Batch driver over gsnapdp_window records (same input format as the
 * product ABI).  Writes results[i] (finalscore, counts, status) and the
 * final pair list of window i into pairs[pair_offsets[i] ...] (at most
 * pair_offsets[i+1]-pair_offsets[i]); npairs[i] = list length.
 * nthreads > 1 uses pthreads, one orc_dp per thread (gmap.c:2270). */
int orc_run_batch(const gsnapdp_window *w, int n, const char *query, const char *query_uc,
                  gsnapdp_result *results, gsnapdp_pair *pairs, const int64_t *pair_offsets,
                  int32_t *npairs, int nthreads);

/* Batch driver over gsnapdp_ggap_window records (single thread). */
int orc_run_ggap_batch(const gsnapdp_ggap_window *w, int n, const char *query, const char *query_uc,
                       gsnapdp_ggap_result *results, gsnapdp_pair *pairs,
                       const int64_t *pair_offsets, int32_t *npairs);

/* Batch maxent: model 0..3 = donor, acceptor, antidonor, antiacceptor. */
void orc_maxent_batch(const uint8_t *model, const uint32_t *pos, const uint32_t *chroffset,
                      double *out, int n);

/* Dynprog_end5_splicejunction (dynprog.c:5412) / Dynprog_end3_splicejunction (:5869) */
void orc_end5_splicejunction(orc_list *out, int *dynprogindex, int *finalscore, int *nmatches,
                             int *nmismatches, int *nopens, int *nindels, orc_dp *dp,
                             const char *revsequence1, const char *revsequenceuc1,
                             const char *revsequence2, const char *revsequenceuc2, int length1,
                             int length2, int revoffset1, int revoffset2_anchor,
                             int revoffset2_far, int cdna_direction, int jump_late_p,
                             int extraband_end, double defect_rate, int contlength);
void orc_end3_splicejunction(orc_list *out, int *dynprogindex, int *finalscore, int *nmatches,
                             int *nmismatches, int *nopens, int *nindels, orc_dp *dp,
                             const char *sequence1, const char *sequenceuc1, const char *sequence2,
                             const char *sequenceuc2, int length1, int length2, int offset1,
                             int offset2_anchor, int offset2_far, int cdna_direction,
                             int jump_late_p, int extraband_end, double defect_rate,
                             int contlength);
int orc_run_sj_batch(const gsnapdp_sj_window *w, int n, const char *query, const char *query_uc,
                     gsnapdp_result *results, gsnapdp_pair *pairs, const int64_t *pair_offsets,
                     int32_t *npairs);

/* Dynprog_microexon_int (dynprog.c:7128) */
typedef struct orc_micro_out {
  double bestprob2, bestprob3;
  int microintrontype, dynprogindex, found, unsupported;
  int bestcL, bestcR, middlelength, offset2M;
} orc_micro_out;
int orc_microexon_int(orc_list *out, orc_micro_out *o, int dynprogindex, const char *sequence1,
                      const char *sequenceuc1, int length1, int offset1, int offset2L,
                      int revoffset2R, int cdna_direction, const char *queryseq,
                      const char *queryuc, uint32_t chroffset, uint32_t chrhigh, uint32_t chrpos,
                      uint32_t genomiclength, int watsonp, double defect_rate);
int orc_run_micro_batch(const gsnapdp_micro_window *w, int n, const char *query,
                        const char *query_uc, gsnapdp_micro_result *results, gsnapdp_pair *pairs,
                        const int64_t *pair_offsets, int32_t *npairs);

#ifdef __cplusplus
}
#endif
#endif
