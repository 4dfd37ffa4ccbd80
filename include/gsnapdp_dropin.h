/*
 * gsnapdp_dropin.h -- the reference's own per-call entry points, served by
 * the MI355X engine (libgsnapdp_dropin.so replaces dynprog.o + maxent_hr.o in
 * the gmap / gsnap link).
 *
 * Every prototype below is ABI-identical to the reference declaration it
 * cites (GMAP/GSNAP 2012-07-03, non-PMAP build): `bool` is the reference's
 * `typedef unsigned char bool` (bool.h:7), Genomicpos_T / UINT4 are
 * `unsigned int` (types.h:12, genomicpos.h:9), the enums are int-sized, and
 * Dynprog_T / List_T / Pairpool_T / IIT_T / Genome_T are opaque pointers.
 * When compiled inside the reference tree, include the reference headers
 * instead of this one; the symbols are the same.
 *
 * Output pairs are materialised with the host program's own
 * Pairpool_push / Pairpool_push_gapholder (pairpool.c:169, 352), in the
 * reference's list order, so callers cannot tell the difference.
 *
 * Per call these run a batch of one window on the GPU (a few tens of
 * microseconds of launch latency); the throughput path is the batched
 * C-ABI of gsnapdp.h.
 */
#ifndef GSNAPDP_DROPIN_H
#define GSNAPDP_DROPIN_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef unsigned char gsnapdp_bool;                 /* bool.h:7 */
typedef unsigned int gsnapdp_Genomicpos_T;          /* genomicpos.h:9 */
typedef int gsnapdp_Endalign_T;                     /* dynprog.h:8 */
typedef int gsnapdp_Mode_T;                         /* mode.h */
typedef int gsnapdp_Splicetype_T;                   /* splicetrie_build.h */
typedef struct Dynprog_T *gsnapdp_Dynprog_T;        /* dynprog.h:9 (opaque) */
typedef struct List_T *gsnapdp_List_T;              /* list.h:6 */
typedef struct Pairpool_T *gsnapdp_Pairpool_T;      /* pairpool.h */
typedef struct IIT_T *gsnapdp_IIT_T;                /* iit-read.h */
typedef struct Genome_T *gsnapdp_Genome_T;          /* genome.h */

/* --- provided by the host program (reference pairpool.c), used by the shim --- */
gsnapdp_List_T Pairpool_push(gsnapdp_List_T list, gsnapdp_Pairpool_T pool, int querypos,
                             int genomepos, char cdna, char comp, char genome,
                             int dynprogindex);                     /* pairpool.h:24 */
gsnapdp_List_T Pairpool_push_gapholder(gsnapdp_List_T list, gsnapdp_Pairpool_T pool,
                                       int queryjump, int genomejump,
                                       gsnapdp_bool knownp);        /* pairpool.h:28 */

/* --- provided by the host program (reference splicetrie.c, list.c, pairpool.c,
 * pair.c), used by Dynprog_end5_known / Dynprog_end3_known (the shim references
 * Splicetrie_solve_end5/3 weakly and looks them up at the first call if the
 * host loaded the shim first) --- */
gsnapdp_List_T Splicetrie_solve_end5(
    gsnapdp_List_T best_pairs, unsigned int* triecontents, unsigned int* trieoffsets, int j,
    gsnapdp_Genomicpos_T knownsplice_limit_low, gsnapdp_Genomicpos_T knownsplice_limit_high,
    int* finalscore, int* nmatches, int* nmismatches, int* nopens, int* nindels,
    gsnapdp_bool* knownsplicep, int* ambig_end_length, int* threshold_miss_score,
    int obsmax_penalty, int perfect_score, gsnapdp_Genomicpos_T anchor_splicesite,
    char* splicejunction, int splicelength, int contlength, gsnapdp_Splicetype_T far_splicetype,
    gsnapdp_Genomicpos_T chroffset, gsnapdp_Genomicpos_T chrhigh, gsnapdp_Genomicpos_T chrpos,
    int genomiclength, int* dynprogindex, gsnapdp_Dynprog_T dynprog, char* revsequence1,
    char* revsequenceuc1, int length1, int length2, int revoffset1, int revoffset2,
    int cdna_direction, gsnapdp_bool watsonp, gsnapdp_bool jump_late_p,
    gsnapdp_Pairpool_T pairpool, int extraband_end, double defect_rate); /* splicetrie.h:32 */
gsnapdp_List_T Splicetrie_solve_end3(
    gsnapdp_List_T best_pairs, unsigned int* triecontents, unsigned int* trieoffsets, int j,
    gsnapdp_Genomicpos_T knownsplice_limit_low, gsnapdp_Genomicpos_T knownsplice_limit_high,
    int* finalscore, int* nmatches, int* nmismatches, int* nopens, int* nindels,
    gsnapdp_bool* knownsplicep, int* ambig_end_length, int* threshold_miss_score,
    int obsmax_penalty, int perfect_score, gsnapdp_Genomicpos_T anchor_splicesite,
    char* splicejunction, int splicelength, int contlength, gsnapdp_Splicetype_T far_splicetype,
    gsnapdp_Genomicpos_T chroffset, gsnapdp_Genomicpos_T chrhigh, gsnapdp_Genomicpos_T chrpos,
    int genomiclength, int* dynprogindex, gsnapdp_Dynprog_T dynprog, char* sequence1,
    char* sequenceuc1, int length1, int length2, int offset1, int offset2, int cdna_direction,
    gsnapdp_bool watsonp, gsnapdp_bool jump_late_p, gsnapdp_Pairpool_T pairpool,
    int extraband_end, double defect_rate);                           /* splicetrie.h:53 */
gsnapdp_List_T List_reverse(gsnapdp_List_T list);                    /* list.h */
gsnapdp_List_T Pairpool_pop(gsnapdp_List_T list, void** x);          /* pairpool.h (Pair_T *x) */
gsnapdp_List_T Pair_protect(gsnapdp_List_T list);                    /* pair.h */

/* --- setup / workspace (dynprog.h:34-72) --- */
char* Dynprog_endalign_string(gsnapdp_Endalign_T endalign);                    /* dynprog.c:335 */
void Dynprog_setup(gsnapdp_bool novelsplicingp, gsnapdp_IIT_T splicesites_iit,
                   int* splicesites_divint_crosstable, int donor_typeint, int acceptor_typeint,
                   gsnapdp_Genomicpos_T* splicesites, gsnapdp_Splicetype_T* splicetypes,
                   gsnapdp_Genomicpos_T* splicedists, int nsplicesites,
                   unsigned int* trieoffsets_obs, unsigned int* triecontents_obs,
                   unsigned int* trieoffsets_max, unsigned int* triecontents_max,
                   gsnapdp_Genome_T genome);                                   /* dynprog.c:350 */
int Dynprog_score(int matches, int mismatches, int qopens, int qindels, int topens, int tindels,
                  double defect_rate);                                         /* dynprog.c:381 */
gsnapdp_Dynprog_T Dynprog_new(int maxlookback, int extraquerygap, int maxpeelback,
                              int extramaterial_end, int extramaterial_paired); /* dynprog.c:856 */
void Dynprog_free(gsnapdp_Dynprog_T* old);                                     /* dynprog.c:877 */
int Dynprog_pairdistance(int c1, int c2);                                      /* dynprog.c:1049 */
void Dynprog_term(void);                                                       /* dynprog.c:1348 */
void Dynprog_init(int maxlookback, int extraquerygap, int maxpeelback, int extramaterial_end,
                  int extramaterial_paired, gsnapdp_Mode_T mode);              /* dynprog.c:1339 */

/* --- the gap fillers served by the GPU (dynprog.h:74-160) --- */
gsnapdp_List_T Dynprog_single_gap(
    int* dynprogindex, int* finalscore, int* nmatches, int* nmismatches, int* nopens,
    int* nindels, gsnapdp_Dynprog_T dynprog, char* sequence1, char* sequenceuc1,
    char* sequence2, char* sequenceuc2, int length1, int length2, int offset1, int offset2,
    gsnapdp_Genomicpos_T chroffset, gsnapdp_Genomicpos_T chrhigh, gsnapdp_Genomicpos_T chrpos,
    gsnapdp_Genomicpos_T genomiclength, int cdna_direction, gsnapdp_bool watsonp,
    gsnapdp_bool jump_late_p, gsnapdp_Pairpool_T pairpool, int extraband_single,
    double defect_rate, int close_indels_mode, gsnapdp_bool widebandp); /* dynprog.c:4450 */

gsnapdp_List_T Dynprog_cdna_gap(
    int* dynprogindex, int* finalscore, gsnapdp_bool* incompletep, gsnapdp_Dynprog_T dynprogL,
    gsnapdp_Dynprog_T dynprogR, char* sequence1L, char* sequenceuc1L, char* revsequence1R,
    char* revsequenceuc1R, char* sequence2, char* sequenceuc2, int length1L, int length1R,
    int length2, int offset1L, int revoffset1R, int offset2, gsnapdp_Genomicpos_T chroffset,
    gsnapdp_Genomicpos_T chrhigh, gsnapdp_Genomicpos_T chrpos,
    gsnapdp_Genomicpos_T genomiclength, int cdna_direction, gsnapdp_bool watsonp,
    gsnapdp_bool jump_late_p, gsnapdp_Pairpool_T pairpool, int extraband_paired,
    double defect_rate); /* dynprog.c:4579 (non-PMAP) */

gsnapdp_List_T Dynprog_genome_gap(
    int* dynprogindex, int* finalscore, int* new_leftgenomepos, int* new_rightgenomepos,
    double* left_prob, double* right_prob, int* nmatches, int* nmismatches, int* nopens,
    int* nindels, int* exonhead, int* introntype, gsnapdp_Dynprog_T dynprogL,
    gsnapdp_Dynprog_T dynprogR, char* sequence1, char* sequenceuc1, char* sequence2L,
    char* sequenceuc2L, char* revsequence2R, char* revsequenceuc2R, int length1, int length2L,
    int length2R, int offset1, int offset2L, int revoffset2R, int chrnum,
    gsnapdp_Genomicpos_T chroffset, gsnapdp_Genomicpos_T chrhigh, gsnapdp_Genomicpos_T chrpos,
    gsnapdp_Genomicpos_T genomiclength, char* genomicuc_ptr, gsnapdp_bool use_genomicseg_p,
    int cdna_direction, gsnapdp_bool watsonp, gsnapdp_bool jump_late_p,
    gsnapdp_Pairpool_T pairpool, int extraband_paired, double defect_rate, int maxpeelback,
    gsnapdp_bool halfp, gsnapdp_bool finalp, gsnapdp_bool use_probabilities_p,
    int score_threshold, gsnapdp_bool splicingp); /* dynprog.c:4798 (non-PMAP; chrnum is Chrnum_T, chrnum.h:8) */

gsnapdp_List_T Dynprog_end5_gap(
    int* dynprogindex, int* finalscore, int* nmatches, int* nmismatches, int* nopens,
    int* nindels, gsnapdp_Dynprog_T dynprog, char* revsequence1, char* revsequenceuc1,
    char* revsequence2, char* revsequenceuc2, int length1, int length2, int revoffset1,
    int revoffset2, gsnapdp_Genomicpos_T chroffset, gsnapdp_Genomicpos_T chrhigh,
    gsnapdp_Genomicpos_T chrpos, gsnapdp_Genomicpos_T genomiclength, int cdna_direction,
    gsnapdp_bool watsonp, gsnapdp_bool jump_late_p, gsnapdp_Pairpool_T pairpool,
    int extraband_end, double defect_rate, gsnapdp_Endalign_T endalign,
    gsnapdp_bool use_genomicseg_p);                                     /* dynprog.c:5094 */

gsnapdp_List_T Dynprog_end3_gap(
    int* dynprogindex, int* finalscore, int* nmatches, int* nmismatches, int* nopens,
    int* nindels, gsnapdp_Dynprog_T dynprog, char* sequence1, char* sequenceuc1,
    char* sequence2, char* sequenceuc2, int length1, int length2, int offset1, int offset2,
    gsnapdp_Genomicpos_T chroffset, gsnapdp_Genomicpos_T chrhigh, gsnapdp_Genomicpos_T chrpos,
    gsnapdp_Genomicpos_T genomiclength, int cdna_direction, gsnapdp_bool watsonp,
    gsnapdp_bool jump_late_p, gsnapdp_Pairpool_T pairpool, int extraband_end,
    double defect_rate, gsnapdp_Endalign_T endalign,
    gsnapdp_bool use_genomicseg_p);                                     /* dynprog.c:5556 */

/* --- splice-junction end gaps and their junction builders (dynprog.h:120-173) --- */
gsnapdp_List_T Dynprog_end5_splicejunction(
    int* dynprogindex, int* finalscore, int* nmatches, int* nmismatches, int* nopens,
    int* nindels, gsnapdp_Dynprog_T dynprog, char* revsequence1, char* revsequenceuc1,
    char* revsequence2, char* revsequenceuc2, int length1, int length2, int revoffset1,
    int revoffset2_anchor, int revoffset2_far, gsnapdp_Genomicpos_T chroffset,
    gsnapdp_Genomicpos_T chrhigh, gsnapdp_Genomicpos_T chrpos,
    gsnapdp_Genomicpos_T genomiclength, int cdna_direction, gsnapdp_bool watsonp,
    gsnapdp_bool jump_late_p, gsnapdp_Pairpool_T pairpool, int extraband_end,
    double defect_rate, int contlength);                                /* dynprog.c:5412 */
gsnapdp_List_T Dynprog_end3_splicejunction(
    int* dynprogindex, int* finalscore, int* nmatches, int* nmismatches, int* nopens,
    int* nindels, gsnapdp_Dynprog_T dynprog, char* sequence1, char* sequenceuc1,
    char* sequence2, char* sequenceuc2, int length1, int length2, int offset1,
    int offset2_anchor, int offset2_far, gsnapdp_Genomicpos_T chroffset,
    gsnapdp_Genomicpos_T chrhigh, gsnapdp_Genomicpos_T chrpos,
    gsnapdp_Genomicpos_T genomiclength, int cdna_direction, gsnapdp_bool watsonp,
    gsnapdp_bool jump_late_p, gsnapdp_Pairpool_T pairpool, int extraband_end,
    double defect_rate, int contlength);                                /* dynprog.c:5869 */
void Dynprog_make_splicejunction_5(char* splicejunction, gsnapdp_Genomicpos_T splicecoord,
                                   int splicelength, int contlength,
                                   gsnapdp_Splicetype_T far_splicetype,
                                   gsnapdp_bool watsonp);               /* dynprog.c:6061 */
void Dynprog_make_splicejunction_3(char* splicejunction, gsnapdp_Genomicpos_T splicecoord,
                                   int splicelength, int contlength,
                                   gsnapdp_Splicetype_T far_splicetype,
                                   gsnapdp_bool watsonp);               /* dynprog.c:6149 */

/* --- end gaps against known splice sites (dynprog.h:194-236; non-GSNAP-shortcut form) --- */
gsnapdp_List_T Dynprog_end5_known(
    gsnapdp_bool* knownsplicep, int* dynprogindex, int* finalscore, int* ambig_end_length,
    gsnapdp_Splicetype_T* ambig_splicetype, int* nmatches, int* nmismatches, int* nopens,
    int* nindels, gsnapdp_Dynprog_T dynprog, char* revsequence1, char* revsequenceuc1,
    char* revsequence2, char* revsequenceuc2, int length1, int length2, int revoffset1,
    int revoffset2, gsnapdp_Genomicpos_T chroffset, gsnapdp_Genomicpos_T chrhigh,
    gsnapdp_Genomicpos_T chrpos, int genomiclength, gsnapdp_Genomicpos_T knownsplice_limit_low,
    gsnapdp_Genomicpos_T knownsplice_limit_high, int cdna_direction, gsnapdp_bool watsonp,
    gsnapdp_bool jump_late_p, gsnapdp_Pairpool_T pairpool, int extraband_end,
    double defect_rate);                                                /* dynprog.c:6414 */
gsnapdp_List_T Dynprog_end3_known(
    gsnapdp_bool* knownsplicep, int* dynprogindex, int* finalscore, int* ambig_end_length,
    gsnapdp_Splicetype_T* ambig_splicetype, int* nmatches, int* nmismatches, int* nopens,
    int* nindels, gsnapdp_Dynprog_T dynprog, char* sequence1, char* sequenceuc1,
    char* sequence2, char* sequenceuc2, int length1, int length2, int offset1, int offset2,
    int querylength, gsnapdp_Genomicpos_T chroffset, gsnapdp_Genomicpos_T chrhigh,
    gsnapdp_Genomicpos_T chrpos, int genomiclength, gsnapdp_Genomicpos_T knownsplice_limit_low,
    gsnapdp_Genomicpos_T knownsplice_limit_high, int cdna_direction, gsnapdp_bool watsonp,
    gsnapdp_bool jump_late_p, gsnapdp_Pairpool_T pairpool, int extraband_end,
    double defect_rate);                                                /* dynprog.c:6680 */

/* --- microexon search (dynprog.h:281-292; _5 / _3 are declared but never
 * defined by the reference, dynprog.c:7467-7762 is #if 0) --- */
gsnapdp_List_T Dynprog_microexon_int(
    double* bestprob2, double* bestprob3, int* dynprogindex, int* microintrontype,
    char* sequence1, char* sequenceuc1, char* sequence2L, char* sequenceuc2L,
    char* revsequence2R, char* revsequenceuc2R, int length1, int length2L, int length2R,
    int offset1, int offset2L, int revoffset2R, int cdna_direction, char* queryseq,
    char* queryuc, char* genomicseg, char* genomicuc, gsnapdp_Genomicpos_T chroffset,
    gsnapdp_Genomicpos_T chrhigh, gsnapdp_Genomicpos_T chrpos,
    gsnapdp_Genomicpos_T genomiclength, gsnapdp_bool watsonp, gsnapdp_bool use_genomicseg_p,
    gsnapdp_Pairpool_T pairpool, double defect_rate);                 /* dynprog.c:7128 */

/* --- MaxEnt splice-site probabilities (maxent_hr.h:6-19) --- */
void Maxent_hr_setup(unsigned int* ref_blocks);                                 /* maxent_hr.c:27195 */
double Maxent_hr_donor_prob(gsnapdp_Genomicpos_T splice_pos, gsnapdp_Genomicpos_T chroffset);
double Maxent_hr_acceptor_prob(gsnapdp_Genomicpos_T splice_pos, gsnapdp_Genomicpos_T chroffset);
double Maxent_hr_antidonor_prob(gsnapdp_Genomicpos_T splice_pos, gsnapdp_Genomicpos_T chroffset);
double Maxent_hr_antiacceptor_prob(gsnapdp_Genomicpos_T splice_pos,
                                   gsnapdp_Genomicpos_T chroffset);

/* score_introns (stage3.c:7935-8162, static there; non-WASTE signature): a
 * stage3.c that calls Gsnapdp_score_introns at its two call sites
 * (stage3.c:9892, 9935) gets the same outputs and the same
 * returned list, with the path's MaxEnt probabilities run in one GPU launch
 * (shared with concurrent callers) instead of four round trips per intron. */
gsnapdp_List_T Gsnapdp_score_introns(double* avg_donor_score, double* avg_acceptor_score, int* nbadintrons,
                                     gsnapdp_List_T path, int cdna_direction, gsnapdp_bool watsonp, int chrnum,
                                     gsnapdp_Genomicpos_T chroffset, gsnapdp_Genomicpos_T chrhigh,
                                     gsnapdp_Genomicpos_T chrpos, char* genomicuc_ptr, int genomiclength,
                                     int nullgap, gsnapdp_bool use_genomicseg_p);

/* build_pairs_introns (stage3.c:7735-7901, static there; non-PMAP, non-WASTE
 * signature): a stage3.c that calls Gsnapdp_build_pairs_introns at its two
 * call sites (stage3.c:8766, 8865) gets the same list, the
 * same counters and flags, with every gap of the path filled by the GPU gap
 * families (gsnapdp_stage3_pass over one path).  The splicing IIT is
 * Dynprog_setup's, asked through the host's own iit-read functions; the
 * genome is the context's.  A caller with many paths at hand calls
 * gsnapdp_stage3_pass (gsnapdp.h) on all of them at once instead. */
gsnapdp_List_T Gsnapdp_build_pairs_introns(
    gsnapdp_bool* shiftp, gsnapdp_bool* incompletep, int* nintrons, int* nnonintrons, int* intronlen,
    int* nonintronlen, int* dynprogindex_minor, int* dynprogindex_major, gsnapdp_List_T path, int chrnum,
    gsnapdp_Genomicpos_T chroffset, gsnapdp_Genomicpos_T chrhigh, gsnapdp_Genomicpos_T chrpos,
    gsnapdp_Genome_T genome, int querylength, int genomiclength, char* queryseq_ptr, char* queryuc_ptr,
    char* genomicseg_ptr, char* genomicuc_ptr, gsnapdp_bool use_genomicseg_p, int cdna_direction,
    gsnapdp_bool watsonp, gsnapdp_bool jump_late_p, int maxpeelback, int nullgap, int extramaterial_paired,
    int extraband_single, int extraband_paired, double defect_rate, int close_indels_mode,
    gsnapdp_Pairpool_T pairpool, gsnapdp_Dynprog_T dynprogL, gsnapdp_Dynprog_T dynprogM,
    gsnapdp_Dynprog_T dynprogR, gsnapdp_bool finalp);

/* build_pairs_singles (stage3.c:7454-7583, static there; non-PMAP, non-WASTE
 * signature): passes 2A / 2C / 7C of path_compute (call sites stage3.c:8671,
 * 8700, 8938).  Same list and dynprogindex as the reference,
 * every single gap filled by traverse_single_gap's GPU family
 * (gsnapdp_stage3_pass, pass GSNAPDP_S3_SINGLES, over one path). */
gsnapdp_List_T Gsnapdp_build_pairs_singles(int* dynprogindex, gsnapdp_List_T path, gsnapdp_Genomicpos_T chroffset,
                                           gsnapdp_Genomicpos_T chrhigh, gsnapdp_Genomicpos_T chrpos,
                                           gsnapdp_Genomicpos_T genomiclength, char* queryseq_ptr,
                                           char* queryuc_ptr, char* genomicseg_ptr, char* genomicuc_ptr,
                                           int cdna_direction, gsnapdp_bool watsonp, gsnapdp_bool jump_late_p,
                                           int maxpeelback, int nullgap, int extraband_single, double defect_rate,
                                           int close_indels_mode, gsnapdp_Pairpool_T pairpool,
                                           gsnapdp_Dynprog_T dynprogM);

/* build_pairs_end5 (stage3.c:7351-7450) and build_path_end3 (:7236-7347),
 * static there (non-GSNAP, non-PMAP signatures): passes 8, 9a / 9b and 10 of
 * path_compute and path_trim (call sites :8966, :9036, :9167, :9660, :9722 and
 * :8990, :9088, :9190, :9683, :9744;
 * INTEGRATION.md 5) with extendp -- the extension's Dynprog_end5_gap /
 * Dynprog_end3_gap in the batched pass.  Same list, dynprogindex_minor,
 * knownsplicep, ambig_end_length and chop_exon_p as the reference without splice
 * sites; distalmedial (extendp false) and the splice-site branch
 * (Dynprog_end5/3_known) are refused with a message. */
gsnapdp_List_T Gsnapdp_build_pairs_end5(
    gsnapdp_bool* knownsplicep, int* ambig_end_length_5, gsnapdp_Splicetype_T* ambig_splicetype_5,
    gsnapdp_bool* chop_exon_p, int* dynprogindex_minor, gsnapdp_List_T pairs, gsnapdp_Genomicpos_T chroffset,
    gsnapdp_Genomicpos_T chrhigh, gsnapdp_Genomicpos_T chrpos, int genomiclength,
    gsnapdp_Genomicpos_T knownsplice_limit_low, gsnapdp_Genomicpos_T knownsplice_limit_high, char* queryseq_ptr,
    char* queryuc_ptr, char* genomicseg_ptr, char* genomicuc_ptr, int cdna_direction, gsnapdp_bool watsonp,
    gsnapdp_bool jump_late_p, int maxpeelback, int maxpeelback_distalmedial, int nullgap, int extramaterial_end,
    int extraband_end, double defect_rate, gsnapdp_Pairpool_T pairpool, gsnapdp_Dynprog_T dynprogR,
    gsnapdp_bool extendp, gsnapdp_Endalign_T endalign);
gsnapdp_List_T Gsnapdp_build_path_end3(
    gsnapdp_bool* knownsplicep, int* ambig_end_length_3, gsnapdp_Splicetype_T* ambig_splicetype_3,
    gsnapdp_bool* chop_exon_p, int* dynprogindex_minor, gsnapdp_List_T path, gsnapdp_Genomicpos_T chroffset,
    gsnapdp_Genomicpos_T chrhigh, gsnapdp_Genomicpos_T chrpos, int querylength, int genomiclength,
    gsnapdp_Genomicpos_T knownsplice_limit_low, gsnapdp_Genomicpos_T knownsplice_limit_high, char* queryseq_ptr,
    char* queryuc_ptr, char* genomicseg_ptr, char* genomicuc_ptr, int cdna_direction, gsnapdp_bool watsonp,
    gsnapdp_bool jump_late_p, int maxpeelback, int maxpeelback_distalmedial, int nullgap, int extramaterial_end,
    int extraband_end, double defect_rate, gsnapdp_Pairpool_T pairpool, gsnapdp_Dynprog_T dynprogL,
    gsnapdp_bool extendp, gsnapdp_Endalign_T endalign);

/* build_dual_breaks (stage3.c:7149-7232, static there; non-PMAP signature, the
 * Oligoindex_T * / Diagpool_T arguments as void *): pass 5 of path_compute
 * (call site :8831).  Same list, dynprogindex_minor and dual_break_p as the
 * reference: the gaps solvable as single gaps run traverse_single_gap (forcep)
 * in the batched pass; the others run traverse_dual_break with the host
 * program's own Stage2_compute_one (stage2.c:4260; looked up in the process)
 * on this call's oligoindices and pools. */
gsnapdp_List_T Gsnapdp_build_dual_breaks(
    gsnapdp_bool* dual_break_p, int* dynprogindex_minor, gsnapdp_List_T path, gsnapdp_Genomicpos_T chroffset,
    gsnapdp_Genomicpos_T chrhigh, gsnapdp_Genomicpos_T chrpos, gsnapdp_Genomicpos_T genomiclength,
    char* queryseq_ptr, char* queryuc_ptr, char* genomicseg_ptr, char* genomicuc_ptr, int cdna_direction,
    gsnapdp_bool watsonp, int genestrand, gsnapdp_bool jump_late_p, gsnapdp_Pairpool_T pairpool,
    gsnapdp_Dynprog_T dynprogM, int maxpeelback, void* oligoindices_minor, int noligoindices_minor, void* diagpool,
    int sufflookback, int nsufflookback, int maxintronlen_bound, int extraband_single, double defect_rate,
    int close_indels_mode);

/* build_pairs_dualintrons (stage3.c:7592-7733, static there; non-PMAP
 * signature; Chrnum_T is an int): pass 3b of path_compute (call site :8746).
 * Same list and dynprogindex_major as the reference; each short exon's
 * traverse_dual_genome_gap (:5980-6364) windows run in the batched pass, with
 * Dynprog_setup's splicing IIT as Gsnapdp_build_pairs_introns takes it. */
gsnapdp_List_T Gsnapdp_build_pairs_dualintrons(
    int* dynprogindex, gsnapdp_List_T path, int chrnum, gsnapdp_Genomicpos_T chroffset,
    gsnapdp_Genomicpos_T chrhigh, gsnapdp_Genomicpos_T chrpos, int genomiclength, char* queryseq_ptr,
    char* queryuc_ptr, char* genomicseg_ptr, char* genomicuc_ptr, gsnapdp_bool use_genomicseg_p,
    int cdna_direction, gsnapdp_bool watsonp, gsnapdp_bool jump_late_p, int maxpeelback, int nullgap,
    int extramaterial_paired, int extraband_paired, double defect_rate, gsnapdp_Pairpool_T pairpool,
    gsnapdp_Dynprog_T dynprogL, gsnapdp_Dynprog_T dynprogR);

/* --- optional additions (not in the reference) ---
 * The shim finds the packed genome on its own: Dynprog_setup's Genome_T
 * (Genome_blocks / Genome_totallength, genome.c:96-107) for an index genome,
 * or the Genome_create_blocks allocation given to Maxent_hr_setup for a user
 * segment.  This call overrides both, before the first DP
 * call: `blocks` and `nwords` = its length in UINT4 words (3 per 32 nt plus
 * any padding), `device` = HIP device index. */
int Gsnapdp_dropin_genome(const unsigned int* blocks, size_t nwords, int device);

/* Counters of this process's GPU work, per entry-point family in the order
 * gap (single / end5 / end3), splice junction, genome gap, cDNA gap, microexon,
 * MaxEnt (concurrent callers of any entry point are combined into shared
 * batches).
 * Gsnapdp_dropin_stats (the round-1 layout): out[0..5] = windows (or
 * positions) run, out[6] = gap batches, out[7] = the largest gap batch.
 * Writes min(n, 8) values; returns 8.
 * Gsnapdp_dropin_stats2: out[0..5] = windows, out[6..11] = GPU batches,
 * out[12..17] = the largest batch, per family.  Writes min(n, 18) values;
 * returns 18.
 * Gsnapdp_dropin_stats3: the same for seven families -- the six above, then
 * score_introns' paths (Gsnapdp_score_introns, one k_introns launch per batch):
 * out[0..6] = windows (paths for score_introns), out[7..13] = batches,
 * out[14..20] = the largest batch.  Writes min(n, 21) values; returns 21.
 * Each symbol keeps its layout; a caller that wants the newer counters calls the
 * newer symbol. */
int Gsnapdp_dropin_stats(unsigned long* out, int n);
int Gsnapdp_dropin_stats2(unsigned long* out, int n);
int Gsnapdp_dropin_stats3(unsigned long* out, int n);

/* ---- genome_hr subset (the reference's genome_hr.c is a missing blob;
 * gmap-gsnap_amd/csrc/genome_hr_sites.c): the setup calls gmap.c makes
 * (gmap.c:3801, 3810) and the splice-site dinucleotide queries of stage 2
 * (stage2.c:916-959, 1504-1919).  Host code, exported by the drop-in so a
 * gmap linked against it needs no genome_hr.o. */
void Genome_hr_setup(unsigned int* ref_blocks_in, unsigned int* snp_blocks_in,  /* genome_hr.h:12 */
                     gsnapdp_bool query_unk_mismatch_p_in, gsnapdp_bool genome_unk_mismatch_p_in,
                     gsnapdp_Mode_T mode_in);
void Genome_hr_user_setup(unsigned int* ref_blocks_in,                          /* genome_hr.h:17 */
                          gsnapdp_bool query_unk_mismatch_p_in,
                          gsnapdp_bool genome_unk_mismatch_p_in, gsnapdp_Mode_T mode_in);
int Genome_prev_donor_position(int pos, gsnapdp_Genomicpos_T genomicstart,      /* genome_hr.h:106 */
                               gsnapdp_Genomicpos_T genomicend, int pos5, gsnapdp_bool plusp);
int Genome_prev_acceptor_position(int pos, gsnapdp_Genomicpos_T genomicstart,   /* genome_hr.h:108 */
                                  gsnapdp_Genomicpos_T genomicend, int pos5, gsnapdp_bool plusp);
int Genome_prev_antidonor_position(int pos, gsnapdp_Genomicpos_T genomicstart,  /* genome_hr.h:110 */
                                   gsnapdp_Genomicpos_T genomicend, int pos5, gsnapdp_bool plusp);
int Genome_prev_antiacceptor_position(int pos,                                  /* genome_hr.h:112 */
                                      gsnapdp_Genomicpos_T genomicstart,
                                      gsnapdp_Genomicpos_T genomicend, int pos5, gsnapdp_bool plusp);

#ifdef __cplusplus
}
#endif

#endif /* GSNAPDP_DROPIN_H */
