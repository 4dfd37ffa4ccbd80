/*
 * gsnapdp.h -- batched C-ABI of the MI355X stage-3 gap-filling DP engine.
 *
 * This is the throughput boundary of the drop-in (the per-call reference
 * entry points Dynprog_* / Maxent_hr_* are declared in gsnapdp_dropin.h and
 * are thin wrappers over this API).  Every entry point is extern "C", takes
 * plain pointers and sizes, and carries no torch / HIP types.
 *
 * Reference interfaces replaced (GMAP/GSNAP 2012-07-03, src/):
 *   - Dynprog_single_gap   dynprog.c:4450-4572   (kind GSNAPDP_SINGLE_GAP)
 *   - Dynprog_end5_gap     dynprog.c:5094-5284   (kind GSNAPDP_END5_GAP)
 *   - Dynprog_end3_gap     dynprog.c:5556-5741   (kind GSNAPDP_END3_GAP)
 *   - Dynprog_microexon_int dynprog.c:7128-7432 (gsnapdp_micro_*)
 *   - Dynprog_end5_splicejunction dynprog.c:5412-5553 / Dynprog_end3_splicejunction
 *     :5869-6057 (gsnapdp_sj_*)
 *   - Maxent_hr_*_prob     maxent_hr.c:27217-27390 (gsnapdp_maxent_batch)
 *   - Genome_user_setup / Maxent_hr_setup (genome.c:9989, maxent_hr.c:27195):
 *     the packed genome blocks are uploaded once per context.
 *
 * Semantics of every window field follow the argument of the same name in
 * the reference entry point (dynprog.h:74-160).  A window never aliases
 * reference memory: query bytes live in a batch buffer addressed by `qpos`.
 */
#ifndef GSNAPDP_H
#define GSNAPDP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GSNAPDP_ABI_VERSION 2

/* Window kinds (one reference entry point each). */
enum {
  GSNAPDP_SINGLE_GAP = 0, /* Dynprog_single_gap, fwd fill, endpoint (L1,L2) */
  GSNAPDP_END5_GAP = 1,   /* Dynprog_end5_gap, rev fill + endpoint search   */
  GSNAPDP_END3_GAP = 2    /* Dynprog_end3_gap, fwd fill + endpoint search   */
};

/* Endalign_T, same order as dynprog.h:8. */
enum {
  GSNAPDP_QUERYEND_GAP = 0,
  GSNAPDP_QUERYEND_INDELS = 1,
  GSNAPDP_QUERYEND_NOGAPS = 2,
  GSNAPDP_BEST_LOCAL = 3
};

/* Mode_T, same order as mode.h. */
enum {
  GSNAPDP_MODE_STANDARD = 0,
  GSNAPDP_MODE_CMET_STRANDED = 1,
  GSNAPDP_MODE_CMET_NONSTRANDED = 2,
  GSNAPDP_MODE_ATOI_STRANDED = 3,
  GSNAPDP_MODE_ATOI_NONSTRANDED = 4
};

/* Comp characters written into pairs (comp.h:5-30). */
#define GSNAPDP_DYNPROG_MATCH_COMP '*'
#define GSNAPDP_AMBIGUOUS_COMP ':'
#define GSNAPDP_MISMATCH_COMP ' '
#define GSNAPDP_INDEL_COMP '-'
#define GSNAPDP_UNKNOWNJUMP (-1000000) /* dynprog.h:30 */
#define GSNAPDP_NEG_INFINITY (-1000000) /* dynprog.c:119 */

/* One DP window.  Field meaning = the reference argument of the same name.
 * For GSNAPDP_END5_GAP, offset1/offset2 are revoffset1/revoffset2 and the
 * query is read backwards from qpos (qpos = index of revsequence1[0], the
 * LAST query base, exactly like the reference's rev pointers). */
typedef struct gsnapdp_window {
  int32_t kind;
  int32_t length1;        /* query rows   */
  int32_t length2;        /* genome cols  */
  int32_t offset1;        /* query offset (or revoffset1)  */
  int32_t offset2;        /* genome offset (or revoffset2) */
  uint32_t chroffset;
  uint32_t chrhigh;
  uint32_t chrpos;
  uint32_t genomiclength;
  uint32_t qpos;          /* index of sequence1[0] in the batch query buffers */
  int32_t cdna_direction;
  int32_t extraband;      /* extraband_single / extraband_end */
  int32_t dynprogindex;   /* value of *dynprogindex at the call */
  int32_t maxlength1;     /* dynprog->maxlength1 of the Dynprog_T passed (dynprog.c:831-852) */
  int32_t maxlength2;     /* dynprog->maxlength2 */
  float defect_rate;      /* only its bin matters: <0.003 HIGHQ, <0.014 MEDQ, else LOWQ */
  uint8_t watsonp;
  uint8_t jump_late_p;
  uint8_t widebandp;      /* single gap only; end gaps always widen (dynprog.c:5189) */
  uint8_t endalign;       /* end gaps only */
} gsnapdp_window;

/* Per-window result.  finalscore/counts are the values the reference entry
 * point leaves in its out-parameters (all post-rules applied: end-gap
 * zeroing dynprog.c:5259/5715, NOGAPS rescoring :5243/:5700, too-long
 * sentinels :4511).  The traceback itself is returned as a compact op stream
 * (see below) that gsnapdp_expand turns into the reference's pair list,
 * push for push. */
typedef struct gsnapdp_result {
  int32_t finalscore;
  int32_t nmatches;
  int32_t nmismatches;
  int32_t nopens;
  int32_t nindels;
  int32_t bestr;          /* traceback start row */
  int32_t bestc;          /* traceback start column */
  int32_t nops;           /* ops written (<= capacity) */
  int32_t status;         /* 0 ok, 1 early return (NULL list), 2 op overflow, 3 zeroed end */
  int32_t length1;        /* effective lengths after end-gap chopping */
  int32_t length2;
  int32_t reserved;
} gsnapdp_result;

/* Op stream: one uint32 per op, in traceback order (from the endpoint back
 * towards (0,0)).  Low 2 bits = type, high 30 bits = count. */
enum {
  GSNAPDP_OP_DIAG = 0,     /* `count` consecutive diagonal steps (pairs pushed unless genome '*') */
  GSNAPDP_OP_HDASH = 1,    /* genome skip of `count`, pushed as INDEL pairs (add_genomeskip dashes) */
  GSNAPDP_OP_HGAP = 2,     /* genome skip of `count` replaced by one gapholder (intron-like) */
  GSNAPDP_OP_VSKIP = 3     /* query skip of `count` (add_queryskip) */
};
#define GSNAPDP_OP(type, count) ((uint32_t)(type) | ((uint32_t)(count) << 2))
#define GSNAPDP_OP_TYPE(op) ((op) & 3u)
#define GSNAPDP_OP_COUNT(op) ((op) >> 2)

/* One pair of the output list (the DP-set fields of Pair_T, pairdef.h:9-49,
 * as written by Pairpool_push / Pairpool_push_gapholder, pairpool.c:169,352). */
typedef struct gsnapdp_pair {
  int32_t querypos;
  int32_t genomepos;
  int32_t queryjump;      /* gapholder only */
  int32_t genomejump;     /* gapholder only */
  int32_t dynprogindex;
  char cdna;
  char comp;
  char genome;
  uint8_t gapp;           /* bit 0: a gapholder (gapp); bit 1: knowngapp, i.e. pushed with
                           * knownp = true (Pairpool_push_gapholder, pairpool.c:383-390) */
} gsnapdp_pair;

/* One intron window (Dynprog_genome_gap, dynprog.c:4798-5061).  The query
 * is sequence1[0..length1) at qpos; genome flanks are addressed through
 * offset2L (left, fwd) and revoffset2R (right, rev) like the reference.
 *
 * Known splice sites (a splicing IIT given to Dynprog_setup, dynprog.c:350;
 * bridge_intron_gap :3375-3697, :4084-4101) are described by known_mode:
 *   GSNAPDP_KNOWN_NONE        splicing_iit == NULL
 *   GSNAPDP_KNOWN_REWARD      novelsplicingp: known sites add
 *                             KNOWN_SPLICESITE_REWARD (20) to the flank scores
 *                             and have probability 1.0
 *   GSNAPDP_KNOWN_SITES       site-level IIT (donor/acceptor types) without
 *                             novel splicing: rewards, and the result requires
 *                             both chosen sites to be known (:4090-4096)
 *   GSNAPDP_KNOWN_INTRONS     intron-level IIT without novel splicing: only
 *                             known introns are candidates (:3552-3697)
 * For every mode but NONE the caller places a known-site record right after
 * the window's query rows, at query[qpos + length1]:
 *   uint8  left_known[length2L]    1 where the reference sets left_known[cL]
 *   uint8  right_known[length2R]   1 where it sets right_known[cR]
 *   uint16 npairs (little endian)  KNOWN_INTRONS: the (cL, cR) pairs, both
 *   uint16 cL, cR  x npairs        flagged, for which the reference's
 *                                  IIT_exists_with_divno_signed holds
 * (gsnapdp_known_site_record builds it from a gsnapdp_iit, below.) */
enum { GSNAPDP_KNOWN_NONE = 0, GSNAPDP_KNOWN_REWARD = 1, GSNAPDP_KNOWN_SITES = 2,
       GSNAPDP_KNOWN_INTRONS = 3 };
typedef struct gsnapdp_ggap_window {
  int32_t length1, length2L, length2R;
  int32_t offset1, offset2L, revoffset2R;
  uint32_t chroffset, chrhigh, chrpos, genomiclength;
  uint32_t qpos;
  int32_t cdna_direction, extraband_paired, maxpeelback, score_threshold, dynprogindex;
  int32_t maxlength1, maxlength2;
  float defect_rate;
  uint8_t watsonp, jump_late_p, halfp, finalp;
  uint8_t use_probabilities_p, splicingp, known_mode, pad1;
} gsnapdp_ggap_window;

/* Out-parameters of Dynprog_genome_gap for one window. */
typedef struct gsnapdp_ggap_result {
  int32_t finalscore, new_leftgenomepos, new_rightgenomepos;
  int32_t nmatches, nmismatches, nopens, nindels, exonhead, introntype;
  int32_t dynprogindex;   /* *dynprogindex after the call */
  int32_t returned_null;  /* 1 if the reference returns NULL */
  int32_t bridge_ok;      /* 0: probability mode found no candidate (reference UB, excluded) */
  double left_prob, right_prob;
} gsnapdp_ggap_result;

/* Where window i's tracebacks start and how its op stream splits: the right
 * flank's ops (reversed fill, traced from (brR, bcR)) come first, then the
 * left flank's (from (brL, bcL)); gsnapdp_ggap_expand replays them.
 * status: 0 ok, 1 early return, 2 op overflow, 4 unsupported (the reference
 * aborts or reads outside its matrices, or no MaxEnt tables were loaded for a
 * window that needs them, 6 kernel invariant failed).  npairs = length of the
 * returned list (0 = NULL).  bridge_accepted = 1 when bridge_intron_gap took a
 * candidate and accepted it (:4084-4101): the new intron ends, exonhead and
 * probabilities are then the reference's out-parameters (0: rejected or early). */
typedef struct gsnapdp_ggap_trace {
  int32_t brL, bcL, brR, bcR;
  int32_t nops_right, nops_left;
  int32_t status;
  int32_t npairs;
  int32_t bridge_accepted;
  int32_t reserved;
} gsnapdp_ggap_trace;

/* One cDNA-insertion window (Dynprog_cdna_gap, dynprog.c:4578-4793).  The
 * genome part (length2, from offset2) forms the rows of both fills, the query
 * the columns: the left fill reads sequence1L = query[qposL ...] forwards, the
 * right fill reads revsequence1R backwards from query[qposR]. */
typedef struct gsnapdp_cgap_window {
  int32_t length1L, length1R, length2;
  int32_t offset1L, revoffset1R, offset2;
  uint32_t chroffset, chrhigh, chrpos, genomiclength;
  uint32_t qposL, qposR;
  int32_t cdna_direction, extraband_paired, dynprogindex, maxlength1, maxlength2;
  float defect_rate;
  uint8_t watsonp, jump_late_p, pad0, pad1;
} gsnapdp_cgap_window;

/* Out-parameters of Dynprog_cdna_gap and where its tracebacks start.
 * status: 0 ok, 1 early return (NULL), 2 op overflow, 4 unsupported, 5 the
 * bridge found no candidate (the reference then traces back from
 * uninitialised indices; excluded).  finalscore_set: 0 on the early returns,
 * which leave *finalscore untouched.  incompletep: 1 if the gapholder was
 * pushed (the only case in which the reference writes *incompletep). */
typedef struct gsnapdp_cgap_result {
  int32_t finalscore, dynprogindex, incompletep, returned_null;
  int32_t status, npairs, finalscore_set, insert_pairs;
  int32_t brL, bcL, brR, bcR;
  int32_t nops_right, nops_left, reserved0, reserved1;
} gsnapdp_cgap_result;

/* ---------------------------------------------------------------- context */

typedef struct gsnapdp_ctx gsnapdp_ctx;

/* Create a context on HIP device `device`.  `blocks` are the reference's
 * packed genome blocks (3 x uint32 per 32 nt: high, low, flags; genome.c:9325)
 * of `nblocks_u32` words; they are copied to HBM once.  The host pointer is
 * borrowed (kept for gsnapdp_expand) and must outlive the context.
 * `mode` is the Mode_T given to Dynprog_init (dynprog.c:1339).
 * Returns NULL on failure (message via gsnapdp_last_error). */
gsnapdp_ctx *gsnapdp_create(int device, const uint32_t *blocks, size_t nblocks_u32, int mode);
void gsnapdp_destroy(gsnapdp_ctx *ctx);
const char *gsnapdp_last_error(void);

/* Device id the library was built for / found ("gfx950"). */
const char *gsnapdp_device_arch(gsnapdp_ctx *ctx);

/* ------------------------------------------------------------ host batches
 * Fill + endpoint + traceback for `n` windows.  Inputs are host buffers;
 * this call copies them to HBM, runs the kernels on the context stream and
 * copies results back (synchronous; concurrent calls on one context run one
 * after the other).  Only the ops each window wrote cross PCIe (compacted on
 * the device, scattered to op_offsets on the host).  Buffers from
 * gsnapdp_host_alloc avoid the driver's pageable staging.  `op_offsets[i]` is where window i's
 * op stream starts in `ops`; window i may write at most
 * op_offsets[i+1]-op_offsets[i] ops (op_offsets has n+1 entries).
 * Returns 0 on success. */
int gsnapdp_run_host(gsnapdp_ctx *ctx, const gsnapdp_window *windows, int n,
                     const char *query, const char *query_uc, size_t query_bytes,
                     gsnapdp_result *results, uint32_t *ops, const int64_t *op_offsets);

/* ---------------------------------------------------------- device batches
 * Same computation with every buffer already resident in HBM (device
 * pointers); asynchronous on `stream` (a hipStream_t, NULL = context stream).
 * This is the path the benchmark times. */
int gsnapdp_run_device(gsnapdp_ctx *ctx, const gsnapdp_window *d_windows, int n,
                       const char *d_query, const char *d_query_uc,
                       gsnapdp_result *d_results, uint32_t *d_ops, const int64_t *d_op_offsets,
                       void *stream);

/* Device scratch needed by gsnapdp_run_device for n windows whose largest
 * dimensions are max_length1 x max_length2 (bytes).  Scratch is owned by
 * the context and grown on demand; this is informational. */
size_t gsnapdp_scratch_bytes(gsnapdp_ctx *ctx, int n, int max_length1, int max_length2);

/* Compact a finished batch's op streams for the multi-GPU gather (SURVEY.md
 * 8(e): result records + compact op streams are all that leave a GPU).
 * Window i's min(results[i].nops, op_offsets[i+1]-op_offsets[i]) ops are
 * written consecutively, windows in batch order, to d_out, so a receiver
 * rebuilds every window's offset from the nops column (exclusive prefix sum).
 * d_header (2 x int64, device) receives {total ops, overflow}: overflow = 1
 * when total > out_cap, in which case only the windows that fit entirely
 * were written.  Asynchronous on `stream` (NULL = context stream); calls on
 * one context run one after another on the GPU whatever streams they are
 * issued on (each waits for the previous call's launch: they share the
 * context's look-back status words).  The other device entry points of one
 * context share its scratch too: issue them on one stream, or order the
 * streams yourself. */
int gsnapdp_compact_ops_device(gsnapdp_ctx *ctx, const gsnapdp_result *d_results, int n,
                               const uint32_t *d_ops, const int64_t *d_op_offsets, uint32_t *d_out,
                               int64_t out_cap, int64_t *d_header, void *stream);

/* Page-locked host memory (hipHostMalloc) for batch buffers handed to the
 * *_run_host entry points: copies from / to it run as DMA without staging.
 * Returns NULL on failure.  Free with gsnapdp_host_free. */
void *gsnapdp_host_alloc(size_t bytes);
void gsnapdp_host_free(void *p);

/* Synchronise the context stream. */
int gsnapdp_sync(gsnapdp_ctx *ctx);

/* Per-kernel timing with HIP events recorded on the stream each kernel is
 * launched on.  After gsnapdp_profile(ctx, 1), every run_device records an
 * event pair around each of its launches; gsnapdp_profile_read synchronises
 * and ADDS the last run's per-stage milliseconds into ms[0..nstages).
 * Returns the number of stages (see gsnapdp_stage_name), or -1. */
int gsnapdp_profile(gsnapdp_ctx *ctx, int enable);
int gsnapdp_profile_read(gsnapdp_ctx *ctx, double *ms, int nstages);
const char *gsnapdp_stage_name(int stage);

/* Test hook (no reference counterpart): the register-band bucketing of the last
 * single/end-gap batch on this context (k_plan + its last-block scan +
 * k_scatter).  Synchronises the context stream, then copies keys[0..n) (each
 * window's bucket key, -1 for a window not on k_fill), the first min(nperm,
 * perm_cap) entries of perm (a window index, or -1 for a bucket's padding),
 * class_start[0..ncls] and the class wave sizes (windows per wave-task) into
 * class_wave[0..ncls).  Returns nperm (= class_start[ncls]), or -1; ncls must
 * be the number of band classes, gsnapdp_debug_buckets(ctx, 0, ...) with all
 * pointers NULL returns it. */
int64_t gsnapdp_debug_buckets(gsnapdp_ctx *ctx, int n, int32_t *keys, int32_t *perm, int64_t perm_cap,
                              int32_t *class_start, int32_t *class_wave, int ncls);

/* ------------------------------------------------------------ maxent_hr
 * Batched Maxent_hr_{donor,acceptor,antidonor,antiacceptor}_prob
 * (maxent_hr.c:27217-27390) on the context genome.  model[i] in 0..3 =
 * donor, acceptor, antidonor, antiacceptor.  Host buffers, synchronous. */
enum { GSNAPDP_DONOR = 0, GSNAPDP_ACCEPTOR = 1, GSNAPDP_ANTIDONOR = 2, GSNAPDP_ANTIACCEPTOR = 3 };
int gsnapdp_maxent_host(gsnapdp_ctx *ctx, const uint8_t *model, const uint32_t *splice_pos,
                        const uint32_t *chroffset, double *out, int n);

/* GSNAP's splice-site scans (stage1hr.c:6300-7046, 8703-8976): every candidate
 * splice position of a read's segment pair asks Maxent_hr_* at
 * segment_left + splice_pos (Genomicpos_T arithmetic) unless the site is known
 * (knowni >= 0: probability 1.0, no model run).  Many reads' candidates in one
 * call: the unknown sites go to one k_maxent launch.  The scans' threshold logic
 * (the mismatch counts and sufficient_splice_prob_local) stays the caller's. */
typedef struct gsnapdp_scan_site {
  uint32_t segment_left;  /* segmenti_left / segmentj_left */
  int32_t splice_pos;
  uint32_t chroffset;
  int32_t knowni;         /* donori_knowni[i] etc.: >= 0 for a known site */
  int32_t model;          /* GSNAPDP_DONOR / _ACCEPTOR / _ANTIDONOR / _ANTIACCEPTOR */
} gsnapdp_scan_site;
int gsnapdp_scan_site_probs(gsnapdp_ctx *ctx, const gsnapdp_scan_site *sites, int n, double *probs);

/* ------------------------------------------------------- score_introns
 * stage3.c:7935-8162 for many paths at once: each path's introns get their
 * donor / acceptor MaxEnt probabilities (1.0 for a site the splicing IIT
 * knows), summed in path order and averaged, and the path's bad-intron count
 * (a canonical intron with both probabilities below 0.9; the reference SETS it
 * to 1 for cdna_direction +1 and counts it for -1, :8048 / :8119).
 *
 * A path's pairs, as score_introns reads them (Pair_T, pairdef.h:9-49), in
 * list order; gsnapdp_path_introns picks the introns out of them (the gaps
 * with genomejump > queryjump + MININTRONLEN_FINAL that are neither past
 * nullgap nor query-heavy, :7960-8146).  An intron's leftpair is the pair
 * after its gap in the list, its rightpair the pair before it. */
typedef struct gsnapdp_path_pair {
  uint32_t genomepos;
  int32_t queryjump, genomejump;
  uint8_t gapp, knowngapp, comp, pad;
} gsnapdp_path_pair;
typedef struct gsnapdp_intron {
  uint32_t left_genomepos, right_genomepos;  /* leftpair->genomepos, rightpair->genomepos */
  int32_t path;                              /* owning path; a path's introns are consecutive, in list order */
  uint8_t comp, knowngapp;                   /* the gap pair's comp and knowngapp */
  uint8_t known_donor, known_acceptor;       /* the splicing IIT has the site (0 without an IIT) */
} gsnapdp_intron;
typedef struct gsnapdp_intron_path {
  uint32_t chroffset, chrpos;
  int32_t genomiclength, cdna_direction, watsonp;
  int32_t first_intron, nintrons, pad;
} gsnapdp_intron_path;
typedef struct gsnapdp_intron_scores {
  double avg_donor_score, avg_acceptor_score;
  int32_t nbadintrons, nintrons;
} gsnapdp_intron_scores;
/* Host-only (no GPU): the introns of one path's pairs, tagged with `path`.
 * Returns how many (at most cap are written), or -1. */
int gsnapdp_path_introns(const gsnapdp_path_pair *pairs, int npairs, int nullgap, int path,
                         gsnapdp_intron *out, int cap);
/* One launch for every path (needs gsnapdp_load_maxent_tables).  The device
 * form is asynchronous on `stream`. */
int gsnapdp_score_introns_device(gsnapdp_ctx *ctx, const gsnapdp_intron_path *d_paths, int npaths,
                                 const gsnapdp_intron *d_introns, gsnapdp_intron_scores *d_out,
                                 void *stream);
int gsnapdp_score_introns_host(gsnapdp_ctx *ctx, const gsnapdp_intron_path *paths, int npaths,
                               const gsnapdp_intron *introns, int nintrons, gsnapdp_intron_scores *out);
int gsnapdp_maxent_device(gsnapdp_ctx *ctx, const uint8_t *d_model, const uint32_t *d_splice_pos,
                          const uint32_t *d_chroffset, double *d_out, int n, void *stream);

/* --------------------------------------------------------- genome gaps
 * Dynprog_genome_gap (dynprog.c:4798-5061) for `n` intron windows: both flank
 * fills, bridge_intron_gap (score or probability mode), the MaxEnt site
 * probabilities and both tracebacks.  Window i may write at most
 * op_offsets[i+1]-op_offsets[i] ops; 2*length1 + length2L + length2R + 4 always
 * suffices.  Windows with use_probabilities_p or finalp need the MaxEnt tables
 * (gsnapdp_load_maxent_tables).  The device form is asynchronous on `stream`;
 * the host form copies in, runs and copies out. */
int gsnapdp_ggap_run_device(gsnapdp_ctx *ctx, const gsnapdp_ggap_window *d_windows, int n,
                            const char *d_query, const char *d_query_uc,
                            gsnapdp_ggap_result *d_results, gsnapdp_ggap_trace *d_traces,
                            uint32_t *d_ops, const int64_t *d_op_offsets, void *stream);
int gsnapdp_ggap_run_host(gsnapdp_ctx *ctx, const gsnapdp_ggap_window *windows, int n,
                          const char *query, const char *query_uc, size_t query_bytes,
                          gsnapdp_ggap_result *results, gsnapdp_ggap_trace *traces, uint32_t *ops,
                          const int64_t *op_offsets);
/* Replay window i's two op streams into the reference's returned list (the
 * right flank's pairs, the gapholder, then the left flank's, dynprog.c:5000-5058).
 * Writes at most `cap` pairs; returns the list length (0 for NULL) or -1. */
int gsnapdp_ggap_expand(gsnapdp_ctx *ctx, const gsnapdp_ggap_window *w,
                        const gsnapdp_ggap_result *res, const gsnapdp_ggap_trace *trace,
                        const uint32_t *ops, const char *query, const char *query_uc,
                        gsnapdp_pair *pairs, int cap);

/* ----------------------------------------------------------- cDNA gaps
 * Dynprog_cdna_gap (dynprog.c:4578-4793) for `n` windows: both genome-row
 * fills, bridge_cdna_gap and both tracebacks.  Op capacity per window:
 * length1L + length1R + 2*length2 + 4.  Expansion rebuilds the list; the
 * INSERT_PAIRS branch reads `sequence2` (the reference's genomic-segment
 * argument, indexed from offset2), or the context genome when it is NULL. */
int gsnapdp_cgap_run_device(gsnapdp_ctx *ctx, const gsnapdp_cgap_window *d_windows, int n,
                            const char *d_query, const char *d_query_uc,
                            gsnapdp_cgap_result *d_results, uint32_t *d_ops,
                            const int64_t *d_op_offsets, void *stream);
int gsnapdp_cgap_run_host(gsnapdp_ctx *ctx, const gsnapdp_cgap_window *windows, int n,
                          const char *query, const char *query_uc, size_t query_bytes,
                          gsnapdp_cgap_result *results, uint32_t *ops, const int64_t *op_offsets);
int gsnapdp_cgap_expand(gsnapdp_ctx *ctx, const gsnapdp_cgap_window *w,
                        const gsnapdp_cgap_result *res, const uint32_t *ops, const char *query,
                        const char *query_uc, const char *sequence2, gsnapdp_pair *pairs, int cap);

/* --------------------------------------------------- splice-junction ends
 * Dynprog_end5_splicejunction (dynprog.c:5412-5553, kind GSNAPDP_END5_GAP) and
 * Dynprog_end3_splicejunction (:5869-6057, kind GSNAPDP_END3_GAP): an end gap
 * against a caller-built genomic segment (the splice junction of
 * Dynprog_make_splicejunction_5/3, `use_genomicseg_p`), endpoint on the last
 * query row (find_best_endpoint_to_queryend_indels :2293), and the traceback
 * split at column `contlength` (traceback_local :2874) around a known
 * gapholder.  The segment lives in the batch query buffers: query[spos...]
 * holds sequence2 (read forwards for END3, backwards from revsequence2[0] for
 * END5, like the query) and query_uc[spos...] sequenceuc2.  The reference
 * never reads chroffset / chrpos here, so the record does not carry them.
 * Segments must consist of A C G T N (what Genome_fill_buffer_blocks_noterm
 * writes, genome.c:8912-8960); other bytes give status UNSUPPORTED. */
typedef struct gsnapdp_sj_window {
  int32_t kind;            /* GSNAPDP_END5_GAP or GSNAPDP_END3_GAP */
  int32_t length1, length2;
  int32_t offset1;         /* offset1 (END3) or revoffset1 (END5) */
  int32_t offset2_anchor;  /* (rev)offset2_anchor: genome offset of the second traceback part */
  int32_t offset2_far;     /* (rev)offset2_far: genome offset of the first part */
  int32_t contlength;      /* endc of the first traceback part */
  uint32_t qpos;           /* sequence1[0] / revsequence1[0] in the query buffers */
  uint32_t spos;           /* sequence2[0] / revsequence2[0] in the query buffers */
  int32_t cdna_direction, extraband_end, dynprogindex, maxlength1, maxlength2;
  float defect_rate;
  uint8_t watsonp, jump_late_p, pad0, pad1;
} gsnapdp_sj_window;

/* Results use gsnapdp_result: finalscore = the reference's recomputed
 * 3*nmatches - 5*nmismatches + nopens*open + nindels*extend (:5541 / :6045),
 * status 1 (early return, NULL list) when a length is <= 0 or above the
 * workspace maxima (:5446-5461), reserved = *dynprogindex after the call.
 * Op capacity per window: length1 + length2 + 2 (as gsnapdp_run_*). */
int gsnapdp_sj_run_device(gsnapdp_ctx *ctx, const gsnapdp_sj_window *d_windows, int n,
                          const char *d_query, const char *d_query_uc, gsnapdp_result *d_results,
                          uint32_t *d_ops, const int64_t *d_op_offsets, void *stream);
int gsnapdp_sj_run_host(gsnapdp_ctx *ctx, const gsnapdp_sj_window *windows, int n,
                        const char *query, const char *query_uc, size_t query_bytes,
                        gsnapdp_result *results, uint32_t *ops, const int64_t *op_offsets);
/* The list the entry point returns: part one (columns > contlength, genome
 * offset offset2_far), the known gapholder (queryjump 0, genomejump
 * anchor - far for END5, far - anchor for END3), part two (offset2_anchor),
 * then INDEL stripping and the END5 List_reverse (:5543-5553 / :6047-6057). */
int gsnapdp_sj_expand(gsnapdp_ctx *ctx, const gsnapdp_sj_window *w, const gsnapdp_result *res,
                      const uint32_t *ops, const char *query, const char *query_uc,
                      gsnapdp_pair *pairs, int cap);

/* ------------------------------------------------------------ microexons
 * Dynprog_microexon_int (dynprog.c:7128-7432, non-PMAP, use_genomicseg_p
 * false as every caller passes it, stage3.c:9865): splice a 3..12 nt
 * microexon into an intron gap.  The left / right boundaries (at most one
 * mismatch, :7241-7290), every GT..AG (CT..AC) pair (cL, cR), every exact hit
 * of the middle query segment in the intron (BoyerMoore_nt, boyer-moore.c:384,
 * hits visited last-found first), the flank test and the MaxEnt site
 * probabilities; the best candidate by prob2 + prob3 under the reference's
 * strict `>` in its scan order.  The query search segment is sequence1 /
 * sequenceuc1 at qpos; the pairs read queryseq / queryuc from offset1 on,
 * staged at ppos (ppos = qpos when sequence1 == &queryseq[offset1], as in
 * stage3.c:5915).  Needs the MaxEnt tables. */
typedef struct gsnapdp_micro_window {
  int32_t length1, offset1, offset2L, revoffset2R, cdna_direction, dynprogindex;
  uint32_t chroffset, chrhigh, chrpos, genomiclength;
  uint32_t qpos, ppos;
  float defect_rate;
  uint8_t watsonp, pad0, pad1, pad2;
} gsnapdp_micro_window;

/* Out-parameters of Dynprog_microexon_int and where its pairs come from.
 * status: 0 ok, 4 unsupported (the reference aborts: cdna_direction 0 or
 * span <= 0, :7204/:7224; or no MaxEnt tables).  found = 1 when a list is
 * returned; then the pairs are: bestcL left-segment pairs, a gapholder, the
 * middle pairs from genome column offset2M (the LAST hit examined, not the
 * best one: dynprog.c:7412-7413), a gapholder, bestcR right-segment pairs;
 * gsnapdp_micro_expand rebuilds them. */
typedef struct gsnapdp_micro_result {
  double bestprob2, bestprob3;
  int32_t microintrontype, dynprogindex, found, status;
  int32_t bestcL, bestcR, middlelength, offset2M;
} gsnapdp_micro_result;

int gsnapdp_micro_run_device(gsnapdp_ctx *ctx, const gsnapdp_micro_window *d_windows, int n,
                             const char *d_query, const char *d_query_uc,
                             gsnapdp_micro_result *d_results, void *stream);
int gsnapdp_micro_run_host(gsnapdp_ctx *ctx, const gsnapdp_micro_window *windows, int n,
                           const char *query, const char *query_uc, size_t query_bytes,
                           gsnapdp_micro_result *results);
/* The list Dynprog_microexon_int returns (make_microexon_pairs_double,
 * :6949-7055: the list head is the last pair pushed).  Returns its length
 * (0 = NULL) or -1. */
int gsnapdp_micro_expand(gsnapdp_ctx *ctx, const gsnapdp_micro_window *w,
                         const gsnapdp_micro_result *res, const char *query, const char *query_uc,
                         gsnapdp_pair *pairs, int cap);

/* -------------------------------------------------------- splicing IIT
 * The splicing IIT gmap / gsnap hand to Dynprog_setup and Stage3_setup
 * (gmap.c:3281-3318, 3721-3837) as the four queries the DP path makes of it:
 *   typed  IIT_exists_with_divno_typed_signed (iit-read.c:4011): an interval
 *          with low == x, high == y, the type (GSNAPDP_DONOR / GSNAPDP_ACCEPTOR:
 *          the IIT's "donor" / "acceptor" type ints) and the sign;
 *   low    IIT_low_exists_signed_p (:3770): an interval whose low end is x;
 *   high   IIT_high_exists_signed_p (:3808): an interval whose high end is x;
 *   exact  IIT_exists_with_divno_signed (:3973): low == x, high == y, sign.
 * chrnum is the caller's chromosome number (the reference maps it to the IIT's
 * division through its divint crosstable).  site_level: the IIT has donor and
 * acceptor types (a splice-sites file, gmap.c:3730), else it holds introns.
 * The callbacks may be called from several threads at once.
 * gsnapdp_iit_from_intervals builds one over intervals as iit_store writes them
 * (start..end; start > end is the minus sign, interval.c:22-40). */
typedef struct gsnapdp_iit {
  void *user;
  int32_t site_level, pad;
  int (*typed)(void *user, int chrnum, uint32_t x, uint32_t y, int type, int sign);
  int (*low)(void *user, int chrnum, uint32_t x, int sign);
  int (*high)(void *user, int chrnum, uint32_t x, int sign);
  int (*exact)(void *user, int chrnum, uint32_t x, uint32_t y, int sign);
} gsnapdp_iit;
typedef struct gsnapdp_iit_interval {
  int32_t chrnum;
  uint32_t start, end;
  int32_t type; /* -1 none (an intron), GSNAPDP_DONOR, GSNAPDP_ACCEPTOR */
} gsnapdp_iit_interval;
gsnapdp_iit *gsnapdp_iit_from_intervals(const gsnapdp_iit_interval *intervals, int n);
void gsnapdp_iit_free(gsnapdp_iit *iit);
/* Host-only: one genome-gap window's known-site record (gsnapdp_ggap_window
 * above), asked of `iit` exactly where bridge_intron_gap asks
 * (dynprog.c:3375-3550, 3598-3612).  Writes *len bytes (length2L + length2R
 * + 2 + 4 * known introns) and returns the window's known_mode (REWARD with
 * novelsplicingp, else SITES or INTRONS); or -1 when cap is short, with *len
 * the bytes the record needs (-1 for an error). */
int gsnapdp_known_site_record(const gsnapdp_iit *iit, int novelsplicingp, int chrnum, uint32_t chrpos,
                              uint32_t genomiclength, int offset2L, int revoffset2R, int length2L, int length2R,
                              int cdna_direction, int watsonp, char *rec, int cap, int *len);
/* Host-only: score_introns' known-site verdicts for `n` introns of paths on
 * chromosome chrnum (stage3.c:7995-8116): intron[i].known_donor /
 * known_acceptor from the IIT, asked in the reference's order. */
int gsnapdp_introns_known(const gsnapdp_iit *iit, int chrnum, uint32_t chrpos, int genomiclength,
                          int cdna_direction, int watsonp, gsnapdp_intron *introns, int n);

/* -------------------------------------------------- stage-3 intron pass
 * build_pairs_introns (stage3.c:7735-7901) for many paths at once.  Each
 * path's gaps are taken in list order, as the reference's loop takes them:
 * classified (past nullgap, cDNA gap, genome gap, short intron, single gap),
 * peeled (peel_leftward / peel_rightward, :4887-5378), filled by the gap
 * families above -- traverse_single_gap (:5381) with its accept test,
 * traverse_cdna_gap (:5518), traverse_genome_gap (:5633) with the SHORTCUT
 * canonical-intron skip, the probability-mode re-run of a final pass (:5828)
 * and the microexon fallback (:5915) -- and then kept, or put back.  All paths
 * advance together: every round gathers the one pending DP window of each
 * path and runs one batch per gap family (gsnapdp_*_run_host), so a pass over
 * P paths with at most G sequential DP calls per path costs G rounds.
 *
 * A path is the reference's List_T of Pair_T in list order (path->first first,
 * i.e. the alignment reversed, as insert_gapholders leaves it); each pair
 * carries the fields the pass reads or writes.  The returned list is written
 * in list order; `src` names the input pair (index within its path) that a
 * returned cell holds, -1 for a pair the pass made.  With a splicing IIT
 * (`iit`, as Dynprog_setup / Stage3_setup got it) every genome-gap window
 * carries its known-site record; NULL for none.  Genome characters come from
 * the context genome.  Needs the MaxEnt tables when a call has finalp
 * (probability re-runs, microexons). */
typedef struct gsnapdp_s3_pair {
  int32_t querypos, genomepos, queryjump, genomejump, dynprogindex;
  int32_t src;
  char cdna, comp, genome;
  uint8_t flags;  /* GSNAPDP_S3_GAPP | GSNAPDP_S3_KNOWNGAPP | GSNAPDP_S3_DISALLOWED |
                   * GSNAPDP_S3_SHORTEXON | GSNAPDP_S3_END_INTRON */
} gsnapdp_s3_pair;
/* Pair_T's gapp, knowngapp, disallowedp, shortexonp (set by Smooth_pairs_by_size,
 * read by build_pairs_dualintrons) and end_intron_p (set by insert_gapholders on
 * the first and last gap, stage3.c:902-916) */
enum {
  GSNAPDP_S3_GAPP = 1,
  GSNAPDP_S3_KNOWNGAPP = 2,
  GSNAPDP_S3_DISALLOWED = 4,
  GSNAPDP_S3_SHORTEXON = 8,
  GSNAPDP_S3_END_INTRON = 16
};
/* gsnapdp_s3_call.ub bits */
enum { GSNAPDP_S3_UB_INTRONLEN = 1, GSNAPDP_S3_UB_DUAL = 2 };
/* gsnapdp_s3_call.pass: which of path_compute's DP passes the call is */
enum {
  GSNAPDP_S3_INTRONS = 0,     /* build_pairs_introns (stage3.c:7735), passes 3c / 6 */
  GSNAPDP_S3_SINGLES = 1,     /* build_pairs_singles (:7454), passes 2A / 2C / 7C */
  GSNAPDP_S3_END5 = 2,        /* build_pairs_end5 (:7351) with extendp, passes 8 / 9a / 10 */
  GSNAPDP_S3_END3 = 3,        /* build_path_end3 (:7236) with extendp, passes 8 / 9b / 10 */
  GSNAPDP_S3_DUALINTRONS = 4, /* build_pairs_dualintrons (:7592), pass 3b */
  GSNAPDP_S3_DUALBREAKS = 5   /* build_dual_breaks (:7149), pass 5: the gaps solvable as single gaps
                               * (traverse_single_gap with forcep); a dual break that needs
                               * traverse_dual_break's stage-2 realignment gives status -1 */
};

/* One build_pairs_introns call: its arguments (the query bytes at query[qpos],
 * querylength of them; the three Dynprog_T workspaces' limits, L, M, R), its
 * in/out counters, and (written by the pass) the returned list's extent in
 * pairs_out, shiftp / incompletep and a status (0, or -1 when the reference
 * would abort on the path: a window outside its domain). */
typedef struct gsnapdp_s3_call {
  int32_t first_pair, npairs;  /* the path in pairs_in */
  int32_t first_out, nout;     /* written: the returned list in pairs_out */
  int32_t qpos, querylength;
  uint32_t chroffset, chrhigh, chrpos;
  int32_t chrnum, genomiclength, cdna_direction;
  int32_t watsonp, jump_late_p, finalp, use_genomicseg_p;
  int32_t maxpeelback, nullgap, extramaterial_paired, extraband_single, extraband_paired, close_indels_mode;
  double defect_rate;
  int32_t maxlength1[3], maxlength2[3];  /* dynprogL, dynprogM, dynprogR */
  int32_t in_minor, in_major, in_nintrons, in_nnonintrons, in_intronlen, in_nonintronlen;
  int32_t out_minor, out_major, out_nintrons, out_nnonintrons, out_intronlen, out_nonintronlen;
  int32_t shiftp, incompletep;       /* written (INTRONS); DUALBREAKS: shiftp = *dual_break_p */
  int32_t novelsplicingp, splicingp;  /* Stage3_setup's module flags (stage3.c:238-239) */
  int32_t status;                     /* written: 0, or -1 (the path is left out, nout = 0) */
  int32_t ub;                         /* written: GSNAPDP_S3_UB_INTRONLEN when out_intronlen /
                                       * out_nonintronlen took traverse_genome_gap's uninitialised
                                       * new_left/rightgenomepos (stage3.c:5651; an early-returning
                                       * Dynprog_genome_gap leaves them unwritten): the reference's own
                                       * value is stack garbage there, and differs between runs */
  int32_t pass;                       /* GSNAPDP_S3_*: which pass.  SINGLES, END5 and END3 step
                                       * dynprogindex_minor (in_minor / out_minor), DUALINTRONS
                                       * dynprogindex_major (in_major / out_major); they read neither
                                       * finalp nor the intron counters (passed through).  END5 gets the
                                       * alignment as `pairs` (ascending querypos), END3 as `path`. */
  int32_t endalign;                   /* END5 / END3: GSNAPDP_QUERYEND_GAP, _NOGAPS or BEST_LOCAL */
  int32_t extramaterial_end, extraband_end;  /* END5 / END3 */
  int32_t splicesitesp;               /* END5 / END3: Stage3_setup got splice sites (the
                                       * Dynprog_end5/3_known branch, not served: status -1) */
  int32_t invocation;                 /* the caller's tag, passed through (golden records: which
                                       * path_compute call of gmap the pass call belongs to) */
  double ref_seconds;                 /* golden records: the reference's own call time (ignored) */
} gsnapdp_s3_call;

typedef struct gsnapdp_s3_stats {
  int32_t rounds;
  int32_t windows[4];   /* single gap, genome gap (score and probability), cDNA gap, microexon */
  int32_t batches[4];
  int32_t undefined;    /* probability re-runs with no qualifying candidate: the reference reads
                         * uninitialised indices (dynprog.c:4055); taken as NULL here */
  int32_t failed;       /* paths with status -1 */
  int32_t pad;
  double seconds[3];    /* wall time: the host's (packing, launches, peels, traversals,
                         * expansion), the time it waited for a batch, the whole pass */
  int64_t new_pairs;    /* pairs the pass made among the returned lists (the new_out a compact
                         * pass needs; written also when new_out was too small) */
  int64_t out_needed;   /* the pairs, cells or runs the returned lists took (written also when the
                         * output was too small) */
} gsnapdp_s3_stats;

/* Runs the pass; pairs_in holds npairs_in pairs and query / query_uc
 * query_bytes bytes each (every call's path and query must lie inside them);
 * pairs_out holds out_cap pairs (2 * (querylength + npairs) + 64 per call
 * always suffices).  Returns 0, or -1 (gsnapdp_last_error) on bad arguments,
 * when a batch fails or when pairs_out is too small; a path the reference would
 * abort on gets status -1 and nout = 0, and the others still run.
 *
 * The pass keeps two rounds in flight (two cohorts of paths): while one
 * cohort's windows run on the GPU, the host peels and expands the other's.
 * The host work runs on a persistent pool of GSNAPDP_S3_THREADS threads
 * (default min(16, hardware threads)). */
int gsnapdp_stage3_pass(gsnapdp_ctx *ctx, gsnapdp_s3_call *calls, int ncalls,
                        const gsnapdp_s3_pair *pairs_in, int64_t npairs_in, const char *query,
                        const char *query_uc, size_t query_bytes, const gsnapdp_iit *iit,
                        gsnapdp_s3_pair *pairs_out, int64_t out_cap, gsnapdp_s3_stats *stats);

/* The same pass with the returned lists written compactly: the pairs a path
 * keeps are named, not copied.  cells_out[first_out + j] for the j-th cell of
 * call i's list is
 *   s (| GSNAPDP_S3_CELL_DISALLOWED)  input pair s of the call's path (the pass
 *                                     set its disallowedp, stage3.c:5873-5880)
 *   -1 - k                            new_out[k], a pair the pass made
 * (a call's new pairs are consecutive in new_out, in list order).  cells_cap
 * as out_cap above; new_cap too small fails the pass with stats->new_pairs
 * set to the size needed.  This is what a caller that owns its Pair_T cells
 * needs (the drop-in relinks them), at 4 bytes per kept pair instead of 28. */
enum { GSNAPDP_S3_CELL_DISALLOWED = 1 << 30 };
int gsnapdp_stage3_pass_compact(gsnapdp_ctx *ctx, gsnapdp_s3_call *calls, int ncalls,
                                const gsnapdp_s3_pair *pairs_in, int64_t npairs_in, const char *query,
                                const char *query_uc, size_t query_bytes, const gsnapdp_iit *iit,
                                int32_t *cells_out, int64_t cells_cap, gsnapdp_s3_pair *new_out, int64_t new_cap,
                                gsnapdp_s3_stats *stats);

/* The same pass with the returned lists as runs, and the gap pairs named by
 * the caller, so that a path costs its gaps, not its pairs (a 5 kbp transcript
 * holds ~5,000 pairs around ~10 gaps).  gaps[gap_off[i] .. gap_off[i + 1]) are
 * the indices (within call i's path, ascending) of exactly the pairs whose
 * flags have GSNAPDP_S3_GAPP -- what insert_gapholders knows as it inserts
 * them (stage3.c:902-916); gaps = gap_off = NULL finds them from the flags (one
 * read of every pair).  runs_out[first_out .. first_out + nout) is call i's
 * list in list order (first_out / nout count runs here), each run
 *   start >= 0: input pairs start, start - 1, .., start - n + 1 of the call's
 *               path (n = count & ~GSNAPDP_S3_CELL_DISALLOWED; with the bit set,
 *               the pass set their disallowedp, stage3.c:5873-5880)
 *   start <  0: new_out[-1 - start .. -1 - start + count), pairs the pass made
 * runs_cap too small fails with stats->out_needed set (2 * (querylength +
 * npairs) + 64 per call always suffices; ~4 per gap is typical), new_cap as
 * gsnapdp_stage3_pass_compact. */
typedef struct gsnapdp_s3_run {
  int32_t start, count;
} gsnapdp_s3_run;
int gsnapdp_stage3_pass_runs(gsnapdp_ctx *ctx, gsnapdp_s3_call *calls, int ncalls,
                             const gsnapdp_s3_pair *pairs_in, int64_t npairs_in, const int32_t *gaps,
                             const int64_t *gap_off, const char *query, const char *query_uc, size_t query_bytes,
                             const gsnapdp_iit *iit, gsnapdp_s3_run *runs_out, int64_t runs_cap,
                             gsnapdp_s3_pair *new_out, int64_t new_cap, gsnapdp_s3_stats *stats);

/* traverse_dual_break's stage-2 realignment (stage3.c:7044-7142): build_dual_breaks
 * runs Stage2_compute_one (stage2.c:4260) on the query bytes [querydp5, querydp3]
 * of a call's query against genomic [mappingstart, mappingend] (the peeled
 * gap's bounds in the call's genomic coordinates, genomedp5 / genomedp3), and
 * stage 2 is the caller's (out of scope here).  The caller writes the list
 * Stage2_compute_one returns, head first (its last pair first), into out[0 ..
 * cap) and returns its length (which may exceed cap: the pass then asks again
 * with room for it), 0 for NULL, or -1 on an error (the path fails).  It is
 * called from the pass's host threads and must be thread-safe; `call` is the
 * pass call (its `invocation` is the caller's own tag).  Without one, a dual
 * break that needs stage 2 fails its path (status -1). */
typedef struct gsnapdp_s3_stage2 {
  void *user;
  int (*compute_one)(void *user, const gsnapdp_s3_call *call, int querydp5, int querydp3, int genomedp5,
                     int genomedp3, uint32_t mappingstart, uint32_t mappingend, gsnapdp_s3_pair *out, int cap);
} gsnapdp_s3_stage2;
int gsnapdp_stage3_set_stage2(gsnapdp_ctx *ctx, const gsnapdp_s3_stage2 *stage2);

/* Passes 2A to 6 of path_compute (stage3.c:8639-8876) for many queries:
 * build_pairs_singles (2A), fix_adjacent_indels + build_pairs_singles (2B, 2C),
 * the defect rate, Smooth_pairs_by_size + build_pairs_dualintrons +
 * build_pairs_introns iterations (3a-3c), chop_ends_by_changepoint, the two HMM
 * filters (4), remove_indel_gaps + build_dual_breaks (5) and the final
 * build_pairs_introns (6, when finalp).  The host steps run on each query's
 * list; every round of DP passes is ONE gsnapdp_stage3_pass over all the
 * queries waiting on one, whichever pass each is at.
 *
 * A query is a gsnapdp_s3_call record: first_pair / npairs = the path pass 2A
 * gets (as path_compute's pass 1 leaves it), finalp = do_final_p, the pass
 * arguments as for gsnapdp_stage3_pass (pass and defect_rate are set by the
 * pipeline), in_minor / in_major / in_* = the counters at pass 2A.  Written:
 * first_out / nout (the list after pass 6, list order, src -1), the out_*
 * counters, shiftp / incompletep of the last build_pairs_introns, defect_rate
 * (pass 4's), ub (OR of the passes'), status (-1 when a pass or a host step
 * would make the reference abort, or a stage-2 dual break has no callback).
 * min_intronlength is gmap's (-j, default 9; remove_indel_gaps). */
typedef struct gsnapdp_s3_compute_stats {
  int32_t passes;         /* gsnapdp_stage3_pass calls */
  int32_t rounds;         /* their rounds */
  int32_t windows[4];     /* as gsnapdp_s3_stats */
  int32_t pass_calls[6];  /* the pass calls, by GSNAPDP_S3_* */
  int32_t failed;
  int32_t sites;          /* MaxEnt site probabilities evaluated for assign_gap_types (path_compute) */
  double seconds[3];      /* wall time: host steps between the passes, the GPU work (passes and MaxEnt
                           * batches), the whole call */
} gsnapdp_s3_compute_stats;
int gsnapdp_stage3_compute(gsnapdp_ctx *ctx, gsnapdp_s3_call *queries, int nqueries,
                           const gsnapdp_s3_pair *paths_in, int64_t npairs_in, const char *query,
                           const char *query_uc, size_t query_bytes, const gsnapdp_iit *iit, int min_intronlength,
                           gsnapdp_s3_pair *out, int64_t out_cap, gsnapdp_s3_compute_stats *stats);

/* path_compute (stage3.c:8586-9220) from pass 2A to its return value, for many
 * queries: passes 2A-6 as gsnapdp_stage3_compute, then
 *   7   the dual breaks at the ends (:8885-8925: dualbreak_distance_from_end,
 *       trim_npairs),
 *   7b  remove_adjacent_ins_del (:1889) and, when it removed any, 7C
 *       build_pairs_singles; remove_indel_gaps,
 *   8   clean_pairs_end5_gap_indels / clean_path_end3_gap_indels (:2056-2126),
 *       build_pairs_end5 / build_path_end3 with QUERYEND_GAP,
 *   9   assign_gap_types (:1015: intron types, cDNA-insertion and short-gap
 *       pairs, the MaxEnt donor / acceptor probabilities of every intron) and
 *       build_pairs_end5 / build_path_end3 with BEST_LOCAL and maxpeelback 0,
 *       then assign_gap_types again,
 *   10  trim_noncanonical_end5_exons / _end3_exons (:2793, :3021) with their
 *       QUERYEND_NOGAPS re-extensions, at most 5 iterations.
 * Every DP pass of every query runs in driven gsnapdp_stage3_pass rounds; the
 * MaxEnt probabilities of each assign_gap_types are one k_maxent batch over all
 * queries that reached it (1.0 for a site the splicing IIT knows, as the
 * reference asks it).  Queries as for gsnapdp_stage3_compute, plus their
 * maxpeelback, extramaterial_end, extraband_end and finalp (= do_final_p).
 * Written: the returned list (list order, src -1) at first_out / nout, and in
 * probs_out (2 doubles per returned pair, NULL to skip) each pair's donor_prob
 * and acceptor_prob; out_minor / out_major, out_intronlen / out_nonintronlen
 * (path_compute's *intronlen / *nonintronlen), defect_rate, ub, status.  Needs
 * the MaxEnt tables. */
typedef struct gsnapdp_s3_path_opts {
  int32_t min_intronlength;    /* Stage3_setup's (gmap -j, default 9): remove_indel_gaps, assign_gap_types */
  int32_t maxintronlen_bound;  /* path_compute's maxintronlen (gmap: maxintronlen_bound, default 1000000) */
  int32_t paired_favor_mode;   /* 0 in GMAP; GSNAP's GMAP-in-GSNAP passes its own */
  int32_t zero_offset;
  int32_t expected_pairlength, pairlength_deviation;  /* Stage3_setup's (read when paired_favor_mode != 0) */
  int32_t gsnap;               /* 1: stage3.c as GSNAP builds it (-DGSNAP: passes 9a / 9b with QUERYEND_NOGAPS,
                                * a sufficiently supported end exon always kept); 0: GMAP */
  int32_t pad;
} gsnapdp_s3_path_opts;
int gsnapdp_stage3_path_compute(gsnapdp_ctx *ctx, gsnapdp_s3_call *queries, int nqueries,
                                const gsnapdp_s3_pair *paths_in, int64_t npairs_in, const char *query,
                                const char *query_uc, size_t query_bytes, const gsnapdp_iit *iit,
                                const gsnapdp_s3_path_opts *opts, gsnapdp_s3_pair *out, int64_t out_cap,
                                double *probs_out, gsnapdp_s3_compute_stats *stats);

/* Host-only: Pbinom (pbinom.c:1680, GSL 1.8's binomial CDF through the
 * incomplete beta function) as chop_ends_by_changepoint calls it (stage3.c:2130:
 * k <= n, theta in [0.1, 1)), bit for bit the reference's double.  Returns 0, or
 * -1 where the reference aborts. */
int gsnapdp_pbinom(int k, int n, double theta, double *p);

/* score_introns (stage3.c:7935-8162) on the lists a pass returned: for every
 * call with status 0, its list reversed into path order (as stage3_compute
 * reverses path_compute's pairs, :9890-9941), the introns picked on the host
 * (gsnapdp_path_introns), the IIT's verdicts (NULL for none) and one k_introns
 * launch for all of them.  scores[i] is call i's (zeros for a failed call). */
int gsnapdp_stage3_score_introns(gsnapdp_ctx *ctx, const gsnapdp_s3_call *calls, int ncalls,
                                 const gsnapdp_s3_pair *pairs_out, const gsnapdp_iit *iit,
                                 gsnapdp_intron_scores *scores);
/* The same on gsnapdp_stage3_pass_runs' output (calls as it left them, its
 * pairs_in, gaps / gap_off (or NULL) and new_out): only each list's gap pairs
 * and their neighbours are read. */
int gsnapdp_stage3_score_introns_runs(gsnapdp_ctx *ctx, const gsnapdp_s3_call *calls, int ncalls,
                                      const gsnapdp_s3_pair *pairs_in, const int32_t *gaps, const int64_t *gap_off,
                                      const gsnapdp_s3_run *runs, const gsnapdp_s3_pair *new_pairs,
                                      const gsnapdp_iit *iit, gsnapdp_intron_scores *scores);

/* Load the MaxEnt parameter tables (12 x 16384 + 4 x 16 doubles, order in
 * DESIGN.md) into the context.  Must be called before gsnapdp_maxent_*. */
int gsnapdp_load_maxent_tables(gsnapdp_ctx *ctx, const double *tables, size_t ndoubles);

/* -------------------------------------------------------------- expansion
 * Replay window i's op stream into the reference's pair list, in final list
 * order (after the entry point's List_reverse / INDEL stripping / zeroing
 * rules).  Host only.  `query`/`query_uc` are the same host buffers given to
 * the run.  Writes at most `cap` pairs; returns the number of pairs in the
 * list (may exceed cap), or -1 on error.  `*finalscore` receives the
 * entry point's final score after its post-rules (end-gap zeroing). */
int gsnapdp_expand(gsnapdp_ctx *ctx, const gsnapdp_window *w, const gsnapdp_result *res,
                   const uint32_t *ops, const char *query, const char *query_uc,
                   gsnapdp_pair *pairs, int cap, int *finalscore);

#ifdef __cplusplus
}
#endif
#endif /* GSNAPDP_H */
