"""numpy views of the C-ABI records of include/gsnapdp.h (byte-for-byte)."""
from __future__ import annotations

import numpy as np

WINDOW = np.dtype([
    ("kind", "<i4"), ("length1", "<i4"), ("length2", "<i4"), ("offset1", "<i4"), ("offset2", "<i4"),
    ("chroffset", "<u4"), ("chrhigh", "<u4"), ("chrpos", "<u4"), ("genomiclength", "<u4"), ("qpos", "<u4"),
    ("cdna_direction", "<i4"), ("extraband", "<i4"), ("dynprogindex", "<i4"),
    ("maxlength1", "<i4"), ("maxlength2", "<i4"), ("defect_rate", "<f4"),
    ("watsonp", "u1"), ("jump_late_p", "u1"), ("widebandp", "u1"), ("endalign", "u1"),
])
assert WINDOW.itemsize == 68

RESULT = np.dtype([
    ("finalscore", "<i4"), ("nmatches", "<i4"), ("nmismatches", "<i4"), ("nopens", "<i4"),
    ("nindels", "<i4"), ("bestr", "<i4"), ("bestc", "<i4"), ("nops", "<i4"), ("status", "<i4"),
    ("length1", "<i4"), ("length2", "<i4"), ("reserved", "<i4"),
])
assert RESULT.itemsize == 48

PAIR = np.dtype([
    ("querypos", "<i4"), ("genomepos", "<i4"), ("queryjump", "<i4"), ("genomejump", "<i4"),
    ("dynprogindex", "<i4"), ("cdna", "S1"), ("comp", "S1"), ("genome", "S1"), ("gapp", "u1"),
])
assert PAIR.itemsize == 24

GGAP_WINDOW = np.dtype([
    ("length1", "<i4"), ("length2L", "<i4"), ("length2R", "<i4"),
    ("offset1", "<i4"), ("offset2L", "<i4"), ("revoffset2R", "<i4"),
    ("chroffset", "<u4"), ("chrhigh", "<u4"), ("chrpos", "<u4"), ("genomiclength", "<u4"), ("qpos", "<u4"),
    ("cdna_direction", "<i4"), ("extraband_paired", "<i4"), ("maxpeelback", "<i4"),
    ("score_threshold", "<i4"), ("dynprogindex", "<i4"), ("maxlength1", "<i4"), ("maxlength2", "<i4"),
    ("defect_rate", "<f4"),
    ("watsonp", "u1"), ("jump_late_p", "u1"), ("halfp", "u1"), ("finalp", "u1"),
    ("use_probabilities_p", "u1"), ("splicingp", "u1"), ("known_mode", "u1"), ("pad1", "u1"),
])
assert GGAP_WINDOW.itemsize == 84

GGAP_RESULT = np.dtype([
    ("finalscore", "<i4"), ("new_leftgenomepos", "<i4"), ("new_rightgenomepos", "<i4"),
    ("nmatches", "<i4"), ("nmismatches", "<i4"), ("nopens", "<i4"), ("nindels", "<i4"),
    ("exonhead", "<i4"), ("introntype", "<i4"), ("dynprogindex", "<i4"),
    ("returned_null", "<i4"), ("bridge_ok", "<i4"), ("left_prob", "<f8"), ("right_prob", "<f8"),
])
assert GGAP_RESULT.itemsize == 64

GGAP_TRACE = np.dtype([
    ("brL", "<i4"), ("bcL", "<i4"), ("brR", "<i4"), ("bcR", "<i4"),
    ("nops_right", "<i4"), ("nops_left", "<i4"), ("status", "<i4"), ("npairs", "<i4"),
    ("bridge_accepted", "<i4"), ("reserved", "<i4"),
])
assert GGAP_TRACE.itemsize == 40

CGAP_WINDOW = np.dtype([
    ("length1L", "<i4"), ("length1R", "<i4"), ("length2", "<i4"),
    ("offset1L", "<i4"), ("revoffset1R", "<i4"), ("offset2", "<i4"),
    ("chroffset", "<u4"), ("chrhigh", "<u4"), ("chrpos", "<u4"), ("genomiclength", "<u4"),
    ("qposL", "<u4"), ("qposR", "<u4"),
    ("cdna_direction", "<i4"), ("extraband_paired", "<i4"), ("dynprogindex", "<i4"),
    ("maxlength1", "<i4"), ("maxlength2", "<i4"), ("defect_rate", "<f4"),
    ("watsonp", "u1"), ("jump_late_p", "u1"), ("pad0", "u1"), ("pad1", "u1"),
])
assert CGAP_WINDOW.itemsize == 76

CGAP_RESULT = np.dtype([
    ("finalscore", "<i4"), ("dynprogindex", "<i4"), ("incompletep", "<i4"), ("returned_null", "<i4"),
    ("status", "<i4"), ("npairs", "<i4"), ("finalscore_set", "<i4"), ("insert_pairs", "<i4"),
    ("brL", "<i4"), ("bcL", "<i4"), ("brR", "<i4"), ("bcR", "<i4"),
    ("nops_right", "<i4"), ("nops_left", "<i4"), ("reserved0", "<i4"), ("reserved1", "<i4"),
])
assert CGAP_RESULT.itemsize == 64

SJ_WINDOW = np.dtype([
    ("kind", "<i4"), ("length1", "<i4"), ("length2", "<i4"), ("offset1", "<i4"),
    ("offset2_anchor", "<i4"), ("offset2_far", "<i4"), ("contlength", "<i4"),
    ("qpos", "<u4"), ("spos", "<u4"),
    ("cdna_direction", "<i4"), ("extraband_end", "<i4"), ("dynprogindex", "<i4"),
    ("maxlength1", "<i4"), ("maxlength2", "<i4"), ("defect_rate", "<f4"),
    ("watsonp", "u1"), ("jump_late_p", "u1"), ("pad0", "u1"), ("pad1", "u1"),
])
assert SJ_WINDOW.itemsize == 64

MICRO_WINDOW = np.dtype([
    ("length1", "<i4"), ("offset1", "<i4"), ("offset2L", "<i4"), ("revoffset2R", "<i4"),
    ("cdna_direction", "<i4"), ("dynprogindex", "<i4"),
    ("chroffset", "<u4"), ("chrhigh", "<u4"), ("chrpos", "<u4"), ("genomiclength", "<u4"),
    ("qpos", "<u4"), ("ppos", "<u4"), ("defect_rate", "<f4"),
    ("watsonp", "u1"), ("pad0", "u1"), ("pad1", "u1"), ("pad2", "u1"),
])
assert MICRO_WINDOW.itemsize == 56

MICRO_RESULT = np.dtype([
    ("bestprob2", "<f8"), ("bestprob3", "<f8"),
    ("microintrontype", "<i4"), ("dynprogindex", "<i4"), ("found", "<i4"), ("status", "<i4"),
    ("bestcL", "<i4"), ("bestcR", "<i4"), ("middlelength", "<i4"), ("offset2M", "<i4"),
])
assert MICRO_RESULT.itemsize == 48

MAXENT_IN = np.dtype([("model", "<u4"), ("splice_pos", "<u4"), ("chroffset", "<u4"), ("pad", "<u4")])

# enums (include/gsnapdp.h)
SINGLE_GAP, END5_GAP, END3_GAP = 0, 1, 2
QUERYEND_GAP, QUERYEND_INDELS, QUERYEND_NOGAPS, BEST_LOCAL = 0, 1, 2, 3
DONOR, ACCEPTOR, ANTIDONOR, ANTIACCEPTOR = 0, 1, 2, 3
OP_DIAG, OP_HDASH, OP_HGAP, OP_VSKIP = 0, 1, 2, 3

# Dynprog_new(600, 10, 11, 10, 8) as called by gmap.c:2270 -> 611 x 2000 (dynprog.c:831-852)
MAXLENGTH1 = 611
MAXLENGTH2 = 2000

# score_introns batches (include/gsnapdp.h: gsnapdp_path_pair, _intron, _intron_path, _intron_scores)
PATH_PAIR = np.dtype([("genomepos", "<u4"), ("queryjump", "<i4"), ("genomejump", "<i4"),
                      ("gapp", "u1"), ("knowngapp", "u1"), ("comp", "u1"), ("pad", "u1")])
assert PATH_PAIR.itemsize == 16
INTRON = np.dtype([("left_genomepos", "<u4"), ("right_genomepos", "<u4"), ("path", "<i4"),
                   ("comp", "u1"), ("knowngapp", "u1"), ("known_donor", "u1"), ("known_acceptor", "u1")])
assert INTRON.itemsize == 16
INTRON_PATH = np.dtype([("chroffset", "<u4"), ("chrpos", "<u4"), ("genomiclength", "<i4"),
                        ("cdna_direction", "<i4"), ("watsonp", "<i4"), ("first_intron", "<i4"),
                        ("nintrons", "<i4"), ("pad", "<i4")])
assert INTRON_PATH.itemsize == 32
INTRON_SCORES = np.dtype([("avg_donor_score", "<f8"), ("avg_acceptor_score", "<f8"),
                          ("nbadintrons", "<i4"), ("nintrons", "<i4")])
assert INTRON_SCORES.itemsize == 24

# the stage-3 intron pass (include/gsnapdp.h: gsnapdp_s3_pair, _s3_call, _s3_stats)
S3_PAIR = np.dtype([("querypos", "<i4"), ("genomepos", "<i4"), ("queryjump", "<i4"), ("genomejump", "<i4"),
                    ("dynprogindex", "<i4"), ("src", "<i4"), ("cdna", "u1"), ("comp", "u1"), ("genome", "u1"),
                    ("flags", "u1")])
assert S3_PAIR.itemsize == 28
S3_GAPP, S3_KNOWNGAPP, S3_DISALLOWED, S3_SHORTEXON, S3_END_INTRON = 1, 2, 4, 8, 16
S3_UB_INTRONLEN = 1  # gsnapdp_s3_call.ub: intronlen / nonintronlen took the reference's uninitialised locals
S3_UB_DUAL = 2  # a dual-intron decision read one of traverse_dual_genome_gap's uninitialised locals
S3_CALL = np.dtype([(n, "<i4") for n in "first_pair npairs first_out nout qpos querylength".split()] +
                   [(n, "<u4") for n in "chroffset chrhigh chrpos".split()] +
                   [(n, "<i4") for n in ("chrnum genomiclength cdna_direction watsonp jump_late_p finalp "
                                         "use_genomicseg_p maxpeelback nullgap extramaterial_paired "
                                         "extraband_single extraband_paired close_indels_mode").split()] +
                   [("defect_rate", "<f8"), ("maxlength1", "<i4", 3), ("maxlength2", "<i4", 3)] +
                   [(n, "<i4") for n in ("in_minor in_major in_nintrons in_nnonintrons in_intronlen in_nonintronlen "
                                         "out_minor out_major out_nintrons out_nnonintrons out_intronlen "
                                         "out_nonintronlen shiftp incompletep novelsplicingp splicingp "
                                         "status ub pass endalign extramaterial_end extraband_end splicesitesp "
                                         "invocation").split()] +
                   [("ref_seconds", "<f8")])
assert S3_CALL.itemsize == 224
# gsnapdp_s3_call.pass: build_pairs_introns, build_pairs_singles, build_pairs_end5, build_path_end3,
# build_pairs_dualintrons, build_dual_breaks
S3_INTRONS, S3_SINGLES, S3_END5, S3_END3, S3_DUALINTRONS, S3_DUALBREAKS = 0, 1, 2, 3, 4, 5
# golden records of gmap_trace (oracle/gmap_trace.c): one Stage2_compute_one call that
# traverse_dual_break made (its pairs in S3_PAIR records), and one path_compute call
S2_CALL = np.dtype([(n, "<i4") for n in "invocation query_offset querylength genomiclength".split()] +
                   [(n, "<u4") for n in "genomicstart genomicend mappingstart mappingend".split()] +
                   [(n, "<i4") for n in "plusp first_pair npairs pad".split()])
assert S2_CALL.itemsize == 48
PC_CALL = np.dtype([(n, "<i4") for n in ("invocation do_final_p stage3debug cdna_direction querylength "
                                         "genomiclength watsonp pad").split()] + [("defect_rate", "<f8")] +
                   [(n, "<i4") for n in ("first_out nout intronlen nonintronlen maxpeelback nullgap "
                                         "extramaterial_end extraband_end maxintronlen_bound paired_favor_mode "
                                         "zero_offset jump_late_p").split()] + [("passes", "<i4", 6)])
assert PC_CALL.itemsize == 112
# GSNAP's splice-site scan candidates (include/gsnapdp.h gsnapdp_scan_site)
SCAN_SITE = np.dtype([("segment_left", "<u4"), ("splice_pos", "<i4"), ("chroffset", "<u4"), ("knowni", "<i4"),
                      ("model", "<i4")])
assert SCAN_SITE.itemsize == 20
S3_COMPUTE_STATS = np.dtype([("passes", "<i4"), ("rounds", "<i4"), ("windows", "<i4", 4), ("pass_calls", "<i4", 6),
                             ("failed", "<i4"), ("sites", "<i4"), ("seconds", "<f8", 3)])
assert S3_COMPUTE_STATS.itemsize == 80
S3_PATH_OPTS = np.dtype([(n, "<i4") for n in ("min_intronlength maxintronlen_bound paired_favor_mode zero_offset "
                                             "expected_pairlength pairlength_deviation gsnap pad").split()])
assert S3_PATH_OPTS.itemsize == 32
S3_STATS = np.dtype([("rounds", "<i4"), ("windows", "<i4", 4), ("batches", "<i4", 4), ("undefined", "<i4"),
                     ("failed", "<i4"), ("pad", "<i4"), ("seconds", "<f8", 3), ("new_pairs", "<i8"),
                     ("out_needed", "<i8")])
assert S3_STATS.itemsize == 88
S3_RUN = np.dtype([("start", "<i4"), ("count", "<i4")])  # gsnapdp_s3_run (gsnapdp_stage3_pass_runs)
S3_CELL_DISALLOWED = 1 << 30  # gsnapdp_stage3_pass_compact: an input pair whose disallowedp the pass set

# a splicing IIT's intervals (include/gsnapdp.h: gsnapdp_iit_interval); start > end is the minus sign,
# type -1 none (an intron), 0 donor, 1 acceptor
IIT_INTERVAL = np.dtype([("chrnum", "<i4"), ("start", "<u4"), ("end", "<u4"), ("type", "<i4")])
assert IIT_INTERVAL.itemsize == 16
