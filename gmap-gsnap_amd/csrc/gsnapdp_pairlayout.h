/* gsnapdp_pairlayout.h -- the byte layout of the host program's Pair_T
 * (pairdef.h:9-49) and List_T (listdef.h) that the drop-in reads and writes in
 * place: the non-PMAP x86-64 build gmap and gsnap use (bool = unsigned char,
 * bool.h; State_T an int-sized enum).  gsnapdp_dropin.cpp static-asserts its
 * mirror structs against these constants, and oracle/pairdef_check.c asserts
 * the same constants against the reference's own pairdef.h / listdef.h
 * (built by `make -C oracle ref` and `make -C oracle asan`), so a host whose
 * Pair_T differs (-DPMAP, a 32-bit ABI) fails the build instead of corrupting
 * lists.  Plain C: included by both. */
#ifndef GSNAPDP_PAIRLAYOUT_H
#define GSNAPDP_PAIRLAYOUT_H

#define GSNAPDP_PAIR_OFF_QUERYPOS 0
#define GSNAPDP_PAIR_OFF_GENOMEPOS 4
#define GSNAPDP_PAIR_OFF_QUERYJUMP 16
#define GSNAPDP_PAIR_OFF_GENOMEJUMP 20
#define GSNAPDP_PAIR_OFF_DYNPROGINDEX 32
#define GSNAPDP_PAIR_OFF_CDNA 36
#define GSNAPDP_PAIR_OFF_COMP 37
#define GSNAPDP_PAIR_OFF_GENOME 38
#define GSNAPDP_PAIR_OFF_GAPP 41
#define GSNAPDP_PAIR_OFF_KNOWNGAPP 42
#define GSNAPDP_PAIR_OFF_SHORTEXONP 44
#define GSNAPDP_PAIR_OFF_DISALLOWEDP 61
#define GSNAPDP_PAIR_OFF_DONOR_PROB 64
#define GSNAPDP_PAIR_OFF_END_INTRON_P 80
#define GSNAPDP_PAIR_SIZE 88
#define GSNAPDP_LIST_OFF_FIRST 0
#define GSNAPDP_LIST_OFF_REST 8
#define GSNAPDP_LIST_SIZE 16

#endif
