/*
 * af_oracle_int.h -- TEST INFRASTRUCTURE ONLY: helpers shared by the oracle's C files
 * (af_oracle.c: seed filter, ksw DP restatements, placement; bwa_pe.c: the bwa-mem
 * paired-end path of S2).  Not part of any product interface.
 */
#ifndef AF_ORACLE_INT_H
#define AF_ORACLE_INT_H
#include <stdint.h>
#include "af_oracle.h"

typedef struct { int32_t h, e; } eh_t;

uint8_t afo_nt4(uint8_t c);
int afo_sc(const afo_params *p, uint8_t x, uint8_t y);
/* ksw_extend2 (bwa ksw.c) */
int afo_ext_dp(int qlen, const uint8_t *query, int tlen, const uint8_t *target, const afo_params *p, int w,
               int end_bonus, int zdrop, int h0, int *_qle, int *_tle, int *_gtle, int *_gscore, int *_max_off);
/* ksw_global2 (bwa ksw.c) with traceback; cigar ops M0 I1 D2, *n_cig may exceed cap */
int afo_global_dp(int qlen, const uint8_t *query, int tlen, const uint8_t *target, const afo_params *p, int w,
                  uint32_t *cig, int cap, int *n_cig);
/* bwamem.c cal_max_gap / infer_bw */
int afo_cal_max_gap(const afo_params *p, int qlen);
int afo_infer_bw(int l1, int l2, int score, int a, int q, int r);
/* bwa_gen_cigar2 (bwa bwa.c) on a doubled text of half length n: the query segment and
 * text[rb, re) are reversed together for reverse-strand spans */
int afo_gen_cigar(const uint8_t *text, int64_t n, const afo_params *p, int w_, int lq, const uint8_t *qseg,
                  int64_t rb, int64_t re, uint32_t *cig, int *n_cig);
/* the same writing at most cap ops (*n_cig counts them all); segments of any length */
int afo_gen_cigar_cap(const uint8_t *text, int64_t n, const afo_params *p, int w_, int lq, const uint8_t *qseg,
                      int64_t rb, int64_t re, uint32_t *cig, int cap, int *n_cig);

/* the bwa text of the S2 anchor (bwa_pe.c): T = pac ++ revcomp(pac) with bwa's N
 * substitution, suffix ranks, and every 16-mer position of T */
typedef struct afo_text afo_text;
afo_text *afo_text_build(const char *anchor, int64_t n);
void afo_text_free(afo_text *X);
const uint8_t *afo_text_codes(const afo_text *X);
/* forward-strand 16-mers of T (those not crossing position n), as (packed kmer << 32 | pos),
 * sorted; count in *m.  Used for the K1 Bloom filter. */
uint64_t *afo_text_kmers_noncrossing(const afo_text *X, int64_t *m);
const afo_text *afo_index_text(const afo_index *I);

#endif
