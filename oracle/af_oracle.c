/*
 * af_oracle.c -- TEST INFRASTRUCTURE ONLY (see af_oracle.h).
 *
 * Plain-C restatement of the S2 path of the reference (Anchored_Fusion.py:181-182:
 * `bwa mem -M -t T anchor fq1 fq2`), written as the bit-exact contract for the HIP
 * kernels in anchored-fusion_amd/csrc.  Every stage cites the published bwa-mem
 * algorithm it restates; nothing here is called by the product path.
 */
#include "af_oracle.h"
#include "af_oracle_int.h"
#include <stdlib.h>
#include <string.h>
#include <math.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define NEG_INF (-0x40000000)

struct afo_index {
    int64_t n;          /* anchor length                                    */
    uint8_t *D;         /* 2n codes: anchor ++ revcomp(anchor), N = 4       */
    int64_t nk;         /* number of indexed 16-mer positions              */
    uint32_t *kmer;     /* sorted by (kmer, pos)                            */
    int32_t *kpos;
    int32_t bl_bits;    /* log2 Bloom words                                */
    uint32_t *bloom;    /* K1 filter over the bwa text's 16-mers            */
    afo_text *X;        /* S2: the bwa text (bwa_pe.c)                      */
};

const afo_text *afo_index_text(const afo_index *I) { return I->X; }

/* ---- encoding ---------------------------------------------------------------------- */
uint8_t afo_nt4(uint8_t c) {
    switch (c) {
    case 'A': case 'a': return 0;
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'T': case 't': return 3;
    default: return 4;
    }
}

void afo_params_default(afo_params *p) {
    /* bwa mem defaults (bwa 0.7.17 `bwa mem` usage text) */
    p->a = 1; p->b = 4; p->o_del = 6; p->e_del = 1; p->o_ins = 6; p->e_ins = 1;
    p->pen_clip5 = 5; p->pen_clip3 = 5; p->w = 100; p->zdrop = 100;
    p->min_seed_len = 19; p->max_occ = 500; p->T = 30; p->max_ext = 16; p->max_mems = 64;
}

/* ---- seed-filter (K1) keys and Bloom filter, restated from the kernel's definition
 * (anchored-fusion_amd/csrc/af_internal.h; not a reference algorithm: the filter
 * only has to keep every read that can hold a bwa seed).
 * code(byte) = 2-bit table 0x8340 indexed by the byte's low 3 bits (A C G T -> 0 1 2 3, N -> 0);
 * key = the 16 codes with base 4w+b at bits 8b+2w; h = key * 0x9E3779B1 (64-bit product hi:lo);
 * word 1 = (hi >> 2) & (2^bits-1) gets one bit per byte at (lo byte & 7), word 2 =
 * lo >> (32-bits) one bit per byte at (hi byte & 7). */
static inline uint32_t k1_code(uint8_t c) { return (0x8340u >> (2 * (c & 7))) & 3u; }
static inline uint64_t k1_hash(uint32_t key) { return (uint64_t)key * 0x9E3779B1u; }
static inline uint32_t k1_mask(uint32_t v) {
    uint32_t m = 0;
    for (int b = 0; b < 4; ++b) m |= 1u << (8 * b + ((v >> (8 * b)) & 7));
    return m;
}
static inline uint32_t k1_w1(uint64_t h, int bits) { return ((uint32_t)(h >> 32) >> 2) & ((1u << bits) - 1u); }
static inline uint32_t k1_w2(uint64_t h, int bits) { return (uint32_t)h >> (32 - bits); }

static int cmp_u64(const void *a, const void *b) {
    uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return x < y ? -1 : x > y;
}

/* 16-mer packing: base i at bits [2i, 2i+1] */
static inline int pack16(const uint8_t *c, uint32_t *k) {
    uint32_t v = 0;
    for (int i = 0; i < AFO_K; ++i) {
        if (c[i] > 3) return 0;
        v |= (uint32_t)c[i] << (2 * i);
    }
    *k = v;
    return 1;
}

afo_index *afo_index_build(const char *anchor, int64_t n) {
    if (n <= 0) return NULL;
    afo_index *I = (afo_index *)calloc(1, sizeof(afo_index));
    I->n = n;
    I->D = (uint8_t *)malloc(2 * n);
    for (int64_t i = 0; i < n; ++i) {
        uint8_t c = afo_nt4((uint8_t)anchor[i]);
        I->D[i] = c;
        I->D[2 * n - 1 - i] = c < 4 ? 3 - c : 4;
    }
    /* every valid 16-mer position of D that does not cross the strand boundary at n */
    uint64_t *tmp = (uint64_t *)malloc(sizeof(uint64_t) * (2 * n + 1));
    int64_t m = 0;
    for (int64_t p = 0; p + AFO_K <= 2 * n; ++p) {
        if (p < n && p + AFO_K > n) continue;
        uint32_t k;
        if (!pack16(I->D + p, &k)) continue;
        tmp[m++] = ((uint64_t)k << 32) | (uint64_t)p;
    }
    qsort(tmp, m, sizeof(uint64_t), cmp_u64);
    I->nk = m;
    I->kmer = (uint32_t *)malloc(sizeof(uint32_t) * (m + 1));
    I->kpos = (int32_t *)malloc(sizeof(int32_t) * (m + 1));
    for (int64_t i = 0; i < m; ++i) {
        I->kmer[i] = (uint32_t)(tmp[i] >> 32);
        I->kpos[i] = (int32_t)(tmp[i] & 0xffffffffu);
    }
    /* Bloom filter of the distinct 16-mers of the bwa text T that do not cross the strand
     * boundary (seeds never do): 2^bl_bits 32-bit words, ~2.4 words per key (at most 2^15),
     * four bits set in each of two words */
    I->X = afo_text_build(anchor, n);
    int64_t mk = 0;
    uint64_t *tk = afo_text_kmers_noncrossing(I->X, &mk);
    int64_t nd = 0;
    for (int64_t i = 0; i < mk; ++i)
        if (i == 0 || (tk[i] >> 32) != (tk[i - 1] >> 32)) ++nd;
    int bits = 8;
    while ((double)(1LL << bits) < 2.4 * (double)nd && bits < 15) ++bits;
    I->bl_bits = bits;
    I->bloom = (uint32_t *)calloc((size_t)1 << bits, sizeof(uint32_t));
    for (int64_t i = 0; i < mk; ++i) {
        if (i > 0 && (tk[i] >> 32) == (tk[i - 1] >> 32)) continue;
        uint32_t km = (uint32_t)(tk[i] >> 32), key = 0;  /* base j (bits 2j) to bits 8(j&3)+2(j>>2) */
        for (int j = 0; j < AFO_K; ++j) key |= ((km >> (2 * j)) & 3u) << (8 * (j & 3) + 2 * (j >> 2));
        uint64_t h = k1_hash(key);
        I->bloom[k1_w1(h, bits)] |= k1_mask((uint32_t)h);
        I->bloom[k1_w2(h, bits)] |= k1_mask((uint32_t)(h >> 32));
    }
    free(tk);
    free(tmp);
    return I;
}

void afo_index_free(afo_index *I) {
    if (!I) return;
    free(I->D); free(I->kmer); free(I->kpos); free(I->bloom); afo_text_free(I->X); free(I);
}
int64_t afo_index_len(const afo_index *I) { return I->n; }
int32_t afo_filter_words(const afo_index *I) { return 1 << I->bl_bits; }
const uint32_t *afo_filter_table(const afo_index *I) { return I->bloom; }

/* a sampled 16-mer (key layout above) is a hit when all six of its Bloom bits are set */
static int filter_query(const afo_index *I, uint32_t key) {
    uint64_t h = k1_hash(key);
    uint32_t m1 = k1_mask((uint32_t)h), m2 = k1_mask((uint32_t)(h >> 32));
    return (I->bloom[k1_w1(h, I->bl_bits)] & m1) == m1 && (I->bloom[k1_w2(h, I->bl_bits)] & m2) == m2;
}

/* K1 semantics: sampled positions are those whose byte offset in the read buffer is a
 * multiple of 4; any MEM >= 19 nt contains such a 16-mer and a Bloom filter has no false
 * negatives, so hits==0 => no seed.  Bytes are
 * projected to 2 bits by k1_code (exact for ACGT/acgt; other bytes land on some code, which
 * can only add hits -- MEMs never contain N, so the superset property holds). */
void afo_seed_filter(const afo_index *I, const uint8_t *reads, int64_t n_reads, int32_t stride,
                     const int32_t *lens, int32_t *hits) {
    for (int64_t r = 0; r < n_reads; ++r) {
        int32_t l = lens ? lens[r] : stride;
        int64_t base = r * (int64_t)stride;
        int32_t h = 0;
        int32_t i0 = (int32_t)((4 - (base & 3)) & 3);
        for (int32_t i = i0; i + AFO_K <= l; i += 4) {
            uint32_t k = 0;
            for (int j = 0; j < AFO_K; ++j) {
                k |= k1_code(reads[base + i + j]) << (8 * (j & 3) + 2 * (j >> 2));
            }
            h += filter_query(I, k);
        }
        hits[r] = h;
    }
}

/* ---- score matrix (bwa_fill_scmat): a / -b for ACGT, -1 for anything with N -------- */
int afo_sc(const afo_params *p, uint8_t x, uint8_t y) {
    if (x > 3 || y > 3) return -1;
    return x == y ? p->a : -p->b;
}

/* ---- ksw_extend restated (bwa ksw.c ksw_extend2): target rows, query columns ------- */

int afo_ext_dp(int qlen, const uint8_t *query, int tlen, const uint8_t *target, const afo_params *p,
                  int w, int end_bonus, int zdrop, int h0, int *_qle, int *_tle, int *_gtle,
                  int *_gscore, int *_max_off) {
    eh_t eh_stack[AFO_MAX_READ + 2];  /* a longer query (afo_blat_long's parts): a heap row */
    eh_t *eh = qlen <= AFO_MAX_READ ? eh_stack : (eh_t *)malloc(sizeof(eh_t) * (qlen + 2));
    int oe_del = p->o_del + p->e_del, oe_ins = p->o_ins + p->e_ins;
    int i, j, max, max_i, max_j, max_ie, gscore, max_off, beg, end;
    memset(eh, 0, sizeof(eh_t) * (qlen + 2));
    /* first row */
    eh[0].h = h0;
    eh[1].h = h0 > oe_ins ? h0 - oe_ins : 0;
    for (j = 2; j <= qlen && eh[j - 1].h > p->e_ins; ++j) eh[j].h = eh[j - 1].h - p->e_ins;
    /* band adjustment: the longest gap that can still score */
    {
        int mx = p->a;
        int max_ins = (int)((double)(qlen * mx + end_bonus - p->o_ins) / p->e_ins + 1.);
        max_ins = max_ins > 1 ? max_ins : 1;
        w = w < max_ins ? w : max_ins;
        int max_del = (int)((double)(qlen * mx + end_bonus - p->o_del) / p->e_del + 1.);
        max_del = max_del > 1 ? max_del : 1;
        w = w < max_del ? w : max_del;
    }
    max = h0; max_i = max_j = -1; max_ie = -1; gscore = -1; max_off = 0;
    beg = 0; end = qlen;
    for (i = 0; i < tlen; ++i) {
        int t, f = 0, h1, m = 0, mj = -1;
        uint8_t ti = target[i];
        if (beg < i - w) beg = i - w;
        if (end > i + w + 1) end = i + w + 1;
        if (end > qlen) end = qlen;
        if (beg == 0) {
            h1 = h0 - (p->o_del + p->e_del * (i + 1));
            if (h1 < 0) h1 = 0;
        } else h1 = 0;
        for (j = beg; j < end; ++j) {
            eh_t *q = &eh[j];
            int h, M = q->h, e = q->e;
            q->h = h1;
            M = M ? M + afo_sc(p, ti, query[j]) : 0;
            h = M > e ? M : e;
            h = h > f ? h : f;
            h1 = h;
            mj = m > h ? mj : j;
            m = m > h ? m : h;
            t = M - oe_del; t = t > 0 ? t : 0;
            e -= p->e_del; e = e > t ? e : t;
            q->e = e;
            t = M - oe_ins; t = t > 0 ? t : 0;
            f -= p->e_ins; f = f > t ? f : t;
        }
        eh[end].h = h1; eh[end].e = 0;
        if (j == qlen) {
            max_ie = gscore > h1 ? max_ie : i;
            gscore = gscore > h1 ? gscore : h1;
        }
        if (m == 0) break;
        if (m > max) {
            max = m; max_i = i; max_j = mj;
            int off = mj - i < 0 ? i - mj : mj - i;
            max_off = max_off > off ? max_off : off;
        } else if (zdrop > 0) {
            if (i - max_i > mj - max_j) {
                if (max - m - ((i - max_i) - (mj - max_j)) * p->e_del > zdrop) break;
            } else {
                if (max - m - ((mj - max_j) - (i - max_i)) * p->e_ins > zdrop) break;
            }
        }
        for (j = beg; j < end && eh[j].h == 0 && eh[j].e == 0; ++j) ;
        beg = j;
        for (j = end; j >= beg && eh[j].h == 0 && eh[j].e == 0; --j) ;
        end = j + 2 < qlen ? j + 2 : qlen;
    }
    *_qle = max_j + 1; *_tle = max_i + 1; *_gtle = max_ie + 1; *_gscore = gscore;
    *_max_off = max_off;
    if (eh != eh_stack) free(eh);
    return max;
}

/* ---- ksw_global restated (bwa ksw.c ksw_global2) with traceback -------------------- */
static int push_cigar(uint32_t *cig, int n, int cap, int op, int len) {
    if (n > 0 && (int)(cig[n - 1] & 0xf) == op) { cig[n - 1] += (uint32_t)len << 4; return n; }
    if (n < cap) cig[n] = (uint32_t)len << 4 | (uint32_t)op;
    return n + 1;
}

/* returns score; writes cigar (ops M=0 I=1 D=2), *n_cig may exceed cap (overflow) */
int afo_global_dp(int qlen, const uint8_t *query, int tlen, const uint8_t *target, const afo_params *p,
                     int w, uint32_t *cig, int cap, int *n_cig) {
    int oe_del = p->o_del + p->e_del, oe_ins = p->o_ins + p->e_ins;
    int n_col = qlen < 2 * w + 1 ? qlen : 2 * w + 1;
    eh_t *eh = (eh_t *)malloc(sizeof(eh_t) * (qlen + 1));
    uint8_t *z = (uint8_t *)malloc((size_t)n_col * (tlen > 0 ? tlen : 1));
    int i, j, k;
    eh[0].h = 0; eh[0].e = NEG_INF;
    for (j = 1; j <= qlen && j <= w; ++j) { eh[j].h = -(p->o_ins + p->e_ins * j); eh[j].e = NEG_INF; }
    for (; j <= qlen; ++j) eh[j].h = eh[j].e = NEG_INF;
    for (i = 0; i < tlen; ++i) {
        int32_t f = NEG_INF, h1, beg, end, t;
        uint8_t *zi = z + (size_t)i * n_col;
        beg = i > w ? i - w : 0;
        end = i + w + 1 < qlen ? i + w + 1 : qlen;
        h1 = beg == 0 ? -(p->o_del + p->e_del * (i + 1)) : NEG_INF;
        for (j = beg; j < end; ++j) {
            eh_t *q = &eh[j];
            int32_t h, m = q->h, e = q->e;
            uint8_t d;
            q->h = h1;
            m += afo_sc(p, target[i], query[j]);
            d = m >= e ? 0 : 1;
            h = m >= e ? m : e;
            d = h >= f ? d : 2;
            h = h >= f ? h : f;
            h1 = h;
            t = m - oe_del;
            e -= p->e_del;
            d |= e > t ? 1 << 2 : 0;
            e = e > t ? e : t;
            q->e = e;
            t = m - oe_ins;
            f -= p->e_ins;
            d |= f > t ? 2 << 4 : 0;
            f = f > t ? f : t;
            zi[j - beg] = d;
        }
        eh[end].h = h1; eh[end].e = NEG_INF;
    }
    int score = eh[qlen].h;
    /* backtrack from the last cell, then reverse */
    int nc = 0, which = 0;
    uint32_t tmp_stack[2 * AFO_MAX_READ + 8];
    int tcap = qlen + tlen + 8 > 2 * AFO_MAX_READ + 8 ? qlen + tlen + 8 : 2 * AFO_MAX_READ + 8;
    uint32_t *tmp = tcap > 2 * AFO_MAX_READ + 8 ? (uint32_t *)malloc(sizeof(uint32_t) * tcap) : tmp_stack;
    i = tlen - 1;
    k = (i + w + 1 < qlen ? i + w + 1 : qlen) - 1;
    while (i >= 0 && k >= 0) {
        which = z[(size_t)i * n_col + (k - (i > w ? i - w : 0))] >> (which << 1) & 3;
        if (which == 0) { nc = push_cigar(tmp, nc, tcap, 0, 1); --i; --k; }
        else if (which == 1) { nc = push_cigar(tmp, nc, tcap, 2, 1); --i; }
        else { nc = push_cigar(tmp, nc, tcap, 1, 1); --k; }
    }
    if (i >= 0) nc = push_cigar(tmp, nc, tcap, 2, i + 1);
    if (k >= 0) nc = push_cigar(tmp, nc, tcap, 1, k + 1);
    for (int x = 0; x < nc && x < cap; ++x) cig[x] = tmp[nc - 1 - x];
    *n_cig = nc;
    free(eh); free(z);
    if (tmp != tmp_stack) free(tmp);
    return score;
}

/* ---- bwa helpers restated (bwamem.c cal_max_gap / infer_bw) ------------------------ */
int afo_cal_max_gap(const afo_params *p, int qlen) {
    int l_del = (int)((double)(qlen * p->a - p->o_del) / p->e_del + 1.);
    int l_ins = (int)((double)(qlen * p->a - p->o_ins) / p->e_ins + 1.);
    int l = l_del > l_ins ? l_del : l_ins;
    l = l > 1 ? l : 1;
    return l < p->w << 1 ? l : p->w << 1;
}

int afo_infer_bw(int l1, int l2, int score, int a, int q, int r) {
    int w;
    if (l1 == l2 && l1 * a - score < (q + r - a) << 1) return 0;
    w = (int)((double)((l1 < l2 ? l1 : l2) * a - score - q) / r + 2.);
    int d = l1 - l2 < 0 ? l2 - l1 : l1 - l2;
    if (w < d) w = d;
    return w;
}

/* bwa_gen_cigar2 restated; query/ref segments in forward-reference orientation; at most cap ops
 * written (*n_cig counts them all) */
int afo_gen_cigar_cap(const uint8_t *text, int64_t n, const afo_params *p, int w_, int lq, const uint8_t *qseg,
                      int64_t rb, int64_t re, uint32_t *cig, int cap, int *n_cig) {
    int rlen = (int)(re - rb);
    int score = 0;
    uint8_t qq_stack[AFO_MAX_READ], rr_stack[2 * AFO_MAX_READ + 512];  /* longer (afo_blat_long): heap */
    uint8_t *qq = lq <= AFO_MAX_READ ? qq_stack : (uint8_t *)malloc(lq);
    uint8_t *rr = rlen <= 2 * AFO_MAX_READ + 512 ? rr_stack : (uint8_t *)malloc(rlen);
    for (int i = 0; i < lq; ++i) qq[i] = qseg[i];
    for (int i = 0; i < rlen; ++i) rr[i] = text[rb + i];
    if (rb >= n) { /* reverse both so indels land leftmost in forward coordinates */
        for (int i = 0; i < lq >> 1; ++i) { uint8_t t = qq[i]; qq[i] = qq[lq - 1 - i]; qq[lq - 1 - i] = t; }
        for (int i = 0; i < rlen >> 1; ++i) { uint8_t t = rr[i]; rr[i] = rr[rlen - 1 - i]; rr[rlen - 1 - i] = t; }
    }
    if (lq == rlen && w_ == 0) {
        cig[0] = (uint32_t)lq << 4;
        *n_cig = 1;
        for (int i = 0; i < lq; ++i) score += afo_sc(p, rr[i], qq[i]);
    } else {
        int max_ins = (int)((double)(((lq + 1) >> 1) * p->a - p->o_ins) / p->e_ins + 1.);
        int max_del = (int)((double)(((lq + 1) >> 1) * p->a - p->o_del) / p->e_del + 1.);
        int max_gap = max_ins > max_del ? max_ins : max_del;
        max_gap = max_gap > 1 ? max_gap : 1;
        int d = rlen - lq < 0 ? lq - rlen : rlen - lq;
        int w = (max_gap + d + 1) >> 1;
        w = w < w_ ? w : w_;
        int min_w = d + 3;
        w = w > min_w ? w : min_w;
        score = afo_global_dp(lq, qq, rlen, rr, p, w, cig, cap, n_cig);
    }
    if (qq != qq_stack) free(qq);
    if (rr != rr_stack) free(rr);
    return score;
}

int afo_gen_cigar(const uint8_t *text, int64_t n, const afo_params *p, int w_, int lq, const uint8_t *qseg,
                  int64_t rb, int64_t re, uint32_t *cig, int *n_cig) {
    return afo_gen_cigar_cap(text, n, p, w_, lq, qseg, rb, re, cig, AFO_MAX_CIGAR, n_cig);
}
