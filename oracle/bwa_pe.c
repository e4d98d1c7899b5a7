/*
 * bwa_pe.c -- TEST INFRASTRUCTURE ONLY (see af_oracle.h).
 *
 * Plain-C restatement of the reference's `bwa mem -M` calls as bwa 0.7.17 computes them:
 *     S2  bwa mem -M -t T <anchor.fa> fq1 fq2          (Anchored_Fusion.py:182), paired-end
 *     S4  bwa mem -M -t T <genome.fa> tmp1 tmp2        (Anchored_Fusion.py:188), paired-end
 *     S5  bwa mem -M -t T <genome.fa> split_reads.fa   (functions.py:716), single-end
 * bwa is a third-party binary (README.md:18, "bwa >= 0.7.17"), not vendored under
 * /root/reference and absent from this image, so this file restates its published source routine
 * by routine; each function names the bwa / klib routine it follows (bwamem.c, bwamem_pair.c,
 * bwt.c, bntseq.c, ksw.c; klib ksort.h and kbtree.h as vendored by bwa).  The product path never
 * loads this file; it is the parity contract of the HIP kernels (csrc/s2.hip for the anchor,
 * csrc/bwa_genome.hip + csrc/fmindex.hip for the genome).
 *
 * The bwa text.  bns_fasta2bntseq concatenates the contigs (no separators) into pac, replacing
 * every non-ACGT base by lrand48() & 3 after srand48(11); the index is built over
 * T = pac ++ revcomp(pac).  Contigs are the bns "anns": seeds crossing a contig or the strand
 * boundary are dropped (bns_intv2rid), extension windows are clipped to the seed's contig
 * (bns_fetch_seq), reported positions are contig-relative (bns_depos, bns_pos2rid).
 *
 * Seeds, two restatements of mem_collect_intv that must agree:
 *  - FM mode (genome texts): bwt_smem1 / bwt_seed_strategy1 over a bidirectional FM index of
 *    T (suffix array by prefix doubling, BWT occurrence checkpoints, bwt_extend), occurrences
 *    by the suffix array (bwt_sa) -- the routines themselves;
 *  - MEM-set mode (the anchor, csrc/s2.hip's contract): the same sets from the read's
 *    position-level maximal exact matches (MEMs >= min_seed_len) against T and T's suffix ranks:
 *      pass 1 (bwt_smem1 with min_intv 1) = the maximal MEM query intervals;
 *      pass 2 (re-seeding, bwt_smem1 at the middle with min_intv = occ + 1) = the maximal
 *             intervals holding the middle position that occur >= occ + 1 times;
 *      pass 3 (bwt_seed_strategy1) = the shortest >= 20-nt prefix from x occurring < 20 times.
 *    tests/test_oracle_fm.py checks the two produce identical seed lists (intervals, counts and
 *    occurrence order) on the anchor and on genomes with repeat families.
 *
 * Caps (part of the GPU/oracle contract): per read at most caps.pmem MEMs
 * (MEM-set mode), caps.intv seed intervals, caps.occ chain seeds, caps.chain chains and caps.reg
 * regions; past one the read is reported unmapped with AF_FLAG_MEM_OVERFLOW (bwa has no caps).
 * The anchor's caps are AFO_PE_MAX_*, the genome's AFO_G_MAX_*.
 */
#include "af_oracle.h"
#include "af_oracle_int.h"
#include <math.h>
#include <stddef.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#ifndef M_SQRT1_2
#define M_SQRT1_2 0.70710678118654752440 /* glibc math.h */
#endif

/* bwa 0.7.17 constants (bwamem.c, bwamem_pair.c) */
#define MEM_MAPQ_COEF 30.0
#define PATCH_MAX_R_BW 0.05f
#define PATCH_MIN_SC_RATIO 0.90f
#define MIN_RATIO 0.8
#define MIN_DIR_CNT 10
#define MIN_DIR_RATIO 0.05
#define OUTLIER_BOUND 2.0
#define MAPPING_BOUND 3.0
#define MAX_STDDEV 4.0
#define KSW_XBYTE 0x10000
#define KSW_XSTOP 0x20000
#define KSW_XSUBO 0x40000
#define KSW_XSTART 0x80000
/* mem_opt_init float options (not settable through the reference's command line) */
static const float opt_split_factor = 1.5f, opt_mask_level = 0.50f, opt_drop_ratio = 0.50f,
                   opt_mask_level_redun = 0.95f;

#define FLAG_MEM_OVERFLOW 0x10000
#define FLAG_CIGAR_OVERFLOW 0x20000

/* ================================================================================ text */
typedef struct { int pmem, intv, occ, chain, reg; } caps_t;
static const caps_t CAPS_ANCHOR = {AFO_PE_MAX_PMEM, AFO_PE_MAX_SEED, AFO_PE_MAX_OCC, AFO_PE_MAX_CHAIN, AFO_PE_MAX_REG};
static const caps_t CAPS_GENOME = {AFO_G_MAX_PMEM, AFO_G_MAX_INTV, AFO_G_MAX_OCC, AFO_G_MAX_CHAIN, AFO_G_MAX_REG};

#define OCC_SHIFT 6  /* FM occurrence checkpoint every 64 rows */

struct afo_text {
    int64_t n, N;       /* l_pac, N = 2 l_pac                                              */
    uint8_t *T;         /* codes 0..3                                                      */
    int n_ctg;          /* bns anns: contig offsets / lengths in pac                        */
    int64_t *ctg_off, *ctg_len;
    caps_t caps;
    /* MEM-set mode */
    int32_t *rank;      /* suffix rank of T[i..] (bwt_sa order)                            */
    uint64_t *km;       /* every 16-mer position of T: (packed << 32 | pos), sorted        */
    int64_t nkm;
    int64_t base_cnt[4];
    /* FM mode: rows 0..N of the suffix array of T$ ('$' smallest; row 0 = the empty suffix) */
    int fm;
    int64_t *sa;        /* sa[row] = text position (sa[0] = N)                              */
    uint8_t *bwt;       /* bwt[row] = T[sa[row] - 1], 4 for the row of sa = 0 (primary)      */
    int64_t *occ;       /* occ[(row >> OCC_SHIFT) * 4 + c]: c in bwt[0, row & ~63)          */
    int64_t C[4];       /* first row of the suffixes starting with c                        */
    int64_t primary;
};

/* srand48(11) / lrand48() as glibc defines them (POSIX drand48 family): bns_fasta2bntseq
 * seeds with bns->seed = 11 and replaces every ambiguous base by lrand48() & 3 */
typedef struct { uint64_t x; } rand48_t;
static void srand48_r11(rand48_t *r, long seed) { r->x = (((uint64_t)(uint32_t)seed) << 16) | 0x330Eu; }
static long lrand48_r11(rand48_t *r) {
    r->x = (0x5DEECE66DULL * r->x + 0xBULL) & ((1ULL << 48) - 1);
    return (long)(r->x >> 17);
}

static int cmp_u64v(const void *a, const void *b) {
    uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return x < y ? -1 : x > y;
}

/* Suffix array of T (length N) with '$' smallest, by prefix doubling (Manber-Myers with the
 * bucket trick): sa has N + 1 rows, sa[0] = N.  Ranks are group starts among rows 1..N.
 * Used for texts too long for the int32 SA-IS below, and as its cross-check. */
static int64_t *suffix_array_doubling(const uint8_t *T, int64_t N) {
    int64_t *sa = (int64_t *)malloc(sizeof(int64_t) * (N + 1));
    int64_t *rk = (int64_t *)malloc(sizeof(int64_t) * (N + 1)), *tmp = (int64_t *)malloc(sizeof(int64_t) * (N + 1));
    int64_t *cur = (int64_t *)malloc(sizeof(int64_t) * (N + 1));
    int64_t cnt[5] = {0, 0, 0, 0, 0};
    for (int64_t i = 0; i < N; ++i) ++cnt[T[i]];
    int64_t st[5];
    st[0] = 0;
    for (int c = 1; c < 5; ++c) st[c] = st[c - 1] + cnt[c - 1];
    int64_t pos[4] = {st[0], st[1], st[2], st[3]};
    for (int64_t i = 0; i < N; ++i) sa[pos[T[i]]++] = i;  /* sa[0, N): suffixes (no '$' row yet) */
    for (int64_t i = 0; i < N; ++i) rk[i] = st[T[i]];
    for (int64_t h = 1; h < N; h <<= 1) {
        /* order by (rk[i], rk[i + h] or -1): the suffixes i >= N - h first (second key -1),
         * then i = sa[j] - h in sa order; a stable pass by rk (group starts) */
        int64_t m = 0;
        for (int64_t i = N - h; i < N; ++i) tmp[m++] = i;
        for (int64_t j = 0; j < N; ++j)
            if (sa[j] >= h) tmp[m++] = sa[j] - h;
        for (int64_t j = 0; j < N; ++j) cur[j] = j;  /* group start -> next free slot */
        for (int64_t j = 0; j < N; ++j) { int64_t i = tmp[j]; sa[cur[rk[i]]++] = i; }
        /* new group starts */
        int64_t done = 1;
        tmp[sa[0]] = 0;
        for (int64_t j = 1; j < N; ++j) {
            int64_t a = sa[j - 1], b = sa[j];
            int64_t ra2 = a + h < N ? rk[a + h] : -1, rb2 = b + h < N ? rk[b + h] : -1;
            if (rk[a] == rk[b] && ra2 == rb2) { tmp[b] = tmp[a]; done = 0; }
            else tmp[b] = j;
        }
        memcpy(rk, tmp, sizeof(int64_t) * N);
        if (done) break;
    }
    /* rows: 0 = the empty suffix, then sa shifted by one */
    memmove(sa + 1, sa, sizeof(int64_t) * N);
    sa[0] = N;
    free(rk); free(tmp); free(cur);
    return sa;
}

/* SA-IS (Nong, Zhang & Chan 2009: induced sorting of the LMS substrings, recursion on their
 * names) over int32 symbols s[0, n) in [0, K) whose last symbol is a unique smallest sentinel.
 * The suffix array is unique, so this equals the doubling construction (and bwa's is.c) row for
 * row; it is linear, which lets the oracle index tens of Mbp in seconds. */
#define SAIS_T(i) ((t[(i) >> 3] >> ((i) & 7)) & 1)
#define SAIS_LMS(i) ((i) > 0 && SAIS_T(i) && !SAIS_T((i) - 1))
static void sais_buckets(const int32_t *s, int32_t n, int32_t K, int32_t *bkt, int end) {
    memset(bkt, 0, sizeof(int32_t) * K);
    for (int32_t i = 0; i < n; ++i) ++bkt[s[i]];
    int32_t sum = 0;
    for (int32_t c = 0; c < K; ++c) { sum += bkt[c]; bkt[c] = end ? sum : sum - bkt[c]; }
}
static void sais_induce(const uint8_t *t, int32_t *SA, const int32_t *s, int32_t *bkt, int32_t n, int32_t K) {
    sais_buckets(s, n, K, bkt, 0);  /* L-type suffixes, left to right from the bucket heads */
    for (int32_t i = 0; i < n; ++i) {
        const int32_t j = SA[i] - 1;
        if (SA[i] > 0 && !SAIS_T(j)) SA[bkt[s[j]]++] = j;
    }
    sais_buckets(s, n, K, bkt, 1);  /* S-type suffixes, right to left from the bucket tails */
    for (int32_t i = n - 1; i >= 0; --i) {
        const int32_t j = SA[i] - 1;
        if (SA[i] > 0 && SAIS_T(j)) SA[--bkt[s[j]]] = j;
    }
}
static void sais(const int32_t *s, int32_t *SA, int32_t n, int32_t K) {
    uint8_t *t = (uint8_t *)calloc((size_t)n / 8 + 1, 1);
    int32_t *bkt = (int32_t *)malloc(sizeof(int32_t) * K);
    /* types: S if s[i] < s[i + 1], or equal and s[i + 1] is S; the sentinel is S */
    t[(n - 1) >> 3] |= (uint8_t)(1 << ((n - 1) & 7));
    for (int32_t i = n - 2; i >= 0; --i)
        if (s[i] < s[i + 1] || (s[i] == s[i + 1] && SAIS_T(i + 1))) t[i >> 3] |= (uint8_t)(1 << (i & 7));
    /* stage 1: the LMS substrings sorted by one induction */
    sais_buckets(s, n, K, bkt, 1);
    for (int32_t i = 0; i < n; ++i) SA[i] = -1;
    for (int32_t i = 1; i < n; ++i)
        if (SAIS_LMS(i)) SA[--bkt[s[i]]] = i;
    sais_induce(t, SA, s, bkt, n, K);
    int32_t n1 = 0;
    for (int32_t i = 0; i < n; ++i)
        if (SAIS_LMS(SA[i])) SA[n1++] = SA[i];
    /* names of the LMS substrings (equal substrings share a name) at SA[n1 + pos / 2] */
    for (int32_t i = n1; i < n; ++i) SA[i] = -1;
    int32_t name = 0, prev = -1;
    for (int32_t i = 0; i < n1; ++i) {
        const int32_t pos = SA[i];
        int diff = 0;
        for (int32_t d = 0; d < n; ++d) {
            if (prev == -1 || pos + d == n - 1 || prev + d == n - 1 || s[pos + d] != s[prev + d] ||
                SAIS_T(pos + d) != SAIS_T(prev + d)) { diff = 1; break; }
            if (d > 0 && (SAIS_LMS(pos + d) || SAIS_LMS(prev + d))) break;
        }
        if (diff) { ++name; prev = pos; }
        SA[n1 + pos / 2] = name - 1;
    }
    for (int32_t i = n - 1, j = n - 1; i >= n1; --i)
        if (SA[i] >= 0) SA[j--] = SA[i];
    /* stage 2: the reduced string's suffix array (recursion while names repeat) */
    int32_t *s1 = SA + n - n1, *SA1 = SA;
    if (name < n1) sais(s1, SA1, n1, name);
    else for (int32_t i = 0; i < n1; ++i) SA1[s1[i]] = i;
    /* stage 3: the LMS suffixes in order at their buckets' tails, then one induction */
    sais_buckets(s, n, K, bkt, 1);
    for (int32_t i = 1, j = 0; i < n; ++i)
        if (SAIS_LMS(i)) s1[j++] = i;
    for (int32_t i = 0; i < n1; ++i) SA1[i] = s1[SA1[i]];
    for (int32_t i = n1; i < n; ++i) SA[i] = -1;
    for (int32_t i = n1 - 1; i >= 0; --i) {
        const int32_t j = SA[i];
        SA[i] = -1;
        SA[--bkt[s[j]]] = j;
    }
    sais_induce(t, SA, s, bkt, n, K);
    free(t);
    free(bkt);
}
#undef SAIS_T
#undef SAIS_LMS

/* Suffix array of T (codes 0..3, length N) with '$' smallest: rows 0..N, sa[0] = N */
static int64_t *suffix_array(const uint8_t *T, int64_t N) {
    if (N + 1 >= INT32_MAX || N < 1) return suffix_array_doubling(T, N);
    const int32_t n = (int32_t)(N + 1);
    int32_t *s = (int32_t *)malloc(sizeof(int32_t) * n), *SA = (int32_t *)malloc(sizeof(int32_t) * n);
    for (int32_t i = 0; i < n - 1; ++i) s[i] = T[i] + 1;
    s[n - 1] = 0;
    sais(s, SA, n, 5);
    free(s);
    int64_t *sa = (int64_t *)malloc(sizeof(int64_t) * (N + 1));
    for (int32_t i = 0; i < n; ++i) sa[i] = SA[i];
    free(SA);
    return sa;
}

/* test hook: SA-IS and the doubling construction agree on T (0 = equal, else first differing row + 1) */
int64_t afo_suffix_array_check(const uint8_t *T, int64_t N) {
    int64_t *a = suffix_array(T, N), *b = suffix_array_doubling(T, N), r = 0;
    for (int64_t i = 0; i <= N && !r; ++i)
        if (a[i] != b[i]) r = i + 1;
    free(a);
    free(b);
    return r;
}

/* FM mode: the BWT of T$ and its occurrence checkpoints (bwt_t: bwt_occ4, primary, L2) */
static void build_fm(afo_text *X) {
    int64_t N = X->N;
    X->sa = suffix_array(X->T, N);
    X->bwt = (uint8_t *)malloc(N + 1);
    X->primary = -1;
    for (int64_t r = 0; r <= N; ++r) {
        int64_t p = X->sa[r];
        if (p == 0) { X->bwt[r] = 4; X->primary = r; }
        else X->bwt[r] = X->T[p - 1];
    }
    int64_t nb = ((N + 1) >> OCC_SHIFT) + 1;
    X->occ = (int64_t *)calloc((size_t)(nb + 1) * 4, sizeof(int64_t));
    int64_t c4[4] = {0, 0, 0, 0};
    for (int64_t r = 0; r <= N; ++r) {
        if ((r & ((1 << OCC_SHIFT) - 1)) == 0) memcpy(X->occ + (r >> OCC_SHIFT) * 4, c4, sizeof(c4));
        if (X->bwt[r] < 4) ++c4[X->bwt[r]];
    }
    X->C[0] = 1;
    for (int c = 1; c < 4; ++c) X->C[c] = X->C[c - 1] + X->base_cnt[c - 1];
    X->fm = 1;
}

/* suffix ranks + 16-mer positions (MEM-set mode) */
static void build_memset(afo_text *X) {
    int64_t N = X->N;
    int64_t *sa = X->sa ? X->sa : suffix_array(X->T, N);
    X->rank = (int32_t *)malloc(sizeof(int32_t) * N);
    for (int64_t r = 1; r <= N; ++r) X->rank[sa[r]] = (int32_t)(r - 1);
    if (!X->sa) free(sa);
    X->nkm = N >= AFO_K ? N - AFO_K + 1 : 0;
    X->km = (uint64_t *)malloc(sizeof(uint64_t) * (X->nkm + 1));
    for (int64_t p = 0; p < X->nkm; ++p) {
        uint32_t v = 0;
        for (int u = 0; u < AFO_K; ++u) v |= (uint32_t)X->T[p + u] << (2 * u);
        X->km[p] = (uint64_t)v << 32 | (uint64_t)p;
    }
    qsort(X->km, X->nkm, sizeof(uint64_t), cmp_u64v);
}

/* bns_fasta2bntseq over contigs [off_k, off_k + len_k) of seq, then the reverse complement */
static afo_text *text_new(const char *seq, const int64_t *off, const int64_t *len, int n_ctg) {
    int64_t n = 0;
    for (int k = 0; k < n_ctg; ++k) n += len[k];
    if (n <= 0) return NULL;
    afo_text *X = (afo_text *)calloc(1, sizeof(afo_text));
    X->n = n; X->N = 2 * n;
    X->T = (uint8_t *)malloc(X->N);
    X->n_ctg = n_ctg;
    X->ctg_off = (int64_t *)malloc(sizeof(int64_t) * n_ctg);
    X->ctg_len = (int64_t *)malloc(sizeof(int64_t) * n_ctg);
    rand48_t rs;
    srand48_r11(&rs, 11);
    int64_t i = 0;
    for (int k = 0; k < n_ctg; ++k) {
        X->ctg_off[k] = i;
        X->ctg_len[k] = len[k];
        for (int64_t j = 0; j < len[k]; ++j, ++i) {
            int c = afo_nt4((uint8_t)seq[off[k] + j]);
            if (c >= 4) c = (int)(lrand48_r11(&rs) & 3);
            X->T[i] = (uint8_t)c;
            X->T[X->N - 1 - i] = (uint8_t)(3 - c);
        }
    }
    for (int64_t j = 0; j < X->N; ++j) ++X->base_cnt[X->T[j]];
    return X;
}

afo_text *afo_text_build(const char *anchor, int64_t n) {
    if (n <= 0) return NULL;
    int64_t off = 0;
    afo_text *X = text_new(anchor, &off, &n, 1);
    X->caps = CAPS_ANCHOR;
    build_memset(X);
    return X;
}

afo_genome *afo_genome_build(const char *blob, const int64_t *ctg_off, const int64_t *ctg_len, int n_ctg,
                             int memset_too) {
    if (n_ctg < 1) return NULL;
    afo_text *X = text_new(blob, ctg_off, ctg_len, n_ctg);
    if (!X) return NULL;
    X->caps = CAPS_GENOME;
    build_fm(X);
    if (memset_too) build_memset(X);
    return X;
}

void afo_text_free(afo_text *X) {
    if (!X) return;
    free(X->T); free(X->rank); free(X->km); free(X->ctg_off); free(X->ctg_len);
    free(X->sa); free(X->bwt); free(X->occ); free(X);
}
void afo_genome_free(afo_genome *G) { afo_text_free(G); }
const uint8_t *afo_text_codes(const afo_text *X) { return X->T; }
int64_t afo_genome_lpac(const afo_genome *G) { return G->n; }
const uint8_t *afo_genome_text(const afo_genome *G) { return G->T; }
const int64_t *afo_genome_sa(const afo_genome *G) { return G->sa; }
int64_t afo_genome_primary(const afo_genome *G) { return G->primary; }

uint64_t *afo_text_kmers_noncrossing(const afo_text *X, int64_t *m) {
    uint64_t *o = (uint64_t *)malloc(sizeof(uint64_t) * (X->nkm + 1));
    int64_t c = 0;
    for (int64_t i = 0; i < X->nkm; ++i) {
        int64_t p = (int64_t)(X->km[i] & 0xffffffffu);
        if (p < X->n && p + AFO_K > X->n) continue;
        o[c++] = X->km[i];
    }
    *m = c;
    return o;
}

/* ======================================================================= bntseq.c */
/* bns_pos2rid: the contig holding forward position pos_f (< l_pac) */
static int pos2rid(const afo_text *X, int64_t pos_f) {
    if (pos_f >= X->n) return -1;
    int left = 0, mid = 0, right = X->n_ctg;
    while (left < right) {
        mid = (left + right) >> 1;
        if (pos_f >= X->ctg_off[mid]) {
            if (mid == X->n_ctg - 1) break;
            if (pos_f < X->ctg_off[mid + 1]) break;
            left = mid + 1;
        } else right = mid;
    }
    return mid;
}
static inline int64_t depos(const afo_text *X, int64_t pos, int *is_rev) {
    return (*is_rev = (pos >= X->n)) ? (X->n << 1) - 1 - pos : pos;
}
/* bns_intv2rid: -2 across the strand boundary, -1 across contigs */
static int intv2rid(const afo_text *X, int64_t rb, int64_t re) {
    int is_rev, rid_b, rid_e;
    if (rb < X->n && re > X->n) return -2;
    rid_b = pos2rid(X, depos(X, rb, &is_rev));
    rid_e = rb < re ? pos2rid(X, depos(X, re - 1, &is_rev)) : rid_b;
    return rid_b == rid_e ? rid_b : -1;
}
/* bns_fetch_seq's clipping: [*beg, *end) limited to the contig (on its strand) holding mid */
static void fetch_clip(const afo_text *X, int64_t *beg, int64_t mid, int64_t *end, int *rid) {
    int is_rev;
    if (*end < *beg) { int64_t t = *end; *end = *beg; *beg = t; }
    *rid = pos2rid(X, depos(X, mid, &is_rev));
    int64_t far_beg = X->ctg_off[*rid], far_end = far_beg + X->ctg_len[*rid];
    if (is_rev) {
        int64_t t = far_beg;
        far_beg = (X->n << 1) - far_end;
        far_end = (X->n << 1) - t;
    }
    *beg = *beg > far_beg ? *beg : far_beg;
    *end = *end < far_end ? *end : far_end;
}

/* ===================================================================== klib ksort.h */
/* ks_introsort / ks_combsort / __ks_insertsort exactly as klib's KSORT_INIT generates them
 * (bwa vendors ksort.h): unstable, so tie orders are part of bwa's behaviour. */
#define AFO_KSORT_INIT(name, type_t, lt)                                                           \
    static void ins_##name(type_t *s, type_t *t) {                                                 \
        type_t *i, *j, sw;                                                                         \
        for (i = s + 1; i < t; ++i)                                                                \
            for (j = i; j > s && lt(*j, *(j - 1)); --j) { sw = *j; *j = *(j - 1); *(j - 1) = sw; } \
    }                                                                                              \
    static void comb_##name(size_t n, type_t a[]) {                                                \
        const double shrink_factor = 1.2473309501039786540366528676643;                            \
        int do_swap;                                                                               \
        size_t gap = n;                                                                            \
        type_t tmp, *i, *j;                                                                        \
        do {                                                                                       \
            if (gap > 2) {                                                                         \
                gap = (size_t)(gap / shrink_factor);                                               \
                if (gap == 9 || gap == 10) gap = 11;                                               \
            }                                                                                      \
            do_swap = 0;                                                                           \
            for (i = a; i < a + n - gap; ++i) {                                                    \
                j = i + gap;                                                                       \
                if (lt(*j, *i)) { tmp = *i; *i = *j; *j = tmp; do_swap = 1; }                      \
            }                                                                                      \
        } while (do_swap || gap > 2);                                                              \
        if (gap != 1) ins_##name(a, a + n);                                                        \
    }                                                                                              \
    static void introsort_##name(size_t n, type_t a[]) {                                           \
        int d;                                                                                     \
        struct { type_t *left, *right; int depth; } stack[160], *top;                              \
        type_t rp, sw;                                                                             \
        type_t *s, *t, *i, *j, *k;                                                                 \
        if (n < 1) return;                                                                         \
        else if (n == 2) {                                                                         \
            if (lt(a[1], a[0])) { sw = a[0]; a[0] = a[1]; a[1] = sw; }                             \
            return;                                                                                \
        }                                                                                          \
        for (d = 2; 1ul << d < n; ++d) ;                                                           \
        top = stack; s = a; t = a + (n - 1); d <<= 1;                                              \
        while (1) {                                                                                \
            if (s < t) {                                                                           \
                if (--d == 0) { comb_##name(t - s + 1, s); t = s; continue; }                      \
                i = s; j = t; k = i + ((j - i) >> 1) + 1;                                          \
                if (lt(*k, *i)) {                                                                  \
                    if (lt(*k, *j)) k = j;                                                         \
                } else k = lt(*j, *i) ? i : j;                                                     \
                rp = *k;                                                                           \
                if (k != t) { sw = *k; *k = *t; *t = sw; }                                         \
                for (;;) {                                                                         \
                    do ++i; while (lt(*i, rp));                                                    \
                    do --j; while (i <= j && lt(rp, *j));                                          \
                    if (j <= i) break;                                                             \
                    sw = *i; *i = *j; *j = sw;                                                     \
                }                                                                                  \
                sw = *i; *i = *t; *t = sw;                                                         \
                if (i - s > t - i) {                                                               \
                    if (i - s > 16) { top->left = s; top->right = i - 1; top->depth = d; ++top; }  \
                    s = t - i > 16 ? i + 1 : t;                                                    \
                } else {                                                                           \
                    if (t - i > 16) { top->left = i + 1; top->right = t; top->depth = d; ++top; }  \
                    t = i - s > 16 ? i - 1 : s;                                                    \
                }                                                                                  \
            } else {                                                                               \
                if (top == stack) { ins_##name(a, a + n); return; }                                \
                --top; s = top->left; t = top->right; d = top->depth;                              \
            }                                                                                      \
        }                                                                                          \
    }

/* ===================================================================== bwa structures */
typedef struct { int64_t rbeg; int32_t qbeg, len, score; } seed_t;  /* mem_seed_t */

typedef struct {                                                     /* mem_chain_t */
    int n, first, rid;
    int w, kept;
    int64_t pos;
    int seed0;      /* index of the chain's first seed in the read's seed pool */
} chain_t;

typedef struct {                                                     /* mem_alnreg_t */
    int64_t rb, re;
    int qb, qe, rid, score, truesc, sub, alt_sc, csub, sub_n, w, seedcov, secondary, secondary_all, seedlen0;
    int n_comp, is_alt;
    uint64_t hash;
} alnreg_t;

typedef struct { int low, high, failed; double avg, std; } pestat_t; /* mem_pestat_t */
typedef struct { uint64_t x, y; } pair64_t;
typedef struct { int64_t k, l, s; int qb, qe; } biv_t;              /* bwtintv_t: x[0..2], info */

#define lt_u64(a, b) ((a) < (b))
#define lt_pair64(a, b) ((a).x < (b).x || ((a).x == (b).x && (a).y < (b).y))
#define lt_flt(a, b) ((a).w > (b).w)                                               /* mem_flt */
#define lt_ars2(a, b) ((a).re < (b).re)                                            /* alnreg_slt2 */
#define lt_ars(a, b) ((a).score > (b).score || ((a).score == (b).score && ((a).rb < (b).rb || ((a).rb == (b).rb && (a).qb < (b).qb))))
#define lt_ars_hash(a, b) ((a).score > (b).score || ((a).score == (b).score && (a).hash < (b).hash))
#define lt_intv(a, b) ((((uint64_t)(a).qb << 32) | (uint32_t)(a).qe) < (((uint64_t)(b).qb << 32) | (uint32_t)(b).qe))
AFO_KSORT_INIT(u64, uint64_t, lt_u64)
AFO_KSORT_INIT(p128, pair64_t, lt_pair64)
AFO_KSORT_INIT(flt, chain_t, lt_flt)
AFO_KSORT_INIT(ars2, alnreg_t, lt_ars2)
AFO_KSORT_INIT(ars, alnreg_t, lt_ars)
AFO_KSORT_INIT(arsh, alnreg_t, lt_ars_hash)
AFO_KSORT_INIT(intv, biv_t, lt_intv)

/* utils.h hash_64 */
static uint64_t hash_64(uint64_t key) {
    key += ~(key << 32);
    key ^= (key >> 22);
    key += ~(key << 13);
    key ^= (key >> 8);
    key += (key << 3);
    key ^= (key >> 15);
    key += ~(key << 27);
    key ^= (key >> 31);
    return key;
}

/* a region list (mem_alnreg_v) that grows up to the text's region cap */
typedef struct { alnreg_t *a; int n, m; } regv_t;
static alnreg_t *regv_push(regv_t *v, int cap) {
    if (v->n >= cap) return NULL;
    if (v->n == v->m) {
        v->m = v->m ? v->m * 2 : 8;
        if (v->m > cap) v->m = cap;
        v->a = (alnreg_t *)realloc(v->a, sizeof(alnreg_t) * v->m);
    }
    return &v->a[v->n++];
}

/* ======================================================================= read state */
typedef struct { int32_t s, t; int64_t r; } pmem_t;            /* position-level MEM */
/* a seed interval: query [qb, qe), cnt occurrences, in MEM-set mode at occ[occ0 ..], in FM
 * mode at sa[sa_k ..] */
typedef struct { int32_t qb, qe; int64_t cnt, sa_k; int32_t occ0; } sintv_t;
typedef struct { seed_t s; int next; } sl_t;

/* per-thread work arrays sized by the caps (grown when a text with larger caps comes) */
typedef struct {
    caps_t caps;
    pmem_t *pm; sintv_t *si; int64_t *occ; seed_t *seed; chain_t *ch, *ch2; sl_t *pool; int *last_of, *order, *ibuf;
    uint64_t *srt;
    biv_t *mem1, *tmpa, *tmpb, *fm_mem;
    void *kbnodes;
} work_t;

typedef struct {
    const afo_text *X;
    const afo_params *p;
    const afo_pe *pe;
    const uint8_t *q;   /* read codes */
    int l;
    int overflow;
    work_t *w;
    int npm; pmem_t *pm;
    int nsi; sintv_t *si;
    int nocc; int64_t *occ;
    int nseed; seed_t *seed;   /* chain seeds, grouped per chain after mem_chain */
    int nch; chain_t *ch;
} rstate_t;

#define KB_T 5
#define KB_MAXK (2 * KB_T - 1)
typedef struct { int n, internal; int key[KB_MAXK]; int ptr[KB_MAXK + 1]; } kbnode_t;

static work_t *work_get(const caps_t *c) {
    static __thread work_t *W = NULL;
    if (W && W->caps.pmem >= c->pmem && W->caps.intv >= c->intv && W->caps.occ >= c->occ &&
        W->caps.chain >= c->chain && W->caps.reg >= c->reg)
        return W;
    if (W) {
        free(W->pm); free(W->si); free(W->occ); free(W->seed); free(W->ch); free(W->ch2); free(W->pool);
        free(W->last_of); free(W->order); free(W->ibuf); free(W->srt); free(W->mem1); free(W->tmpa); free(W->tmpb);
        free(W->fm_mem); free(W->kbnodes); free(W);
    }
    W = (work_t *)calloc(1, sizeof(work_t));
    W->caps = *c;
    int occ_cap = c->occ > c->pmem ? c->occ : c->pmem;  /* MEM-set mode stores every occurrence */
    W->pm = (pmem_t *)malloc(sizeof(pmem_t) * (c->pmem + 1));
    W->si = (sintv_t *)malloc(sizeof(sintv_t) * (c->intv + 1));
    W->occ = (int64_t *)malloc(sizeof(int64_t) * (occ_cap + 1));
    W->seed = (seed_t *)malloc(sizeof(seed_t) * (c->occ + 1));
    W->ch = (chain_t *)malloc(sizeof(chain_t) * (c->chain + 1));
    W->ch2 = (chain_t *)malloc(sizeof(chain_t) * (c->chain + 1));
    W->pool = (sl_t *)malloc(sizeof(sl_t) * (c->occ + 1));
    W->last_of = (int *)malloc(sizeof(int) * (c->chain + 1));
    W->order = (int *)malloc(sizeof(int) * (c->chain + 1));
    int ib = c->pmem > c->chain ? c->pmem : c->chain;
    W->ibuf = (int *)malloc(sizeof(int) * 3 * (ib + 1));
    W->srt = (uint64_t *)malloc(sizeof(uint64_t) * (c->occ + 1));
    W->mem1 = (biv_t *)malloc(sizeof(biv_t) * (AFO_MAX_READ + 2));
    W->tmpa = (biv_t *)malloc(sizeof(biv_t) * (AFO_MAX_READ + 2));
    W->tmpb = (biv_t *)malloc(sizeof(biv_t) * (AFO_MAX_READ + 2));
    W->fm_mem = (biv_t *)malloc(sizeof(biv_t) * (c->intv + AFO_MAX_READ + 2));
    W->kbnodes = malloc(sizeof(kbnode_t) * (2 * (size_t)c->chain + 4));
    return W;
}

/* ============================================================ seeds (mem_collect_intv) */
/* ---- MEM-set mode ------------------------------------------------------------------- */
static void find_pmems(rstate_t *S) {
    const afo_text *X = S->X;
    const uint8_t *q = S->q;
    int l = S->l;
    S->npm = 0;
    for (int s = 0; s + AFO_K <= l; ++s) {
        uint32_t v = 0;
        int ok = 1;
        for (int u = 0; u < AFO_K; ++u) {
            if (q[s + u] > 3) { ok = 0; break; }
            v |= (uint32_t)q[s + u] << (2 * u);
        }
        if (!ok) continue;
        uint64_t key = (uint64_t)v << 32;
        int64_t lo = 0, hi = X->nkm;
        while (lo < hi) { int64_t mid = (lo + hi) >> 1; if (X->km[mid] < key) lo = mid + 1; else hi = mid; }
        for (int64_t e = lo; e < X->nkm && (uint32_t)(X->km[e] >> 32) == v; ++e) {
            int64_t r = (int64_t)(X->km[e] & 0xffffffffu);
            if (s > 0 && q[s - 1] < 4 && r > 0 && X->T[r - 1] == q[s - 1]) continue;  /* not left-maximal */
            int len = AFO_K;
            while (s + len < l && r + len < X->N && q[s + len] == X->T[r + len]) ++len;
            if (len < S->p->min_seed_len) continue;
            if (S->npm >= X->caps.pmem) { S->overflow = 1; return; }
            S->pm[S->npm].s = s; S->pm[S->npm].t = s + len; S->pm[S->npm].r = r;
            ++S->npm;
        }
    }
}

/* number of occurrences of q[b, e) in T (e - b >= min_seed_len): MEMs covering [b, e) */
static int count_cov(const rstate_t *S, int b, int e) {
    int c = 0;
    for (int k = 0; k < S->npm; ++k) c += S->pm[k].s <= b && e <= S->pm[k].t;
    return c;
}

/* push seed interval [b, e) with its occurrences (bwt_sa order) */
static void push_intv(rstate_t *S, int b, int e) {
    if (S->overflow) return;
    if (S->nsi >= S->X->caps.intv) { S->overflow = 1; return; }
    sintv_t *v = &S->si[S->nsi++];
    v->qb = b; v->qe = e; v->occ0 = S->nocc; v->cnt = 0; v->sa_k = -1;
    /* every occurrence is stored (the anchor: AFO_PE_MAX_OCC = AFO_PE_MAX_PMEM, the S2 contract) */
    int occ_cap = S->X->caps.occ > S->X->caps.pmem ? S->X->caps.occ : S->X->caps.pmem;
    for (int k = 0; k < S->npm; ++k) {
        if (!(S->pm[k].s <= b && e <= S->pm[k].t)) continue;
        if (S->nocc >= occ_cap) { S->overflow = 1; return; }
        S->occ[S->nocc++] = S->pm[k].r + (b - S->pm[k].s);
        ++v->cnt;
    }
    /* suffix-rank order: insertion sort (counts are small) */
    int64_t *o = S->occ + v->occ0;
    for (int i = 1; i < v->cnt; ++i)
        for (int j = i; j > 0 && S->X->rank[o[j]] < S->X->rank[o[j - 1]]; --j) { int64_t t = o[j]; o[j] = o[j - 1]; o[j - 1] = t; }
}

/* bwt_smem1(x, min_intv = m) restricted to outputs >= min_seed_len (see file header) */
static void smem_at(rstate_t *S, int x, int m) {
    const uint8_t *q = S->q;
    int l = S->l, msl = S->p->min_seed_len;
    int64_t c0 = S->X->base_cnt[q[x]];
    if (c0 < m) {
        /* degenerate: the single base occurs < m times; bwt_smem1 returns [x, e1) with e1 the
         * first end where the forward count changes (or an N / the read end) */
        if (x + msl > l) return;
        for (int i = x + 1; i < x + msl; ++i) if (q[i] > 3) return;
        if (count_cov(S, x, x + msl) != c0) return;
        int e1 = x + msl;
        while (e1 < l && q[e1] < 4 && count_cov(S, x, e1 + 1) == c0) ++e1;
        if (c0 == 0) {  /* no occurrence: pushed with x[2] = 0 (no chain seeds) */
            if (S->nsi >= S->X->caps.intv) { S->overflow = 1; return; }
            sintv_t *v = &S->si[S->nsi++];
            v->qb = x; v->qe = e1; v->cnt = 0; v->occ0 = S->nocc; v->sa_k = -1;
            return;
        }
        push_intv(S, x, e1);
        return;
    }
    /* MEMs holding x, their distinct starts ascending */
    int *ks = S->w->ibuf, *starts = ks + S->npm + 1, *ts = starts + S->npm + 1;
    int nk = 0;
    for (int k = 0; k < S->npm; ++k)
        if (S->pm[k].s <= x && x < S->pm[k].t) ks[nk++] = k;
    int ns = 0;
    for (int a = 0; a < nk; ++a) {
        int s = S->pm[ks[a]].s, dup = 0;
        for (int b = 0; b < ns; ++b) dup |= starts[b] == s;
        if (!dup) starts[ns++] = s;
    }
    for (int i = 1; i < ns; ++i)
        for (int j = i; j > 0 && starts[j] < starts[j - 1]; --j) { int t = starts[j]; starts[j] = starts[j - 1]; starts[j - 1] = t; }
    int prev_e = -1;
    for (int a = 0; a < ns; ++a) {
        int b = starts[a];
        /* e(b) = m-th largest end among MEMs holding x that start at or before b */
        int nt = 0;
        for (int u = 0; u < nk; ++u) if (S->pm[ks[u]].s <= b) ts[nt++] = S->pm[ks[u]].t;
        if (nt < m) continue;
        for (int i = 1; i < nt; ++i)
            for (int j = i; j > 0 && ts[j] > ts[j - 1]; --j) { int t = ts[j]; ts[j] = ts[j - 1]; ts[j - 1] = t; }
        int e = ts[m - 1];
        if (e > prev_e) {
            if (e - b >= msl) push_intv(S, b, e);
            prev_e = e;
        }
    }
}

static int cmp_sintv(const void *a, const void *b) {
    const sintv_t *x = (const sintv_t *)a, *y = (const sintv_t *)b;
    if (x->qb != y->qb) return x->qb - y->qb;
    return x->qe - y->qe;
}

static void collect_intv_memset(rstate_t *S) {
    const afo_pe *pe = S->pe;
    int l = S->l, msl = S->p->min_seed_len;
    int split_len = (int)(msl * opt_split_factor + .499);
    S->nsi = 0; S->nocc = 0;
    find_pmems(S);
    if (S->overflow) return;
    /* pass 1: maximal MEM query intervals, each once */
    for (int k = 0; k < S->npm; ++k) {
        int s = S->pm[k].s, t = S->pm[k].t, keep = 1;
        for (int j = 0; j < S->npm && keep; ++j) {
            if (S->pm[j].s == s && S->pm[j].t == t) { if (j < k) keep = 0; continue; }
            if (S->pm[j].s <= s && t <= S->pm[j].t) keep = 0;
        }
        if (keep) push_intv(S, s, t);
    }
    /* pass 2 */
    int old_n = S->nsi;
    for (int k = 0; k < old_n && !S->overflow; ++k) {
        int start = S->si[k].qb, end = S->si[k].qe;
        if (end - start < split_len || S->si[k].cnt > pe->split_width) continue;
        smem_at(S, (start + end) >> 1, (int)S->si[k].cnt + 1);
    }
    /* pass 3 */
    if (pe->max_mem_intv > 0) {
        int x = 0;
        while (x < l && !S->overflow) {
            if (S->q[x] > 3) { ++x; continue; }
            int i, nx = l;
            for (i = x + 1; i < l; ++i) {
                if (S->q[i] > 3) { nx = i + 1; break; }
                if (i - x >= msl) {
                    int c = count_cov(S, x, i + 1);
                    if (c < pe->max_mem_intv) {
                        if (c > 0) push_intv(S, x, i + 1);
                        nx = i + 1;
                        break;
                    }
                }
            }
            x = nx;
        }
    }
    if (S->overflow) return;
    qsort(S->si, S->nsi, sizeof(sintv_t), cmp_sintv);
}

/* ---- FM mode: bwt.c --------------------------------------------------------------------- */
/* occurrences of c in bwt[0, i) */
static inline int64_t fm_occ(const afo_text *X, int c, int64_t i) {
    int64_t b = i >> OCC_SHIFT, v = X->occ[b * 4 + c];
    for (int64_t r = b << OCC_SHIFT; r < i; ++r) v += X->bwt[r] == c;
    return v;
}
/* bwt_extend, backward direction, all four bases: ok[c] = the bi-interval of cW from W's */
static void fm_back4(const afo_text *X, const biv_t *ik, biv_t ok[4]) {
    for (int c = 0; c < 4; ++c) {
        int64_t a = fm_occ(X, c, ik->k), b = fm_occ(X, c, ik->k + ik->s);
        ok[c].k = X->C[c] + a;
        ok[c].s = b - a;
    }
    /* the reverse-complement side: rc(cW) = rc(W) comp(c) inside rc(W)'s interval, after the one
     * suffix equal to rc(W) (when W is a prefix of T) and ordered by comp(c) */
    ok[3].l = ik->l + (ik->k <= X->primary && ik->k + ik->s - 1 >= X->primary);
    ok[2].l = ok[3].l + ok[3].s;
    ok[1].l = ok[2].l + ok[2].s;
    ok[0].l = ok[1].l + ok[1].s;
}
/* bwt_extend(is_back = 0): ok[c'] for the forward extension W -> W comp(c') */
static void fm_fwd4(const afo_text *X, const biv_t *ik, biv_t ok[4]) {
    biv_t sw = *ik;
    sw.k = ik->l; sw.l = ik->k;
    biv_t o[4];
    fm_back4(X, &sw, o);
    for (int c = 0; c < 4; ++c) { ok[c] = o[c]; ok[c].k = o[c].l; ok[c].l = o[c].k; }
}
static inline biv_t fm_set_intv(const afo_text *X, int c) {
    biv_t b;
    b.k = X->C[c]; b.s = X->base_cnt[c]; b.l = X->C[3 - c]; b.qb = 0; b.qe = 0;
    return b;
}

/* bwt_smem1 (bwt_smem1a with max_intv = 0): the SMEMs holding x with >= min_intv occurrences;
 * returns the end of the longest forward match */
static int fm_smem1(const afo_text *X, int len, const uint8_t *q, int x, int64_t min_intv, biv_t *mem, int *n_mem,
                    biv_t *bufa, biv_t *bufb) {
    int i, j, c, ret, np = 0, nc = 0;
    biv_t ik, ok[4], *prev = bufa, *curr = bufb, *swp;
    *n_mem = 0;
    if (q[x] > 3) return x + 1;
    if (min_intv < 1) min_intv = 1;
    ik = fm_set_intv(X, q[x]);
    ik.qe = x + 1;
    for (i = x + 1; i < len; ++i) {  /* forward search */
        if (q[i] < 4) {
            c = 3 - q[i];
            fm_fwd4(X, &ik, ok);
            if (ok[c].s != ik.s) {
                curr[nc++] = ik;
                if (ok[c].s < min_intv) break;
            }
            ik = ok[c]; ik.qe = i + 1;
        } else {
            curr[nc++] = ik;
            break;
        }
    }
    if (i == len) curr[nc++] = ik;
    for (j = 0; j < nc >> 1; ++j) { biv_t t = curr[j]; curr[j] = curr[nc - 1 - j]; curr[nc - 1 - j] = t; }
    ret = curr[0].qe;
    swp = curr; curr = prev; prev = swp; np = nc;
    for (i = x - 1; i >= -1; --i) {  /* backward search for MEMs */
        c = i < 0 ? -1 : q[i] < 4 ? q[i] : -1;
        nc = 0;
        for (j = 0; j < np; ++j) {
            biv_t *p = &prev[j];
            if (c >= 0) fm_back4(X, p, ok);
            if (c < 0 || ok[c].s < min_intv) {
                if (nc == 0) {
                    if (*n_mem == 0 || i + 1 < mem[*n_mem - 1].qb) {
                        ik = *p; ik.qb = i + 1;
                        mem[(*n_mem)++] = ik;
                    }
                }
            } else if (nc == 0 || ok[c].s != curr[nc - 1].s) {
                ok[c].qe = p->qe;
                ok[c].qb = 0;
                curr[nc++] = ok[c];
            }
        }
        if (nc == 0) break;
        swp = curr; curr = prev; prev = swp; np = nc;
    }
    for (j = 0; j < *n_mem >> 1; ++j) { biv_t t = mem[j]; mem[j] = mem[*n_mem - 1 - j]; mem[*n_mem - 1 - j] = t; }
    return ret;
}

/* bwt_seed_strategy1 */
static int fm_seed_strategy1(const afo_text *X, int len, const uint8_t *q, int x, int min_len, int max_intv, biv_t *mem) {
    int i, c;
    biv_t ik, ok[4];
    memset(mem, 0, sizeof(*mem));
    if (q[x] > 3) return x + 1;
    ik = fm_set_intv(X, q[x]);
    for (i = x + 1; i < len; ++i) {
        if (q[i] < 4) {
            c = 3 - q[i];
            fm_fwd4(X, &ik, ok);
            if (ok[c].s < max_intv && i - x >= min_len) {
                *mem = ok[c];
                mem->qb = x; mem->qe = i + 1;
                return i + 1;
            }
            ik = ok[c];
        } else return i + 1;
    }
    return len;
}

static void fm_push(rstate_t *S, const biv_t *m) {
    if (S->overflow) return;
    if (S->nsi >= S->X->caps.intv) { S->overflow = 1; return; }
    biv_t *o = &S->w->fm_mem[S->nsi++];
    *o = *m;
}

/* mem_collect_intv over the FM index */
static void collect_intv_fm(rstate_t *S) {
    const afo_text *X = S->X;
    const afo_pe *pe = S->pe;
    const uint8_t *q = S->q;
    int len = S->l, msl = S->p->min_seed_len, x = 0, n1 = 0;
    int split_len = (int)(msl * opt_split_factor + .499);
    biv_t *m1 = S->w->mem1;
    S->nsi = 0; S->nocc = 0;
    while (x < len) {
        if (q[x] < 4) {
            x = fm_smem1(X, len, q, x, 1, m1, &n1, S->w->tmpa, S->w->tmpb);
            for (int i = 0; i < n1; ++i)
                if (m1[i].qe - m1[i].qb >= msl) fm_push(S, &m1[i]);
        } else ++x;
    }
    int old_n = S->nsi;
    for (int k = 0; k < old_n && !S->overflow; ++k) {
        biv_t p = S->w->fm_mem[k];
        if (p.qe - p.qb < split_len || p.s > pe->split_width) continue;
        fm_smem1(X, len, q, (p.qb + p.qe) >> 1, p.s + 1, m1, &n1, S->w->tmpa, S->w->tmpb);
        for (int i = 0; i < n1; ++i)
            if (m1[i].qe - m1[i].qb >= msl) fm_push(S, &m1[i]);
    }
    if (pe->max_mem_intv > 0) {
        x = 0;
        while (x < len && !S->overflow) {
            if (q[x] < 4) {
                biv_t m;
                x = fm_seed_strategy1(X, len, q, x, msl, pe->max_mem_intv, &m);
                if (m.s > 0) fm_push(S, &m);
            } else ++x;
        }
    }
    if (S->overflow) return;
    introsort_intv(S->nsi, S->w->fm_mem);
    for (int i = 0; i < S->nsi; ++i) {
        const biv_t *b = &S->w->fm_mem[i];
        sintv_t *v = &S->si[i];
        v->qb = b->qb; v->qe = b->qe; v->cnt = b->s; v->sa_k = b->k; v->occ0 = 0;
    }
}

static void collect_intv(rstate_t *S) {
    if (S->X->fm) collect_intv_fm(S);
    else collect_intv_memset(S);
}

/* occurrence k of interval v (bwt_sa order) */
static inline int64_t intv_occ(const rstate_t *S, const sintv_t *v, int64_t k) {
    return v->sa_k >= 0 ? S->X->sa[v->sa_k + k] : S->occ[v->occ0 + k];
}

/* ============================================================= kbtree of chains (t = 5) */
/* klib kbtree.h with KB_DEFAULT_SIZE 512 and sizeof(mem_chain_t) = 40 (bwa 0.7.17, 64-bit):
 * t = ((512 - 4 - 8) / (8 + 40) + 1) >> 1 = 5, at most 9 keys per node.  Keys are chain
 * indices compared by chain pos.  Equal positions follow kbtree's own placement. */
typedef struct { kbnode_t *node; int nn, root; const chain_t *ch; } kbtree_t;

static inline int kb_cmp(const kbtree_t *b, int x, int64_t kpos) {
    int64_t a = b->ch[x].pos;
    return (kpos < a) - (a < kpos);  /* chain_cmp(a, k) = (k < a) - (a < k) */
}
/* __kb_getp_aux: first index equal to k if present, else the last index below k (-1) */
static int kb_getp_aux(const kbtree_t *b, const kbnode_t *x, int64_t kpos, int *r) {
    int tr, *rr, begin = 0, end = x->n;
    if (x->n == 0) return -1;
    rr = r ? r : &tr;
    while (begin < end) {
        int mid = (begin + end) >> 1;
        if (kb_cmp(b, x->key[mid], kpos) < 0) begin = mid + 1;
        else end = mid;
    }
    if (begin == x->n) { *rr = 1; return x->n - 1; }
    if ((*rr = -kb_cmp(b, x->key[begin], kpos)) < 0) --begin;
    return begin;
}
static int kb_new(kbtree_t *b, int internal) {
    kbnode_t *z = &b->node[b->nn];
    memset(z, 0, sizeof(*z));
    z->internal = internal;
    return b->nn++;
}
static void kb_init(kbtree_t *b, kbnode_t *nodes, const chain_t *ch) { b->node = nodes; b->nn = 0; b->ch = ch; b->root = kb_new(b, 0); }
/* kb_intervalp: the lower neighbour of k */
static int kb_lower(const kbtree_t *b, int64_t kpos) {
    int i, r = 0, lower = -1;
    int xi = b->root;
    while (xi >= 0) {
        const kbnode_t *x = &b->node[xi];
        i = kb_getp_aux(b, x, kpos, &r);
        if (i >= 0 && r == 0) return x->key[i];
        if (i >= 0) lower = x->key[i];
        if (!x->internal) return lower;
        xi = x->ptr[i + 1];
    }
    return lower;
}
static void kb_split(kbtree_t *b, int xi, int i, int yi) {
    int zi = kb_new(b, b->node[yi].internal);
    kbnode_t *x = &b->node[xi], *y = &b->node[yi], *z = &b->node[zi];
    z->n = KB_T - 1;
    memcpy(z->key, y->key + KB_T, sizeof(int) * (KB_T - 1));
    if (y->internal) memcpy(z->ptr, y->ptr + KB_T, sizeof(int) * KB_T);
    y->n = KB_T - 1;
    memmove(x->ptr + i + 2, x->ptr + i + 1, sizeof(int) * (x->n - i));
    x->ptr[i + 1] = zi;
    memmove(x->key + i + 1, x->key + i, sizeof(int) * (x->n - i));
    x->key[i] = y->key[KB_T - 1];
    ++x->n;
}
static void kb_putp_aux(kbtree_t *b, int xi, int k) {
    int64_t kpos = b->ch[k].pos;
    kbnode_t *x = &b->node[xi];
    if (!x->internal) {
        int i = kb_getp_aux(b, x, kpos, 0);
        if (i != x->n - 1) memmove(x->key + i + 2, x->key + i + 1, sizeof(int) * (x->n - i - 1));
        x->key[i + 1] = k;
        ++x->n;
    } else {
        int i = kb_getp_aux(b, x, kpos, 0) + 1;
        if (b->node[x->ptr[i]].n == KB_MAXK) {
            kb_split(b, xi, i, x->ptr[i]);
            x = &b->node[xi];
            if (kb_cmp(b, x->key[i], kpos) < 0) ++i;  /* b->cmp(*k, key[i]) > 0: k past the promoted key */
        }
        kb_putp_aux(b, x->ptr[i], k);
    }
}
static void kb_putp(kbtree_t *b, int k) {
    int ri = b->root;
    if (b->node[ri].n == KB_MAXK) {
        int si = kb_new(b, 1);
        b->node[si].ptr[0] = ri;
        b->root = si;
        kb_split(b, si, 0, ri);
        kb_putp_aux(b, si, k);
    } else kb_putp_aux(b, ri, k);
}
static void kb_traverse(const kbtree_t *b, int xi, int *out, int *n) {
    const kbnode_t *x = &b->node[xi];
    for (int i = 0; i < x->n; ++i) {
        if (x->internal) kb_traverse(b, x->ptr[i], out, n);
        out[(*n)++] = x->key[i];
    }
    if (x->internal) kb_traverse(b, x->ptr[x->n], out, n);
}

/* ============================================================= mem_chain / mem_chain_flt */
/* chain storage during mem_chain: each chain's seeds in a per-chain list (linked through the
 * pool); compacted per chain afterwards */
static int test_and_merge(const rstate_t *S, chain_t *c, sl_t *pool, int *last_of, int ci, const seed_t *p, int rid,
                          int *npool) {
    const afo_pe *pe = S->pe;
    int64_t l_pac = S->X->n;
    const seed_t *first = &pool[c->seed0].s, *last = &pool[last_of[ci]].s;
    int64_t qend = last->qbeg + last->len, rend = last->rbeg + last->len;
    if (rid != c->rid) return 0;
    if (p->qbeg >= first->qbeg && p->qbeg + p->len <= qend && p->rbeg >= first->rbeg && p->rbeg + p->len <= rend)
        return 1;  /* contained seed; do nothing */
    if ((last->rbeg < l_pac || first->rbeg < l_pac) && p->rbeg >= l_pac) return 0;  /* different strand */
    int64_t x = p->qbeg - last->qbeg, y = p->rbeg - last->rbeg;
    if (y >= 0 && x - y <= S->p->w && y - x <= S->p->w && x - last->len < pe->max_chain_gap &&
        y - last->len < pe->max_chain_gap) {
        if (*npool >= S->X->caps.occ) return -1;
        int k = (*npool)++;
        pool[k].s = *p; pool[k].next = -1;
        pool[last_of[ci]].next = k;
        last_of[ci] = k;
        ++c->n;
        return 1;
    }
    return 0;
}

/* mem_chain: seeds into chains keyed by reference position (kbtree), chains in tree order */
static void mem_chain(rstate_t *S) {
    S->nch = 0; S->nseed = 0;
    if (S->l < S->p->min_seed_len) return;
    collect_intv(S);
    if (S->overflow) return;
    work_t *W = S->w;
    sl_t *pool = W->pool;
    kbtree_t tree;
    chain_t *ch = W->ch2;
    int *last_of = W->last_of;
    int nch = 0, npool = 0;
    const caps_t *cp = &S->X->caps;
    kb_init(&tree, (kbnode_t *)W->kbnodes, ch);
    for (int i = 0; i < S->nsi; ++i) {
        const sintv_t *v = &S->si[i];
        int slen = v->qe - v->qb;
        int64_t step = v->cnt > S->p->max_occ ? v->cnt / S->p->max_occ : 1;
        int64_t k;
        int count;
        for (k = 0, count = 0; k < v->cnt && count < S->p->max_occ; k += step, ++count) {
            seed_t s;
            s.rbeg = intv_occ(S, v, k);
            s.qbeg = v->qb;
            s.score = s.len = slen;
            int rid = intv2rid(S->X, s.rbeg, s.rbeg + s.len);
            if (rid < 0) continue;  /* bridging contigs or the forward-reverse boundary */
            int to_add = 0;
            if (nch) {
                int lower = kb_lower(&tree, s.rbeg);
                if (lower < 0) to_add = 1;
                else {
                    int r = test_and_merge(S, &ch[lower], pool, last_of, lower, &s, rid, &npool);
                    if (r < 0) { S->overflow = 1; return; }
                    if (!r) to_add = 1;
                }
            } else to_add = 1;
            if (to_add) {
                if (nch >= cp->chain || npool >= cp->occ) { S->overflow = 1; return; }
                int kk = npool++;
                pool[kk].s = s; pool[kk].next = -1;
                chain_t *c = &ch[nch];
                c->n = 1; c->first = -1; c->rid = rid; c->w = 0; c->kept = 0; c->pos = s.rbeg; c->seed0 = kk;
                last_of[nch] = kk;
                kb_putp(&tree, nch);
                ++nch;
            }
        }
    }
    int *order = W->order, no = 0;
    kb_traverse(&tree, tree.root, order, &no);
    /* compact: chain seeds contiguous in S->seed, chains in traversal order */
    for (int a = 0; a < no; ++a) {
        chain_t c = ch[order[a]];
        int s0 = S->nseed;
        for (int k = c.seed0; k >= 0; k = pool[k].next) S->seed[S->nseed++] = pool[k].s;
        c.seed0 = s0;
        S->ch[S->nch++] = c;
    }
}

static int mem_chain_weight(const rstate_t *S, const chain_t *c) {
    int64_t end;
    int j, w = 0, tmp;
    const seed_t *sd = S->seed + c->seed0;
    for (j = 0, end = 0; j < c->n; ++j) {
        const seed_t *s = &sd[j];
        if (s->qbeg >= end) w += s->len;
        else if (s->qbeg + s->len > end) w += (int)(s->qbeg + s->len - end);
        end = end > s->qbeg + s->len ? end : s->qbeg + s->len;
    }
    tmp = w; w = 0;
    for (j = 0, end = 0; j < c->n; ++j) {
        const seed_t *s = &sd[j];
        if (s->rbeg >= end) w += s->len;
        else if (s->rbeg + s->len > end) w += (int)(s->rbeg + s->len - end);
        end = end > s->rbeg + s->len ? end : s->rbeg + s->len;
    }
    w = w < tmp ? w : tmp;
    return w < 1 << 30 ? w : (1 << 30) - 1;
}

#define chn_beg(S, c) ((S)->seed[(c).seed0].qbeg)
#define chn_end(S, c) ((S)->seed[(c).seed0 + (c).n - 1].qbeg + (S)->seed[(c).seed0 + (c).n - 1].len)

/* mem_chain_flt (min_chain_weight 0, max_chain_extend 1 << 30) */
static void mem_chain_flt(rstate_t *S) {
    int i, k, n_chn = S->nch;
    chain_t *a = S->ch;
    if (n_chn == 0) return;
    for (i = 0; i < n_chn; ++i) { a[i].first = -1; a[i].kept = 0; a[i].w = mem_chain_weight(S, &a[i]); }
    introsort_flt(n_chn, a);
    int *chains = S->w->order, nc = 0;
    a[0].kept = 3;
    chains[nc++] = 0;
    for (i = 1; i < n_chn; ++i) {
        int large_ovlp = 0;
        for (k = 0; k < nc; ++k) {
            int j = chains[k];
            int b_max = chn_beg(S, a[j]) > chn_beg(S, a[i]) ? chn_beg(S, a[j]) : chn_beg(S, a[i]);
            int e_min = chn_end(S, a[j]) < chn_end(S, a[i]) ? chn_end(S, a[j]) : chn_end(S, a[i]);
            if (e_min > b_max) {  /* is_alt never set (no ALT contigs) */
                int li = chn_end(S, a[i]) - chn_beg(S, a[i]);
                int lj = chn_end(S, a[j]) - chn_beg(S, a[j]);
                int min_l = li < lj ? li : lj;
                if (e_min - b_max >= min_l * opt_mask_level && min_l < S->pe->max_chain_gap) {
                    large_ovlp = 1;
                    if (a[j].first < 0) a[j].first = i;
                    if (a[i].w < a[j].w * opt_drop_ratio && a[j].w - a[i].w >= S->p->min_seed_len << 1) break;
                }
            }
        }
        if (k == nc) {
            chains[nc++] = i;
            a[i].kept = large_ovlp ? 2 : 3;
        }
    }
    for (i = 0; i < nc; ++i) {
        chain_t *c = &a[chains[i]];
        if (c->first >= 0) a[c->first].kept = 1;
    }
    /* max_chain_extend = 1 << 30: no further drops */
    for (i = k = 0; i < n_chn; ++i)
        if (a[i].kept != 0) a[k++] = a[i];
    S->nch = k;
}

/* ==================================================================== mem_chain2aln */
static void mem_chain2aln(rstate_t *S, const chain_t *c, regv_t *av) {
    const afo_params *p = S->p;
    const afo_text *X = S->X;
    int l_query = S->l;
    const uint8_t *query = S->q;
    int64_t l_pac = X->n, rmax[2];
    const seed_t *sd = S->seed + c->seed0;
    if (c->n == 0) return;
    rmax[0] = l_pac << 1; rmax[1] = 0;
    for (int i = 0; i < c->n; ++i) {
        const seed_t *t = &sd[i];
        int64_t b = t->rbeg - (t->qbeg + afo_cal_max_gap(p, t->qbeg));
        int64_t e = t->rbeg + t->len + ((l_query - t->qbeg - t->len) + afo_cal_max_gap(p, l_query - t->qbeg - t->len));
        rmax[0] = rmax[0] < b ? rmax[0] : b;
        rmax[1] = rmax[1] > e ? rmax[1] : e;
    }
    rmax[0] = rmax[0] > 0 ? rmax[0] : 0;
    rmax[1] = rmax[1] < l_pac << 1 ? rmax[1] : l_pac << 1;
    if (rmax[0] < l_pac && l_pac < rmax[1]) {
        if (sd[0].rbeg < l_pac) rmax[1] = l_pac;
        else rmax[0] = l_pac;
    }
    {   /* bns_fetch_seq: clipped to the contig (on its strand) holding seeds[0] */
        int rid;
        fetch_clip(X, &rmax[0], sd[0].rbeg, &rmax[1], &rid);
    }
    const uint8_t *rseq = X->T + rmax[0];
    uint64_t *srt = S->w->srt;
    for (int i = 0; i < c->n; ++i) srt[i] = (uint64_t)sd[i].score << 32 | (uint32_t)i;
    introsort_u64(c->n, srt);
    for (int k = c->n - 1; k >= 0; --k) {
        const seed_t *s = &sd[(uint32_t)srt[k]];
        int i;
        for (i = 0; i < av->n; ++i) {  /* test whether extension has been made before */
            const alnreg_t *pr = &av->a[i];
            int64_t rd;
            int qd, w, max_gap;
            if (s->rbeg < pr->rb || s->rbeg + s->len > pr->re || s->qbeg < pr->qb || s->qbeg + s->len > pr->qe) continue;
            if (s->len - pr->seedlen0 > .1 * l_query) continue;
            qd = s->qbeg - pr->qb; rd = s->rbeg - pr->rb;
            max_gap = afo_cal_max_gap(p, qd < rd ? qd : (int)rd);
            w = max_gap < pr->w ? max_gap : pr->w;
            if (qd - rd < w && rd - qd < w) break;
            qd = pr->qe - (s->qbeg + s->len); rd = pr->re - (s->rbeg + s->len);
            max_gap = afo_cal_max_gap(p, qd < rd ? qd : (int)rd);
            w = max_gap < pr->w ? max_gap : pr->w;
            if (qd - rd < w && rd - qd < w) break;
        }
        if (i < av->n) {  /* (almost) contained: extend only if an overlapping seed could differ */
            for (i = k + 1; i < c->n; ++i) {
                const seed_t *t;
                if (srt[i] == 0) continue;
                t = &sd[(uint32_t)srt[i]];
                if (t->len < s->len * .95) continue;
                if (s->qbeg <= t->qbeg && s->qbeg + s->len - t->qbeg >= s->len >> 2 &&
                    t->qbeg - s->qbeg != t->rbeg - s->rbeg) break;
                if (t->qbeg <= s->qbeg && t->qbeg + t->len - s->qbeg >= s->len >> 2 &&
                    s->qbeg - t->qbeg != s->rbeg - t->rbeg) break;
            }
            if (i == c->n) { srt[k] = 0; continue; }
        }
        alnreg_t *a = regv_push(av, X->caps.reg);
        if (!a) { S->overflow = 1; return; }
        memset(a, 0, sizeof(*a));
        int aw[2], max_off[2];
        a->w = aw[0] = aw[1] = p->w;
        a->score = a->truesc = -1;
        a->rid = c->rid;
        if (s->qbeg) {  /* left extension */
            uint8_t qs[AFO_MAX_READ], rs[2 * AFO_MAX_READ + 1024];
            int qle, tle, gtle, gscore;
            for (i = 0; i < s->qbeg; ++i) qs[i] = query[s->qbeg - 1 - i];
            int64_t tmp = s->rbeg - rmax[0];
            for (i = 0; i < tmp; ++i) rs[i] = rseq[tmp - 1 - i];
            for (i = 0; i < 2; ++i) {  /* MAX_BAND_TRY */
                int prev = a->score;
                aw[0] = p->w << i;
                a->score = afo_ext_dp(s->qbeg, qs, (int)tmp, rs, p, aw[0], p->pen_clip5, p->zdrop, s->len * p->a, &qle,
                                      &tle, &gtle, &gscore, &max_off[0]);
                if (a->score == prev || max_off[0] < (aw[0] >> 1) + (aw[0] >> 2)) break;
            }
            if (gscore <= 0 || gscore <= a->score - p->pen_clip5) {
                a->qb = s->qbeg - qle; a->rb = s->rbeg - tle; a->truesc = a->score;
            } else {
                a->qb = 0; a->rb = s->rbeg - gtle; a->truesc = gscore;
            }
        } else {
            a->score = a->truesc = s->len * p->a; a->qb = 0; a->rb = s->rbeg;
        }
        if (s->qbeg + s->len != l_query) {  /* right extension */
            int qle, tle, qe, gtle, gscore, sc0 = a->score;
            int64_t re;
            qe = s->qbeg + s->len;
            re = s->rbeg + s->len - rmax[0];
            for (i = 0; i < 2; ++i) {
                int prev = a->score;
                aw[1] = p->w << i;
                a->score = afo_ext_dp(l_query - qe, query + qe, (int)(rmax[1] - rmax[0] - re), rseq + re, p, aw[1],
                                      p->pen_clip3, p->zdrop, sc0, &qle, &tle, &gtle, &gscore, &max_off[1]);
                if (a->score == prev || max_off[1] < (aw[1] >> 1) + (aw[1] >> 2)) break;
            }
            if (gscore <= 0 || gscore <= a->score - p->pen_clip3) {
                a->qe = qe + qle; a->re = rmax[0] + re + tle; a->truesc += a->score - sc0;
            } else {
                a->qe = l_query; a->re = rmax[0] + re + gtle; a->truesc += gscore - sc0;
            }
        } else {
            a->qe = l_query; a->re = s->rbeg + s->len;
        }
        a->seedcov = 0;
        for (i = 0; i < c->n; ++i) {
            const seed_t *t = &sd[i];
            if (t->qbeg >= a->qb && t->qbeg + t->len <= a->qe && t->rbeg >= a->rb && t->rbeg + t->len <= a->re)
                a->seedcov += t->len;
        }
        a->w = aw[0] > aw[1] ? aw[0] : aw[1];
        a->seedlen0 = s->len;
    }
}

/* ========================================================= mem_sort_dedup_patch */
static int mem_patch_reg(const rstate_t *S, const alnreg_t *a, const alnreg_t *b, int *_w) {
    const afo_params *p = S->p;
    int64_t l_pac = S->X->n;
    int w, score, q_s, r_s;
    double r;
    if (a->rb < l_pac && b->rb >= l_pac) return 0;
    if (a->qb >= b->qb || a->qe >= b->qe || a->re >= b->re) return 0;
    if (b->re - a->rb > AFO_PE_MAX_TSPAN) return 0;  /* cap: the GPU's 1 KiB target window */
    w = (int)((a->re - b->rb) - (a->qe - b->qb));
    w = w > 0 ? w : -w;
    r = (double)(a->re - b->rb) / (b->re - a->rb) - (double)(a->qe - b->qb) / (b->qe - a->qb);
    r = r > 0. ? r : -r;
    if (a->re < b->rb || a->qe < b->qb) {
        if (w > p->w << 1 || r >= PATCH_MAX_R_BW) return 0;
    } else if (w > p->w << 2 || r >= PATCH_MAX_R_BW * 2) return 0;
    w += a->w + b->w;
    w = w < p->w << 2 ? w : p->w << 2;
    {   /* bwa_gen_cigar2 of query[a->qb, b->qe) against [a->rb, b->re): only its score */
        int lq = b->qe - a->qb;
        if (lq <= 0 || a->rb >= b->re || (a->rb < l_pac && b->re > l_pac)) score = 0;  /* never on this path */
        else {
            uint32_t cig[AFO_MAX_CIGAR];
            int nc = 0;
            score = afo_gen_cigar(S->X->T, l_pac, p, w, lq, S->q + a->qb, a->rb, b->re, cig, &nc);
        }
    }
    q_s = (int)((double)(b->qe - a->qb) / ((b->qe - b->qb) + (a->qe - a->qb)) * (b->score + a->score) + .499);
    r_s = (int)((double)(b->re - a->rb) / ((b->re - b->rb) + (a->re - a->rb)) * (b->score + a->score) + .499);
    if ((double)score / (q_s > r_s ? q_s : r_s) < PATCH_MIN_SC_RATIO) return 0;
    *_w = w;
    return score;
}

static int mem_sort_dedup_patch(const rstate_t *S, int patch, int n, alnreg_t *a) {
    int m, i, j;
    if (n <= 1) return n;
    introsort_ars2(n, a);
    for (i = 0; i < n; ++i) a[i].n_comp = 1;
    for (i = 1; i < n; ++i) {
        alnreg_t *p = &a[i];
        if (p->rid != a[i - 1].rid || p->rb >= a[i - 1].re + S->pe->max_chain_gap) continue;
        for (j = i - 1; j >= 0 && p->rid == a[j].rid && p->rb < a[j].re + S->pe->max_chain_gap; --j) {
            alnreg_t *q = &a[j];
            int64_t or_, oq, mr, mq;
            int score, w;
            if (q->qe == q->qb) continue;
            or_ = q->re - p->rb;
            oq = q->qb < p->qb ? q->qe - p->qb : p->qe - q->qb;
            mr = q->re - q->rb < p->re - p->rb ? q->re - q->rb : p->re - p->rb;
            mq = q->qe - q->qb < p->qe - p->qb ? q->qe - q->qb : p->qe - p->qb;
            if (or_ > opt_mask_level_redun * mr && oq > opt_mask_level_redun * mq) {
                if (p->score < q->score) { p->qe = p->qb; break; }
                else q->qe = q->qb;
            } else if (q->rb < p->rb && patch && (score = mem_patch_reg(S, q, p, &w)) > 0) {
                p->n_comp += q->n_comp + 1;
                p->seedcov = p->seedcov > q->seedcov ? p->seedcov : q->seedcov;
                p->sub = p->sub > q->sub ? p->sub : q->sub;
                p->csub = p->csub > q->csub ? p->csub : q->csub;
                p->qb = q->qb; p->rb = q->rb;
                p->truesc = p->score = score;
                p->w = w;
                q->qb = q->qe;
            }
        }
    }
    for (i = 0, m = 0; i < n; ++i)
        if (a[i].qe > a[i].qb) {
            if (m != i) a[m++] = a[i];
            else ++m;
        }
    n = m;
    introsort_ars(n, a);
    for (i = 1; i < n; ++i)
        if (a[i].score == a[i - 1].score && a[i].rb == a[i - 1].rb && a[i].qb == a[i - 1].qb) a[i].qe = a[i].qb;
    for (i = 1, m = 1; i < n; ++i)
        if (a[i].qe > a[i].qb) {
            if (m != i) a[m++] = a[i];
            else ++m;
        }
    return m;
}

/* ======================================================================= mem_align1_core */
static void rstate_init(rstate_t *S, const afo_text *X, const afo_params *p, const afo_pe *pe, const uint8_t *q, int l) {
    memset(S, 0, sizeof(*S));
    S->X = X; S->p = p; S->pe = pe; S->q = q; S->l = l; S->overflow = 0;
    S->w = work_get(&X->caps);
    S->pm = S->w->pm; S->si = S->w->si; S->occ = S->w->occ; S->seed = S->w->seed; S->ch = S->w->ch;
}

static int align1_core(const afo_text *X, const afo_params *p, const afo_pe *pe, const uint8_t *q, int l, regv_t *regs) {
    rstate_t S;
    rstate_init(&S, X, p, pe, q, l);
    regs->n = 0;
    mem_chain(&S);
    if (!S.overflow) mem_chain_flt(&S);
    /* mem_flt_chained_seeds: min_l = 5.5 * log(l) exceeds 0.05 * l for every l <= AFO_MAX_READ, a no-op */
    for (int i = 0; i < S.nch && !S.overflow; ++i) mem_chain2aln(&S, &S.ch[i], regs);
    if (S.overflow) { regs->n = 0; return -1; }
    regs->n = mem_sort_dedup_patch(&S, 1, regs->n, regs->a);
    return 0;
}

/* ============================================================================ pestat */
static int cal_sub(const alnreg_t *a, int n, int min_seed_len, int a_sc) {
    int j;
    for (j = 1; j < n; ++j) {
        int b_max = a[j].qb > a[0].qb ? a[j].qb : a[0].qb;
        int e_min = a[j].qe < a[0].qe ? a[j].qe : a[0].qe;
        if (e_min > b_max) {
            int min_l = a[j].qe - a[j].qb < a[0].qe - a[0].qb ? a[j].qe - a[j].qb : a[0].qe - a[0].qb;
            if (e_min - b_max >= min_l * opt_mask_level) break;
        }
    }
    return j < n ? a[j].score : min_seed_len * a_sc;
}

static inline int mem_infer_dir(int64_t l_pac, int64_t b1, int64_t b2, int64_t *dist) {
    int64_t p2;
    int r1 = (b1 >= l_pac), r2 = (b2 >= l_pac);
    p2 = r1 == r2 ? b2 : (l_pac << 1) - 1 - b2;
    *dist = p2 > b1 ? p2 - b1 : b1 - p2;
    return (r1 == r2 ? 0 : 1) ^ (p2 > b1 ? 0 : 3);
}

static void mem_pestat(const afo_params *p, const afo_pe *pe, int64_t l_pac, int64_t n_pairs, regv_t *regs, pestat_t pes[4]) {
    int64_t cap = n_pairs > 0 ? n_pairs : 1;
    uint64_t *isz[4];
    int64_t nn[4] = {0, 0, 0, 0};
    for (int d = 0; d < 4; ++d) isz[d] = (uint64_t *)malloc(sizeof(uint64_t) * cap);
    memset(pes, 0, 4 * sizeof(pestat_t));
    for (int64_t i = 0; i < n_pairs; ++i) {
        regv_t *r0 = &regs[2 * i], *r1 = &regs[2 * i + 1];
        int64_t is;
        if (r0->n == 0 || r1->n == 0) continue;
        if (cal_sub(r0->a, r0->n, p->min_seed_len, p->a) > MIN_RATIO * r0->a[0].score) continue;
        if (cal_sub(r1->a, r1->n, p->min_seed_len, p->a) > MIN_RATIO * r1->a[0].score) continue;
        if (r0->a[0].rid != r1->a[0].rid) continue;
        int dir = mem_infer_dir(l_pac, r0->a[0].rb, r1->a[0].rb, &is);
        if (is && is <= pe->max_ins) isz[dir][nn[dir]++] = (uint64_t)is;
    }
    for (int d = 0; d < 4; ++d) {
        pestat_t *r = &pes[d];
        uint64_t *q = isz[d];
        int64_t n = nn[d];
        int p25, p50, p75, x;
        if (n < MIN_DIR_CNT) { r->failed = 1; continue; }
        introsort_u64(n, q);
        p25 = (int)q[(int)(.25 * n + .499)];
        p50 = (int)q[(int)(.50 * n + .499)];
        p75 = (int)q[(int)(.75 * n + .499)];
        (void)p50;
        r->low = (int)(p25 - OUTLIER_BOUND * (p75 - p25) + .499);
        if (r->low < 1) r->low = 1;
        r->high = (int)(p75 + OUTLIER_BOUND * (p75 - p25) + .499);
        int64_t i;
        for (i = x = 0, r->avg = 0; i < n; ++i)
            if (q[i] >= (uint64_t)(int64_t)r->low && q[i] <= (uint64_t)(int64_t)r->high) r->avg += q[i], ++x;
        r->avg /= x;
        for (i = 0, r->std = 0; i < n; ++i)
            if (q[i] >= (uint64_t)(int64_t)r->low && q[i] <= (uint64_t)(int64_t)r->high)
                r->std += (q[i] - r->avg) * (q[i] - r->avg);
        r->std = sqrt(r->std / x);
        r->low = (int)(p25 - MAPPING_BOUND * (p75 - p25) + .499);
        r->high = (int)(p75 + MAPPING_BOUND * (p75 - p25) + .499);
        if (r->low > r->avg - MAX_STDDEV * r->std) r->low = (int)(r->avg - MAX_STDDEV * r->std + .499);
        if (r->high < r->avg + MAX_STDDEV * r->std) r->high = (int)(r->avg + MAX_STDDEV * r->std + .499);
        if (r->low < 1) r->low = 1;
    }
    int64_t max = 0;
    for (int d = 0; d < 4; ++d) max = max > nn[d] ? max : nn[d];
    for (int d = 0; d < 4; ++d)
        if (pes[d].failed == 0 && nn[d] < max * MIN_DIR_RATIO) pes[d].failed = 1;
    for (int d = 0; d < 4; ++d) free(isz[d]);
}

/* ================================================================ ksw_u8 / ksw_i16 */
typedef struct { int score, te, qe, score2, te2, tb, qb; } kswr_t;

/* Farrar's striped local SW exactly as ksw.c computes it: P lanes (16 for ksw_u8, 8 for
 * ksw_i16), query position k*slen + j in lane k of segment j, first pass with F chained
 * inside a lane, then the lazy-F loop (E is not revisited: no D->I adjacency through it). */
static kswr_t ksw_sw(int size, int qlen, const uint8_t *query, int tlen, const uint8_t *target, const int8_t *mat,
                     int o_del, int e_del, int o_ins, int e_ins, int xtra) {
    const int P = size == 1 ? 16 : 8;
    const int slen = (qlen + P - 1) / P;
    const int m = 5;
    int shift = 0, mdiff = 0;
    kswr_t r = {0, -1, -1, -1, -1, -1, -1};
    int minsc = (xtra & KSW_XSUBO) ? xtra & 0xffff : 0x10000;
    int endsc = (xtra & KSW_XSTOP) ? xtra & 0xffff : 0x10000;
    /* ksw_qinit */
    {
        int8_t sh = 127, md = 0;
        for (int a = 0; a < m * m; ++a) {
            if (mat[a] < sh) sh = mat[a];
            if (mat[a] > md) md = mat[a];
        }
        shift = size == 1 ? (uint8_t)(256 - (uint8_t)sh) : 0;
        mdiff = md;
    }
    int vmax = size == 1 ? 255 : 32767;  /* saturation of the add; subtractions floor at 0 */
    int *qp = (int *)malloc(sizeof(int) * m * slen * P);
    for (int a = 0; a < m; ++a)
        for (int j = 0; j < slen; ++j)
            for (int k = 0; k < P; ++k) {
                int pos = k * slen + j;
                qp[(a * slen + j) * P + k] = pos >= qlen ? 0 : mat[a * m + query[pos]];
            }
    int *H0 = (int *)calloc(slen * P, sizeof(int)), *H1 = (int *)calloc(slen * P, sizeof(int));
    int *E = (int *)calloc(slen * P, sizeof(int)), *Hmax = (int *)calloc(slen * P, sizeof(int));
    int gmax = 0, te = -1;
    int oe_del = o_del + e_del, oe_ins = o_ins + e_ins;
#define SUBS(x, y) ((x) - (y) > 0 ? (x) - (y) : 0)
    for (int i = 0; i < tlen; ++i) {
        int f[16], mx[16], h[16];
        const int *S = qp + (size_t)target[i] * slen * P;
        for (int k = 0; k < P; ++k) { f[k] = 0; mx[k] = 0; }
        /* h = H0[slen-1] shifted up one lane (lane 0 <- 0) */
        for (int k = P - 1; k >= 1; --k) h[k] = H0[(slen - 1) * P + k - 1];
        h[0] = 0;
        for (int j = 0; j < slen; ++j) {
            for (int k = 0; k < P; ++k) {
                int v;
                if (size == 1) { v = h[k] + S[j * P + k] + shift; if (v > 255) v = 255; v = SUBS(v, shift); }
                else { v = h[k] + S[j * P + k]; if (v > vmax) v = vmax; if (v < -32768) v = -32768; }
                int e = E[j * P + k];
                v = v > e ? v : e;
                v = v > f[k] ? v : f[k];
                mx[k] = mx[k] > v ? mx[k] : v;
                H1[j * P + k] = v;
                e = SUBS(e, e_del);
                int t = SUBS(v, oe_del);
                E[j * P + k] = e > t ? e : t;
                f[k] = SUBS(f[k], e_ins);
                t = SUBS(v, oe_ins);
                f[k] = f[k] > t ? f[k] : t;
                h[k] = H0[j * P + k];
            }
        }
        for (int kk = 0; kk < 16; ++kk) {  /* lazy-F loop */
            for (int k = P - 1; k >= 1; --k) f[k] = f[k - 1];
            f[0] = 0;
            int done = 0;
            for (int j = 0; j < slen; ++j) {
                int all = 1;
                for (int k = 0; k < P; ++k) {
                    int v = H1[j * P + k];
                    v = v > f[k] ? v : f[k];
                    H1[j * P + k] = v;
                    int hh = SUBS(v, oe_ins);
                    f[k] = SUBS(f[k], e_ins);
                    if (f[k] > hh) all = 0;
                }
                if (all) { done = 1; break; }
            }
            if (done) break;
        }
        int imax = 0;
        for (int k = 0; k < P; ++k) imax = imax > mx[k] ? imax : mx[k];
        (void)minsc;  /* the suboptimal-hit array (score2, for MAPQ) is not produced */
        if (imax > gmax) {
            gmax = imax; te = i;
            memcpy(Hmax, H1, sizeof(int) * slen * P);
            if ((size == 1 && gmax + shift >= 255) || gmax >= endsc) break;
        }
        int *sw = H1; H1 = H0; H0 = sw;
    }
#undef SUBS
    r.score = (size == 1 && gmax + shift >= 255) ? 255 : gmax;
    r.te = te;
    if (r.score != 255 || size != 1) {
        int max = -1, tmp, ql = slen * P;
        for (int i = 0; i < ql; ++i) {
            int j = i / P, k = i % P;  /* byte i of Hmax: segment i / P, lane i % P */
            int v = Hmax[j * P + k];
            tmp = i / P + i % P * slen;
            if (v > max) max = v, r.qe = tmp;
            else if (v == max && tmp < r.qe) r.qe = tmp;
        }
    }
    (void)mdiff;
    free(qp); free(H0); free(H1); free(E); free(Hmax);
    return r;
}

/* ksw_align2 with KSW_XSTART: the start from a second, reversed pass that stops at the score */
static kswr_t ksw_align2(int qlen, uint8_t *query, int tlen, uint8_t *target, const int8_t *mat, int o_del, int e_del,
                         int o_ins, int e_ins, int xtra) {
    int size = (xtra & KSW_XBYTE) ? 1 : 2;
    kswr_t r = ksw_sw(size, qlen, query, tlen, target, mat, o_del, e_del, o_ins, e_ins, xtra), rr;
    if ((xtra & KSW_XSTART) == 0 || ((xtra & KSW_XSUBO) && r.score < (xtra & 0xffff))) return r;
    /* revseq(r.qe + 1, query); revseq(r.te + 1, target) */
    for (int i = 0; i < (r.qe + 1) >> 1; ++i) { uint8_t t = query[i]; query[i] = query[r.qe - i]; query[r.qe - i] = t; }
    for (int i = 0; i < (r.te + 1) >> 1; ++i) { uint8_t t = target[i]; target[i] = target[r.te - i]; target[r.te - i] = t; }
    rr = ksw_sw(size, r.qe + 1, query, tlen, target, mat, o_del, e_del, o_ins, e_ins, KSW_XSTOP | r.score);
    for (int i = 0; i < (r.qe + 1) >> 1; ++i) { uint8_t t = query[i]; query[i] = query[r.qe - i]; query[r.qe - i] = t; }
    for (int i = 0; i < (r.te + 1) >> 1; ++i) { uint8_t t = target[i]; target[i] = target[r.te - i]; target[r.te - i] = t; }
    if (r.score == rr.score) r.tb = r.te - rr.te, r.qb = r.qe - rr.qe;
    return r;
}

/* ======================================================================= mem_matesw */
static int mem_matesw(const afo_text *X, const afo_params *p, const afo_pe *pe, const pestat_t pes[4],
                      const alnreg_t *a, int l_ms, const uint8_t *ms, regv_t *ma, const rstate_t *Sdedup) {
    int64_t l_pac = X->n;
    int i, r, skip[4], n = 0, rid = -1;
    int8_t mat[25];
    for (int x = 0, k = 0; x < 4; ++x) {  /* bwa_fill_scmat */
        for (int y = 0; y < 4; ++y) mat[k++] = x == y ? p->a : -p->b;
        mat[k++] = -1;
    }
    for (int y = 0; y < 5; ++y) mat[20 + y] = -1;
    for (r = 0; r < 4; ++r) skip[r] = pes[r].failed ? 1 : 0;
    for (i = 0; i < ma->n; ++i) {
        int64_t dist;
        r = mem_infer_dir(l_pac, a->rb, ma->a[i].rb, &dist);
        if (dist >= pes[r].low && dist <= pes[r].high) skip[r] = 1;
    }
    if (skip[0] + skip[1] + skip[2] + skip[3] == 4) return 0;
    for (r = 0; r < 4; ++r) {
        int is_rev, is_larger;
        uint8_t seq[AFO_MAX_READ], *ref = 0;
        int64_t rb, re;
        if (skip[r]) continue;
        is_rev = (r >> 1 != (r & 1));
        is_larger = !(r >> 1);
        if (is_rev) for (i = 0; i < l_ms; ++i) seq[l_ms - 1 - i] = ms[i] < 4 ? 3 - ms[i] : 4;
        else memcpy(seq, ms, l_ms);
        if (!is_rev) {
            rb = is_larger ? a->rb + pes[r].low : a->rb - pes[r].high;
            re = (is_larger ? a->rb + pes[r].high : a->rb - pes[r].low) + l_ms;
        } else {
            rb = (is_larger ? a->rb + pes[r].low : a->rb - pes[r].high) - l_ms;
            re = is_larger ? a->rb + pes[r].high : a->rb - pes[r].low;
        }
        if (rb < 0) rb = 0;
        if (re > l_pac << 1) re = l_pac << 1;
        if (rb < re) {  /* bns_fetch_seq: clipped to the contig (on its strand) holding the middle */
            fetch_clip(X, &rb, (rb + re) >> 1, &re, &rid);
            ref = (uint8_t *)malloc(re - rb > 0 ? re - rb : 1);
            memcpy(ref, X->T + rb, re - rb);
        }
        /* (rid keeps its previous value when rb >= re, as the uninitialised variable in bwa;
         * re - rb < min_seed_len then rejects the window anyway) */
        if (a->rid == rid && re - rb >= p->min_seed_len) {
            kswr_t aln;
            alnreg_t b;
            int tmp, xtra = KSW_XSUBO | KSW_XSTART | (l_ms * p->a < 250 ? KSW_XBYTE : 0) | (p->min_seed_len * p->a);
            aln = ksw_align2(l_ms, seq, (int)(re - rb), ref, mat, p->o_del, p->e_del, p->o_ins, p->e_ins, xtra);
            memset(&b, 0, sizeof(alnreg_t));
            if (aln.score >= p->min_seed_len && aln.qb >= 0) {
                b.rid = a->rid;
                b.is_alt = a->is_alt;
                b.qb = is_rev ? l_ms - (aln.qe + 1) : aln.qb;
                b.qe = is_rev ? l_ms - aln.qb : aln.qe + 1;
                b.rb = is_rev ? (l_pac << 1) - (rb + aln.te + 1) : rb + aln.tb;
                b.re = is_rev ? (l_pac << 1) - (rb + aln.tb) : rb + aln.te + 1;
                b.score = aln.score;
                b.csub = aln.score2;
                b.secondary = -1;
                b.seedcov = (int)((b.re - b.rb < b.qe - b.qb ? b.re - b.rb : b.qe - b.qb) >> 1);
                if (!regv_push(ma, X->caps.reg)) { free(ref); return -1; }
                ma->a[ma->n - 1] = b;
                for (i = 0; i < ma->n - 1; ++i)
                    if (ma->a[i].score < b.score) break;
                tmp = i;
                for (i = ma->n - 1; i > tmp; --i) ma->a[i] = ma->a[i - 1];
                ma->a[i] = b;
            }
            ++n;
        }
        if (n) ma->n = mem_sort_dedup_patch(Sdedup, 0, ma->n, ma->a);
        free(ref);
    }
    return n;
}

/* ================================================================ mem_mark_primary_se */
static void mark_primary_core(const afo_params *p, int n, alnreg_t *a) {
    int i, k, tmp, nz = 0;
    int *z = (int *)malloc(sizeof(int) * (n + 1));
    tmp = p->a + p->b;
    tmp = p->o_del + p->e_del > tmp ? p->o_del + p->e_del : tmp;
    tmp = p->o_ins + p->e_ins > tmp ? p->o_ins + p->e_ins : tmp;
    z[nz++] = 0;
    for (i = 1; i < n; ++i) {
        for (k = 0; k < nz; ++k) {
            int j = z[k];
            int b_max = a[j].qb > a[i].qb ? a[j].qb : a[i].qb;
            int e_min = a[j].qe < a[i].qe ? a[j].qe : a[i].qe;
            if (e_min > b_max) {
                int min_l = a[i].qe - a[i].qb < a[j].qe - a[j].qb ? a[i].qe - a[i].qb : a[j].qe - a[j].qb;
                if (e_min - b_max >= min_l * opt_mask_level) {
                    if (a[j].sub == 0) a[j].sub = a[i].score;
                    if (a[j].score - a[i].score <= tmp && (a[j].is_alt || !a[i].is_alt)) ++a[j].sub_n;
                    break;
                }
            }
        }
        if (k == nz) z[nz++] = i;
        else a[i].secondary = z[k];
    }
    free(z);
}

static int mark_primary_se(const afo_params *p, int n, alnreg_t *a, int64_t id) {
    if (n == 0) return 0;
    for (int i = 0; i < n; ++i) {
        a[i].sub = a[i].alt_sc = 0; a[i].secondary = a[i].secondary_all = -1;
        a[i].hash = hash_64((uint64_t)(id + i));
    }
    introsort_arsh(n, a);
    mark_primary_core(p, n, a);
    for (int i = 0; i < n; ++i) a[i].secondary_all = a[i].secondary;  /* no ALT contigs: n_pri == n */
    return n;
}

/* ========================================================================= mem_pair */
static int mem_pair(const afo_text *X, const afo_params *p, const pestat_t pes[4], regv_t a[2], int id, int *sub,
                    int *n_sub, int z[2], const int n_pri[2]) {
    int64_t l_pac = X->n;
    pair64_t *v = (pair64_t *)malloc(sizeof(pair64_t) * (n_pri[0] + n_pri[1] + 1));
    int64_t mu = 64;
    pair64_t *u = (pair64_t *)malloc(sizeof(pair64_t) * mu);
    int nv = 0, nu = 0, r, i, k, y[4], ret;
    for (r = 0; r < 2; ++r)
        for (i = 0; i < n_pri[r]; ++i) {
            pair64_t key;
            const alnreg_t *e = &a[r].a[i];
            key.x = e->rb < l_pac ? e->rb : (l_pac << 1) - 1 - e->rb;
            key.x = (uint64_t)e->rid << 32 | (key.x - X->ctg_off[e->rid]);
            key.y = (uint64_t)e->score << 32 | (uint64_t)i << 2 | (e->rb >= l_pac) << 1 | r;
            v[nv++] = key;
        }
    introsort_p128(nv, v);
    y[0] = y[1] = y[2] = y[3] = -1;
    for (i = 0; i < nv; ++i) {
        for (r = 0; r < 2; ++r) {
            int dir = r << 1 | (v[i].y >> 1 & 1), which;
            if (pes[dir].failed) continue;
            which = r << 1 | ((v[i].y & 1) ^ 1);
            if (y[which] < 0) continue;
            for (k = y[which]; k >= 0; --k) {
                int64_t dist;
                int q;
                double ns;
                if ((v[k].y & 3) != (uint64_t)which) continue;
                dist = (int64_t)v[i].x - (int64_t)v[k].x;
                if (dist > pes[dir].high) break;
                if (dist < pes[dir].low) continue;
                ns = (dist - pes[dir].avg) / pes[dir].std;
                q = (int)((v[i].y >> 32) + (v[k].y >> 32) + .721 * log(2. * erfc(fabs(ns) * M_SQRT1_2)) * p->a + .499);
                if (q < 0) q = 0;
                if (nu == mu) { mu <<= 1; u = (pair64_t *)realloc(u, sizeof(pair64_t) * mu); }
                pair64_t *pp = &u[nu++];
                pp->y = (uint64_t)k << 32 | (uint64_t)i;
                pp->x = (uint64_t)q << 32 | (hash_64(pp->y ^ (uint64_t)(int64_t)(int32_t)((uint32_t)id << 8)) & 0xffffffffU);
            }
        }
        y[v[i].y & 3] = i;
    }
    if (nu) {
        int tmp = p->a + p->b;
        tmp = tmp > p->o_del + p->e_del ? tmp : p->o_del + p->e_del;
        tmp = tmp > p->o_ins + p->e_ins ? tmp : p->o_ins + p->e_ins;
        introsort_p128(nu, u);
        i = (int)(u[nu - 1].y >> 32); k = (int)(u[nu - 1].y << 32 >> 32);
        z[v[i].y & 1] = (int)(v[i].y << 32 >> 34);
        z[v[k].y & 1] = (int)(v[k].y << 32 >> 34);
        ret = (int)(u[nu - 1].x >> 32);
        *sub = nu > 1 ? (int)(u[nu - 2].x >> 32) : 0;
        for (i = nu - 2, *n_sub = 0; i >= 0; --i)
            if (*sub - (int)(u[i].x >> 32) <= tmp) ++*n_sub;
    } else ret = 0, *sub = 0, *n_sub = 0;
    free(v); free(u);
    return ret;
}

/* ========================================================= mem_reg2aln + mem_aln2sam */
typedef struct { int rid; int64_t pos; int is_rev, flag, score, n_cigar, of; uint32_t cigar[AFO_MAX_CIGAR]; } aln_t;

static void reg2aln(const afo_text *X, const afo_params *p, int l_query, const uint8_t *query, const alnreg_t *ar,
                    aln_t *o) {
    memset(o, 0, sizeof(*o));
    if (!ar || ar->rb < 0 || ar->re < 0) { o->rid = -1; o->pos = -1; o->flag |= 0x4; return; }
    int64_t l_pac = X->n;
    int qb = ar->qb, qe = ar->qe;
    int64_t rb = ar->rb, re = ar->re;
    if (ar->secondary >= 0) o->flag |= 0x100;
    int tmp = afo_infer_bw(qe - qb, (int)(re - rb), ar->truesc, p->a, p->o_del, p->e_del);
    int w2 = afo_infer_bw(qe - qb, (int)(re - rb), ar->truesc, p->a, p->o_ins, p->e_ins);
    w2 = w2 > tmp ? w2 : tmp;
    if (w2 > p->w) w2 = w2 < ar->w ? w2 : ar->w;
    uint32_t cig[AFO_MAX_CIGAR];
    int nc = 0, score = 0, last_sc = -(1 << 30), i = 0;
    do {
        w2 = w2 < p->w << 2 ? w2 : p->w << 2;
        score = afo_gen_cigar(X->T, l_pac, p, w2, qe - qb, query + qb, rb, re, cig, &nc);
        if (score == last_sc || w2 == p->w << 2) break;
        last_sc = score;
        w2 <<= 1;
    } while (++i < 3 && score < ar->truesc - p->a);
    int is_rev;
    int64_t pos = depos(X, rb < l_pac ? rb : re - 1, &is_rev);
    int ncap = nc < AFO_MAX_CIGAR ? nc : AFO_MAX_CIGAR, of = nc > AFO_MAX_CIGAR;
    if (ncap > 0) {  /* squeeze out leading or trailing deletions */
        if ((cig[0] & 0xf) == 2) {
            pos += cig[0] >> 4;
            memmove(cig, cig + 1, sizeof(uint32_t) * (ncap - 1));
            --ncap;
        } else if ((cig[ncap - 1] & 0xf) == 2) --ncap;
    }
    uint32_t fin[AFO_MAX_CIGAR + 2];
    int nf = 0;
    int clip5 = is_rev ? l_query - qe : qb, clip3 = is_rev ? qb : l_query - qe;
    if (clip5) fin[nf++] = (uint32_t)clip5 << 4 | 4;  /* primary record: soft clip (S = 4 in BAM) */
    for (int x = 0; x < ncap; ++x) fin[nf++] = cig[x];
    if (clip3) fin[nf++] = (uint32_t)clip3 << 4 | 4;
    if (nf > AFO_MAX_CIGAR) { of = 1; nf = AFO_MAX_CIGAR; }
    memcpy(o->cigar, fin, sizeof(uint32_t) * nf);
    o->n_cigar = nf;
    o->of = of;
    if (of) o->flag |= FLAG_CIGAR_OVERFLOW;
    o->rid = pos2rid(X, pos);
    o->pos = pos - X->ctg_off[o->rid];
    o->is_rev = is_rev;
    o->score = ar->score;
}

/* mem_aln2sam's flag/position rules for the primary record of a read with mate m (S2 output:
 * one record per read, positions on the single anchor contig) */
static void aln2rec(const aln_t *p_, const aln_t *m_, int extra, afo_out *out, int64_t r) {
    aln_t p = *p_, m = *m_;
    int flag = p.flag | extra;
    flag |= 0x1;
    flag |= p.rid < 0 ? 0x4 : 0;
    flag |= m.rid < 0 ? 0x8 : 0;
    if (p.rid < 0 && m.rid >= 0) { p.rid = m.rid; p.pos = m.pos; p.is_rev = m.is_rev; p.n_cigar = 0; }
    if (m.rid < 0 && p.rid >= 0) { m.rid = p.rid; m.pos = p.pos; m.is_rev = p.is_rev; m.n_cigar = 0; }
    flag |= p.is_rev ? 0x10 : 0;
    flag |= m.is_rev ? 0x20 : 0;
    out->flag[r] = flag;
    out->pos[r] = p.rid >= 0 ? (int32_t)p.pos : -1;
    out->score[r] = p_->rid >= 0 ? p.score : 0;
    out->n_cigar[r] = p_->rid >= 0 ? p.n_cigar : 0;
    for (int c = 0; c < AFO_MAX_CIGAR; ++c) out->cigar[r * AFO_MAX_CIGAR + c] = c < out->n_cigar[r] ? p.cigar[c] : 0;
}

/* mem_aln2sam for the genome calls: record `which` of a read's list, mate m (NULL single-end).
 * Under -M a supplementary part (internal 0x10000) prints as 0x100; parts after the first take
 * hard clips and a SEQ trimmed to the aligned query span (SEQ orientation). */
static void aln2grec(const aln_t *p_, const aln_t *m_, int which, int l_seq, int32_t read, afo_grec *o) {
    aln_t p = *p_, m;
    if (m_) m = *m_;
    p.flag |= m_ ? 0x1 : 0;
    p.flag |= p.rid < 0 ? 0x4 : 0;
    p.flag |= m_ && m.rid < 0 ? 0x8 : 0;
    if (p.rid < 0 && m_ && m.rid >= 0) { p.rid = m.rid; p.pos = m.pos; p.is_rev = m.is_rev; p.n_cigar = 0; }
    if (m_ && m.rid < 0 && p.rid >= 0) { m.rid = p.rid; m.pos = p.pos; m.is_rev = p.is_rev; m.n_cigar = 0; }
    p.flag |= p.is_rev ? 0x10 : 0;
    p.flag |= m_ && m.is_rev ? 0x20 : 0;
    memset(o, 0, sizeof(*o));
    o->read = read;
    o->flag = (p.flag & 0xffff) | ((p.flag & 0x10000) ? 0x100 : 0) | (p_->of ? FLAG_CIGAR_OVERFLOW : 0);
    o->rid = p.rid;
    o->pos = p.rid >= 0 ? p.pos : -1;
    o->score = p.rid >= 0 && p_->rid >= 0 ? p.score : 0;
    o->n_cigar = p.n_cigar;
    for (int c = 0; c < p.n_cigar; ++c) {
        uint32_t op = p.cigar[c] & 0xf;
        if (op == 4 && which) op = 5;  /* hard clips on the parts after the first */
        o->cigar[c] = (p.cigar[c] & ~0xfu) | op;
    }
    o->mrid = m_ && m.rid >= 0 ? m.rid : -1;
    o->mpos = m_ && m.rid >= 0 ? m.pos : -1;
    o->seq_b = 0; o->seq_e = l_seq;
    if (p.n_cigar && which) {
        if ((p.cigar[0] & 0xf) == 4) o->seq_b = (int32_t)(p.cigar[0] >> 4);
        if ((p.cigar[p.n_cigar - 1] & 0xf) == 4) o->seq_e = l_seq - (int32_t)(p.cigar[p.n_cigar - 1] >> 4);
    }
}

/* mem_reg2sam (-M, no -a): the records of one read from its marked regions; returns their
 * count (written up to max_rec) */
static int reg2sam(const afo_text *X, const afo_params *p, int l, const uint8_t *q, const regv_t *a, int extra_flag,
                   const aln_t *m, int32_t read, afo_grec *out, int max_rec) {
    int k, nrec = 0;
    aln_t al[AFO_G_MAX_REC];
    int na = 0;
    for (k = 0; k < a->n; ++k) {
        const alnreg_t *r = &a->a[k];
        if (r->score < p->T) continue;
        if (r->secondary >= 0) continue;
        if (na >= AFO_G_MAX_REC) { ++na; continue; }
        reg2aln(X, p, l, q, r, &al[na]);
        al[na].flag |= extra_flag;
        if (na && r->secondary < 0) al[na].flag |= 0x10000;  /* -M: supplementary -> 0x100 */
        ++na;
    }
    if (na == 0) {
        aln_t t;
        reg2aln(X, p, l, q, NULL, &t);
        t.flag |= extra_flag;
        if (max_rec > 0) aln2grec(&t, m, 0, l, read, &out[0]);
        return 1;
    }
    for (k = 0; k < na && k < AFO_G_MAX_REC; ++k) {
        if (nrec < max_rec) aln2grec(&al[k], m, k, l, read, &out[nrec]);
        ++nrec;
    }
    return na;  /* > AFO_G_MAX_REC: the caller flags the read */
}

/* ======================================================================== mem_sam_pe */
/* out: S2's one-record-per-read arrays (the anchor), or (grec) every record of the pair (the
 * genome, S4: read 1's records then read 2's); returns the number of records written to grec */
static int mem_sam_pe(const afo_text *X, const afo_params *p, const afo_pe *pe, const pestat_t pes[4], uint64_t id,
                      const uint8_t *q0, int l0, const uint8_t *q1, int l1, regv_t a[2], int ovf[2], afo_out *out,
                      int64_t r0, afo_grec *grec, int max_rec, int32_t *n_rec) {
    int i, j, z[2], o, subo, n_sub, extra_flag = 1, n_pri[2];
    aln_t h[2];
    const uint8_t *qs[2] = {q0, q1};
    int ls[2] = {l0, l1};
    rstate_t Sd;  /* mem_sort_dedup_patch context (no patching in mate rescue) */
    memset(&Sd, 0, sizeof(Sd));
    Sd.X = X; Sd.p = p; Sd.pe = pe;
    {   /* mate rescue: mem_matesw for the top hits of each end */
        regv_t b[2];
        b[0].n = b[1].n = 0; b[0].m = b[1].m = 0; b[0].a = b[1].a = NULL;
        for (i = 0; i < 2; ++i)
            for (j = 0; j < a[i].n; ++j)
                if (a[i].a[j].score >= a[i].a[0].score - pe->pen_unpaired) *regv_push(&b[i], 1 << 30) = a[i].a[j];
        for (i = 0; i < 2; ++i)
            for (j = 0; j < b[i].n && j < pe->max_matesw; ++j) {
                if (ovf[!i]) continue;
                if (mem_matesw(X, p, pe, pes, &b[i].a[j], ls[!i], qs[!i], &a[!i], &Sd) < 0) {
                    ovf[!i] = 1; a[!i].n = 0;
                }
            }
        free(b[0].a); free(b[1].a);
    }
    n_pri[0] = mark_primary_se(p, a[0].n, a[0].a, (int64_t)(id << 1 | 0));
    n_pri[1] = mark_primary_se(p, a[1].n, a[1].a, (int64_t)(id << 1 | 1));
    if (n_pri[0] && n_pri[1] && (o = mem_pair(X, p, pes, a, (int)(uint32_t)id, &subo, &n_sub, z, n_pri)) > 0) {
        int is_multi[2], score_un;
        for (i = 0; i < 2; ++i) {
            for (j = 1; j < n_pri[i]; ++j)
                if (a[i].a[j].secondary < 0 && a[i].a[j].score >= p->T) break;
            is_multi[i] = j < n_pri[i] ? 1 : 0;
        }
        if (is_multi[0] || is_multi[1]) goto no_pairing;
        score_un = a[0].a[0].score + a[1].a[0].score - pe->pen_unpaired;
        if (o > score_un) {
            for (i = 0; i < 2; ++i) {
                alnreg_t *c = &a[i].a[z[i]];
                if (c->secondary >= 0) c->sub = a[i].a[c->secondary].score, c->secondary = -2;
            }
            extra_flag |= 2;
        } else {
            z[0] = z[1] = 0;
        }
        for (i = 0; i < 2; ++i) reg2aln(X, p, ls[i], qs[i], &a[i].a[z[i]], &h[i]);
        if (grec) {
            for (i = 0; i < 2; ++i) {
                h[i].flag |= 0x40 << i | extra_flag;
                if (max_rec > 0) aln2grec(&h[i], &h[!i], 0, ls[i], (int32_t)(r0 + i), &grec[i * max_rec]);
                n_rec[i] = 1;
            }
            goto flags_done;
        }
        aln2rec(&h[0], &h[1], 0x40 | extra_flag, out, r0);
        aln2rec(&h[1], &h[0], 0x80 | extra_flag, out, r0 + 1);
        goto flags_done;
    }
no_pairing:
    for (i = 0; i < 2; ++i) {
        int which = -1;
        if (a[i].n && a[i].a[0].score >= p->T) which = 0;
        reg2aln(X, p, ls[i], qs[i], which >= 0 ? &a[i].a[which] : NULL, &h[i]);
    }
    if (h[0].rid == h[1].rid && h[0].rid >= 0) {
        int64_t dist;
        int d = mem_infer_dir(X->n, a[0].a[0].rb, a[1].a[0].rb, &dist);
        if (!pes[d].failed && dist >= pes[d].low && dist <= pes[d].high) extra_flag |= 2;
    }
    if (grec) {
        for (i = 0; i < 2; ++i)
            n_rec[i] = reg2sam(X, p, ls[i], qs[i], &a[i], (0x40 << i) | extra_flag, &h[!i], (int32_t)(r0 + i),
                               grec + i * max_rec, max_rec);
        goto flags_done;
    }
    aln2rec(&h[0], &h[1], 0x40 | extra_flag, out, r0);
    aln2rec(&h[1], &h[0], 0x80 | extra_flag, out, r0 + 1);
flags_done:
    if (grec) {
        for (i = 0; i < 2; ++i)
            if (ovf[i] || n_rec[i] > max_rec)
                for (j = 0; j < (n_rec[i] < max_rec ? n_rec[i] : max_rec); ++j) grec[i * max_rec + j].flag |= FLAG_MEM_OVERFLOW;
        return 0;
    }
    for (i = 0; i < 2; ++i)
        if (ovf[i]) out->flag[r0 + i] |= FLAG_MEM_OVERFLOW;
    return 0;
}

/* ====================================================================== driver */
void afo_pe_default(afo_pe *pe) {
    /* bwa 0.7.17 mem_opt_init, paired-end defaults; chunk = 10,000,000 bases x the thread
     * count of the reference's --thread (default 1, Anchored_Fusion.py:29) */
    pe->pen_unpaired = 17; pe->max_ins = 10000; pe->max_matesw = 50; pe->split_width = 10;
    pe->max_mem_intv = 20; pe->max_chain_gap = 10000;
    pe->chunk_bases = 10000000; pe->pair_base = 0;
}

static int read_codes(const uint8_t *reads, int64_t r, int32_t stride, const int32_t *lens, uint8_t *q) {
    int l = lens ? lens[r] : stride;
    if (l > stride) l = stride;
    if (l > AFO_MAX_READ) l = AFO_MAX_READ;
    if (l < 0) l = 0;
    for (int i = 0; i < l; ++i) q[i] = afo_nt4(reads[r * (int64_t)stride + i]);
    return l;
}

/* paired-end over a text (anchor: out; genome: grec) */
static int align_pairs_text(const afo_text *X, const afo_index *I, const uint8_t *reads, int64_t n_pairs,
                            int32_t stride, const int32_t *lens, const afo_params *p, const afo_pe *pe_in, int n_threads,
                            afo_out *out, afo_grec *grec, int32_t max_rec, int32_t *n_rec) {
    afo_pe pe;
    if (pe_in) pe = *pe_in;
    else afo_pe_default(&pe);
    int64_t nr = 2 * n_pairs;
    if (n_pairs <= 0) return 0;
    if (out && out->hits && I) afo_seed_filter(I, reads, nr, stride, lens, out->hits);
    regv_t *regs = (regv_t *)calloc(nr, sizeof(regv_t));
    uint8_t *codes = (uint8_t *)malloc((size_t)nr * AFO_MAX_READ);
    int *len = (int *)malloc(sizeof(int) * nr), *ovf = (int *)calloc(nr, sizeof(int));
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#pragma omp parallel for schedule(dynamic, 64)
#endif
    for (int64_t r = 0; r < nr; ++r) {
        uint8_t *q = codes + r * AFO_MAX_READ;
        int l = read_codes(reads, r, stride, lens, q);
        len[r] = l;
        /* K1: a read with no sampled 16-mer in the filter has no seed (exact), so no regions */
        if (out && out->hits && I && out->hits[r] == 0) { regs[r].n = 0; continue; }
        if (align1_core(X, p, &pe, q, l, &regs[r]) < 0) ovf[r] = 1;
    }
    /* chunks of >= chunk_bases bases (bseq_read): insert-size statistics per chunk */
    int64_t c0 = 0;
    while (c0 < n_pairs) {
        int64_t size = 0, c1 = c0;
        while (c1 < n_pairs) {
            size += len[2 * c1] + len[2 * c1 + 1];
            ++c1;
            if (size >= pe.chunk_bases) break;
        }
        pestat_t pes[4];
        mem_pestat(p, &pe, X->n, c1 - c0, regs + 2 * c0, pes);
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 64)
#endif
        for (int64_t pp = c0; pp < c1; ++pp) {
            mem_sam_pe(X, p, &pe, pes, (uint64_t)(pe.pair_base + pp), codes + 2 * pp * AFO_MAX_READ, len[2 * pp],
                       codes + (2 * pp + 1) * AFO_MAX_READ, len[2 * pp + 1], &regs[2 * pp], &ovf[2 * pp], out, 2 * pp,
                       grec ? grec + 2 * pp * max_rec : NULL, max_rec, n_rec ? n_rec + 2 * pp : NULL);
        }
        c0 = c1;
    }
    for (int64_t r = 0; r < nr; ++r) free(regs[r].a);
    free(regs); free(codes); free(len); free(ovf);
    return 0;
}

int afo_align_pairs(const afo_index *I, const uint8_t *reads, int64_t n_pairs, int32_t stride, const int32_t *lens,
                    const afo_params *p, const afo_pe *pe_in, int n_threads, afo_out *out) {
    return align_pairs_text(afo_index_text(I), I, reads, n_pairs, stride, lens, p, pe_in, n_threads, out, NULL, 0, NULL);
}

/* S4: `bwa mem -M genome fq1 fq2`, every record of every pair (grec[(2 pair + mate) * max_rec + k]) */
int afo_genome_align_pe(const afo_genome *G, const uint8_t *reads, int64_t n_pairs, int32_t stride, const int32_t *lens,
                        const afo_params *p, const afo_pe *pe, int n_threads, int32_t max_rec, afo_grec *recs,
                        int32_t *n_rec) {
    if (max_rec < 1) return -1;
    return align_pairs_text(G, NULL, reads, n_pairs, stride, lens, p, pe, n_threads, NULL, recs, max_rec, n_rec);
}

/* S5: `bwa mem -M genome reads.fa` (single-end), read ids id_base + r, or ids[r] when ids is given
 * (a shard of a wider query list: the reads' ordinals in that list) */
static int genome_align_se(const afo_genome *G, const uint8_t *reads, int64_t n, int32_t stride, const int32_t *lens,
                           const afo_params *p, const afo_pe *pe_in, int64_t id_base, const int64_t *ids, int n_threads,
                           int32_t max_rec, afo_grec *recs, int32_t *n_rec) {
    afo_pe pe;
    if (pe_in) pe = *pe_in;
    else afo_pe_default(&pe);
    if (max_rec < 1) return -1;
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#pragma omp parallel for schedule(dynamic, 16)
#endif
    for (int64_t r = 0; r < n; ++r) {
        uint8_t q[AFO_MAX_READ];
        int l = read_codes(reads, r, stride, lens, q);
        regv_t rg = {NULL, 0, 0};
        int ovf = align1_core(G, p, &pe, q, l, &rg) < 0;
        mark_primary_se(p, rg.n, rg.a, ids ? ids[r] : id_base + r);
        n_rec[r] = reg2sam(G, p, l, q, &rg, 0, NULL, (int32_t)r, recs + r * max_rec, max_rec);
        if (ovf || n_rec[r] > max_rec)
            for (int j = 0; j < (n_rec[r] < max_rec ? n_rec[r] : max_rec); ++j) recs[r * max_rec + j].flag |= FLAG_MEM_OVERFLOW;
        free(rg.a);
    }
    return 0;
}

int afo_genome_align_se(const afo_genome *G, const uint8_t *reads, int64_t n, int32_t stride, const int32_t *lens,
                        const afo_params *p, const afo_pe *pe_in, int64_t id_base, int n_threads, int32_t max_rec,
                        afo_grec *recs, int32_t *n_rec) {
    return genome_align_se(G, reads, n, stride, lens, p, pe_in, id_base, NULL, n_threads, max_rec, recs, n_rec);
}

int afo_genome_align_se_ids(const afo_genome *G, const uint8_t *reads, int64_t n, int32_t stride, const int32_t *lens,
                            const afo_params *p, const afo_pe *pe_in, const int64_t *ids, int n_threads, int32_t max_rec,
                            afo_grec *recs, int32_t *n_rec) {
    return genome_align_se(G, reads, n, stride, lens, p, pe_in, 0, ids, n_threads, max_rec, recs, n_rec);
}

/* mem_collect_intv + mem_chain's occurrence sampling for one read, as the seed list mem_chain
 * walks: seeds[k] = {rbeg, qbeg, len} in order (before contig / strand checks); returns the
 * count, -1 on overflow.  memset_mode: the MEM-set restatement instead of the FM index. */
int afo_genome_seeds(const afo_genome *G, const uint8_t *read, int32_t l, const afo_params *p, const afo_pe *pe_in,
                     int memset_mode, int64_t *rbeg, int32_t *qbeg, int32_t *len, int32_t cap) {
    afo_pe pe;
    if (pe_in) pe = *pe_in;
    else afo_pe_default(&pe);
    afo_text tmp = *G;
    if (memset_mode) {
        if (!G->rank) return -2;
        tmp.fm = 0;
    }
    uint8_t q[AFO_MAX_READ];
    if (l > AFO_MAX_READ) l = AFO_MAX_READ;
    for (int i = 0; i < l; ++i) q[i] = afo_nt4(read[i]);
    rstate_t S;
    rstate_init(&S, &tmp, p, &pe, q, l);
    if (l < p->min_seed_len) return 0;
    collect_intv(&S);
    if (S.overflow) return -1;
    int n = 0;
    for (int i = 0; i < S.nsi; ++i) {
        const sintv_t *v = &S.si[i];
        int64_t step = v->cnt > p->max_occ ? v->cnt / p->max_occ : 1, k;
        int count;
        for (k = 0, count = 0; k < v->cnt && count < p->max_occ; k += step, ++count) {
            if (n >= cap) return -1;
            rbeg[n] = intv_occ(&S, v, k); qbeg[n] = v->qb; len[n] = v->qe - v->qb;
            ++n;
        }
    }
    return n;
}

/* mem_collect_intv for each read (FM index): its seed intervals in mem_chain's order, as int64
 * words {sa_k, s, qb, qe} at out[(r * max_iv + i) * 4]; n_iv[r] the count (-1: past caps.intv) */
int afo_genome_intervals(const afo_genome *G, const uint8_t *reads, int64_t n, int32_t stride, const int32_t *lens,
                         const afo_params *p, const afo_pe *pe_in, int n_threads, int32_t max_iv, int64_t *out,
                         int32_t *n_iv) {
    afo_pe pe;
    if (pe_in) pe = *pe_in;
    else afo_pe_default(&pe);
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#pragma omp parallel for schedule(dynamic, 16)
#endif
    for (int64_t r = 0; r < n; ++r) {
        uint8_t q[AFO_MAX_READ];
        const int l = read_codes(reads, r, stride, lens, q);
        rstate_t S;
        rstate_init(&S, G, p, &pe, q, l);
        n_iv[r] = 0;
        if (l < p->min_seed_len) continue;
        collect_intv(&S);
        if (S.overflow) { n_iv[r] = -1; continue; }
        n_iv[r] = S.nsi;
        for (int i = 0; i < S.nsi && i < max_iv; ++i) {
            int64_t *o = out + ((size_t)r * max_iv + i) * 4;
            o[0] = S.si[i].sa_k; o[1] = S.si[i].cnt; o[2] = S.si[i].qb; o[3] = S.si[i].qe;
        }
    }
    return 0;
}

/* mem_align1_core for each read: its regions in mem_sort_dedup_patch order */
int afo_genome_regions(const afo_genome *G, const uint8_t *reads, int64_t n, int32_t stride, const int32_t *lens,
                       const afo_params *p, const afo_pe *pe_in, int n_threads, int32_t max_reg, afo_reg *regs,
                       int32_t *n_reg) {
    afo_pe pe;
    if (pe_in) pe = *pe_in;
    else afo_pe_default(&pe);
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#pragma omp parallel for schedule(dynamic, 16)
#endif
    for (int64_t r = 0; r < n; ++r) {
        uint8_t q[AFO_MAX_READ];
        int l = read_codes(reads, r, stride, lens, q);
        regv_t rg = {NULL, 0, 0};
        if (align1_core(G, p, &pe, q, l, &rg) < 0) n_reg[r] = -1;
        else {
            n_reg[r] = rg.n;
            for (int k = 0; k < rg.n && k < max_reg; ++k) {
                afo_reg *o = &regs[r * max_reg + k];
                const alnreg_t *a = &rg.a[k];
                o->rb = a->rb; o->re = a->re; o->qb = a->qb; o->qe = a->qe; o->rid = a->rid; o->score = a->score;
                o->truesc = a->truesc; o->w = a->w; o->seedcov = a->seedcov; o->seedlen0 = a->seedlen0;
            }
        }
        free(rg.a);
    }
    return 0;
}
