/*
 * blat.c -- TEST INFRASTRUCTURE ONLY: CPU restatement of the BLAT searches of the partner
 * stages (functions.py:341, 530, 966, 1007, 1071, 1122, 1244), the contract of the GPU kernel
 * anchored-fusion_amd/csrc/blat.hip (bit-exact).
 *
 * BLAT (Kent 2002, Genome Res. 12:656; blat >= v.35, README.md:19) is a third-party binary,
 * absent from /root/reference and from this image.  Its published search is restated with the
 * options the reference passes (-stepSize, -minMatch, -repMatch, -minScore, -minIdentity,
 * defaults otherwise); the steps and the choices this restatement makes are in afgpu.h
 * (af_blat_params) and DESIGN.md §2.  Parity with the BLAT binary is unpinned.
 *
 * Alignment as the paper publishes it for nucleotides: the hits of a clump that lie on one
 * diagonal with touching tiles form a range (an exact match), each range is extended WITHOUT gaps
 * into a high-scoring segment pair (HSP: +1 per match, -1 per mismatch, an end stops XDOWN
 * positions after its last new best -- blat's extendHitLeft / extendHitRight), and gaps appear
 * only where HSPs are stitched into one alignment (the chain DP below).  The round-5 contract --
 * one part per clump from a banded ksw_extend2 + global alignment, gaps inside parts -- is kept
 * behind afo_blat_set_gapped(1) so that the two can be compared (tests, scripts/blat_modes.py).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "af_oracle.h"
#include "af_oracle_int.h"

#define TILE 11
#define NKEYS (1u << (2 * TILE))
#define MAXH 32768     /* tile hits per query strand (the first MAXH in query order) */
#define MAXCL 4096     /* clumps per query strand (the first MAXCL in diagonal order) */
#define MAXP MAXCL     /* aligned clumps per query strand: one per clump at most (no cap of its own) */
/* stitching work per query strand (predecessor candidates the chain DP rescans after a chain is
 * emitted; the first pass is always made): once past it,
 * no further chain is emitted and the strand is counted as cap[2] */
#define STITCH_WORK (1LL << 24)
/* an HSP end stops this many positions after its running score last reached a new best */
#define XDOWN 10

struct afo_tiles {
    uint8_t *T;        /* codes 0-3, 4 = N */
    int64_t n;
    int32_t step;
    uint32_t *start;   /* NKEYS + 1 */
    uint32_t *pos;     /* tile positions, ascending per key */
    uint32_t *ncum;    /* N count before each 64-base block: stitching never crosses an N */
    uint64_t *nmask;   /* N bits, 64 bases per word */
};

afo_tiles *afo_tiles_build(const char *seq, int64_t n, int32_t step) {
    if (n < TILE || step < 1 || step > TILE) return NULL;
    afo_tiles *X = (afo_tiles *)calloc(1, sizeof(afo_tiles));
    X->n = n; X->step = step;
    X->T = (uint8_t *)malloc(n);
    for (int64_t i = 0; i < n; ++i) X->T[i] = afo_nt4((uint8_t)seq[i]);
    X->start = (uint32_t *)calloc(NKEYS + 1, sizeof(uint32_t));
    int64_t nt = 0;
    for (int64_t p = 0; p + TILE <= n; p += step) {
        uint32_t k = 0;
        int ok = 1;
        for (int u = 0; u < TILE; ++u) {
            if (X->T[p + u] > 3) { ok = 0; break; }
            k |= (uint32_t)X->T[p + u] << (2 * u);
        }
        if (ok) { ++X->start[k + 1]; ++nt; }
    }
    for (uint32_t k = 0; k < NKEYS; ++k) X->start[k + 1] += X->start[k];
    X->pos = (uint32_t *)malloc(sizeof(uint32_t) * (nt > 0 ? nt : 1));
    uint32_t *fill = (uint32_t *)malloc(sizeof(uint32_t) * NKEYS);
    memcpy(fill, X->start, sizeof(uint32_t) * NKEYS);
    for (int64_t p = 0; p + TILE <= n; p += step) {
        uint32_t k = 0;
        int ok = 1;
        for (int u = 0; u < TILE; ++u) {
            if (X->T[p + u] > 3) { ok = 0; break; }
            k |= (uint32_t)X->T[p + u] << (2 * u);
        }
        if (ok) X->pos[fill[k]++] = (uint32_t)p;
    }
    free(fill);
    int64_t nb = (n >> 6) + 2;
    X->ncum = (uint32_t *)calloc(nb, sizeof(uint32_t));
    X->nmask = (uint64_t *)calloc(nb, sizeof(uint64_t));
    for (int64_t i = 0; i < n; ++i)
        if (X->T[i] > 3) X->nmask[i >> 6] |= 1ull << (i & 63);
    for (int64_t b = 0; b + 1 < nb; ++b) X->ncum[b + 1] = X->ncum[b] + (uint32_t)__builtin_popcountll(X->nmask[b]);
    return X;
}

void afo_tiles_free(afo_tiles *X) {
    if (!X) return;
    free(X->T); free(X->start); free(X->pos); free(X->ncum); free(X->nmask); free(X);
}

/* N bases in T[a, b): the 64-base blocks' prefix counts, corrected by the end blocks' masks */
static int64_t n_in(const afo_tiles *X, int64_t a, int64_t b) {
    if (b <= a) return 0;
    int64_t ba = a >> 6, bb = b >> 6;
    int64_t c = (int64_t)X->ncum[bb] - (int64_t)X->ncum[ba];
    c -= __builtin_popcountll(X->nmask[ba] & ((1ull << (a & 63)) - 1));
    c += __builtin_popcountll(X->nmask[bb] & ((1ull << (b & 63)) - 1));
    return c;
}

void afo_blat_params_default(afo_blat_params *p) {
    p->step_size = TILE; p->min_match = 2; p->rep_match = 1024; p->min_score = 30;
    p->min_identity = 90; p->max_gap = 2; p->max_intron = 750000;
}

/* the alignment scores of a clump's extension (afgpu.h) */
static void blat_dp_params(afo_params *p) {
    memset(p, 0, sizeof(*p));
    p->a = 1; p->b = 1; p->o_del = 3; p->e_del = 1; p->o_ins = 3; p->e_ins = 1;
    p->pen_clip5 = 0; p->pen_clip3 = 0; p->w = 16; p->zdrop = 20;
}

typedef struct { int64_t diag, t; int32_t q; } hit_t;
typedef struct { int32_t sz, q; int64_t t; } blk_t;
/* a growable list of blocks (the parts' and, in long mode, the rows') */
typedef struct { blk_t *b; int64_t n, cap; } blk_arena;
static void arena_push(blk_arena *a, int32_t sz, int32_t q, int64_t t) {
    if (a->n == a->cap) {
        a->cap = a->cap ? 2 * a->cap : 1024;
        a->b = (blk_t *)realloc(a->b, sizeof(blk_t) * a->cap);
    }
    a->b[a->n].sz = sz; a->b[a->n].q = q; a->b[a->n].t = t;
    ++a->n;
}
/* one aligned clump ("part"): its blocks are ar[boff, boff + nb); block 0 is (b0sz, b0q, b0t),
 * which trim_front shortens */
typedef struct {
    int32_t qb, qe, score, matches, mismatches, ncount, qni, qbi, tni, tbi, nb;
    int64_t tb, te;
    int32_t b0sz, b0q;
    int64_t b0t, boff;
    int used;
} reg_b;
typedef struct { int32_t cnt, q; int64_t diag, t, h0, h1; } clump_t;  /* h0, h1: its hits in diagonal order */

/* The caps of a search mode.  Short queries (afo_blat: reads and tails, <= AFO_MAX_READ bases)
 * are the GPU kernel k_blat's contract; long queries (afo_blat_long: the anchor transcript of
 * fn:341 / fn:966, one query of up to AFO_BLAT_LONG_MAX bases) searched whole, as BLAT searches a
 * query, with larger caps and rows of any block count. */
typedef struct {
    int64_t maxh;     /* tile hits per strand (the first maxh in query order) */
    int maxcl;        /* clumps per strand (the first maxcl in diagonal order) */
    int part_blocks;  /* blocks per part (a part with more is dropped) */
    int cig_cap;      /* CIGAR ops per part (more: dropped) */
    int row_blocks;   /* blocks per row (more: the row is dropped); 0: any */
} blat_mode;
static const blat_mode MODE_SHORT = {MAXH, MAXCL, AFO_PSL_MAX_BLOCKS, AFO_MAX_CIGAR, AFO_PSL_MAX_BLOCKS};
static const blat_mode MODE_LONG = {AFO_BLAT_LONG_HITS, AFO_BLAT_LONG_CLUMPS, AFO_BLAT_LONG_PART_BLOCKS,
                                    2 * AFO_BLAT_LONG_PART_BLOCKS + 1, 0};

static int cmp_hit(const void *a, const void *b) {
    const hit_t *x = (const hit_t *)a, *y = (const hit_t *)b;
    if (x->diag != y->diag) return x->diag < y->diag ? -1 : 1;
    return x->q - y->q;
}
static int cmp_clump(const void *a, const void *b) {
    const clump_t *x = (const clump_t *)a, *y = (const clump_t *)b;
    if (x->cnt != y->cnt) return y->cnt - x->cnt;
    if (x->diag != y->diag) return x->diag < y->diag ? -1 : 1;
    return x->q - y->q;
}

static inline blk_t blk_of(const blk_arena *ar, const reg_b *r, int k) {
    if (k == 0) { blk_t b = {r->b0sz, r->b0q, r->b0t}; return b; }
    return ar->b[r->boff + k];
}

/* one clump's seed tile (q, t) -> an aligned region with blocks (appended to ar); 0 if dropped */
static int align_clump(const afo_tiles *X, const uint8_t *Q, int L, int32_t q, int64_t t, reg_b *r,
                       const blat_mode *md, blk_arena *ar, uint8_t *qs, uint8_t *ts, uint32_t *cig) {
    afo_params P;
    blat_dp_params(&P);
    int qle, tle, gtle, gscore, max_off;
    int score, truesc, qb, qe;
    int64_t tb, te;
    if (q > 0) {
        int tl = (int)(t < q + P.w ? t : q + P.w);
        for (int i = 0; i < q; ++i) qs[i] = Q[q - 1 - i];
        for (int i = 0; i < tl; ++i) ts[i] = X->T[t - 1 - i];
        score = afo_ext_dp(q, qs, tl, ts, &P, P.w, 0, P.zdrop, TILE * P.a, &qle, &tle, &gtle, &gscore, &max_off);
        if (gscore <= 0 || gscore <= score) { qb = q - qle; tb = t - tle; truesc = score; }
        else { qb = 0; tb = t - gtle; truesc = gscore; }
    } else {
        score = truesc = TILE * P.a; qb = 0; tb = t;
    }
    if (q + TILE < L) {
        int qs0 = q + TILE;
        int64_t t0 = t + TILE;
        int64_t room = X->n - t0;
        int tl = (int)(room < (L - qs0) + P.w ? room : (L - qs0) + P.w);
        int sc0 = score;
        score = afo_ext_dp(L - qs0, Q + qs0, tl, X->T + t0, &P, P.w, 0, P.zdrop, sc0, &qle, &tle, &gtle, &gscore,
                           &max_off);
        if (gscore <= 0 || gscore <= score) { qe = qs0 + qle; te = t0 + tle; truesc += score - sc0; }
        else { qe = L; te = t0 + gtle; truesc += gscore - sc0; }
    } else {
        qe = L; te = t + TILE;
    }
    int lq = qe - qb, rl = (int)(te - tb);
    if (lq <= 0 || rl <= 0) return 0;
    int w2 = afo_infer_bw(lq, rl, truesc, P.a, P.o_del, P.e_del);
    int w3 = afo_infer_bw(lq, rl, truesc, P.a, P.o_ins, P.e_ins);
    w2 = w2 > w3 ? w2 : w3;
    w2 = w2 < 64 ? w2 : 64;
    int nc = 0;
    afo_gen_cigar_cap(X->T, (int64_t)1 << 62, &P, w2, lq, Q + qb, tb, te, cig, md->cig_cap, &nc);
    if (nc > md->cig_cap) return 0;
    int xs = 0, xe = nc;
    if (nc > 0 && (cig[0] & 0xf) == 2) { tb += cig[0] >> 4; xs = 1; }
    else if (nc > 0 && (cig[nc - 1] & 0xf) == 2) { te -= cig[nc - 1] >> 4; xe = nc - 1; }
    memset(r, 0, sizeof(*r));
    const int64_t a0 = ar->n;
    r->boff = a0;
    int32_t x = qb;
    int64_t y = tb;
    for (int k = xs; k < xe; ++k) {
        int len = (int)(cig[k] >> 4), op = (int)(cig[k] & 0xf);
        if (op == 0) {
            if (r->nb >= md->part_blocks) { ar->n = a0; return 0; }
            arena_push(ar, len, x, y);
            ++r->nb;
            for (int u = 0; u < len; ++u) {
                uint8_t a = Q[x + u], b = X->T[y + u];
                if (a > 3 || b > 3) ++r->ncount;
                else if (a == b) ++r->matches;
                else ++r->mismatches;
            }
            x += len; y += len;
        } else if (op == 1) {
            ++r->qni; r->qbi += len; x += len;
        } else {
            ++r->tni; r->tbi += len; y += len;
        }
    }
    if (r->nb == 0) { ar->n = a0; return 0; }
    r->b0sz = ar->b[a0].sz; r->b0q = ar->b[a0].q; r->b0t = ar->b[a0].t;
    r->qb = qb; r->qe = qe; r->tb = tb; r->te = te;
    r->score = r->matches - r->mismatches - r->qni - r->tni;
    return 1;
}

/* +1 / -1 per aligned base pair (an N on either side mismatches): the HSP extension's score */
static inline int hsp_sc(uint8_t a, uint8_t b) { return (a > 3 || b > 3 || a != b) ? -1 : 1; }

/* a range (the exact match [q0, q1) on diagonal t0 - q0) -> its HSP: extended without gaps to the
 * left of q0 and the right of q1, each end at the first best running score, the walk stopped XDOWN
 * positions after its last new best (blat's extendHitLeft / extendHitRight); one block */
static void hsp_range(const afo_tiles *X, const uint8_t *Q, int L, int32_t q0, int32_t q1, int64_t t0, reg_b *r,
                      blk_arena *ar) {
    int s = 0, best = 0, nb = 0;
    for (int i = 1; q0 - i >= 0 && t0 - i >= 0; ++i) {
        s += hsp_sc(Q[q0 - i], X->T[t0 - i]);
        if (s > best) { best = s; nb = i; }
        else if (i - nb > XDOWN) break;
    }
    const int32_t qb = q0 - nb;
    const int64_t tb = t0 - nb, t1 = t0 + (q1 - q0);
    s = best = nb = 0;
    for (int i = 1; q1 + i - 1 < L && t1 + i - 1 < X->n; ++i) {
        s += hsp_sc(Q[q1 + i - 1], X->T[t1 + i - 1]);
        if (s > best) { best = s; nb = i; }
        else if (i - nb > XDOWN) break;
    }
    memset(r, 0, sizeof(*r));
    r->qb = qb; r->qe = q1 + nb; r->tb = tb; r->te = t1 + nb;
    for (int32_t x = r->qb; x < r->qe; ++x) {
        const uint8_t a = Q[x], b = X->T[tb + (x - qb)];
        if (a > 3 || b > 3) ++r->ncount;
        else if (a == b) ++r->matches;
        else ++r->mismatches;
    }
    r->score = r->matches - r->mismatches;
    r->boff = ar->n;
    arena_push(ar, r->qe - r->qb, r->qb, r->tb);
    r->nb = 1;
    r->b0sz = r->qe - r->qb; r->b0q = r->qb; r->b0t = r->tb;
}

/* r without its first k aligned bases (k inside the first block): the chain's query / target
 * overlap with the previous part is given to that part; 0 if k does not fit */
static int trim_front(const afo_tiles *X, const uint8_t *Q, const reg_b *r, int k, reg_b *o) {
    *o = *r;
    if (k <= 0) return 1;
    if (k >= r->b0sz) return 0;
    for (int u = 0; u < k; ++u) {
        uint8_t a = Q[r->b0q + u], b = X->T[r->b0t + u];
        if (a > 3 || b > 3) --o->ncount;
        else if (a == b) --o->matches;
        else --o->mismatches;
    }
    o->b0sz -= k; o->b0q += k; o->b0t += k;
    o->qb = o->b0q; o->tb = o->b0t;
    o->score = o->matches - o->mismatches - o->qni - o->tni;
    return 1;
}

/* trim of region b chained after region a: max(query overlap, target overlap, 0) */
static int chain_trim(const reg_b *a, const reg_b *b) {
    int64_t k = a->qe - b->qb;
    if (a->te - b->tb > k) k = a->te - b->tb;
    return k > 0 ? (int)k : 0;
}

static int psl_millibad(const afo_psl *o) {
    int q_ali = o->q_end - o->q_start;
    int64_t t_ali = o->t_end - o->t_start;
    int64_t ali = q_ali < t_ali ? q_ali : t_ali;
    if (ali <= 0) return 0;
    int64_t size_dif = q_ali - t_ali;
    if (size_dif < 0) size_dif = 0;  /* mRNA: a shorter query span is an intron, not an error */
    int total = o->matches + o->mismatches;
    if (total == 0) return 0;
    return (int)((1000 * (o->mismatches + o->q_num_insert + round(3 * log(1. + (double)size_dif)))) / total);
}

static int tile_key(const uint8_t *Q, int q, uint32_t *k) {
    *k = 0;
    for (int u = 0; u < TILE; ++u) {
        if (Q[q + u] > 3) return 0;
        *k |= (uint32_t)Q[q + u] << (2 * u);
    }
    return 1;
}

static int cmp_psl(const void *a, const void *b);

/* test switch: 1 = the chain DP recomputes every unused part each round (afo_blat_set_literal) */
static int g_blat_literal = 0;
void afo_blat_set_literal(int on) { g_blat_literal = on; }
/* comparison switch: 1 = the round-5 parts (one gapped ksw extension per clump), 0 = HSPs */
static int g_blat_gapped = 0;
void afo_blat_set_gapped(int on) { g_blat_gapped = on; }

/* the chain DP of part i (position i of ord) over the unused parts before it: a predecessor a
 * must end before i on both sequences; i is trimmed by the overlap (chain_trim) and must keep part
 * of its first block; the target gap must be <= max_intron and hold no N; the score is best[a] +
 * the trimmed part's score - 1 per query / target gap; the first a with the highest score wins
 * over i alone.  pre: room for the first block's length + 1 */
static void chain_node(const afo_tiles *X, const afo_blat_params *bp, const uint8_t *Q, const reg_b *regs,
                       const int *ord, int *best, int *prev, const int *fl, int i, int *pre) {
    const reg_b *ri = &regs[ord[i]];
    best[i] = ri->score; prev[i] = -1;
    if (g_blat_literal) {  /* the plain statement: trim_front per candidate */
        for (int j = 0; j < i; ++j) {
            if (fl[j] & 1) continue;
            const reg_b *a = &regs[ord[j]];
            reg_b b;
            if (ri->qe <= a->qe || ri->te <= a->te) continue;
            if (!trim_front(X, Q, ri, chain_trim(a, ri), &b)) continue;
            if (b.tb - a->te > bp->max_intron || n_in(X, a->te, b.tb)) continue;
            int s = best[j] + b.score - (b.qb > a->qe) - (b.tb > a->te);
            if (s > best[i]) { best[i] = s; prev[i] = j; }
        }
        return;
    }
    /* pre[k] = the score of the first block's first k bases (what trim_front removes) */
    pre[0] = 0;
    for (int u = 0; u < ri->b0sz; ++u) {
        uint8_t x = Q[ri->b0q + u], y = X->T[ri->b0t + u];
        pre[u + 1] = pre[u] + ((x > 3 || y > 3) ? 0 : (x == y ? 1 : -1));
    }
    for (int j = 0; j < i; ++j) {
        if (fl[j] & 1) continue;
        const reg_b *a = &regs[ord[j]];
        if (ri->qe <= a->qe || ri->te <= a->te) continue;
        const int k = chain_trim(a, ri);
        if (k > 0 && k >= ri->b0sz) continue;
        const int32_t bqb = ri->qb + k;
        const int64_t btb = ri->tb + k;
        if (btb - a->te > bp->max_intron || n_in(X, a->te, btb)) continue;
        int s = best[j] + (ri->score - pre[k]) - (bqb > a->qe) - (btb > a->te);
        if (s > best[i]) { best[i] = s; prev[i] = j; }
    }
}

/* where a strand's rows go: short mode, the best cap_out in cmp_psl order (out; *n_out counts every
 * row); long mode, every row with all its blocks (rows / rblk, growable) */
typedef struct { afo_psl h; int64_t boff; int32_t seq; } long_row;  /* seq: the strand's emission order */
typedef struct {
    afo_psl *out;
    int *n_out, cap_out;
    long_row *rows;
    int64_t n_rows, cap_rows;
    int32_t emitted[2];
    blk_arena rblk;
} row_sink;

/* per-strand working memory, grown for the query and the mode */
typedef struct {
    hit_t *hits;
    reg_b *regs;
    clump_t *cl;
    int *ord, *pre;
    uint8_t *qs, *ts;
    uint32_t *cig;
    blk_arena ar;
} strand_mem;

static void strand_mem_init(strand_mem *m, const blat_mode *md, int L) {
    memset(m, 0, sizeof(*m));
    m->hits = (hit_t *)malloc(sizeof(hit_t) * md->maxh);
    m->regs = (reg_b *)malloc(sizeof(reg_b) * md->maxcl);
    m->cl = (clump_t *)malloc(sizeof(clump_t) * md->maxcl);
    m->ord = (int *)malloc(sizeof(int) * 5 * (size_t)md->maxcl);
    m->pre = (int *)malloc(sizeof(int) * (L + 2));
    m->qs = (uint8_t *)malloc(L + 1);
    m->ts = (uint8_t *)malloc(L + 64);
    m->cig = (uint32_t *)malloc(sizeof(uint32_t) * (md->cig_cap + 1));
}
static void strand_mem_free(strand_mem *m) {
    free(m->hits); free(m->regs); free(m->cl); free(m->ord); free(m->pre); free(m->qs); free(m->ts); free(m->cig);
    free(m->ar.b);
}

/* one strand of one query: its rows to the sink; cap[3]: the hit, clump and stitching caps bound */
static void blat_strand(const afo_tiles *X, const afo_blat_params *bp, const uint8_t *Q, int L, int strand,
                        int32_t qi, const blat_mode *md, row_sink *sink, strand_mem *M, int *cap) {
    hit_t *hits = M->hits;
    reg_b *regs = M->regs;
    M->ar.n = 0;
    int64_t nh = 0;
    int64_t all = 0;
    for (int q = 0; q + TILE <= L; ++q) {
        uint32_t k;
        if (!tile_key(Q, q, &k)) continue;
        const int64_t c = (int64_t)X->start[k + 1] - X->start[k];
        if (c <= bp->rep_match) all += c;
    }
    if (all > md->maxh) cap[0] = 1;
    for (int q = 0; q + TILE <= L && nh < md->maxh; ++q) {
        uint32_t k;
        if (!tile_key(Q, q, &k)) continue;
        uint32_t lo = X->start[k], hi = X->start[k + 1];
        if (hi == lo || (int64_t)(hi - lo) > bp->rep_match) continue;
        for (uint32_t i = lo; i < hi && nh < md->maxh; ++i) {
            hits[nh].t = X->pos[i]; hits[nh].q = q; hits[nh].diag = (int64_t)X->pos[i] - q;
            ++nh;
        }
    }
    if (nh == 0) return;
    qsort(hits, nh, sizeof(hit_t), cmp_hit);
    clump_t *cl = M->cl;
    int ncl = 0;
    for (int64_t i = 0; i < nh && ncl < md->maxcl;) {
        int64_t j = i, bq = i;
        while (j + 1 < nh && hits[j + 1].diag - hits[j].diag <= bp->max_gap + 2) {
            ++j;
            if (hits[j].q < hits[bq].q || (hits[j].q == hits[bq].q && hits[j].t < hits[bq].t)) bq = j;
        }
        if (j - i + 1 >= bp->min_match) {
            cl[ncl].cnt = (int32_t)(j - i + 1); cl[ncl].q = hits[bq].q; cl[ncl].t = hits[bq].t;
            cl[ncl].diag = hits[bq].diag; cl[ncl].h0 = i; cl[ncl].h1 = j + 1;
            ++ncl;
        }
        i = j + 1;
    }
    if (ncl == md->maxcl) cap[1] = 1;
    qsort(cl, ncl, sizeof(clump_t), cmp_clump);  /* (hits desc, diagonal): keys are unique */
    int nr = 0, c = 0;
    if (g_blat_gapped) {
        for (; c < ncl && nr < md->maxcl; ++c) {
            int32_t q = cl[c].q;
            int64_t t = cl[c].t;
            int skip = 0;
            for (int r = 0; r < nr; ++r)
                if (regs[r].qb <= q && q + TILE <= regs[r].qe && regs[r].tb <= t && t + TILE <= regs[r].te) { skip = 1; break; }
            if (skip) continue;
            if (align_clump(X, Q, L, q, t, &regs[nr], md, &M->ar, M->qs, M->ts, M->cig)) ++nr;
        }
        if (nr == md->maxcl && c < ncl) cap[2] = 1;
    } else {
        /* HSPs: per clump in order, its hits in (diagonal, offset) order; a range = hits of one
         * diagonal whose tiles touch (the next tile starts at or before the range's end); a range
         * inside (as a box) an HSP made before makes none; the first maxcl HSPs are kept (cap[2]) */
        for (; c < ncl; ++c) {
            for (int64_t h = cl[c].h0; h < cl[c].h1;) {
                const int64_t r0 = h;
                int32_t q1 = hits[h].q + TILE;
                while (h + 1 < cl[c].h1 && hits[h + 1].diag == hits[r0].diag && hits[h + 1].q <= q1) {
                    ++h;
                    q1 = hits[h].q + TILE;
                }
                ++h;
                const int32_t q0 = hits[r0].q;
                const int64_t t0 = hits[r0].t, t1 = t0 + (q1 - q0);
                int skip = 0;
                for (int r = 0; r < nr && !skip; ++r)
                    skip = regs[r].qb <= q0 && q1 <= regs[r].qe && regs[r].tb <= t0 && t1 <= regs[r].te;
                if (skip) continue;
                if (nr == md->maxcl) { cap[2] = 1; c = ncl; break; }
                hsp_range(X, Q, L, q0, q1, t0, &regs[nr++], &M->ar);
            }
        }
    }
    if (nr == 0) return;
    /* regions in (qb, tb, qe) order for the chain DP (stable: ties keep their creation order) */
    int *ord = M->ord;
    int *best = ord + nr, *prev = best + nr, *fl = prev + nr, *chain = fl + nr;
    for (int i = 0; i < nr; ++i) ord[i] = i;
    for (int i = 1; i < nr; ++i)
        for (int j = i; j > 0; --j) {
            const reg_b *a = &regs[ord[j - 1]], *b = &regs[ord[j]];
            int gt = a->qb > b->qb || (a->qb == b->qb && (a->tb > b->tb || (a->tb == b->tb && a->qe > b->qe)));
            if (!gt) break;
            int tmp = ord[j - 1]; ord[j - 1] = ord[j]; ord[j] = tmp;
        }
    for (int i = 0; i < nr; ++i) { regs[i].used = 0; fl[i] = 0; }
    /* BLAT-style stitching: each round emits the chain with the highest score over the unused
     * parts (the first in order on ties).  chain_node is the literal DP of one part; after a
     * chain is emitted only the parts whose predecessor path meets a used (or recomputed) part
     * are recomputed -- the others' values cannot change, as removing parts only lowers scores
     * (g_blat_literal = 1 recomputes every part each round, the plain statement of the rule). */
    int64_t work = 0;  /* the recomputations' candidates (the first pass is always made) */
    for (int i = 0; i < nr; ++i) chain_node(X, bp, Q, regs, ord, best, prev, fl, i, M->pre);
    for (;;) {
        if (work > STITCH_WORK && !g_blat_literal) { cap[2] = 1; break; }
        int bi = -1;
        for (int i = 0; i < nr; ++i)
            if (!fl[i] && (bi < 0 || best[i] > best[bi])) bi = i;
        if (bi < 0) break;
        int m = 0;
        for (int i = bi; i >= 0; i = prev[i]) chain[m++] = i;
        afo_psl o;
        memset(&o, 0, sizeof(o));
        o.query = qi; o.strand = strand; o.q_size = L;
        int ok = 1;
        const int64_t rb0 = sink->rblk.n;
        reg_b pp, first, last, cur;
        memset(&first, 0, sizeof first); memset(&last, 0, sizeof last); memset(&pp, 0, sizeof pp);
        for (int k = m - 1; k >= 0; --k) {
            fl[chain[k]] = 1;
            const reg_b *src = &regs[ord[chain[k]]];
            if (k == m - 1) cur = *src;
            else trim_front(X, Q, src, chain_trim(&pp, src), &cur);
            if (k < m - 1) {
                if (cur.qb > pp.qe) { ++o.q_num_insert; o.q_base_insert += cur.qb - pp.qe; }
                if (cur.tb > pp.te) { ++o.t_num_insert; o.t_base_insert += (int32_t)(cur.tb - pp.te); }
            }
            o.matches += cur.matches; o.mismatches += cur.mismatches; o.n_count += cur.ncount;
            o.q_num_insert += cur.qni; o.q_base_insert += cur.qbi; o.t_num_insert += cur.tni; o.t_base_insert += cur.tbi;
            for (int b = 0; b < cur.nb && ok; ++b) {
                const blk_t bk = blk_of(&M->ar, &cur, b);
                if (md->row_blocks && o.block_count >= md->row_blocks) { ok = 0; break; }
                if (o.block_count < AFO_PSL_MAX_BLOCKS) {
                    o.block_sizes[o.block_count] = bk.sz; o.q_starts[o.block_count] = bk.q;
                    o.t_starts[o.block_count] = bk.t;
                }
                if (!md->row_blocks) arena_push(&sink->rblk, bk.sz, bk.q, bk.t);
                ++o.block_count;
            }
            if (k == m - 1) first = cur;
            if (k == 0) last = cur;
            pp = cur;
        }
        o.q_start = strand ? L - last.qe : first.qb;
        o.q_end = strand ? L - first.qb : last.qe;
        o.t_start = first.tb; o.t_end = last.te;
        o.score = o.matches - o.mismatches - o.q_num_insert - o.t_num_insert;
        if (ok && o.score >= bp->min_score && psl_millibad(&o) <= (100 - bp->min_identity) * 10) {
            if (sink->out) {
                /* the strand's best cap_out rows in cmp_psl order, stable; every row counted */
                int n = *sink->n_out < sink->cap_out ? *sink->n_out : sink->cap_out, at = n;
                while (at > 0 && cmp_psl(&o, &sink->out[at - 1]) < 0) --at;
                if (at < sink->cap_out) {
                    for (int x = n < sink->cap_out ? n : sink->cap_out - 1; x > at; --x) sink->out[x] = sink->out[x - 1];
                    sink->out[at] = o;
                }
                ++*sink->n_out;
            } else {
                if (sink->n_rows == sink->cap_rows) {
                    sink->cap_rows = sink->cap_rows ? 2 * sink->cap_rows : 64;
                    sink->rows = (long_row *)realloc(sink->rows, sizeof(long_row) * sink->cap_rows);
                }
                sink->rows[sink->n_rows].h = o;
                sink->rows[sink->n_rows].boff = rb0;
                sink->rows[sink->n_rows].seq = sink->emitted[strand]++;
                ++sink->n_rows;
            }
        } else if (!sink->out) {
            sink->rblk.n = rb0;  /* the row's blocks, not kept */
        }
        if (g_blat_literal) {
            for (int i = 0; i < nr; ++i)
                if (!fl[i]) chain_node(X, bp, Q, regs, ord, best, prev, fl, i, M->pre);
        } else {
            for (int i = chain[m - 1] + 1; i < nr; ++i) {
                if (fl[i] & 1) continue;
                if (prev[i] >= 0 && fl[prev[i]]) {
                    chain_node(X, bp, Q, regs, ord, best, prev, fl, i, M->pre);
                    work += i;
                    fl[i] = 2;
                }
            }
            for (int i = 0; i < nr; ++i) fl[i] &= 1;
        }
    }
}

static int cmp_psl(const void *a, const void *b) {
    const afo_psl *x = (const afo_psl *)a, *y = (const afo_psl *)b;
    if (x->score != y->score) return y->score - x->score;
    if (x->strand != y->strand) return x->strand - y->strand;
    if (x->t_start != y->t_start) return x->t_start < y->t_start ? -1 : 1;
    if (x->q_start != y->q_start) return x->q_start - y->q_start;
    if (x->t_end != y->t_end) return x->t_end < y->t_end ? -1 : 1;
    return x->q_end - y->q_end;
}

int afo_blat(const afo_tiles *X, const uint8_t *queries, int64_t n_queries, int32_t stride, const int32_t *lens,
             const afo_blat_params *bp, int32_t max_rows, afo_psl *rows, int32_t *n_rows, int threads) {
    return afo_blat_caps(X, queries, n_queries, stride, lens, bp, max_rows, rows, n_rows, threads, NULL);
}

int afo_blat_caps(const afo_tiles *X, const uint8_t *queries, int64_t n_queries, int32_t stride, const int32_t *lens,
                  const afo_blat_params *bp, int32_t max_rows, afo_psl *rows, int32_t *n_rows, int threads,
                  int32_t *caps) {
    /* max_rows up to MAXP: every row of a query (the GPU's kept rows + its spill pool, tests) */
    if (!X || max_rows < 1 || max_rows > MAXP || bp->step_size != X->step) return -1;
#pragma omp parallel num_threads(threads > 0 ? threads : 1)
    {
        strand_mem M;
        strand_mem_init(&M, &MODE_SHORT, AFO_MAX_READ);
        afo_psl *cand[2];
        cand[0] = (afo_psl *)malloc(sizeof(afo_psl) * 2 * (size_t)max_rows);
        cand[1] = cand[0] + max_rows;
#pragma omp for schedule(dynamic, 64)
        for (int64_t qi = 0; qi < n_queries; ++qi) {
            int L = lens ? lens[qi] : stride;
            if (L > stride) L = stride;
            if (L > AFO_MAX_READ) L = AFO_MAX_READ;
            if (L < 0) L = 0;
            uint8_t Q[2][AFO_MAX_READ];
            for (int i = 0; i < L; ++i) {
                uint8_t c = afo_nt4(queries[qi * stride + i]);
                Q[0][i] = c;
                Q[1][L - 1 - i] = c > 3 ? 4 : 3 - c;
            }
            int nc[2] = {0, 0};
            int cap[2][3] = {{0, 0, 0}, {0, 0, 0}};
            for (int s = 0; s < 2; ++s) {
                row_sink sink;
                memset(&sink, 0, sizeof sink);
                sink.out = cand[s]; sink.n_out = &nc[s]; sink.cap_out = max_rows;
                blat_strand(X, bp, Q[s], L, s, (int32_t)qi, &MODE_SHORT, &sink, &M, cap[s]);
            }
            if (caps) {
                for (int s = 0; s < 2; ++s)
                    for (int k = 0; k < 3; ++k)
                        if (cap[s][k]) {
#pragma omp atomic
                            caps[k] += 1;
                        }
                if (nc[0] + nc[1] > max_rows) {
#pragma omp atomic
                    caps[3] += 1;
                }
            }
            /* the two strands' sorted lists merged (strand 0 first on equal keys: cmp_psl orders by
             * strand, so never) */
            int na = nc[0] < max_rows ? nc[0] : max_rows, nb = nc[1] < max_rows ? nc[1] : max_rows;
            int i = 0, j = 0, k = 0;
            for (; k < max_rows && (i < na || j < nb); ++k) {
                int take_b = j < nb && (i >= na || cmp_psl(&cand[1][j], &cand[0][i]) < 0);
                rows[qi * max_rows + k] = take_b ? cand[1][j++] : cand[0][i++];
            }
            n_rows[qi] = k;
        }
        free(cand[0]);
        strand_mem_free(&M);
    }
    return 0;
}

/* cmp_psl, then the strand's emission order (a total order: the sort's result is unique) */
static int cmp_long_row(const void *a, const void *b) {
    const long_row *x = (const long_row *)a, *y = (const long_row *)b;
    const int c = cmp_psl(&x->h, &y->h);
    return c ? c : x->seq - y->seq;
}

int afo_blat_long(const afo_tiles *X, const uint8_t *query, int32_t len, const afo_blat_params *bp, int32_t max_rows,
                  afo_psl *rows, int32_t *n_rows, afo_psl_block *blocks, int64_t block_cap, int64_t *block_off,
                  int64_t *n_blocks, int32_t *caps) {
    if (!X || len < 0 || len > AFO_BLAT_LONG_MAX || max_rows < 0 || bp->step_size != X->step) return -1;
    const int L = len;
    uint8_t *Q[2];
    Q[0] = (uint8_t *)malloc((size_t)L + 1);
    Q[1] = (uint8_t *)malloc((size_t)L + 1);
    for (int i = 0; i < L; ++i) {
        uint8_t c = afo_nt4(query[i]);
        Q[0][i] = c;
        Q[1][L - 1 - i] = c > 3 ? 4 : 3 - c;
    }
    strand_mem M;
    strand_mem_init(&M, &MODE_LONG, L);
    row_sink sink;
    memset(&sink, 0, sizeof sink);
    int cap[2][3] = {{0, 0, 0}, {0, 0, 0}};
    for (int s = 0; s < 2; ++s) blat_strand(X, bp, Q[s], L, s, 0, &MODE_LONG, &sink, &M, cap[s]);
    strand_mem_free(&M);
    free(Q[0]); free(Q[1]);
    if (caps)
        for (int s = 0; s < 2; ++s)
            for (int k = 0; k < 3; ++k) caps[k] += cap[s][k];
    /* every row of both strands, best first (strand 0's rows before strand 1's: cmp_psl's order) */
    qsort(sink.rows, sink.n_rows, sizeof(long_row), cmp_long_row);
    const int64_t m = sink.n_rows < max_rows ? sink.n_rows : max_rows;
    int64_t nb = 0;
    for (int64_t k = 0; k < m; ++k) nb += sink.rows[k].h.block_count;
    *n_rows = (int32_t)sink.n_rows;
    *n_blocks = nb;
    int rc = 0;
    if (nb > block_cap) {
        rc = -3;
    } else {
        int64_t off = 0;
        for (int64_t k = 0; k < m; ++k) {
            rows[k] = sink.rows[k].h;
            block_off[k] = off;
            for (int b = 0; b < sink.rows[k].h.block_count; ++b, ++off) {
                const blk_t bk = sink.rblk.b[sink.rows[k].boff + b];
                blocks[off].size = bk.sz; blocks[off].q_start = bk.q; blocks[off].t_start = bk.t;
            }
        }
        block_off[m] = off;
    }
    free(sink.rows);
    free(sink.rblk.b);
    return rc;
}
