// bwa_dev.h -- device restatements of bwa / klib routines shared by the S2 kernels (s2.hip,
// the anchor) and the genome calls S4 / S5 (bwa_genome.hip): klib's introsort (unstable, so its
// exact tie order is part of bwa's behaviour), utils.h hash_64, and one pass of ksw.c's striped
// local SW (ksw_u8 / ksw_i16) on the wave.  Header-only, anonymous namespace (see ksw_dp.h).
#pragma once
#include "ksw_dp.h"

#ifndef S2DBGL
#ifdef AF_S2_DEBUG
#define S2DBGL(...) printf(__VA_ARGS__)
#else
#define S2DBGL(...) do { } while (0)
#endif
#endif

namespace {

__device__ __forceinline__ int wave_min(int v) { return -wave_max(-v); }
__device__ __forceinline__ int lanes_below(uint64_t m, int lane) {
    return __builtin_popcountll(m & ((1ull << lane) - 1ull));
}

// ---- klib ksort.h introsort (lane 0; unstable -- tie orders are bwa's) --------------------
template <class T, class LT>
__device__ void ks_ins(T *a, int s, int t, LT lt) {
    for (int i = s + 1; i < t; ++i)
        for (int j = i; j > s && lt(a[j], a[j - 1]); --j) { T sw = a[j]; a[j] = a[j - 1]; a[j - 1] = sw; }
}
template <class T, class LT>
__device__ void ks_comb(T *a, int n, LT lt) {
    const double shrink_factor = 1.2473309501039786540366528676643;
    int do_swap;
    size_t gap = (size_t)n;
    do {
        if (gap > 2) {
            gap = (size_t)((double)gap / shrink_factor);
            if (gap == 9 || gap == 10) gap = 11;
        }
        do_swap = 0;
        for (int i = 0; i < n - (int)gap; ++i) {
            const int j = i + (int)gap;
            if (lt(a[j], a[i])) { T t = a[i]; a[i] = a[j]; a[j] = t; do_swap = 1; }
        }
    } while (do_swap || gap > 2);
    if (gap != 1) ks_ins(a, 0, n, lt);
}
template <class T, class LT>
__device__ void ks_introsort(T *a, int n, LT lt) {
    if (n < 1) return;
    if (n == 2) {
        if (lt(a[1], a[0])) { T sw = a[0]; a[0] = a[1]; a[1] = sw; }
        return;
    }
    int d;
    for (d = 2; (1ul << d) < (unsigned long)n; ++d) ;
    // klib pushes the larger part and continues with the smaller (segments of <= 16 are left to
    // the final insertion sort), so the stack holds at most
    // log2(n / 17) + 1 segments: 20 covers n <= 17 << 19 (call sites sort <= 16384 items)
    int stl[20], str[20], std_[20], top = 0;
    int s = 0, t = n - 1;
    d <<= 1;
    for (;;) {
        S2DBGL("introsort s %d t %d d %d top %d\n", s, t, d, top);
        if (s < t) {
            if (--d == 0) { ks_comb(a + s, t - s + 1, lt); t = s; continue; }
            int i = s, j = t, k = i + ((j - i) >> 1) + 1;
            if (lt(a[k], a[i])) {
                if (lt(a[k], a[j])) k = j;
            } else k = lt(a[j], a[i]) ? i : j;
            const T rp = a[k];
            if (k != t) { T sw = a[k]; a[k] = a[t]; a[t] = sw; }
            for (;;) {
                // a[t] == rp ends the first scan; the explicit bound keeps a broken comparator from
                // walking off the array
                do ++i; while (i < t && lt(a[i], rp));
                S2DBGL("introsort scan i %d lt(a[t], rp) %d\n", i, (int)lt(a[t], rp));
                do --j; while (i <= j && lt(rp, a[j]));
                if (j <= i) break;
                T sw = a[i]; a[i] = a[j]; a[j] = sw;
                S2DBGL("introsort swap i %d j %d\n", i, j);
            }
            S2DBGL("introsort part i %d j %d k %d\n", i, j, k);
            { T sw = a[i]; a[i] = a[t]; a[t] = sw; }
            if (i - s > t - i) {
                if (i - s > 16) { stl[top] = s; str[top] = i - 1; std_[top] = d; ++top; }
                s = t - i > 16 ? i + 1 : t;
            } else {
                if (t - i > 16) { stl[top] = i + 1; str[top] = t; std_[top] = d; ++top; }
                t = i - s > 16 ? i - 1 : s;
            }
        } else {
            if (top == 0) { ks_ins(a, 0, n, lt); return; }
            --top; s = stl[top]; t = str[top]; d = std_[top];
        }
    }
}

// klib's introsort with its exact output (ties included), partitions on the wave.  A Hoare
// partition's swaps are fixed by two lists of the ORIGINAL segment: the left stoppers L (indices in
// (s, t] holding no key below the pivot, t -- the pivot's slot -- last) and the right stoppers R
// (indices in [s, t) holding no key above it, descending).  Swap k exchanges L[k] and R[k] for
// every k before the first K with R[k] <= L[k] (R[k] = -1 past R's end); the i scan of round K then
// stops at L[K] or, when the swapped-in key at R[K - 1] comes first, there: the pivot lands at
// min(L[K], R[K - 1]).  Segments are independent (their order of processing does not matter),
// each child of more than 16 keys is partitioned with its parent's depth (at depth 0 klib's comb
// sort on lane 0).  klib's closing insertion sort is stable (strict comparisons), so its output is
// the stable sort of the partitioned array: a bitonic network over (key, position) pairs.
// scr: 5 n ints of scratch (L, R, the segment queue; then the positions).  Wave-uniform call.
template <class T, class LT>
__device__ void wave_introsort(T *a, int n, LT lt, int32_t *scr, int lane) {
    if (n < 3) {
        if (n == 2 && lane == 0 && lt(a[1], a[0])) { T sw = a[0]; a[0] = a[1]; a[1] = sw; }
        __threadfence_block();
        wave_sync();
        return;
    }
    int d = 2;
    while ((1 << d) < n) ++d;
    d <<= 1;
    int32_t *const Lp = scr, *const Rp = scr + n, *const Q = scr + 2 * n;
    int qh = 0, qt = 1;
    if (lane == 0) { Q[0] = 0; Q[1] = n - 1; Q[2] = d; }
    __threadfence_block();
    wave_sync();
    while (qh < qt) {
        const int s = Q[3 * qh], t = Q[3 * qh + 1];
        int dd = Q[3 * qh + 2];
        ++qh;
        if (s >= t) continue;
        if (--dd == 0) {
            if (lane == 0) ks_comb(a + s, t - s + 1, lt);
            __threadfence_block();
            wave_sync();
            continue;
        }
        if (lane == 0) {
            const int i = s, j = t;
            int k = i + ((j - i) >> 1) + 1;
            if (lt(a[k], a[i])) {
                if (lt(a[k], a[j])) k = j;
            } else k = lt(a[j], a[i]) ? i : j;
            if (k != t) { T sw = a[k]; a[k] = a[t]; a[t] = sw; }
        }
        __threadfence_block();
        wave_sync();
        const T rp = a[t];
        int nl = 0, nr = 0;
        for (int x0 = s + 1; x0 <= t; x0 += 64) {
            const int x = x0 + lane;
            const bool st = x <= t && !lt(a[x], rp);
            const uint64_t m = __ballot(st);
            if (st) Lp[nl + lanes_below(m, lane)] = x;
            nl += __builtin_popcountll(m);
        }
        for (int x0 = t - 1; x0 >= s; x0 -= 64) {
            const int x = x0 - lane;
            const bool st = x >= s && !lt(rp, a[x]);
            const uint64_t m = __ballot(st);
            if (st) Rp[nr + lanes_below(m, lane)] = x;
            nr += __builtin_popcountll(m);
        }
        __threadfence_block();
        wave_sync();
        int K = -1;
        for (int k0 = 0; K < 0 && k0 < nl; k0 += 64) {
            const int k = k0 + lane;
            bool c = false;
            if (k < nl) c = (k < nr ? Rp[k] : -1) <= Lp[k];
            const uint64_t m = __ballot(c);
            if (m) K = k0 + (int)__builtin_ctzll(m);
        }
        const int fi = K == 0 ? Lp[0] : min(Lp[K], Rp[K - 1]);
        for (int k0 = 0; k0 < K; k0 += 64) {
            const int k = k0 + lane;
            if (k < K) {
                const int li = Lp[k], ri = Rp[k];
                const T x = a[li];
                a[li] = a[ri];
                a[ri] = x;
            }
        }
        __threadfence_block();
        wave_sync();
        if (lane == 0) {
            T sw = a[fi]; a[fi] = a[t]; a[t] = sw;
            int q = qt;
            if (fi - s > 16) { Q[3 * q] = s; Q[3 * q + 1] = fi - 1; Q[3 * q + 2] = dd; ++q; }
            if (t - fi > 16) { Q[3 * q] = fi + 1; Q[3 * q + 1] = t; Q[3 * q + 2] = dd; ++q; }
        }
        if (fi - s > 16) ++qt;
        if (t - fi > 16) ++qt;
        __threadfence_block();
        wave_sync();
    }
    // the closing insertion sort: (key, position) ascending, the network whose comparators all put
    // the lesser pair low (missing pairs past n act as +inf)
    int32_t *const P = scr;
    for (int i = lane; i < n; i += 64) P[i] = i;
    __threadfence_block();
    wave_sync();
    int N = 1;
    while (N < n) N <<= 1;
    for (int k = 2; k <= N; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i0 = 0; i0 < N; i0 += 64) {
                const int i = i0 + lane;
                const int l = j == (k >> 1) ? (i ^ (k - 1)) : (i ^ j);
                if (l > i && l < n) {
                    const T x = a[i], y = a[l];
                    const int px = P[i], py = P[l];
                    if (lt(y, x) || (!lt(x, y) && py < px)) { a[i] = y; a[l] = x; P[i] = py; P[l] = px; }
                }
            }
            __threadfence_block();
            wave_sync();
        }
    }
}

// a[0, n) sorted on the wave by rank when the comparator orders every pair strictly (no two items
// equivalent): every correct sort, klib's introsort included, then gives this one order.  Each
// lane ranks its items against all n (LDS broadcast reads); tmp: n items of scratch.  Returns
// false, a unchanged, when some pair is equivalent (the caller runs the introsort for bwa's tie
// order).  Wave-uniform call.
// Long lists (the region lists of repeat-rich reads and pairs: hundreds of entries) take a bitonic
// network instead of the n^2 / 64 ranking: the variant whose comparators all put the lesser item at
// the lower index (each merge opens with i against its mirror i ^ (k - 1), then half-cleaners i ^
// j), so the missing items past n act as +inf and their comparators are skipped.  The original is
// kept in tmp; an equivalent adjacent pair after the sort means a tie: a is restored, false.
constexpr int WAVE_BITONIC_MIN = 96;
template <class T, class LT>
__device__ bool wave_bitonic_sort(T *a, int n, LT lt, T *tmp, int lane) {
    for (int i = lane; i < n; i += 64) tmp[i] = a[i];
    __threadfence_block();
    wave_sync();
    int N = 1;
    while (N < n) N <<= 1;
    for (int k = 2; k <= N; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i0 = 0; i0 < N; i0 += 64) {
                const int i = i0 + lane;
                const int l = j == (k >> 1) ? (i ^ (k - 1)) : (i ^ j);
                if (l > i && l < n) {
                    const T x = a[i], y = a[l];
                    if (lt(y, x)) { a[i] = y; a[l] = x; }
                }
            }
            __threadfence_block();
            wave_sync();
        }
    }
    bool tie = false;
    for (int i = lane; i + 1 < n; i += 64) tie = tie || !lt(a[i], a[i + 1]);
    if (!__ballot(tie)) return true;
    for (int i = lane; i < n; i += 64) a[i] = tmp[i];
    __threadfence_block();
    wave_sync();
    return false;
}

template <class T, class LT>
__device__ bool wave_rank_sort(T *a, int n, LT lt, T *tmp, int lane) {
    if (n >= WAVE_BITONIC_MIN) return wave_bitonic_sort(a, n, lt, tmp, lane);
    bool tie = false;
    for (int i0 = 0; i0 < n; i0 += 64) {
        const int i = i0 + lane;
        if (i < n) {
            const T x = a[i];
            int r = 0;
            for (int j = 0; j < n; ++j) {
                const T y = a[j];
                if (lt(y, x)) ++r;
                else if (j != i && !lt(x, y)) tie = true;
            }
            if (!tie) tmp[r] = x;
        }
    }
    if (__ballot(tie)) return false;
    __threadfence_block();
    wave_sync();
    for (int i = lane; i < n; i += 64) a[i] = tmp[i];
    __threadfence_block();
    wave_sync();
    return true;
}

// utils.h hash_64
__device__ __forceinline__ uint64_t hash_64(uint64_t key) {
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

struct SwRes { int score, te, qe; };

// One pass of ksw_u8 / ksw_i16 (oracle ksw_sw) on the wave.  The striped kernel's result is
// H(i,j) = max(G, F) with G = max(H(i-1,j-1) + S, E, 0) and F the full horizontal-gap term,
// while E(i+1,j) is fed by the first-pass value max(G, F within the query's stripe block
// [blk * slen, (blk + 1) * slen)) -- the lazy-F loop does not revisit E.  Lanes hold C query
// columns each; both F terms are prefix maxima (one plain, one keyed by block).  The target base
// of row i is tg[i] (rev: tg[te0 - i] for i <= te0, as the start pass's partly reversed target);
// tg is the LDS window when it holds the whole target.  Stops at the first row reaching endsc.
template <int C>
__device__ SwRes ksw_pass(const uint8_t *q, int qlen, const uint8_t *tg, int tlen, int rev_te, int P,
                             const af_params &p, int endsc, int lane) {
    const int slen = (qlen + P - 1) / P;
    const int oe_del = p.o_del + p.e_del, oe_ins = p.o_ins + p.e_ins;
    const int shift = p.b > 1 ? p.b : 1;  // ksw_qinit: minus the smallest score of the matrix (N: -1)
    const int j0 = lane * C;
    int H[C], E[C], qc[C], blk[C];
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const int j = j0 + c;
        H[c] = 0; E[c] = 0;
        qc[c] = j < qlen ? q[j] : 4;
        blk[c] = j < qlen ? j / slen : 0;
    }
    SwRes r{0, -1, -1};
    int gmax = 0;
    int t_next = tlen > 0 ? tg[rev_te >= 0 ? rev_te : 0] : 4;
    for (int i = 0; i < tlen; ++i) {
        const int ti = __builtin_amdgcn_readfirstlane(t_next);
        if (i + 1 < tlen) t_next = tg[rev_te >= 0 && i + 1 <= rev_te ? rev_te - i - 1 : i + 1];
        const int from_left = wave_shr1(0, H[C - 1]);
        int G[C], runX = kNeg, runK = -1, bxX[C], bxK[C];
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const int j = j0 + c;
            const bool in = j < qlen;
            const int hd = c == 0 ? from_left : H[c - 1];
            const int s = (ti > 3 || qc[c] > 3) ? -1 : (ti == qc[c] ? p.a : -p.b);
            G[c] = max(max(hd + s, 0), E[c]);
            bxX[c] = runX; bxK[c] = runK;
            if (in) {
                const int X = G[c] - oe_ins + j * p.e_ins;
                runX = max(runX, X);
                runK = max(runK, (blk[c] << 20) | (X + (1 << 19)));
            }
        }
        const int lexX = wave_shr1(kNeg, wave_incl_max(runX));
        const int lexK = wave_shr1(-1, wave_incl_max(runK));
        int rowmax = 0;
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const int j = j0 + c;
            const bool in = j < qlen;
            const int PX = max(lexX, bxX[c]);
            const int F = PX <= kNeg / 2 ? 0 : max(PX - (j - 1) * p.e_ins, 0);
            const int PK = max(lexK, bxK[c]);
            const int Fs = (PK >= 0 && (PK >> 20) == blk[c]) ? max((PK & 0xFFFFF) - (1 << 19) - (j - 1) * p.e_ins, 0) : 0;
            const int h = max(G[c], F);
            const int hfp = max(G[c], Fs);
            E[c] = max(max(E[c] - p.e_del, hfp - oe_del), 0);
            H[c] = in ? h : 0;
            if (in) rowmax = max(rowmax, h);
        }
        rowmax = wave_max(rowmax);
        if (rowmax > gmax) {
            gmax = rowmax;
            r.te = i;
            int qj = 1 << 30;
#pragma unroll
            for (int c = 0; c < C; ++c)
                if (j0 + c < qlen && H[c] == gmax) qj = min(qj, j0 + c);
            r.qe = wave_min(qj);
            if ((P == 16 && gmax + shift >= 255) || gmax >= endsc) break;
        }
    }
    r.score = (P == 16 && gmax + shift >= 255) ? 255 : gmax;
    if (r.score == 255) r.qe = -1;
    return r;
}

__device__ SwRes ksw_pass_any(const uint8_t *q, int qlen, const uint8_t *tg, int tlen, int rev_te, int P,
                                 const af_params &p, int endsc, int lane) {
    const int cpl = (qlen + 63) >> 6;  // <= 5 (AF_MAX_READ 320)
    if (cpl <= 1) return ksw_pass<1>(q, qlen, tg, tlen, rev_te, P, p, endsc, lane);
    if (cpl == 2) return ksw_pass<2>(q, qlen, tg, tlen, rev_te, P, p, endsc, lane);
    if (cpl == 3) return ksw_pass<3>(q, qlen, tg, tlen, rev_te, P, p, endsc, lane);
    if (cpl == 4) return ksw_pass<4>(q, qlen, tg, tlen, rev_te, P, p, endsc, lane);
    return ksw_pass<5>(q, qlen, tg, tlen, rev_te, P, p, endsc, lane);
}

}  // namespace
