// blat.hip -- the BLAT searches of the partner stages on the GPU (functions.py:341, 530, 966, 1007,
// 1071, 1122, 1244): the tile index and k_blat, one wave per query strand.  oracle/blat.c is the
// bit-exact contract; the restated algorithm and its choices are in afgpu.h (af_blat_params) and
// DESIGN.md §2.
//
// Tile index (af_tile_index_build*): codes of the target (1 B/base), every step_size-th 11-mer
// without N as (key, position) pairs radix-sorted by key (stable: positions ascending within a
// key), key starts by a count + scan over all 4^11 keys, per 64-base block an N bitmask, the N
// count before it and the first N at or after it (the stitcher never joins parts across an N).
//
// k_blat per query strand (strand 1 = the reverse-complemented query):
//   hits     the query's 11-mer keys (lanes over offsets); every hit, the first NMAX in (offset,
//            position) order, as a 64-bit key (diagonal + 1024) << 9 | offset; hits with no other
//            hit within the drift are dropped on the way (hashed diagonal-bucket bitmaps in LDS)
//   sort     stable LSD radix sort of the keys by diagonal (offsets ascending within a diagonal)
//   clumps   runs of diagonals (a step > max_gap + 2 starts one) with >= min_match hits, the first
//            MAXCL in diagonal order, ordered (hits desc, diagonal); each knows its hits S[h0, h1)
//   HSPs     Kent 2002: a clump's hits of one diagonal whose tiles touch form a range (an exact
//            match); per range in order, unless it lies inside an HSP made before, a gapless
//            extension both ways (+1 / -1, an end stops XDOWN positions after its last new best),
//            the walks as wave scans over 64 positions at a time
//   stitch   chain DP over the HSPs in (qb, tb, qe) order with overlap trimming (the only place a
//            gap enters an alignment); every chain passing minScore / minIdentity is a PSL row
//   output   rows of both strands ordered (score desc, strand, tStart, qStart, tEnd, qEnd)
//
// LDS: one BlatLds per wave, declared in each kernel and handed down by reference to helpers that
// are all force-inlined, so every LDS access is a ds_* instruction on the kernel's own layout and
// no helper reaches LDS through the LDS lowering's per-kernel offset table (the
// round-5 fault).
#include <cstdlib>

#include <hipcub/hipcub.hpp>

#include "ksw_dp.h"

#ifndef AF_BLAT_ROUNDS
#define AF_BLAT_ROUNDS 6  // drift-filter rounds at most (round 0 is marked while the hits are collected)
#endif
#ifndef AF_BLAT_FILTER_MIN
#define AF_BLAT_FILTER_MIN 256  // hits below which another drift-filter round is not worth its passes
#endif
#ifndef AF_BLAT_WPS
#define AF_BLAT_WPS 6  // k_blat waves per SIMD (launch bound: VGPR budget)
#endif

namespace {

constexpr int TILE = AF_TILE;
constexpr uint32_t NKEYS = 1u << (2 * TILE);
// HSPs per query strand: the first MAXP in range order (AF_BLAT_CAP_PARTS when more ranges remain)
constexpr int NMAX = 32768, MAXCL = 4096, MAXP = 4096;
// stitching work per query strand (predecessor candidates the chain DP rescans after a chain is
// emitted; the first pass over every part is always made): once past it, no further chain is
// emitted and the strand is counted in AF_BLAT_CAP_PARTS (oracle/blat.c: the same)
constexpr int64_t STITCH_WORK = 1 << 24;
constexpr int XDOWN = 10;  // oracle/blat.c XDOWN: an HSP end stops 10 positions after its last new best

struct Clump { int32_t cnt, h0, h1, pad; };  // hit count, its hits S[h0, h1) in diagonal order
// one HSP (= one block): query [qb, qe) against target [tb, te), te - tb = qe - qb
struct Reg {
    int32_t qb, qe, score, matches, mismatches, ncount;
    int64_t tb, te;
};
static_assert(sizeof(Reg) == 40, "Reg layout");
// per-slot scratch layout (bytes): hit keys (two buffers; the one not holding the sorted hits
// later holds the range starts at +64 KB and the clump order in its first 64 KB), clumps, HSPs,
// the chain DP's per-part words (sorted order, best, predecessor, flags, chain, qe, te, first N),
// the strand's rows
constexpr size_t SC_KEYS_A = 0, SC_KEYS_B = SC_KEYS_A + NMAX * 8, SC_CLUMP = SC_KEYS_B + NMAX * 8,
                 SC_REGS = SC_CLUMP + MAXCL * sizeof(Clump), SC_DP = SC_REGS + (size_t)MAXP * sizeof(Reg),
                 SC_ROWS = SC_DP + 8 * 4 * (size_t)MAXP, SC_END = SC_ROWS + (8 << 10);
constexpr size_t SC_RANGES = 64 << 10;  // offset of the range starts inside the spare key buffer
static_assert(SC_END == AF_BLAT_SLOT_BYTES, "BLAT slot layout");
static_assert(AF_BLAT_MAX_ROWS * sizeof(af_psl) <= (8 << 10), "BLAT rows scratch");
static_assert(SC_RANGES + 4 * (size_t)NMAX <= (size_t)NMAX * 8, "range starts fit the spare key buffer");
static_assert(2 * 8 * (size_t)MAXCL <= SC_RANGES, "clump order fits below the range starts");

// one wave's LDS (declared in each kernel, passed down by reference)
struct __attribute__((aligned(16))) BlatLds {
    uint32_t hist[AF_MAX_READ];     // radix digit counts (256) / per offset: first position index - first hit index / PRE
    int32_t base[AF_MAX_READ + 1];  // first hit index per query offset (exclusive scan of the counts)
    uint32_t once[512];             // drift filter: 16K-bit "seen" map
    uint32_t twice[256];            // drift filter: 8K-bit "seen twice" map
    uint8_t q[AF_MAX_READ + 16];    // the strand's codes
    int32_t nrow, tmp[7];
};

#ifdef AF_K2_PROF
// profiling build only: per query [0..4] cycles in hits / sort / clumps / HSPs / chain, [5] hits,
// [6] clumps, [7] HSPs, [8] length, [9] total cycles, [10] drift-filter cycles, [11] hits kept,
// [12] deferred, [13] ranges
__device__ int32_t *g_blprof = nullptr;
#define BP(...) __VA_ARGS__
#define BPM(k) BP({ const int64_t _n = clock64(); pc[k] += _n - tq; tq = _n; })
#else
#define BP(...)
#define BPM(k)
#endif

__device__ __forceinline__ uint8_t nt4(uint8_t c) {
    switch (c) {
    case 'A': case 'a': return 0;
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'T': case 't': return 3;
    default: return 4;
    }
}

__device__ __forceinline__ int lanes_below_blat(uint64_t m, int lane) {
    return lane ? __builtin_popcountll(m << (64 - lane)) : 0;
}

__device__ __forceinline__ bool tile_key(const uint8_t *Q, int q, uint32_t &k) {
    k = 0;
    bool ok = true;
    for (int u = 0; u < TILE; ++u) {
        const uint8_t b = Q[q + u];
        ok = ok && b < 4;
        k |= (uint32_t)(b & 3) << (2 * u);
    }
    return ok;
}

__device__ __forceinline__ int wave_incl_sum(int v, int lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int u = __shfl_up(v, d);
        if (lane >= d) v += u;
    }
    return v;
}

__device__ __forceinline__ uint32_t bucket_hash(uint64_t b, int round, int bits) {
    const uint32_t x = (uint32_t)b ^ (uint32_t)(b >> 32) ^ (0x632BE59Bu * (uint32_t)(round + 1));
    return (x * 0x9E3779B1u) >> (32 - bits);
}

// The drift filter: a key (diagonal = key >> 9) is kept when another key may lie within drift of
// its diagonal.  Buckets of 1 << wsh diagonals hashed into a 16K-bit "seen" map and an 8K-bit
// "seen twice" map; a hash collision only keeps a key.
__device__ __forceinline__ void drift_clear(BlatLds &B, int lane) {
    for (int x = lane; x < 512; x += 64) B.once[x] = 0;
    for (int x = lane; x < 256; x += 64) B.twice[x] = 0;
}
__device__ __forceinline__ void drift_mark(BlatLds &B, uint64_t key, int wsh, int round) {
    const uint32_t h = bucket_hash(key >> (9 + wsh), round, 14), bit = 1u << (h & 31);
    if (atomicOr(&B.once[h >> 5], bit) & bit) {
        const uint32_t g = h & 8191;
        atomicOr(&B.twice[g >> 5], 1u << (g & 31));
    }
}
// whether key k (marked for this round) may have another key within drift of its diagonal
__device__ __forceinline__ bool drift_kept(const BlatLds &B, uint64_t k, int64_t drift, int wsh, int round) {
    const int64_t d = (int64_t)(k >> 9);
    const uint64_t b = (uint64_t)d >> wsh, b0 = (uint64_t)(d - drift) >> wsh, b1 = (uint64_t)(d + drift) >> wsh;
    const uint32_t h = bucket_hash(b, round, 14), g = h & 8191;
    bool keep = (B.twice[g >> 5] >> (g & 31)) & 1u;
    const uint64_t bn = b0 != b ? b0 : b1;  // the bucket width is >= 2 drift: one neighbour at most
    if (bn != b) { const uint32_t hn = bucket_hash(bn, round, 14); keep = keep || ((B.once[hn >> 5] >> (hn & 31)) & 1u); }
    return keep;
}
// src[0, n) -> dst: the keys this round keeps, in order; returns their count
__device__ __forceinline__ int drift_filter(BlatLds &B, const uint64_t *src, uint64_t *dst, int n, int64_t drift, int wsh,
                                            int round, int lane) {
    drift_clear(B, lane);
    wave_sync();
    for (int i = lane; i < n; i += 64) drift_mark(B, src[i], wsh, round);
    wave_sync();
    int nk = 0;
    for (int i0 = 0; i0 < n; i0 += 64) {
        const int i = i0 + lane;
        bool keep = false;
        uint64_t k = 0;
        if (i < n) {
            k = src[i];
            keep = drift_kept(B, k, drift, wsh, round);
        }
        const uint64_t m = __ballot(keep);
        if (keep) dst[nk + lanes_below_blat(m, lane)] = k;
        nk += (int)__builtin_popcountll(m);
    }
    __threadfence_block();
    wave_sync();
    return nk;
}

// stable LSD radix sort of a[0, n) by bits [lo, lo + 8 * passes) on the wave, ping-ponging with
// b; returns the buffer holding the result
__device__ __forceinline__ uint64_t *wave_radix_sort(BlatLds &B, uint64_t *a, uint64_t *b, int n, int lo, int passes,
                                                     int lane) {
    uint32_t *H = B.hist;
    for (int p = 0; p < passes; ++p) {
        const int sh = lo + 8 * p;
        for (int x = lane; x < 256; x += 64) H[x] = 0;
        wave_sync();
        for (int i = lane; i < n; i += 64) atomicAdd(&H[(uint32_t)(a[i] >> sh) & 255u], 1u);
        wave_sync();
        const uint32_t v0 = H[4 * lane], v1 = H[4 * lane + 1], v2 = H[4 * lane + 2], v3 = H[4 * lane + 3];
        const int tot = (int)(v0 + v1 + v2 + v3);
        const uint32_t ex = (uint32_t)(wave_incl_sum(tot, lane) - tot);
        H[4 * lane] = ex; H[4 * lane + 1] = ex + v0; H[4 * lane + 2] = ex + v0 + v1; H[4 * lane + 3] = ex + v0 + v1 + v2;
        wave_sync();
        for (int i0 = 0; i0 < n; i0 += 64) {
            const int i = i0 + lane;
            const bool valid = i < n;
            const uint64_t k = valid ? a[i] : 0;
            const uint32_t d = (uint32_t)(k >> sh) & 255u;
            uint64_t m = __ballot(valid);
#pragma unroll
            for (int bit = 0; bit < 8; ++bit) {
                const bool on = (d >> bit) & 1u;
                const uint64_t bl = __ballot(valid && on);
                m &= on ? bl : ~bl;
            }
            const uint32_t base = H[d];
            if (valid) b[base + lanes_below_blat(m, lane)] = k;
            wave_sync();
            if (valid && (m >> lane) == 1ull) H[d] = base + (uint32_t)__builtin_popcountll(m);
            wave_sync();
        }
        __threadfence_block();
        wave_sync();
        uint64_t *t = a; a = b; b = t;
    }
    return a;
}

// Bases one end of an HSP takes: the walk from query offset qa / target position ta outwards
// (dir +1: qa, qa + 1, ...; dir -1: qa, qa - 1, ...) over at most n pairs, +1 per match, -1 per
// mismatch or N; the walk stops at the first step more than XDOWN after its last new best (a
// strictly higher running score) and takes the bases up to that best (oracle hsp_range).  Lanes
// over 64 steps at a time: prefix sums, the running best before each step as an exclusive prefix
// max, the last new-best step as a prefix max of step indices.
__device__ __forceinline__ int hsp_walk(const uint8_t *Q, const uint8_t *T, int qa, int64_t ta, int dir, int n,
                                        int lane) {
    int carry = 0, best = 0, nb = 0;
    for (int i0 = 0; i0 < n; i0 += 64) {
        const int i = i0 + lane + 1;  // this lane's step (1-based)
        const bool v = i <= n;
        int sc = 0;
        if (v) {
            const uint8_t a = Q[qa + dir * (i - 1)], b = T[ta + dir * (int64_t)(i - 1)];
            sc = (a > 3 || b > 3 || a != b) ? -1 : 1;
        }
        const int s = carry + wave_incl_sum(sc, lane);
        const int sv = v ? s : kMaxId;
        const int mincl = wave_incl_max(sv);
        const int mprev = max(best, wave_shr1(kMaxId, mincl));  // the best before this step
        const bool f = v && s > mprev;
        const int nbi = max(nb, wave_incl_max(f ? i : 0));      // the last new best up to this step
        const uint64_t stop = __ballot(v && !f && i - nbi > XDOWN);
        if (stop) return __builtin_amdgcn_readlane(nbi, (int)__builtin_ctzll(stop));
        const uint64_t vm = __ballot(v);
        const int last = 63 - (int)__builtin_clzll(vm);
        carry = __builtin_amdgcn_readlane(s, last);
        best = max(best, __builtin_amdgcn_readlane(mincl, last));
        nb = __builtin_amdgcn_readlane(nbi, last);
    }
    return nb;
}

// the range [q0, q1) on diagonal t0 - q0 (an exact match) -> its HSP (oracle hsp_range); every
// lane returns it
__device__ __forceinline__ Reg hsp_range(const DevTile &X, const uint8_t *Q, int L, int q0, int q1, int64_t t0, int lane) {
    const int64_t t1 = t0 + (q1 - q0);
    const int nl = (int)min((int64_t)q0, t0);
    const int left = nl > 0 ? hsp_walk(Q, X.T, q0 - 1, t0 - 1, -1, nl, lane) : 0;
    const int nr = (int)min((int64_t)(L - q1), X.n - t1);
    const int right = nr > 0 ? hsp_walk(Q, X.T, q1, t1, 1, nr, lane) : 0;
    Reg r;
    r.qb = q0 - left; r.qe = q1 + right;
    r.tb = t0 - left; r.te = t1 + right;
    int mt = 0, mm = 0, nn = 0;
    for (int x = r.qb + lane; x < r.qe; x += 64) {
        const uint8_t a = Q[x], b = X.T[r.tb + (x - r.qb)];
        if (a > 3 || b > 3) ++nn;
        else if (a == b) ++mt;
        else ++mm;
    }
    r.matches = wave_sum(mt); r.mismatches = wave_sum(mm); r.ncount = wave_sum(nn);
    r.score = r.matches - r.mismatches;
    return r;
}

__device__ __forceinline__ int psl_millibad(const af_psl &o) {
    const int q_ali = o.q_end - o.q_start;
    const int64_t t_ali = o.t_end - o.t_start;
    const int64_t ali = q_ali < t_ali ? q_ali : t_ali;
    if (ali <= 0) return 0;
    int64_t size_dif = q_ali - t_ali;
    if (size_dif < 0) size_dif = 0;
    const int total = o.matches + o.mismatches;
    if (total == 0) return 0;
    return (int)((1000 * (o.mismatches + o.q_num_insert + round(3 * log(1. + (double)size_dif)))) / total);
}

__device__ __forceinline__ bool psl_before(const af_psl &x, const af_psl &y) {
    if (x.score != y.score) return x.score > y.score;
    if (x.strand != y.strand) return x.strand < y.strand;
    if (x.t_start != y.t_start) return x.t_start < y.t_start;
    if (x.q_start != y.q_start) return x.q_start < y.q_start;
    if (x.t_end != y.t_end) return x.t_end < y.t_end;
    return x.q_end < y.q_end;
}

// The chain DP's per-part words (parts in (qb, tb, qe) order, position k): ORD[k] = the part's
// index in RG, BEST / PREV its chain score and predecessor, FL bit 0 = used by an emitted chain,
// bit 1 = recomputed in this pass, CH the chain being emitted
struct ChainDp {
    int32_t *ORD, *BEST, *PREV, *FL, *CH;
    int32_t *QE;    // the part's qe, -1 once used (one load tells both)
    uint32_t *TE;   // its te
    uint32_t *NXT;  // the first N of the target at or after te (no N: 0xFFFFFFFF)
};

// the first N of the target at or after p (the oracle's n_in(p, b) == 0 <=> first_n(p) >= b)
__device__ __forceinline__ uint32_t first_n(const DevTile &X, int64_t p) {
    const int64_t b = p >> 6;
    const uint64_t m = X.nmask[b] >> (p & 63);
    return m ? (uint32_t)(p + __builtin_ctzll(m)) : X.nnext[b + 1];
}

// best[i] / prev[i] over the unused parts j < i (oracle/blat.c chain_node, the literal rule): a
// predecessor must end before i on both sequences, leave part of i after the overlap trim, lie
// within max_intron on the target with no N in between; the first j with the highest best[j] +
// trimmed score - gap flags wins over i alone.  Lanes over j on the parts' sorted per-part words
// (coalesced; four 64-part chunks per pass); the trimmed score from a prefix sum of i's bases
// (PRE, LDS), the N test against the part's first N after te.
__device__ __forceinline__ void chain_node(BlatLds &B, const DevTile &X, const Reg *RG, const ChainDp &C, int i,
                                           int64_t max_intron, int lane) {
    const Reg &ri = RG[C.ORD[i]];
    const uint8_t *Q = B.q;
    int32_t *PRE = reinterpret_cast<int32_t *>(B.hist);  // PRE[k] = score of the part's first k bases
    const int iqb = ri.qb, iqe = ri.qe, isc = ri.score, ilen = ri.qe - ri.qb;
    const int64_t itb = ri.tb, ite = ri.te;
    const int b0 = ilen < AF_MAX_READ ? ilen : AF_MAX_READ;
    int carry = 0;
    for (int u0 = 0; u0 < b0; u0 += 64) {
        const int u = u0 + lane;
        int m = 0;
        if (u < b0) {
            const uint8_t x = Q[iqb + u], y = X.T[itb + u];
            m = (x > 3 || y > 3) ? 0 : (x == y ? 1 : -1);
        }
        const int inc = wave_incl_sum(m, lane);
        if (u < b0) PRE[u] = carry + inc - m;
        carry += __builtin_amdgcn_readlane(inc, 63);
    }
    wave_sync();
    int best = isc, prev = -1;
    for (int j0 = 0; j0 < i; j0 += 256) {
        int sc[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int j = j0 + 64 * c + lane;
            int v = INT_MIN;
            if (j < i) {
                const int aqe = C.QE[j];
                const int64_t ate = C.TE[j];
                const int64_t nx = C.NXT[j];
                const int bj = C.BEST[j];
                if (aqe >= 0 && iqe > aqe && ite > ate) {
                    int64_t kk = aqe - iqb;
                    if (ate - itb > kk) kk = ate - itb;
                    const int k = kk > 0 ? (int)kk : 0;
                    const int64_t btb = itb + k;
                    if (!(k > 0 && k >= ilen) && btb - ate <= max_intron && nx >= btb)
                        v = bj + (isc - (k > 0 ? PRE[k] : 0)) - (iqb + k > aqe) - (btb > ate);
                }
            }
            sc[c] = v;
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int mx = wave_max(sc[c]);
            if (mx > best) { best = mx; prev = j0 + 64 * c + (int)__builtin_ctzll(__ballot(sc[c] == mx)); }
        }
    }
    if (lane == 0) { C.BEST[i] = best; C.PREV[i] = prev; }
    wave_sync();
}

// the box [q0, q1) x [t0, t1) inside one of the parts RG[0, nr) (lanes over the parts)
__device__ __forceinline__ bool inside_part(const Reg *RG, int nr, int q0, int q1, int64_t t0, int64_t t1, int lane) {
    bool inside = false;
    for (int r0 = 0; r0 < nr && !inside; r0 += 64) {
        const int r = r0 + lane;
        bool in = false;
        if (r < nr) {
            const Reg &g = RG[r];
            in = g.qb <= q0 && q1 <= g.qe && g.tb <= t0 && t1 <= g.te;
        }
        inside = __ballot(in) != 0;
    }
    return inside;
}

// the chains of one strand's parts RG[0, nr) (B.q its codes), best first, into its row list (RW,
// B.nrow; rows past max_rows to the spill pool).  parts_capped: AF_BLAT_CAP_PARTS already counted
// for the strand (a strand counts each cap once, as the oracle's per-strand flags)
__device__ __forceinline__ void strand_chains(BlatLds &B, const DevTile &X, const af_blat_params &bp, Reg *RG,
                                              const ChainDp &CD, int nr, int64_t qi, int strand, int L, uint64_t *KA,
                                              uint64_t *KB, af_psl *RW, int32_t max_rows, const BlatCaps &caps,
                                              const BlatSpill &spill, bool parts_capped, int lane) {
    // ---- parts in (qb, tb, qe) order, ties in creation order: ORD ----------------------------
    // key: qb in bits 54-63, tb in 21-53, qe in 12-20, the part index in 0-11
    static_assert(AF_MAX_READ < 512, "qb / qe take 9 bits of the ORD key");
    static_assert(MAXP <= 4096, "the part index takes 12 bits of the ORD key");
    {
        const auto key = [&](int r) {
            const Reg &g = RG[r];
            return ((uint64_t)g.qb << 54) | ((uint64_t)g.tb << 21) | ((uint64_t)g.qe << 12) | (uint64_t)r;
        };
        if (nr <= 64) {
            if (lane < nr) {
                const uint64_t k = key(lane);
                int rank = 0;
                for (int r = 0; r < nr; ++r) rank += key(r) < k;
                CD.ORD[rank] = lane;
            }
        } else {
            for (int r = lane; r < nr; r += 64) KA[r] = key(r);
            __threadfence_block();
            wave_sync();
            const uint64_t *SK = wave_radix_sort(B, KA, KB, nr, 12, 7, lane);
            for (int r = lane; r < nr; r += 64) CD.ORD[r] = (int32_t)(SK[r] & 4095u);
        }
        __threadfence_block();
        wave_sync();
        for (int r = lane; r < nr; r += 64) {
            const Reg &g = RG[CD.ORD[r]];
            CD.FL[r] = 0;
            CD.QE[r] = g.qe;
            CD.TE[r] = (uint32_t)g.te;
            CD.NXT[r] = first_n(X, g.te);
        }
        __threadfence_block();
        wave_sync();
    }
    // ---- chains, best first (oracle/blat.c: each round takes the unused part with the
    // highest chain score, first in order on ties; only the parts whose predecessor path
    // met a used part are recomputed, the others keep their exact value) ----------------
    int64_t work = 0;  // the recomputations' candidates (the first pass is always made)
    for (int i = 0; i < nr; ++i) {
        chain_node(B, X, RG, CD, i, bp.max_intron, lane);
        __threadfence_block();
        wave_sync();
    }
    const uint8_t *Q = B.q;
    for (;;) {
        if (work > STITCH_WORK) {
            if (lane == 0 && !parts_capped) caps.hit(qi, AF_BLAT_CAP_PARTS);
            break;
        }
        // the unused part with the highest chain score, the first on ties
        int bv = INT_MIN, bi = -1;
        for (int i0 = 0; i0 < nr; i0 += 64) {
            const int i = i0 + lane;
            const bool free_ = i < nr && !(CD.FL[i] & 1);
            if (!__ballot(free_)) continue;
            const int v = free_ ? CD.BEST[i] : INT_MIN;
            const int mx = wave_max(v);
            if (bi < 0 || mx > bv) { bv = mx; bi = i0 + (int)__builtin_ctzll(__ballot(free_ && v == mx)); }
        }
        if (bi < 0) break;
        // the chain (lane 0 follows the predecessors), its parts marked used
        int m = 0;
        if (lane == 0) {
            for (int i = bi; i >= 0; i = CD.PREV[i]) CD.CH[m++] = i;
        }
        m = __builtin_amdgcn_readfirstlane(m);
        __threadfence_block();
        wave_sync();
        const int first = CD.CH[m - 1];
        for (int c = lane; c < m; c += 64) { CD.FL[CD.CH[c]] |= 1; CD.QE[CD.CH[c]] = -1; }
        if (m <= AF_PSL_MAX_BLOCKS) {  // a chain of more HSPs than a row holds blocks: no row
            // lane b: block b, the chain's b-th part (CH[m - 1 - b]), its front trimmed by the
            // overlap with part b - 1 (trim_front; the oracle's literal accounting)
            const int b = lane;
            int32_t qb = 0, qe = 0, blen = 0;
            int64_t tb = 0, te = 0;
            int mt = 0, mm = 0, nn = 0, qni = 0, qbi = 0, tni = 0, tbi = 0;
            if (b < m) {
                const Reg &src = RG[CD.ORD[CD.CH[m - 1 - b]]];
                qb = src.qb; qe = src.qe; tb = src.tb; te = src.te;
                mt = src.matches; mm = src.mismatches; nn = src.ncount;
                if (b > 0) {
                    const Reg &prv = RG[CD.ORD[CD.CH[m - b]]];
                    int64_t kk = prv.qe - qb;
                    if (prv.te - tb > kk) kk = prv.te - tb;
                    const int trim = kk > 0 && kk < src.qe - src.qb ? (int)kk : 0;
                    for (int u = 0; u < trim; ++u) {
                        const uint8_t x = Q[qb + u], y = X.T[tb + u];
                        if (x > 3 || y > 3) --nn;
                        else if (x == y) --mt;
                        else --mm;
                    }
                    qb += trim; tb += trim;
                    if (qb > prv.qe) { qni = 1; qbi = qb - prv.qe; }
                    if (tb > prv.te) { tni = 1; tbi = (int)(tb - prv.te); }
                }
                blen = qe - qb;
            }
            const int s_mt = wave_sum(mt), s_mm = wave_sum(mm), s_nn = wave_sum(nn);
            const int s_qni = wave_sum(qni), s_qbi = wave_sum(qbi), s_tni = wave_sum(tni), s_tbi = wave_sum(tbi);
            const int fqb = __builtin_amdgcn_readlane(qb, 0);
            const int64_t ftb = ((int64_t)__builtin_amdgcn_readlane((int)(tb >> 32), 0) << 32) |
                                (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)tb, 0);
            const int lqe = __builtin_amdgcn_readlane(qe, m - 1);
            const int64_t lte = ((int64_t)__builtin_amdgcn_readlane((int)(te >> 32), m - 1) << 32) |
                                (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)te, m - 1);
            af_psl h;  // the header fields (lane-uniform); the block arrays are written lane by lane
            h.query = (int32_t)qi; h.strand = strand; h.q_size = L;
            h.matches = s_mt; h.mismatches = s_mm; h.n_count = s_nn;
            h.q_num_insert = s_qni; h.q_base_insert = s_qbi; h.t_num_insert = s_tni; h.t_base_insert = s_tbi;
            h.q_start = strand ? L - lqe : fqb;
            h.q_end = strand ? L - fqb : lqe;
            h.t_start = ftb; h.t_end = lte;
            h.block_count = m;
            h.score = h.matches - h.mismatches - h.q_num_insert - h.t_num_insert;
            if (h.score >= bp.min_score && psl_millibad(h) <= (100 - bp.min_identity) * 10) {
                // the strand's best max_rows rows in psl_before order (stable), all counted; the
                // row that falls off the list goes to the spill pool
                const int n = B.nrow < max_rows ? B.nrow : max_rows;
                const bool after = lane < n && !psl_before(h, RW[lane]);  // RW sorted: a prefix
                const int at = (int)__builtin_popcountll(__ballot(after));
                af_psl *dst = nullptr;  // where the new row goes
                if (at < max_rows) {
                    if (n == max_rows && spill.cap > 0) {  // the last kept row falls off
                        int k = 0;
                        if (lane == 0) k = atomicAdd(spill.n, 1);
                        k = __builtin_amdgcn_readfirstlane(k);
                        if (k < spill.cap) {
                            const int32_t *src = reinterpret_cast<const int32_t *>(RW + max_rows - 1);
                            int32_t *d = reinterpret_cast<int32_t *>(spill.rows + k);
                            for (int w = lane; w < (int)(sizeof(af_psl) / 4); w += 64) d[w] = src[w];
                            if (lane == 0) spill.query[k] = (int32_t)qi;
                        } else if (lane == 0) {
                            caps.hit(qi, AF_BLAT_CAP_ROWS);
                        }
                    }
                    for (int x = (n < max_rows ? n : max_rows - 1); x > at; --x) {
                        const int32_t *src = reinterpret_cast<const int32_t *>(RW + x - 1);
                        int32_t *d = reinterpret_cast<int32_t *>(RW + x);
                        for (int w = lane; w < (int)(sizeof(af_psl) / 4); w += 64) d[w] = src[w];
                        __threadfence_block();
                        wave_sync();
                    }
                    dst = RW + at;
                } else if (spill.cap > 0) {
                    int k = 0;
                    if (lane == 0) k = atomicAdd(spill.n, 1);
                    k = __builtin_amdgcn_readfirstlane(k);
                    if (k < spill.cap) {
                        dst = spill.rows + k;
                        if (lane == 0) spill.query[k] = (int32_t)qi;
                    } else if (lane == 0) {
                        caps.hit(qi, AF_BLAT_CAP_ROWS);
                    }
                }
                if (dst) {
                    if (lane == 0) {
                        dst->query = h.query; dst->strand = h.strand; dst->score = h.score;
                        dst->matches = h.matches; dst->mismatches = h.mismatches; dst->n_count = h.n_count;
                        dst->q_num_insert = h.q_num_insert; dst->q_base_insert = h.q_base_insert;
                        dst->t_num_insert = h.t_num_insert; dst->t_base_insert = h.t_base_insert;
                        dst->q_start = h.q_start; dst->q_end = h.q_end; dst->q_size = h.q_size;
                        dst->block_count = h.block_count; dst->t_start = h.t_start; dst->t_end = h.t_end;
                    }
                    if (lane < AF_PSL_MAX_BLOCKS) {
                        const bool v = lane < m;
                        dst->block_sizes[lane] = v ? blen : 0;
                        dst->q_starts[lane] = v ? qb : 0;
                        dst->t_starts[lane] = v ? tb : 0;
                    }
                }
                if (lane == 0) ++B.nrow;
            }
        }
        __threadfence_block();
        wave_sync();
        // parts after the chain's first whose predecessor path meets a used or recomputed
        // part: recomputed in order (a recomputed part marks its successors in turn)
        for (int i0 = first + 1 - ((first + 1) & 63); i0 < nr; i0 += 64) {
            const int i = i0 + lane;
            bool live = i > first && i < nr && !(CD.FL[i] & 1);
            const int pv = live ? CD.PREV[i] : -1;
            bool dirty = live && pv >= 0 && pv < i0 && (CD.FL[pv] & 3);
            // predecessors inside this chunk: the marks spread lane to lane
            uint64_t dm = __ballot(dirty);
            for (;;) {
                const bool more = !dirty && live && pv >= i0 && ((CD.FL[pv] & 1) || ((dm >> (pv - i0)) & 1));
                const uint64_t nm = __ballot(more);
                if (!nm) break;
                dirty = dirty || more;
                dm |= nm;
            }
            while (dm) {
                const int l = (int)__builtin_ctzll(dm);
                dm &= dm - 1;
                chain_node(B, X, RG, CD, i0 + l, bp.max_intron, lane);
                work += i0 + l;
                if (lane == 0) CD.FL[i0 + l] |= 2;
                __threadfence_block();
                wave_sync();
            }
        }
        for (int i = lane; i < nr; i += 64) CD.FL[i] &= 1;
        __threadfence_block();
        wave_sync();
    }
}

// the first index in A[0, n) holding a value >= v (A ascending; every lane the same answer)
__device__ __forceinline__ int lower_bound_u32(const uint32_t *A, int n, uint32_t v) {
    int a = 0, b = n;
    while (a < b) {
        const int m = (a + b) >> 1;
        if (A[m] < v) a = m + 1; else b = m;
    }
    return a;
}

// the query codes of (qi, strand) into B.q (strand 1: the reverse complement); returns its length
__device__ __forceinline__ int load_strand(BlatLds &B, const uint8_t *queries, int32_t stride, const int32_t *lens, int64_t qi,
                                           int strand, int lane) {
    int L = lens ? lens[qi] : stride;
    if (L > stride) L = stride;
    if (L > AF_MAX_READ) L = AF_MAX_READ;
    if (L < 0) L = 0;
    const uint8_t *row = queries + qi * (int64_t)stride;
    for (int x = lane; x < L; x += 64) {
        const uint8_t c = nt4(row[strand ? L - 1 - x : x]);
        B.q[x] = strand ? (c > 3 ? 4 : 3 - c) : c;
    }
    wave_sync();
    return L;
}

// One query strand (item 2 qi + strand) on the wave, with the slot's scratch zg: its rows to the
// item's stage; true when it was left to k_blat_heavy instead (allow_defer, a strand table with
// room, more than hv.min_clumps clumps).
__device__ __forceinline__ bool search_strand(BlatLds &B, const DevTile &X, const uint8_t *queries, int32_t stride,
                                              const int32_t *lens, const af_blat_params &bp, int64_t qi, int strand,
                                              uint8_t *zg, int32_t diag_passes, af_psl *stage, int32_t *stage_n,
                                              int32_t max_rows, const BlatCaps &caps, const BlatSpill &spill,
                                              const BlatHeavy &hv, bool allow_defer, int lane) {
    uint64_t *KA = reinterpret_cast<uint64_t *>(zg + SC_KEYS_A), *KB = reinterpret_cast<uint64_t *>(zg + SC_KEYS_B);
    Clump *CL = reinterpret_cast<Clump *>(zg + SC_CLUMP);
    Reg *RG = reinterpret_cast<Reg *>(zg + SC_REGS);
    af_psl *RW = reinterpret_cast<af_psl *>(zg + SC_ROWS);
    int32_t *dpw = reinterpret_cast<int32_t *>(zg + SC_DP);
    const ChainDp CD{dpw, dpw + MAXP, dpw + 2 * MAXP, dpw + 3 * MAXP, dpw + 4 * MAXP, dpw + 5 * MAXP,
                     reinterpret_cast<uint32_t *>(dpw + 6 * MAXP), reinterpret_cast<uint32_t *>(dpw + 7 * MAXP)};
    const int L = load_strand(B, queries, stride, lens, qi, strand, lane);
    if (lane == 0) B.nrow = 0;
    wave_sync();
    const int64_t drift = (int64_t)bp.max_gap + 2;
    int wsh = 3;  // bucket width 1 << wsh >= 2 * drift: [d - drift, d + drift] meets <= 2 buckets
    while ((1ll << wsh) < 2 * drift) ++wsh;
    BP(int64_t tq0 = clock64(), tq = tq0; int64_t pc[6] = {0, 0, 0, 0, 0, 0}; int ch = 0, cc_ = 0, cr = 0, cs = 0, crg = 0;)
    bool deferred = false;
    do {
        // ---- per offset: its tile's position range (count 0: N inside, absent or over rep_match) --
        const bool filt = bp.min_match >= 2;
        if (filt) drift_clear(B, lane);  // round 0 of the drift filter is marked while collecting
        uint32_t *DEL = B.hist;          // first position index - first hit index, per offset
        int carry = 0;
        for (int q0 = 0; q0 < L; q0 += 64) {
            const int q = q0 + lane;
            uint32_t k, c = 0, lo = 0;
            if (q + TILE <= L && tile_key(B.q, q, k)) {
                lo = X.start[k];
                c = X.start[k + 1] - lo;
                if ((int64_t)c > bp.rep_match) c = 0;
            }
            const int inc = wave_incl_sum((int)c, lane);
            const int bq = carry + inc - (int)c;
            if (q < L) { DEL[q] = lo - (uint32_t)bq; B.base[q] = bq; }
            carry += __builtin_amdgcn_readlane(inc, 63);
        }
        wave_sync();
        // ---- every hit, the first NMAX in (offset, position) order: lanes over hits, 4 chunks
        // in flight.  With the drift filter (min_match >= 2) the hits are gathered twice: the
        // first pass only marks their buckets (LDS), the second keeps round 0's survivors
        const int nh_all = min(carry, NMAX);
        // (a deferred strand's hit and clump caps were counted by k_blat: not again here)
        if (lane == 0 && carry > NMAX && allow_defer) caps.hit(qi, AF_BLAT_CAP_HITS);
        auto gather = [&](int h0, int &qc, int (&qv)[4], uint32_t (&pv)[4]) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int h = h0 + 64 * j + lane;
                int q = qc;  // the last offset whose first hit index is <= h
                if (h < nh_all)
                    while (q + 1 < L && B.base[q + 1] <= h) ++q;
                qv[j] = q;
            }
            qc = __builtin_amdgcn_readlane(qv[3], 63);  // (a full group: lane 63 of chunk 3 is a hit)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int h = h0 + 64 * j + lane;
                pv[j] = h < nh_all ? X.pos[DEL[qv[j]] + (uint32_t)h] : 0u;
            }
        };
        int qc = 0;  // offset of the group's first hit (hit offsets are nondecreasing)
        for (int h0 = 0; h0 < nh_all; h0 += 256) {
            int qv[4];
            uint32_t pv[4];
            gather(h0, qc, qv, pv);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int h = h0 + 64 * j + lane;
                if (h < nh_all) {
                    const uint64_t key = ((uint64_t)((int64_t)pv[j] - qv[j] + 1024) << 9) | (uint32_t)qv[j];
                    if (filt) drift_mark(B, key, wsh, 0);
                    else KA[h] = key;
                }
            }
        }
        int nh = nh_all;
        __threadfence_block();
        wave_sync();
        if (nh == 0) break;
        BPM(0);
        BP(ch += nh;)
        // ---- drop hits with no other hit within the drift (they cannot join a clump of
        // min_match >= 2 hits, and removing them changes no other run) ----------------------
        uint64_t *H0 = KA, *H1 = KB;
        if (filt) {
            int nk = 0;
            qc = 0;
            for (int h0 = 0; h0 < nh_all; h0 += 256) {
                int qv[4];
                uint32_t pv[4];
                gather(h0, qc, qv, pv);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int h = h0 + 64 * j + lane;
                    const uint64_t key = ((uint64_t)((int64_t)pv[j] - qv[j] + 1024) << 9) | (uint32_t)qv[j];
                    const bool keep = h < nh_all && drift_kept(B, key, drift, wsh, 0);
                    const uint64_t m = __ballot(keep);
                    if (keep) H0[nk + lanes_below_blat(m, lane)] = key;
                    nk += (int)__builtin_popcountll(m);
                }
            }
            __threadfence_block();
            wave_sync();
            bool stop = nk * 8 > nh * 7;
            nh = nk;
            for (int round = 1; !stop && round < AF_BLAT_ROUNDS && nh > AF_BLAT_FILTER_MIN; ++round) {
                const int nk2 = drift_filter(B, H0, H1, nh, drift, wsh, round, lane);
                uint64_t *t = H0; H0 = H1; H1 = t;
                stop = nk2 * 8 > nh * 7;
                nh = nk2;
            }
        }
        BPM(5);
        BP(cs += nh;)
        if (nh == 0) break;
        // ---- sort by diagonal (stable: offsets ascending within a diagonal) ------------------
        const uint64_t *S = wave_radix_sort(B, H0, H1, nh, 9, diag_passes, lane);
        uint8_t *SO = reinterpret_cast<uint8_t *>(S == H0 ? H1 : H0);  // the spare key buffer
        uint32_t *ST = reinterpret_cast<uint32_t *>(SO);
        BPM(1);
        // ---- run starts, then the clumps (runs of min_match hits) in diagonal order -----------
        int nrun = 0;
        for (int i0 = 0; i0 < nh; i0 += 64) {
            const int i = i0 + lane;
            bool st = false;
            if (i < nh) st = i == 0 || (int64_t)(S[i] >> 9) - (int64_t)(S[i - 1] >> 9) > drift;
            const uint64_t m = __ballot(st);
            if (st) ST[nrun + lanes_below_blat(m, lane)] = (uint32_t)i;
            nrun += (int)__builtin_popcountll(m);
        }
        __threadfence_block();
        wave_sync();
        int ncl = 0;
        for (int r0 = 0; r0 < nrun && ncl < MAXCL; r0 += 64) {
            const int r = r0 + lane;
            bool keep = false;
            Clump cc{};
            if (r < nrun) {
                const int s0 = (int)ST[r], e0 = r + 1 < nrun ? (int)ST[r + 1] : nh;
                if (e0 - s0 >= bp.min_match) {
                    keep = true;
                    cc.cnt = e0 - s0; cc.h0 = s0; cc.h1 = e0;
                }
            }
            const uint64_t m = __ballot(keep);
            const int slot = ncl + lanes_below_blat(m, lane);
            if (keep && slot < MAXCL) CL[slot] = cc;
            ncl = min(MAXCL, ncl + (int)__builtin_popcountll(m));
        }
        __threadfence_block();
        wave_sync();
        if (lane == 0 && ncl == MAXCL && allow_defer) caps.hit(qi, AF_BLAT_CAP_CLUMPS);
        if (ncl == 0) break;
        // ---- range starts over the sorted hits (ranges never cross a run): a hit starts one
        // when its diagonal differs from the previous hit's or its tile starts past that one's end
        uint32_t *RS = reinterpret_cast<uint32_t *>(SO + SC_RANGES);
        int nrs = 0;
        for (int i0 = 0; i0 < nh; i0 += 64) {
            const int i = i0 + lane;
            bool st = false;
            if (i < nh) {
                const uint64_t k = S[i];
                if (i == 0) st = true;
                else {
                    const uint64_t kp = S[i - 1];
                    st = (k >> 9) != (kp >> 9) || (int)(k & 511u) > (int)(kp & 511u) + TILE;
                }
            }
            const uint64_t m = __ballot(st);
            if (st) RS[nrs + lanes_below_blat(m, lane)] = (uint32_t)i;
            nrs += (int)__builtin_popcountll(m);
        }
        // ---- clump order: hits desc, then diagonal (= run order) ------------------------------
        uint64_t *OA = reinterpret_cast<uint64_t *>(SO), *OB = OA + MAXCL;
        for (int i = lane; i < ncl; i += 64) OA[i] = ((uint64_t)(65535 - CL[i].cnt) << 32) | (uint32_t)i;
        __threadfence_block();
        wave_sync();
        const uint64_t *CO = wave_radix_sort(B, OA, OB, ncl, 32, 2, lane);
        BPM(2);
        BP(cc_ += ncl;)
        // ---- a heavy strand is left to k_blat_heavy, which searches it after the caller's
        // live flags are known (S6: after S5's check) ------------------------------------------
        if (allow_defer && hv.min_clumps > 0 && ncl > hv.min_clumps) {
            int ok = 0;
            if (lane == 0) {
                const int s = atomicAdd(hv.strands_n, 1);
                if (s < hv.strands_cap) {
                    hv.strands[s] = make_int4((int)(2 * qi + strand), 0, ncl, 0);
                    atomicAdd(hv.jobs_n, ncl);
                    ok = 1;
                }
            }
            if (__builtin_amdgcn_readfirstlane(ok)) { deferred = true; break; }
        }
        // ---- HSPs: per clump in order, its ranges in order; a range inside an HSP made before
        // makes none ---------------------------------------------------------------------------
        int nr = 0;
        bool capped = false;
        for (int c = 0; c < ncl && !capped; ++c) {
            const Clump cc = CL[(uint32_t)CO[c]];
            const int k0 = lower_bound_u32(RS, nrs, (uint32_t)cc.h0), k1 = lower_bound_u32(RS, nrs, (uint32_t)cc.h1);
            for (int k = k0; k < k1; ++k) {
                const int hs = (int)RS[k], he = (k + 1 < nrs ? (int)RS[k + 1] : nh) - 1;
                const uint64_t ks = S[hs], ke = S[he];
                const int q0 = (int)(ks & 511u), q1 = (int)(ke & 511u) + TILE;
                const int64_t t0 = (int64_t)(ks >> 9) - 1024 + q0, t1 = t0 + (q1 - q0);
                BP(++crg;)
                if (inside_part(RG, nr, q0, q1, t0, t1, lane)) continue;
                if (nr == MAXP) { capped = true; break; }
                const Reg r = hsp_range(X, B.q, L, q0, q1, t0, lane);
                if (lane == 0) RG[nr] = r;
                ++nr;
                __threadfence_block();
                wave_sync();
            }
        }
        if (lane == 0 && capped) caps.hit(qi, AF_BLAT_CAP_PARTS);
        BPM(3);
        BP(cr += nr;)
        if (nr > 0) strand_chains(B, X, bp, RG, CD, nr, qi, strand, L, KA, KB, RW, max_rows, caps, spill, capped, lane);
    } while (false);
    BPM(4);
    if (!deferred && lane == 0) {  // the strand's rows (RW holds the first max_rows of B.nrow in order)
        const int n = B.nrow;
        const int m = n < max_rows ? n : max_rows;
        const int64_t sl = 2 * qi + strand;
        for (int k = 0; k < m; ++k) stage[sl * max_rows + k] = RW[k];
        stage_n[sl] = n;  // all of the strand's rows (k_blat_merge takes the first max_rows)
    }
    BP(if (lane == 0 && g_blprof && qi < (1 << 22)) {
        int32_t *pf = g_blprof + qi * 16;
        for (int k = 0; k < 5; ++k) pf[k] = (int32_t)min(pc[k], (int64_t)0x7fffffff);
        pf[5] = ch; pf[6] = cc_; pf[7] = cr; pf[8] = L;
        pf[9] = (int32_t)min(clock64() - tq0, (int64_t)0x7fffffff);
        pf[10] = (int32_t)min(pc[5], (int64_t)0x7fffffff); pf[11] = cs; pf[12] = deferred ? 1 : 0; pf[13] = crg;
    })
    __threadfence_block();
    wave_sync();
    return deferred;
}

// next work item of a persistent grid from 8 per-XCD heads (item = first + head + 8 * k), or n
// when drained
__device__ __forceinline__ int64_t next_item(int32_t *heads, int64_t first, int64_t n, int &head, int &heads_left, int lane) {
    while (heads_left > 0) {
        int v = 0;
        if (lane == 0) v = atomicAdd(&heads[AF_HEAD_STRIDE * head], 1);
        v = __builtin_amdgcn_readfirstlane(v);
        const int64_t it = first + head + 8 * (int64_t)v;
        if (it < n) return it;
        head = (head + 1) & 7;
        --heads_left;
    }
    return n;
}

// every query strand of [q_first, n_q), heaviest queries first (order): items 2k + s = strand s of
// the k-th query, so a heavy query's strands run on two waves at once
__global__ __launch_bounds__(64, AF_BLAT_WPS) void k_blat(DevTile X, const uint8_t *__restrict__ queries, int32_t stride,
                                                        const int32_t *__restrict__ lens, af_blat_params bp,
                                                        const int32_t *__restrict__ n_q, const int32_t *__restrict__ q_first,
                                                        int64_t cap, int32_t *__restrict__ heads,
                                                        uint8_t *__restrict__ bscratch, int32_t diag_passes,
                                                        af_psl *__restrict__ stage, int32_t *__restrict__ stage_n,
                                                        int32_t max_rows, const int32_t *__restrict__ order, BlatCaps caps,
                                                        BlatSpill spill, BlatHeavy hv) {
    __shared__ BlatLds B;
    const int lane = threadIdx.x;
    const int64_t nq64 = *n_q < cap ? *n_q : cap;
    const int nq = (int)(nq64 < 0 ? 0 : nq64);
    const int q0 = q_first ? max(0, min(*q_first, nq)) : 0;  // queries [q0, nq)
    uint8_t *zg = bscratch + (size_t)blockIdx.x * SC_END;
    int head = (int)(blockIdx.x & 7), heads_left = 8;
    for (;;) {
        const int64_t item = next_item(heads, 2 * (int64_t)q0, 2 * (int64_t)nq, head, heads_left, lane);
        if (item >= 2 * (int64_t)nq) break;
        const int64_t qi = order ? order[item >> 1] : (item >> 1);
        search_strand(B, X, queries, stride, lens, bp, qi, (int)(item & 1), zg, diag_passes, stage, stage_n, max_rows,
                      caps, spill, hv, true, lane);
    }
}

// the deferred strands of the live queries, one per wave, searched in full
__global__ __launch_bounds__(64, AF_BLAT_WPS) void k_blat_heavy(DevTile X, const uint8_t *__restrict__ queries,
                                                              int32_t stride, const int32_t *__restrict__ lens,
                                                              af_blat_params bp, BlatHeavy hv,
                                                              const uint8_t *__restrict__ live,
                                                              int32_t *__restrict__ heads, uint8_t *__restrict__ bscratch,
                                                              int32_t diag_passes, af_psl *__restrict__ stage,
                                                              int32_t *__restrict__ stage_n, int32_t max_rows,
                                                              BlatCaps caps, BlatSpill spill) {
    __shared__ BlatLds B;
    const int lane = threadIdx.x;
    uint8_t *zg = bscratch + (size_t)blockIdx.x * SC_END;
    int64_t ns = *hv.strands_n;
    if (ns > hv.strands_cap) ns = hv.strands_cap;
    int head = (int)(blockIdx.x & 7), heads_left = 8;
    for (;;) {
        const int64_t s = next_item(heads, 0, ns, head, heads_left, lane);
        if (s >= ns) break;
        const int4 st = hv.strands[s];
        const int64_t qi = st.x >> 1;
        if (live && !live[qi]) continue;
        search_strand(B, X, queries, stride, lens, bp, qi, st.x & 1, zg, diag_passes, stage, stage_n, max_rows, caps,
                      spill, hv, false, lane);
        if (lane == 0) {
            atomicAdd(hv.ctrl + AF_BLAT_HV_JOBS_DONE, st.z);
            atomicAdd(hv.ctrl + AF_BLAT_HV_STRANDS_DONE, 1);
        }
    }
}

// ---- tile index build -------------------------------------------------------------------------
__global__ void k_tile_codes(const uint8_t *__restrict__ seq, int64_t n, uint8_t *__restrict__ T) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) T[i] = nt4(seq[i]);
}

__global__ void k_tile_keys(const uint8_t *__restrict__ T, int64_t n, int32_t step, int64_t n_tiles,
                            uint32_t *__restrict__ keys, uint32_t *__restrict__ pos, uint32_t *__restrict__ cnt) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n_tiles) return;
    const int64_t p = k * step;
    uint32_t key = 0;
    bool ok = p + TILE <= n;
    for (int u = 0; u < TILE && ok; ++u) {
        const uint8_t b = T[p + u];
        ok = b < 4;
        key |= (uint32_t)(b & 3) << (2 * u);
    }
    keys[k] = ok ? key : NKEYS;  // invalid tiles sort last
    pos[k] = (uint32_t)p;
    if (ok) atomicAdd(&cnt[key], 1u);
}

// one thread per 64-base block b: its N bits (bit u = base 64 b + u), nblk[b + 1] = their count and
// rfirst[nb - 1 - b] = its first N (0xFFFFFFFF: none), reversed for the suffix min of k_tile_nnext
__global__ void k_tile_nblocks(const uint8_t *__restrict__ T, int64_t n, int64_t nb, uint64_t *__restrict__ mask,
                               uint32_t *__restrict__ nblk, uint32_t *__restrict__ rfirst) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    const int64_t a = b << 6;
    uint64_t m = 0;
    for (int u = 0; u < 64 && a + u < n; ++u) m |= (uint64_t)(T[a + u] > 3) << u;
    mask[b] = m;
    nblk[b + 1] = (uint32_t)__builtin_popcountll(m);
    rfirst[nb - 1 - b] = m ? (uint32_t)(a + __builtin_ctzll(m)) : 0xFFFFFFFFu;
}
// nnext[b] = the first N at or after block b (the reversed prefix min back in order)
__global__ void k_tile_nnext(const uint32_t *__restrict__ rmin, int64_t nb, uint32_t *__restrict__ nnext) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b < nb) nnext[b] = rmin[nb - 1 - b];
}
struct MinU32 {
    __host__ __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a < b ? a : b; }
};

}  // namespace

// the rows of a query's two strands (each sorted, <= max_rows) merged in psl_before order: the
// stable sort of the union, as one wave doing both strands would have produced
__global__ void k_blat_merge(const af_psl *__restrict__ stage, const int32_t *__restrict__ stage_n,
                             const int32_t *__restrict__ n_q, const int32_t *__restrict__ q_first, int64_t cap,
                             int32_t max_rows, af_psl *__restrict__ rows, int32_t *__restrict__ n_rows,
                             BlatCaps caps, BlatSpill spill, const uint8_t *__restrict__ live) {
    const int64_t nq = *n_q < cap ? *n_q : cap;
    const int64_t q0 = q_first ? max((int64_t)0, min((int64_t)*q_first, nq)) : 0;
    const int64_t qi = q0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (qi >= nq) return;
    if (live && !live[qi]) {  // a query the caller dropped: no rows (its strands may not be searched)
        n_rows[qi] = 0;
        return;
    }
    const af_psl *A = stage + 2 * qi * max_rows, *Bs = A + max_rows;
    const int sa = stage_n[2 * qi], sb = stage_n[2 * qi + 1];
    const int na = sa < max_rows ? sa : max_rows, nb = sb < max_rows ? sb : max_rows;
    if (sa + sb > max_rows && spill.cap <= 0) caps.hit(qi, AF_BLAT_CAP_ROWS);
#ifdef AF_BLAT_CHECK
    if (na < 0 || nb < 0) {
        printf("k_blat_merge: query %ld rows %d %d\n", (long)qi, na, nb);
        return;
    }
#endif
    int i = 0, j = 0, k = 0;
    for (; k < max_rows && (i < na || j < nb); ++k) {
        const bool take_b = j < nb && (i >= na || psl_before(Bs[j], A[i]));
        rows[qi * max_rows + k] = take_b ? Bs[j++] : A[i++];
    }
    n_rows[qi] = k;
    // the strands' kept rows that the merge leaves out follow the max_rows taken: to the pool
    if (spill.cap > 0) {
        for (; i < na || j < nb;) {
            const af_psl &r = j < nb && (i >= na || psl_before(Bs[j], A[i])) ? Bs[j++] : A[i++];
            const int x = atomicAdd(spill.n, 1);
            if (x < spill.cap) { spill.rows[x] = r; spill.query[x] = (int32_t)qi; }
            else caps.hit(qi, AF_BLAT_CAP_ROWS);
        }
    }
}

// the queries' forward tile hits (tiles over repMatch excluded): the scheduling key of k_blat,
// heaviest first (the order changes no result, only which wave takes a query when)
__global__ void k_blat_cost(DevTile X, const uint8_t *__restrict__ queries, int32_t stride,
                            const int32_t *__restrict__ lens, const int32_t *__restrict__ n_q, int64_t cap,
                            int32_t rep_match, uint32_t *__restrict__ keys, int32_t *__restrict__ vals) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= cap) return;
    const int64_t nq = *n_q < cap ? *n_q : cap;
    vals[i] = (int32_t)i;
    if (i >= nq) { keys[i] = 0xFFFFFFFFu; return; }
    int L = lens ? lens[i] : stride;
    L = max(0, min(L, min(stride, AF_MAX_READ)));
    const uint8_t *q = queries + i * (int64_t)stride;
    uint64_t cost = 0;
    uint32_t k = 0;
    int run = 0;
    for (int j = 0; j < L; ++j) {
        const uint8_t b = nt4(q[j]);
        if (b > 3) { run = 0; continue; }
        k = (k >> 2) | ((uint32_t)b << (2 * (TILE - 1)));
        if (++run >= TILE) {
            const uint32_t c = X.start[k + 1] - X.start[k];
            if ((int64_t)c <= rep_match) cost += c;
        }
    }
    keys[i] = 0xFFFFFFFEu - (uint32_t)(cost < 0xFFFFFFFEull ? cost : 0xFFFFFFFEull);
}


size_t af_blat_order_bytes(int64_t cap) {
    size_t tb = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tb, (uint32_t *)nullptr, (uint32_t *)nullptr,
                                             (int32_t *)nullptr, (int32_t *)nullptr, (int)cap, 0, 32);
    return 16 * (size_t)cap + ((tb + 255) & ~(size_t)255) + 256;
}

// order[0, cap): the queries [0, *n_queries) by k_blat_cost, heaviest first, then the empty slots
hipError_t af_launch_blat_order(const DevTile &X, const uint8_t *queries, const int32_t *n_queries, int64_t cap,
                                int32_t stride, const int32_t *lens, int32_t rep_match, void *work,
                                int32_t *order, hipStream_t s) {
    uint8_t *w = static_cast<uint8_t *>(work);
    uint32_t *k0 = reinterpret_cast<uint32_t *>(w), *k1 = k0 + cap;
    int32_t *v0 = reinterpret_cast<int32_t *>(k1 + cap);
    void *temp = w + 16 * (size_t)cap;
    size_t tb = af_blat_order_bytes(cap) - 16 * (size_t)cap - 256;
    hipLaunchKernelGGL(k_blat_cost, dim3((unsigned)((cap + 255) / 256)), dim3(256), 0, s, X, queries, stride, lens,
                       n_queries, cap, rep_match, k0, v0);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return hipcub::DeviceRadixSort::SortPairs(temp, tb, k0, k1, v0, order, (int)cap, 0, 32, s);
}


hipError_t af_launch_blat_begin(const BlatLaunch &B, hipStream_t s) {
    hipError_t e;
    const BlatHeavy &hv = B.hv;
    if (hv.min_clumps > 0) {
        // the strand table's fill, its counters and dequeue heads
        if ((e = hipMemsetAsync(hv.ctrl, 0, sizeof(int32_t) * AF_BLAT_HV_CTRL_WORDS, s)) != hipSuccess) return e;
    }
    // radix passes over the diagonal bits: (diagonal + 1024) < n + 1024
    int bits = 64 - __builtin_clzll((unsigned long long)(B.X.n + 1024));
    const int diag_passes = (bits + 7) / 8;
    hipLaunchKernelGGL(k_blat, dim3(B.n_slots), dim3(64), 0, s, B.X, B.queries, B.stride, B.lens, B.p, B.n_queries,
                       B.q_first, B.cap, B.heads, B.bscratch, diag_passes, B.stage, B.stage_n, B.max_rows, B.order,
                       B.caps, B.spill, hv);
    return hipGetLastError();
}

hipError_t af_launch_blat_end(const BlatLaunch &B, const uint8_t *live, hipStream_t s) {
    const BlatHeavy &hv = B.hv;
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (hv.min_clumps > 0) {
        int bits = 64 - __builtin_clzll((unsigned long long)(B.X.n + 1024));
        const int diag_passes = (bits + 7) / 8;
        hipLaunchKernelGGL(k_blat_heavy, dim3(B.n_slots), dim3(64), 0, s, B.X, B.queries, B.stride, B.lens, B.p, hv, live,
                           hv.ctrl + AF_BLAT_HV_STRAND_HEADS, B.bscratch, diag_passes, B.stage, B.stage_n, B.max_rows,
                           B.caps, B.spill);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_blat_merge, dim3((unsigned)((B.cap + 255) / 256)), dim3(256), 0, s, B.stage, B.stage_n,
                       B.n_queries, B.q_first, B.cap, B.max_rows, B.rows, B.n_rows, B.caps, B.spill, live);
    return hipGetLastError();
}

hipError_t af_launch_blat(const BlatLaunch &B, hipStream_t s) {
    hipError_t e = af_launch_blat_begin(B, s);
    return e != hipSuccess ? e : af_launch_blat_end(B, nullptr, s);
}

int af_blat_slots(int n_cu) {
    if (const char *e = getenv("AF_BLAT_WAVES_PER_CU")) {  // experiment knob: resident BLAT waves per CU
        const int w = atoi(e);
        if (w > 0) return n_cu * w;
    }
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, reinterpret_cast<const void *>(k_blat), 64, 0) !=
            hipSuccess || occ < 1)
        occ = 8;
    return n_cu * occ;
}

// Test hook (tests/test_gpu_ext_dp.py; not part of afgpu.h): ksw_extend2 through ext_dp, the
// dispatch k_blat's clump extensions take (ext_dp_w1 / ext_dp_band / ext_dp_w2 / ext_dp_wave by
// qlen and the clamped band), on n independent cases, one wave each.  Case k: query codes
// q[k * stride, + qlen[k]), target codes t[k * stride, + tlen[k]), par[10 k ..] = a, b, o_del,
// e_del, o_ins, e_ins, w, end_bonus, zdrop, h0; out[7 k ..] = max, qle, tle, gtle, gscore,
// max_off, rows.
__global__ __launch_bounds__(64) void k_debug_ext_dp(const uint8_t *__restrict__ q, const uint8_t *__restrict__ t,
                                                     int32_t stride, const int32_t *__restrict__ qlen,
                                                     const int32_t *__restrict__ tlen, const int32_t *__restrict__ par,
                                                     int32_t n, int32_t *__restrict__ out) {
    const int k = blockIdx.x, lane = threadIdx.x;
    if (k >= n) return;
    DpLds &D = g_dp;
    const int ql = qlen[k], tl = tlen[k];
    for (int x = lane; x < ql; x += 64) D.qs[x] = q[(int64_t)k * stride + x];
    for (int x = lane; x < tl; x += 64) D.t[x] = t[(int64_t)k * stride + x];
    wave_sync();
    const int32_t *c = par + 10 * (int64_t)k;
    af_params P{};
    P.a = c[0]; P.b = c[1]; P.o_del = c[2]; P.e_del = c[3]; P.o_ins = c[4]; P.e_ins = c[5];
    const ExtRes r = ext_dp<6>(ql, D.qs, tl, D.t, P, c[6], c[7], c[8], c[9], lane);
    if (lane == 0) {
        int32_t *o = out + 7 * (int64_t)k;
        o[0] = r.max; o[1] = r.qle; o[2] = r.tle; o[3] = r.gtle; o[4] = r.gscore; o[5] = r.max_off; o[6] = r.rows;
    }
}
static_assert(AF_MAX_READ + 1 <= 6 * 64, "k_debug_ext_dp's ext_dp<6> covers every query length");

extern "C" int af_debug_ext_dp(const uint8_t *q, const uint8_t *t, int32_t stride, const int32_t *qlen,
                               const int32_t *tlen, const int32_t *par, int32_t n, int32_t *out) {
    if (n <= 0) return 0;
    if (!q || !t || !qlen || !tlen || !par || !out || stride <= 0) return -1;
    for (int32_t k = 0; k < n; ++k)
        if (qlen[k] < 1 || qlen[k] > AF_MAX_READ || qlen[k] > stride || tlen[k] < 0 || tlen[k] > 1024 ||
            tlen[k] > stride)
            return -1;
    uint8_t *dq = nullptr, *dt = nullptr;
    int32_t *dql = nullptr, *dtl = nullptr, *dp = nullptr, *dout = nullptr;
    const size_t nb = (size_t)n * stride;
    int rc = -1;
    if (hipMalloc(&dq, nb) == hipSuccess && hipMalloc(&dt, nb) == hipSuccess && hipMalloc(&dql, 4 * n) == hipSuccess &&
        hipMalloc(&dtl, 4 * n) == hipSuccess && hipMalloc(&dp, 40 * (size_t)n) == hipSuccess &&
        hipMalloc(&dout, 28 * (size_t)n) == hipSuccess && hipMemcpy(dq, q, nb, hipMemcpyHostToDevice) == hipSuccess &&
        hipMemcpy(dt, t, nb, hipMemcpyHostToDevice) == hipSuccess &&
        hipMemcpy(dql, qlen, 4 * n, hipMemcpyHostToDevice) == hipSuccess &&
        hipMemcpy(dtl, tlen, 4 * n, hipMemcpyHostToDevice) == hipSuccess &&
        hipMemcpy(dp, par, 40 * (size_t)n, hipMemcpyHostToDevice) == hipSuccess) {
        hipLaunchKernelGGL(k_debug_ext_dp, dim3(n), dim3(64), 0, 0, dq, dt, stride, dql, dtl, dp, n, dout);
        if (hipGetLastError() == hipSuccess && hipDeviceSynchronize() == hipSuccess &&
            hipMemcpy(out, dout, 28 * (size_t)n, hipMemcpyDeviceToHost) == hipSuccess)
            rc = 0;
    }
    (void)hipFree(dq); (void)hipFree(dt); (void)hipFree(dql); (void)hipFree(dtl); (void)hipFree(dp); (void)hipFree(dout);
    return rc;
}

#ifdef AF_K2_PROF
extern "C" int af_debug_blat_prof_enable() {
    int32_t *d = nullptr;
    if (hipMalloc(&d, sizeof(int32_t) * 16 << 22) != hipSuccess) return -1;
    (void)hipMemset(d, 0, sizeof(int32_t) * 16 << 22);
    return hipMemcpyToSymbol(HIP_SYMBOL(g_blprof), &d, sizeof d) == hipSuccess ? 16 : -1;
}
extern "C" int af_debug_blat_prof_read(int32_t *host, int64_t n) {
    int32_t *d = nullptr;
    if (hipMemcpyFromSymbol(&d, HIP_SYMBOL(g_blprof), sizeof d) != hipSuccess || !d) return -1;
    return hipMemcpy(host, d, sizeof(int32_t) * 16 * n, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

// builds X's device arrays from d_seq (device bytes): allocations go to allocs[*na] (freed with
// the index); returns a HIP error or hipSuccess
hipError_t af_build_tile_index(const uint8_t *d_seq, int64_t n, int32_t step, DevTile *X, void **allocs, int *na,
                               hipStream_t s) {
    hipError_t e;
    const int64_t n_tiles = n >= TILE ? (n - TILE) / step + 1 : 0;
    const int64_t nb = (n >> 6) + 2;  // N counts before each 64-base block (and one past the last)
    uint8_t *T = nullptr;
    uint32_t *start = nullptr, *pos = nullptr, *ncum = nullptr, *nnext = nullptr;
    uint64_t *nmask = nullptr;
    uint32_t *keys = nullptr, *keys2 = nullptr, *pos2 = nullptr, *cnt = nullptr, *rf = nullptr, *rm = nullptr;
    void *temp = nullptr;
    auto cleanup = [&]() {
        if (rf) (void)hipFree(rf);
        if (rm) (void)hipFree(rm);
        if (keys) (void)hipFree(keys);
        if (keys2) (void)hipFree(keys2);
        if (pos2) (void)hipFree(pos2);
        if (cnt) (void)hipFree(cnt);
        if (temp) (void)hipFree(temp);
    };
    if ((e = hipMalloc(&T, (size_t)n)) != hipSuccess) return e;
    allocs[(*na)++] = T;
    if ((e = hipMalloc(&start, sizeof(uint32_t) * (NKEYS + 1))) != hipSuccess) return e;
    allocs[(*na)++] = start;
    if ((e = hipMalloc(&pos, sizeof(uint32_t) * (size_t)(n_tiles > 0 ? n_tiles : 1))) != hipSuccess) return e;
    allocs[(*na)++] = pos;
    if ((e = hipMalloc(&ncum, sizeof(uint32_t) * (size_t)nb)) != hipSuccess) return e;
    allocs[(*na)++] = ncum;
    if ((e = hipMalloc(&nmask, sizeof(uint64_t) * (size_t)nb)) != hipSuccess) return e;
    allocs[(*na)++] = nmask;
    if ((e = hipMalloc(&nnext, sizeof(uint32_t) * (size_t)nb)) != hipSuccess) return e;
    allocs[(*na)++] = nnext;
    if ((e = hipMalloc(&keys, sizeof(uint32_t) * (size_t)(n_tiles > 0 ? n_tiles : 1))) != hipSuccess ||
        (e = hipMalloc(&keys2, sizeof(uint32_t) * (size_t)(n_tiles > 0 ? n_tiles : 1))) != hipSuccess ||
        (e = hipMalloc(&pos2, sizeof(uint32_t) * (size_t)(n_tiles > 0 ? n_tiles : 1))) != hipSuccess ||
        (e = hipMalloc(&cnt, sizeof(uint32_t) * (NKEYS + 1))) != hipSuccess ||
        (e = hipMalloc(&rf, sizeof(uint32_t) * (size_t)nb)) != hipSuccess ||
        (e = hipMalloc(&rm, sizeof(uint32_t) * (size_t)nb)) != hipSuccess) {
        cleanup();
        return e;
    }
    size_t tb_sort = 0, tb_scan = 0, tb_scan2 = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tb_sort, keys, keys2, pos, pos2, n_tiles, 0, 2 * TILE + 1);
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, tb_scan, cnt, start, NKEYS + 1);
    (void)hipcub::DeviceScan::InclusiveSum(nullptr, tb_scan2, ncum, ncum, nb);
    size_t tb_min = 0;
    (void)hipcub::DeviceScan::InclusiveScan(nullptr, tb_min, rf, rm, MinU32(), nb - 1);
    size_t tb = std::max(std::max(tb_sort, tb_min), std::max(tb_scan, tb_scan2));
    if ((e = hipMalloc(&temp, tb > 0 ? tb : 16)) != hipSuccess) { cleanup(); return e; }
    const int bs = 256;
    if ((e = hipMemsetAsync(cnt, 0, sizeof(uint32_t) * (NKEYS + 1), s)) != hipSuccess ||
        (e = hipMemsetAsync(ncum, 0, sizeof(uint32_t) * (size_t)nb, s)) != hipSuccess ||
        (e = hipMemsetAsync(nnext, 0xFF, sizeof(uint32_t) * (size_t)nb, s)) != hipSuccess) { cleanup(); return e; }
    hipLaunchKernelGGL(k_tile_codes, dim3((unsigned)((n + bs - 1) / bs)), dim3(bs), 0, s, d_seq, n, T);
    if (n_tiles > 0)
        hipLaunchKernelGGL(k_tile_keys, dim3((unsigned)((n_tiles + bs - 1) / bs)), dim3(bs), 0, s, T, n, step, n_tiles,
                           keys, pos2, cnt);
    hipLaunchKernelGGL(k_tile_nblocks, dim3((unsigned)((nb - 1 + bs - 1) / bs)), dim3(bs), 0, s, T, n, nb - 1, nmask,
                       ncum, rf);
    if ((e = hipGetLastError()) != hipSuccess) { cleanup(); return e; }
    size_t t1 = tb;
    if (n_tiles > 0 &&
        (e = hipcub::DeviceRadixSort::SortPairs(temp, t1, keys, keys2, pos2, pos, n_tiles, 0, 2 * TILE + 1, s)) !=
            hipSuccess) { cleanup(); return e; }
    t1 = tb;
    if ((e = hipcub::DeviceScan::ExclusiveSum(temp, t1, cnt, start, NKEYS + 1, s)) != hipSuccess) { cleanup(); return e; }
    t1 = tb;
    if ((e = hipcub::DeviceScan::InclusiveSum(temp, t1, ncum, ncum, nb, s)) != hipSuccess) { cleanup(); return e; }
    t1 = tb;
    if ((e = hipcub::DeviceScan::InclusiveScan(temp, t1, rf, rm, MinU32(), nb - 1, s)) != hipSuccess) { cleanup(); return e; }
    hipLaunchKernelGGL(k_tile_nnext, dim3((unsigned)((nb - 1 + bs - 1) / bs)), dim3(bs), 0, s, rm, nb - 1, nnext);
    if ((e = hipGetLastError()) != hipSuccess) { cleanup(); return e; }
    if ((e = hipStreamSynchronize(s)) != hipSuccess) { cleanup(); return e; }
    cleanup();
    X->T = T; X->start = start; X->pos = pos; X->ncum = ncum; X->nmask = nmask; X->nnext = nnext; X->n = n;
    X->step = step;
    return hipSuccess;
}
