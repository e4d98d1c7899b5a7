// blat_long.hip -- one long BLAT query searched whole on the GPU (af_blat_long): the anchor
// transcript, kilobases long, that functions.py:341 (`Find_homo_genes`, homologs vs the genome) and
// fn:966 (`Build_candidate_fasta`, the anchor vs the candidate blocks) hand BLAT as one query.
//
// The algorithm is k_blat's (blat.hip; contract oracle/blat.c afo_blat_long, bit-exact): every
// 11-mer of the query and of its reverse complement looked up, hits sorted by diagonal, clumps of
// >= min_match hits ordered (hits desc, diagonal), a clump's hits of one diagonal with touching
// tiles forming a range, each range -- unless it lies inside an HSP made from an earlier range --
// extended without gaps into an HSP, then the chain DP over the HSPs and every chain passing
// -minScore / -minIdentity as a row.  What differs is the size (a query of up to AF_BLAT_LONG_MAX
// bases: 1.7 M hits per strand for the 6.8 kb anchor against hg38 at step 3), so every step is
// spread over the chip instead of walked by one wave:
//   - hits listed by a thread per hit, sorted by hipCUB; runs, clumps and ranges a thread each;
//   - every range's HSP extended at once, a thread per range (lk_hsp);
//   - the serial rule "a range inside an HSP kept before makes none" as rounds (lk_keep_round):
//     a range is kept once every earlier HSP containing it is known to be dropped, dropped once one
//     of them is kept -- the rule's unique outcome, reached in as many rounds as its longest chain of
//     containments (the candidates of a range: the HSPs sorted by target start, within the longest
//     HSP's span before it);
//   - the chain DP (lk_chain, a wave per strand) looks for predecessors only among the parts whose
//     target end lies within max_intron before the part (sorted by target end: a window), picks the
//     next chain from per-64-part maxima, and after a chain is emitted recomputes exactly the parts
//     whose predecessor path ended in it (the parts with the chain's root as their root);
//   - rows hold any number of blocks (a 23-exon anchor's locus is one row with 23 blocks) in a block
//     arena, reserved only for the rows that pass the filters.
// Rows come back unsorted with their strand and emission order; the host orders them (score desc,
// strand, tStart, qStart, tEnd, qEnd; then emission).
#include <algorithm>
#include <vector>

#include <hipcub/hipcub.hpp>

#pragma clang diagnostic ignored "-Wunneeded-internal-declaration"  // ksw_dp.h's DPs this file does not use
#include "ksw_dp.h"

namespace {

constexpr int TILE = AF_TILE;
constexpr int QBITS = 17;                       // query offsets < 2^17 (AF_BLAT_LONG_MAX)
constexpr int64_t DIAG0 = (int64_t)1 << QBITS;  // diagonal + DIAG0 >= 0
constexpr int64_t STITCH_WORK = 1 << 24;        // blat.hip / oracle/blat.c: the same budget
constexpr int XDOWN = 10;                       // blat.hip / oracle/blat.c XDOWN
static_assert(AF_BLAT_LONG_MAX <= (1 << QBITS), "query offsets in the hit keys");

struct Blk { int32_t sz, q; int64_t t; };
// one HSP (one block) with its range's box
struct RegL {
    int32_t qb, qe, score, matches, mismatches, ncount;
    int64_t tb, te;
    int32_t rq0, rq1;  // the range [rq0, rq1) it was extended from (target: rq0 + (tb - qb) on)
};

__device__ __forceinline__ int64_t key_diag(uint64_t k) { return (int64_t)(k >> QBITS) - DIAG0; }
__device__ __forceinline__ int32_t key_q(uint64_t k) { return (int32_t)(k & ((1u << QBITS) - 1)); }

// ---- hits, clumps, ranges -------------------------------------------------------------------------
// per offset q of the strand's codes Q: its tile's first position index and count (0: N inside,
// absent, or over rep_match); cnt[L] = 0 so the scan's last entry is the total
__global__ void lk_count(DevTile X, const uint8_t *__restrict__ Q, int L, int32_t rep_match, uint32_t *__restrict__ lo,
                         int64_t *__restrict__ cnt) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q > L) return;
    int64_t c = 0;
    uint32_t l = 0;
    if (q + TILE <= L) {
        uint32_t k = 0;
        bool ok = true;
        for (int u = 0; u < TILE; ++u) {
            const uint8_t b = Q[q + u];
            ok = ok && b < 4;
            k |= (uint32_t)(b & 3) << (2 * u);
        }
        if (ok) {
            l = X.start[k];
            c = (int64_t)(X.start[k + 1] - l);
            if (c > rep_match) c = 0;
        }
    }
    lo[q] = l;
    cnt[q] = c;
}

// hit h < nh (the first nh in (offset, position) order): key = (diagonal + DIAG0) << QBITS | offset
__global__ void lk_hits(DevTile X, int L, const uint32_t *__restrict__ lo, const int64_t *__restrict__ base, int64_t nh,
                        uint64_t *__restrict__ keys) {
    const int64_t h = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (h >= nh) return;
    int a = 0, b = L;  // the last offset whose first hit is <= h (base[q + 1] > h)
    while (a < b) {
        const int m = (a + b + 1) >> 1;
        if (base[m] <= h) a = m; else b = m - 1;
    }
    const int64_t t = X.pos[lo[a] + (uint32_t)(h - base[a])];
    keys[h] = ((uint64_t)(t - a + DIAG0) << QBITS) | (uint32_t)a;
}

// run starts over the diagonal-sorted keys (a diagonal step > max_gap + 2 starts a run) and range
// starts (a new diagonal, or a tile starting past the previous tile's end)
__global__ void lk_flags(const uint64_t *__restrict__ keys, int64_t nh, int64_t drift, uint8_t *__restrict__ run,
                         uint8_t *__restrict__ rng) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nh) return;
    if (i == 0) { run[i] = 1; rng[i] = 1; return; }
    const uint64_t k = keys[i], kp = keys[i - 1];
    run[i] = key_diag(k) - key_diag(kp) > drift ? 1 : 0;
    rng[i] = (key_diag(k) != key_diag(kp) || key_q(k) > key_q(kp) + TILE) ? 1 : 0;
}

struct ClumpL { int32_t cnt; int32_t pad; int64_t h0, h1; };
// run r -> a clump when it holds >= min_match hits: its hit count and hits [h0, h1)
__global__ void lk_clumps(int64_t nh, const int64_t *__restrict__ starts, int64_t nrun, int32_t min_match,
                          ClumpL *__restrict__ cl, uint8_t *__restrict__ keep) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nrun) return;
    const int64_t s0 = starts[r], e0 = r + 1 < nrun ? starts[r + 1] : nh;
    keep[r] = e0 - s0 >= min_match ? 1 : 0;
    cl[r] = ClumpL{(int32_t)(e0 - s0), 0, s0, e0};
}

// clump order keys: hits desc, then diagonal (= the clump's index in diagonal order)
__global__ void lk_clump_keys(const ClumpL *__restrict__ cl, int64_t ncl, uint64_t *__restrict__ k,
                              int32_t *__restrict__ v) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ncl) return;
    k[i] = ((uint64_t)(0xFFFFFFu - (uint32_t)min(cl[i].cnt, 0xFFFFFF)) << 32) | (uint64_t)i;
    v[i] = (int32_t)i;
}

__device__ __forceinline__ int64_t lower_bound_i64(const int64_t *A, int64_t n, int64_t v) {
    int64_t a = 0, b = n;
    while (a < b) {
        const int64_t m = (a + b) >> 1;
        if (A[m] < v) a = m + 1; else b = m;
    }
    return a;
}

// per clump in clump order: its first range and range count (ranges never cross a run)
__global__ void lk_clump_ranges(const ClumpL *__restrict__ cl, const int32_t *__restrict__ co, int64_t ncl,
                                const int64_t *__restrict__ rs, int64_t nrs, int64_t *__restrict__ k0,
                                int64_t *__restrict__ cnt) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c > ncl) return;
    if (c == ncl) { cnt[c] = 0; return; }
    const ClumpL cc = cl[co[c]];
    const int64_t a = lower_bound_i64(rs, nrs, cc.h0), b = lower_bound_i64(rs, nrs, cc.h1);
    k0[c] = a;
    cnt[c] = b - a;
}

// the ranges in order: range list entry off[c] + j = range k0[c] + j (a thread per clump)
__global__ void lk_range_list(int64_t ncl, const int64_t *__restrict__ k0, const int64_t *__restrict__ cnt,
                              const int64_t *__restrict__ off, int64_t *__restrict__ rl) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= ncl) return;
    for (int64_t j = 0; j < cnt[c]; ++j) rl[off[c] + j] = k0[c] + j;
}

__device__ __forceinline__ int hsp_sc(uint8_t a, uint8_t b) { return (a > 3 || b > 3 || a != b) ? -1 : 1; }

// the HSP of ordered range o (oracle hsp_range): extended without gaps both ways, each end at
// the first best running score, a walk stopped XDOWN positions after its last new best
__global__ void lk_hsp(DevTile X, const uint8_t *__restrict__ Q, int L, const uint64_t *__restrict__ keys, int64_t nh,
                       const int64_t *__restrict__ rs, int64_t nrs, const int64_t *__restrict__ rl, int64_t nr,
                       RegL *__restrict__ hsp, int64_t *__restrict__ tb_key, int32_t *__restrict__ tb_val,
                       int64_t *__restrict__ span) {
    const int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= nr) return;
    const int64_t k = rl[o];
    const int64_t hs = rs[k], he = (k + 1 < nrs ? rs[k + 1] : nh) - 1;
    const int32_t q0 = key_q(keys[hs]), q1 = key_q(keys[he]) + TILE;
    const int64_t t0 = key_diag(keys[hs]) + q0, t1 = t0 + (q1 - q0);
    int s = 0, best = 0, nb = 0;
    for (int i = 1; q0 - i >= 0 && t0 - i >= 0; ++i) {
        s += hsp_sc(Q[q0 - i], X.T[t0 - i]);
        if (s > best) { best = s; nb = i; }
        else if (i - nb > XDOWN) break;
    }
    RegL r;
    r.qb = q0 - nb; r.tb = t0 - nb;
    s = best = nb = 0;
    for (int i = 1; q1 + i - 1 < L && t1 + i - 1 < X.n; ++i) {
        s += hsp_sc(Q[q1 + i - 1], X.T[t1 + i - 1]);
        if (s > best) { best = s; nb = i; }
        else if (i - nb > XDOWN) break;
    }
    r.qe = q1 + nb; r.te = t1 + nb;
    int mt = 0, mm = 0, nn = 0;
    for (int32_t x = r.qb; x < r.qe; ++x) {
        const uint8_t a = Q[x], b = X.T[r.tb + (x - r.qb)];
        if (a > 3 || b > 3) ++nn;
        else if (a == b) ++mt;
        else ++mm;
    }
    r.matches = mt; r.mismatches = mm; r.ncount = nn; r.score = mt - mm;
    r.rq0 = q0; r.rq1 = q1;
    hsp[o] = r;
    tb_key[o] = r.tb;
    tb_val[o] = (int32_t)o;
    span[o] = r.te - r.tb;
}

// One round of the keep rule over the ranges still undecided (st 0): a range is dropped (2) when an
// earlier HSP containing its box is kept, kept (1) when every earlier HSP containing it is dropped;
// candidates: the HSPs with target start in [t1 - maxspan, t0] (tbs: the starts sorted, tbo their
// range index).  A decision needs only decided earlier ranges, so updating in place is exact.
__global__ void lk_keep_round(const RegL *__restrict__ hsp, int64_t nr, const int64_t *__restrict__ tbs,
                              const int32_t *__restrict__ tbo, const int64_t *__restrict__ maxspan,
                              uint8_t *__restrict__ st, int32_t *__restrict__ n_undecided) {
    const int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= nr || st[o]) return;
    const RegL r = hsp[o];
    const int32_t q0 = r.rq0, q1 = r.rq1;
    const int64_t t0 = r.tb + (q0 - r.qb), t1 = t0 + (q1 - q0);
    const int64_t lo = lower_bound_i64(tbs, nr, t1 - *maxspan);
    bool undecided = false;
    for (int64_t x = lo; x < nr && tbs[x] <= t0; ++x) {
        const int32_t s = tbo[x];
        if (s >= o) continue;
        const RegL &g = hsp[s];
        if (!(g.qb <= q0 && q1 <= g.qe && g.tb <= t0 && t1 <= g.te)) continue;
        const uint8_t v = st[s];
        if (v == 1) { st[o] = 2; return; }
        if (v == 0) undecided = true;
    }
    if (undecided) atomicAdd(n_undecided, 1);
    else st[o] = 1;
}

// kept flags (the first cap kept ranges, in order) from the states and their inclusive count
__global__ void lk_kept_flags(const uint8_t *__restrict__ st, const int64_t *__restrict__ cum, int64_t nr, int64_t cap,
                              uint8_t *__restrict__ flag) {
    const int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (o < nr) flag[o] = st[o] == 1 && cum[o] <= cap ? 1 : 0;
}
__global__ void lk_is_kept(const uint8_t *__restrict__ st, int64_t nr, int64_t *__restrict__ one) {
    const int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (o < nr) one[o] = st[o] == 1 ? 1 : 0;
}

// the chain DP's sort keys of the kept parts: (qb, tb) and (qe, creation order), for two stable
// passes; and (te, creation order) for the predecessor window
__global__ void lk_ord_keys(const RegL *__restrict__ parts, int n, uint64_t *__restrict__ k_hi, uint64_t *__restrict__ k_lo,
                            int32_t *__restrict__ idx) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const RegL &g = parts[r];
    k_hi[r] = ((uint64_t)g.qb << 40) | (uint64_t)g.tb;
    k_lo[r] = ((uint64_t)g.qe << 32) | (uint32_t)r;
    idx[r] = r;
}
// out[p] = keys[perm[p]]
__global__ void lk_gather_keys(const uint64_t *__restrict__ keys, const int32_t *__restrict__ perm, int n,
                               uint64_t *__restrict__ out) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < n) out[p] = keys[perm[p]];
}
// per DP position k (ord[k] = its part): the te-window keys (te, k)
__global__ void lk_te_keys(const RegL *__restrict__ parts, const int32_t *__restrict__ ord, int n, uint64_t *__restrict__ tk,
                           int32_t *__restrict__ tv) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    tk[k] = (uint64_t)parts[ord[k]].te;
    tv[k] = k;
}

// ---- chains and rows ---------------------------------------------------------------------------
struct ChainL {
    const RegL *parts;
    const int32_t *ord;   // part index at DP position k
    const uint64_t *tes;  // the parts' te, ascending (tev: their DP positions)
    const int32_t *tev;
    int32_t *best, *prev, *fl, *ch, *pre, *root, *cnt;
    int32_t *qe;          // -1 once used
    int64_t *te;
    uint32_t *nxt;        // first N of the target at or after te (0xFFFFFFFF: none)
    uint64_t *bmax;       // per 64 DP positions: the max of (best, -k) over the unused ones (0: none)
};

__device__ __forceinline__ uint32_t first_n_l(const DevTile &X, int64_t p) {
    const int64_t b = p >> 6;
    const uint64_t m = X.nmask[b] >> (p & 63);
    return m ? (uint32_t)(p + __builtin_ctzll(m)) : X.nnext[b + 1];
}

// the selection key of DP position k: higher best first, then lower k
__device__ __forceinline__ uint64_t sel_key(int best, int k) {
    return ((uint64_t)(uint32_t)(best + 0x40000000) << 32) | (uint32_t)(0x7FFFFFFF - k);
}
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const uint64_t o = __shfl_xor(v, d);
        v = o > v ? o : v;
    }
    return v;
}
// recompute the block maximum of DP positions [64 b, 64 b + 64)
__device__ __forceinline__ void block_max(const ChainL &C, int nr, int b, int lane) {
    const int k = 64 * b + lane;
    const uint64_t v = (k < nr && C.qe[k] >= 0) ? sel_key(C.best[k], k) : 0;
    const uint64_t m = wave_max_u64(v);
    if (lane == 0) C.bmax[b] = m;
}

// best / prev of DP position i over the unused parts before it (oracle chain_node): the candidates
// are the parts with te in [tb_i - max_intron, te_i) (tes window), lanes over them; the highest
// score wins over i alone, the lowest position among equal scores
__device__ void chain_node_l(const DevTile &X, const uint8_t *Q, const ChainL &C, int nr, int i, int64_t max_intron,
                             int lane) {
    const RegL &ri = C.parts[C.ord[i]];
    const int ilen = ri.qe - ri.qb;
    int carry = 0;
    for (int u0 = 0; u0 < ilen; u0 += 64) {
        const int u = u0 + lane;
        int m = 0;
        if (u < ilen) {
            const uint8_t a = Q[ri.qb + u], b = X.T[ri.tb + u];
            m = (a > 3 || b > 3) ? 0 : (a == b ? 1 : -1);
        }
        int inc = m;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int v = __shfl_up(inc, d);
            if (lane >= d) inc += v;
        }
        if (u < ilen) C.pre[u] = carry + inc - m;
        carry += __builtin_amdgcn_readlane(inc, 63);
    }
    __threadfence_block();
    wave_sync();
    // the window: te in [itb - max_intron, ite)
    const int64_t wlo = ri.tb - max_intron;
    int a = 0, b = nr;
    while (a < b) { const int m = (a + b) >> 1; if ((int64_t)C.tes[m] < wlo) a = m + 1; else b = m; }
    const int x0 = a;
    b = nr;
    while (a < b) { const int m = (a + b) >> 1; if ((int64_t)C.tes[m] < ri.te) a = m + 1; else b = m; }
    const int x1 = a;
    int best = ri.score, prev = -1;
    for (int y0 = x0; y0 < x1; y0 += 64) {
        const int y = y0 + lane;
        int v = INT_MIN, j = INT_MAX;
        if (y < x1) {
            j = C.tev[y];
            const int aqe = j < i ? C.qe[j] : -1;
            if (aqe >= 0 && ri.qe > aqe) {
                const int64_t ate = C.te[j];
                int64_t kk = aqe - ri.qb;
                if (ate - ri.tb > kk) kk = ate - ri.tb;
                const int k = kk > 0 ? (int)kk : 0;
                const int64_t btb = ri.tb + k;
                if (!(k > 0 && k >= ilen) && btb - ate <= max_intron && (int64_t)C.nxt[j] >= btb)
                    v = C.best[j] + (ri.score - (k > 0 ? C.pre[k] : 0)) - (ri.qb + k > aqe) - (btb > ate);
            }
        }
        const int mx = wave_max(v);
        if (mx == INT_MIN || mx < best) continue;
        const int mj = -wave_max(v == mx ? -j : INT_MIN + 1);  // the lowest position with the max
        if (mx > best) { best = mx; prev = mj; }
        else if (prev >= 0 && mj < prev) prev = mj;  // equal to a chain found before: the lower position
    }
    if (lane == 0) { C.best[i] = best; C.prev[i] = prev; }
    __threadfence_block();
    wave_sync();
}

// the row output of af_blat_long: headers (the first 16 blocks inside), per row its strand's emission
// order and first block in the row block arena
struct RowsL {
    af_psl *rows;
    int32_t *seq;
    int64_t *boff;
    Blk *blk;
    int32_t *n_rows;
    unsigned long long *n_blk;
    int64_t rows_cap, blk_cap;
    int32_t *caps;      // the context's af_blat_caps counters
    int32_t *overflow;  // set when a row or its blocks found no room
};

// one wave per strand: the chain DP over its parts in DP order, chains best first as rows
__global__ __launch_bounds__(64) void lk_chain(DevTile X, const uint8_t *__restrict__ Q2, int L, af_blat_params bp,
                                                const RegL *__restrict__ parts_all, const int32_t *__restrict__ ord_all,
                                                const uint64_t *__restrict__ tes_all, const int32_t *__restrict__ tev_all,
                                                const int32_t *__restrict__ n_parts, int64_t base1,
                                                uint8_t *__restrict__ work_all, int64_t work_bytes, RowsL R,
                                                int32_t capped_mask) {
    const int lane = threadIdx.x, strand = blockIdx.x;
    const int nr = n_parts[strand];
    const int64_t base = strand ? base1 : 0;
    const uint8_t *Q = Q2 + (int64_t)strand * L;
    uint8_t *wk = work_all + strand * work_bytes;
    ChainL C;
    C.parts = parts_all + base; C.ord = ord_all + base; C.tes = tes_all + base; C.tev = tev_all + base;
    int32_t *w32 = reinterpret_cast<int32_t *>(wk);
    C.best = w32; C.prev = w32 + nr; C.fl = w32 + 2 * nr; C.ch = w32 + 3 * nr; C.qe = w32 + 4 * nr;
    C.nxt = reinterpret_cast<uint32_t *>(w32 + 5 * nr);
    C.root = w32 + 6 * nr; C.cnt = w32 + 7 * nr;
    C.pre = w32 + 8 * nr;
    C.te = reinterpret_cast<int64_t *>(((uintptr_t)(C.pre + L + 64) + 15) & ~(uintptr_t)15);
    C.bmax = reinterpret_cast<uint64_t *>(C.te + nr + 2);
    const int nblk = (nr + 63) / 64;
    for (int r = lane; r < nr; r += 64) {
        const RegL &g = C.parts[C.ord[r]];
        C.fl[r] = 0; C.qe[r] = g.qe; C.te[r] = g.te; C.nxt[r] = first_n_l(X, g.te); C.cnt[r] = 0;
    }
    __threadfence_block();
    wave_sync();
    for (int i = 0; i < nr; ++i) {
        chain_node_l(X, Q, C, nr, i, bp.max_intron, lane);
        if (lane == 0) {
            const int p = C.prev[i];
            const int rt = p < 0 ? i : C.root[p];
            C.root[i] = rt;
            ++C.cnt[rt];
        }
        __threadfence_block();
        wave_sync();
    }
    for (int bk = 0; bk < nblk; ++bk) block_max(C, nr, bk, lane);
    __threadfence_block();
    wave_sync();
    int64_t work = 0;
    int emitted = 0;
    for (;;) {
        if (work > STITCH_WORK) {
            // (a strand counts each cap once: not again when its parts cap bound)
            if (lane == 0 && !((capped_mask >> strand) & 1)) atomicAdd(&R.caps[AF_BLAT_CAP_PARTS], 1);
            break;
        }
        // the unused part with the highest chain score, the first on ties: the best block, then its part
        uint64_t bv = 0;
        for (int b0 = 0; b0 < nblk; b0 += 64) {
            const uint64_t v = b0 + lane < nblk ? C.bmax[b0 + lane] : 0;
            const uint64_t m = wave_max_u64(v);
            bv = m > bv ? m : bv;
        }
        if (bv == 0) break;
        const int bi = 0x7FFFFFFF - (int)(uint32_t)bv;
        int m = 0;
        if (lane == 0) {
            for (int i = bi; i >= 0; i = C.prev[i]) C.ch[m++] = i;
        }
        m = __builtin_amdgcn_readfirstlane(m);
        __threadfence_block();
        wave_sync();
        const int first = C.ch[m - 1];
        const int rt = first;  // the chain ends at its root
        const bool rescan = C.cnt[rt] > m;  // parts other than the chain's have this root
        for (int c = lane; c < m; c += 64) { C.fl[C.ch[c]] = 1; C.qe[C.ch[c]] = -1; }
        __threadfence_block();
        wave_sync();
        if (lane == 0) {
            af_psl o{};
            o.query = 0; o.strand = strand; o.q_size = L;
            int32_t pqe = 0, fqb = 0, lqe = 0;
            int64_t pte = 0, ftb = 0, lte = 0;
            for (int c = m - 1; c >= 0; --c) {
                const RegL &src = C.parts[C.ord[C.ch[c]]];
                int32_t qb = src.qb;
                int64_t tb = src.tb;
                int mt = src.matches, mm = src.mismatches, nn = src.ncount;
                if (c < m - 1) {
                    int64_t kk = pqe - qb;
                    if (pte - tb > kk) kk = pte - tb;
                    const int trim = kk > 0 && kk < src.qe - src.qb ? (int)kk : 0;  // trim_front
                    for (int u = 0; u < trim; ++u) {
                        const uint8_t a = Q[qb + u], b = X.T[tb + u];
                        if (a > 3 || b > 3) --nn;
                        else if (a == b) --mt;
                        else --mm;
                    }
                    qb += trim; tb += trim;
                    if (qb > pqe) { ++o.q_num_insert; o.q_base_insert += qb - pqe; }
                    if (tb > pte) { ++o.t_num_insert; o.t_base_insert += (int32_t)(tb - pte); }
                }
                o.matches += mt; o.mismatches += mm; o.n_count += nn;
                if (o.block_count < AF_PSL_MAX_BLOCKS) {
                    o.block_sizes[o.block_count] = src.qe - qb; o.q_starts[o.block_count] = qb;
                    o.t_starts[o.block_count] = tb;
                }
                ++o.block_count;
                if (c == m - 1) { fqb = qb; ftb = tb; }
                if (c == 0) { lqe = src.qe; lte = src.te; }
                pqe = src.qe; pte = src.te;
            }
            o.q_start = strand ? L - lqe : fqb;
            o.q_end = strand ? L - fqb : lqe;
            o.t_start = ftb; o.t_end = lte;
            o.score = o.matches - o.mismatches - o.q_num_insert - o.t_num_insert;
            // pslCalcMilliBad (mRNA), as k_blat's psl_millibad
            int mb = 0;
            {
                const int q_ali = o.q_end - o.q_start;
                const int64_t t_ali = o.t_end - o.t_start;
                const int64_t ali = q_ali < t_ali ? q_ali : t_ali;
                int64_t dif = q_ali - t_ali;
                if (dif < 0) dif = 0;
                const int total = o.matches + o.mismatches;
                if (ali > 0 && total > 0)
                    mb = (int)((1000 * (o.mismatches + o.q_num_insert + round(3 * log(1. + (double)dif)))) / total);
            }
            if (o.score >= bp.min_score && mb <= (100 - bp.min_identity) * 10) {
                // the row's blocks: a stretch of the arena reserved for a passing row only
                const int64_t b0 = (int64_t)atomicAdd(R.n_blk, (unsigned long long)m);
                const int r = atomicAdd(R.n_rows, 1);
                if (r < R.rows_cap && b0 + m <= R.blk_cap) {
                    R.rows[r] = o; R.seq[r] = emitted; R.boff[r] = b0;
                    int64_t bo = b0;
                    pqe = 0; pte = 0;
                    for (int c = m - 1; c >= 0; --c, ++bo) {
                        const RegL &src = C.parts[C.ord[C.ch[c]]];
                        int32_t qb = src.qb;
                        int64_t tb = src.tb;
                        if (c < m - 1) {
                            int64_t kk = pqe - qb;
                            if (pte - tb > kk) kk = pte - tb;
                            const int trim = kk > 0 && kk < src.qe - src.qb ? (int)kk : 0;
                            qb += trim; tb += trim;
                        }
                        R.blk[bo] = Blk{src.qe - qb, qb, tb};
                        pqe = src.qe; pte = src.te;
                    }
                } else {
                    atomicOr(R.overflow, 1);
                }
                ++emitted;
            }
        }
        emitted = __builtin_amdgcn_readfirstlane(emitted);
        __threadfence_block();
        wave_sync();
        // the parts whose predecessor path ended in the chain (root rt, unused): recomputed in order
        if (rescan) {
            for (int i0 = first + 1 - ((first + 1) & 63); i0 < nr; i0 += 64) {
                const int i = i0 + lane;
                uint64_t dm = __ballot(i > first && i < nr && !C.fl[i] && C.root[i] == rt);
                while (dm) {
                    const int l = (int)__builtin_ctzll(dm);
                    dm &= dm - 1;
                    chain_node_l(X, Q, C, nr, i0 + l, bp.max_intron, lane);
                    work += i0 + l;
                    if (lane == 0) {
                        const int p = C.prev[i0 + l];
                        const int r2 = p < 0 ? i0 + l : C.root[p];
                        C.root[i0 + l] = r2;
                        ++C.cnt[r2];
                    }
                    __threadfence_block();
                    wave_sync();
                }
            }
        }
        // the block maxima of the chain's parts and of the recomputed ones (all in [first, nr))
        if (rescan) {
            for (int bk = first / 64; bk < nblk; ++bk) block_max(C, nr, bk, lane);
        } else {
            for (int c = 0; c < m; ++c) {
                const int bk = C.ch[c] / 64;
                if (c == 0 || bk != C.ch[c - 1] / 64) block_max(C, nr, bk, lane);
            }
        }
        __threadfence_block();
        wave_sync();
    }
}

}  // namespace

// Host-driven search of one long query (codes of both strands in d_q2: strand s at d_q2 + s L).
// Returns hipSuccess or an error; *overflow = 1 when the row lists or the block arena overflowed.
hipError_t af_blat_long_run(const DevTile &X, const uint8_t *d_q2, int L, const af_blat_params &bp, int32_t *caps,
                            std::vector<af_psl> &rows, std::vector<int32_t> &seq, std::vector<int64_t> &boff,
                            std::vector<af_psl_block> &blocks, int n_cu, hipStream_t s, int *overflow) {
    (void)n_cu;
    *overflow = 0;
    hipError_t e = hipSuccess;
    std::vector<void *> allocs;
    auto dalloc = [&](size_t bytes) -> void * {
        void *p = nullptr;
        if (e == hipSuccess && (e = hipMalloc(&p, bytes > 0 ? bytes : 16)) == hipSuccess) allocs.push_back(p);
        return p;
    };
    auto finish = [&](hipError_t r) {
        (void)hipStreamSynchronize(s);
        for (void *p : allocs) (void)hipFree(p);
        return r;
    };
    auto grid = [](int64_t n) { return dim3((unsigned)((n + 255) / 256)); };
    auto d2h = [&](void *dst, const void *src, size_t bytes) {
        if (e == hipSuccess) e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        return e == hipSuccess;
    };
    const int bs = 256;
    const int64_t maxh = AF_BLAT_LONG_HITS, maxcl = AF_BLAT_LONG_CLUMPS;
    RegL *parts[2] = {nullptr, nullptr};
    int32_t nparts[2] = {0, 0};
    int32_t host_caps[3] = {0, 0, 0};
    int32_t capped_mask = 0;  // strands whose parts cap bound
    for (int st = 0; st < 2; ++st) {
        const uint8_t *Q = d_q2 + (int64_t)st * L;
        uint32_t *lo = (uint32_t *)dalloc(sizeof(uint32_t) * (L + 1));
        int64_t *cnt = (int64_t *)dalloc(sizeof(int64_t) * (L + 1));
        int64_t *base = (int64_t *)dalloc(sizeof(int64_t) * (L + 1));
        if (e != hipSuccess) return finish(e);
        hipLaunchKernelGGL(lk_count, grid(L + 1), dim3(bs), 0, s, X, Q, L, bp.rep_match, lo, cnt);
        size_t tb = 0;
        (void)hipcub::DeviceScan::ExclusiveSum(nullptr, tb, cnt, base, L + 1);
        void *tmp = dalloc(tb);
        if (e != hipSuccess) return finish(e);
        if ((e = hipcub::DeviceScan::ExclusiveSum(tmp, tb, cnt, base, L + 1, s)) != hipSuccess) return finish(e);
        int64_t all = 0;
        if (!d2h(&all, base + L, sizeof(int64_t))) return finish(e);
        if (all > maxh) host_caps[0] += 1;
        const int64_t nh = std::min(all, maxh);
        if (nh == 0) continue;
        uint64_t *k0 = (uint64_t *)dalloc(sizeof(uint64_t) * nh), *k1 = (uint64_t *)dalloc(sizeof(uint64_t) * nh);
        if (e != hipSuccess) return finish(e);
        hipLaunchKernelGGL(lk_hits, grid(nh), dim3(bs), 0, s, X, L, lo, base, nh, k0);
        const int dbits = 64 - __builtin_clzll((unsigned long long)(X.n + DIAG0));
        tb = 0;
        (void)hipcub::DeviceRadixSort::SortKeys(nullptr, tb, k0, k1, (int)nh, 0, QBITS + dbits);
        void *tmp2 = dalloc(tb);
        if (e != hipSuccess) return finish(e);
        if ((e = hipcub::DeviceRadixSort::SortKeys(tmp2, tb, k0, k1, (int)nh, 0, QBITS + dbits, s)) != hipSuccess)
            return finish(e);
        // runs and ranges
        uint8_t *rflag = (uint8_t *)dalloc(nh), *gflag = (uint8_t *)dalloc(nh);
        int64_t *starts = (int64_t *)dalloc(sizeof(int64_t) * nh), *rs = (int64_t *)dalloc(sizeof(int64_t) * nh);
        int64_t *nsel = (int64_t *)dalloc(sizeof(int64_t) * 2);
        if (e != hipSuccess) return finish(e);
        hipLaunchKernelGGL(lk_flags, grid(nh), dim3(bs), 0, s, k1, nh, (int64_t)bp.max_gap + 2, rflag, gflag);
        tb = 0;
        (void)hipcub::DeviceSelect::Flagged(nullptr, tb, hipcub::CountingInputIterator<int64_t>(0), rflag, starts, nsel, nh);
        void *tmp3 = dalloc(tb);
        if (e != hipSuccess) return finish(e);
        if ((e = hipcub::DeviceSelect::Flagged(tmp3, tb, hipcub::CountingInputIterator<int64_t>(0), rflag, starts, nsel,
                                               nh, s)) != hipSuccess ||
            (e = hipcub::DeviceSelect::Flagged(tmp3, tb, hipcub::CountingInputIterator<int64_t>(0), gflag, rs, nsel + 1,
                                               nh, s)) != hipSuccess)
            return finish(e);
        int64_t nn[2] = {0, 0};
        if (!d2h(nn, nsel, sizeof nn)) return finish(e);
        const int64_t nrun = nn[0], nrs = nn[1];
        // clumps (the first maxcl in diagonal order), ordered (hits desc, diagonal)
        ClumpL *all_cl = (ClumpL *)dalloc(sizeof(ClumpL) * nrun);
        uint8_t *keep = (uint8_t *)dalloc(nrun);
        ClumpL *cl = (ClumpL *)dalloc(sizeof(ClumpL) * nrun);
        if (e != hipSuccess) return finish(e);
        hipLaunchKernelGGL(lk_clumps, grid(nrun), dim3(bs), 0, s, nh, starts, nrun, bp.min_match, all_cl, keep);
        tb = 0;
        (void)hipcub::DeviceSelect::Flagged(nullptr, tb, all_cl, keep, cl, nsel, nrun);
        void *tmp4 = dalloc(tb);
        if (e != hipSuccess) return finish(e);
        if ((e = hipcub::DeviceSelect::Flagged(tmp4, tb, all_cl, keep, cl, nsel, nrun, s)) != hipSuccess) return finish(e);
        int64_t nk = 0;
        if (!d2h(&nk, nsel, sizeof(int64_t))) return finish(e);
        if (nk >= maxcl) host_caps[1] += 1;  // oracle: the clump loop stops at maxcl
        const int64_t ncl = std::min(nk, maxcl);
        if (ncl == 0) continue;
        uint64_t *ck0 = (uint64_t *)dalloc(sizeof(uint64_t) * ncl), *ck1 = (uint64_t *)dalloc(sizeof(uint64_t) * ncl);
        int32_t *iv0 = (int32_t *)dalloc(sizeof(int32_t) * ncl), *co = (int32_t *)dalloc(sizeof(int32_t) * ncl);
        if (e != hipSuccess) return finish(e);
        hipLaunchKernelGGL(lk_clump_keys, grid(ncl), dim3(bs), 0, s, cl, ncl, ck0, iv0);
        tb = 0;
        (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tb, ck0, ck1, iv0, co, (int)ncl, 0, 64);
        void *tmp5 = dalloc(tb);
        if (e != hipSuccess) return finish(e);
        if ((e = hipcub::DeviceRadixSort::SortPairs(tmp5, tb, ck0, ck1, iv0, co, (int)ncl, 0, 64, s)) != hipSuccess)
            return finish(e);
        // the ranges of the clumps in clump order
        int64_t *rk0 = (int64_t *)dalloc(sizeof(int64_t) * (ncl + 1)), *rcnt = (int64_t *)dalloc(sizeof(int64_t) * (ncl + 1));
        int64_t *roff = (int64_t *)dalloc(sizeof(int64_t) * (ncl + 1));
        if (e != hipSuccess) return finish(e);
        hipLaunchKernelGGL(lk_clump_ranges, grid(ncl + 1), dim3(bs), 0, s, cl, co, ncl, rs, nrs, rk0, rcnt);
        tb = 0;
        (void)hipcub::DeviceScan::ExclusiveSum(nullptr, tb, rcnt, roff, ncl + 1);
        void *tmp6 = dalloc(tb);
        if (e != hipSuccess) return finish(e);
        if ((e = hipcub::DeviceScan::ExclusiveSum(tmp6, tb, rcnt, roff, ncl + 1, s)) != hipSuccess) return finish(e);
        int64_t nr = 0;
        if (!d2h(&nr, roff + ncl, sizeof(int64_t))) return finish(e);
        if (nr == 0) continue;
        int64_t *rl = (int64_t *)dalloc(sizeof(int64_t) * nr);
        RegL *hsp = (RegL *)dalloc(sizeof(RegL) * nr);
        int64_t *tbk = (int64_t *)dalloc(sizeof(int64_t) * nr), *tbs = (int64_t *)dalloc(sizeof(int64_t) * nr);
        int32_t *tbv = (int32_t *)dalloc(sizeof(int32_t) * nr), *tbo = (int32_t *)dalloc(sizeof(int32_t) * nr);
        int64_t *span = (int64_t *)dalloc(sizeof(int64_t) * nr), *maxspan = (int64_t *)dalloc(sizeof(int64_t));
        uint8_t *state = (uint8_t *)dalloc(nr);
        int32_t *nund = (int32_t *)dalloc(sizeof(int32_t));
        if (e != hipSuccess) return finish(e);
        hipLaunchKernelGGL(lk_range_list, grid(ncl), dim3(bs), 0, s, ncl, rk0, rcnt, roff, rl);
        hipLaunchKernelGGL(lk_hsp, grid(nr), dim3(bs), 0, s, X, Q, L, k1, nh, rs, nrs, rl, nr, hsp, tbk, tbv, span);
        // the HSPs by target start, the longest target span
        tb = 0;
        size_t tb2 = 0;
        (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tb, tbk, tbs, tbv, tbo, (int)nr, 0, 64);
        (void)hipcub::DeviceReduce::Max(nullptr, tb2, span, maxspan, (int)nr);
        void *tmp7 = dalloc(std::max(tb, tb2));
        if (e != hipSuccess) return finish(e);
        if ((e = hipcub::DeviceRadixSort::SortPairs(tmp7, tb, tbk, tbs, tbv, tbo, (int)nr, 0, 64, s)) != hipSuccess ||
            (e = hipcub::DeviceReduce::Max(tmp7, tb2, span, maxspan, (int)nr, s)) != hipSuccess ||
            (e = hipMemsetAsync(state, 0, nr, s)) != hipSuccess)
            return finish(e);
        // the keep rule, round by round (each round decides at least the first undecided range)
        for (;;) {
            if ((e = hipMemsetAsync(nund, 0, sizeof(int32_t), s)) != hipSuccess) return finish(e);
            hipLaunchKernelGGL(lk_keep_round, grid(nr), dim3(bs), 0, s, hsp, nr, tbs, tbo, maxspan, state, nund);
            int32_t left = 0;
            if ((e = hipGetLastError()) != hipSuccess || !d2h(&left, nund, sizeof left)) return finish(e);
            if (left == 0) break;
        }
        // the first maxcl kept HSPs in range order become the strand's parts
        int64_t *one = (int64_t *)dalloc(sizeof(int64_t) * nr), *cum = (int64_t *)dalloc(sizeof(int64_t) * nr);
        uint8_t *kflag = (uint8_t *)dalloc(nr);
        parts[st] = (RegL *)dalloc(sizeof(RegL) * std::min(nr, maxcl));
        if (e != hipSuccess) return finish(e);
        hipLaunchKernelGGL(lk_is_kept, grid(nr), dim3(bs), 0, s, state, nr, one);
        tb = 0;
        (void)hipcub::DeviceScan::InclusiveSum(nullptr, tb, one, cum, (int)nr);
        void *tmp8 = dalloc(tb);
        if (e != hipSuccess) return finish(e);
        if ((e = hipcub::DeviceScan::InclusiveSum(tmp8, tb, one, cum, (int)nr, s)) != hipSuccess) return finish(e);
        hipLaunchKernelGGL(lk_kept_flags, grid(nr), dim3(bs), 0, s, state, cum, nr, maxcl, kflag);
        int64_t nkept = 0;
        if (!d2h(&nkept, cum + nr - 1, sizeof(int64_t))) return finish(e);
        if (nkept > maxcl) { host_caps[2] += 1; capped_mask |= 1 << st; }
        tb = 0;
        (void)hipcub::DeviceSelect::Flagged(nullptr, tb, hsp, kflag, parts[st], nsel, (int)nr);
        void *tmp9 = dalloc(tb);
        if (e != hipSuccess) return finish(e);
        if ((e = hipcub::DeviceSelect::Flagged(tmp9, tb, hsp, kflag, parts[st], nsel, (int)nr, s)) != hipSuccess)
            return finish(e);
        nparts[st] = (int32_t)std::min(nkept, maxcl);
    }
    const int64_t np = (int64_t)nparts[0] + nparts[1];
    if (np > 0) {
        // both strands' parts side by side (strand 1 from nparts[0]); DP order (qb, tb, qe), ties in
        // creation order (two stable passes); the te window of each strand
        RegL *pall = (RegL *)dalloc(sizeof(RegL) * np);
        int32_t *ord = (int32_t *)dalloc(sizeof(int32_t) * np), *tev = (int32_t *)dalloc(sizeof(int32_t) * np);
        uint64_t *tes = (uint64_t *)dalloc(sizeof(uint64_t) * np);
        int32_t *d_np = (int32_t *)dalloc(sizeof(int32_t) * 2);
        if (e != hipSuccess) return finish(e);
        for (int st = 0; st < 2; ++st)
            if (nparts[st] && (e = hipMemcpyAsync(pall + (st ? nparts[0] : 0), parts[st], sizeof(RegL) * nparts[st],
                                                  hipMemcpyDeviceToDevice, s)) != hipSuccess)
                return finish(e);
        if ((e = hipMemcpyAsync(d_np, nparts, sizeof nparts, hipMemcpyHostToDevice, s)) != hipSuccess) return finish(e);
        for (int st = 0; st < 2; ++st) {
            const int n = nparts[st];
            if (n == 0) continue;
            const int64_t off = st ? nparts[0] : 0;
            uint64_t *a0 = (uint64_t *)dalloc(8 * n), *a1 = (uint64_t *)dalloc(8 * n), *l0 = (uint64_t *)dalloc(8 * n),
                     *l1 = (uint64_t *)dalloc(8 * n);
            int32_t *i0 = (int32_t *)dalloc(4 * n), *i1 = (int32_t *)dalloc(4 * n), *tv0 = (int32_t *)dalloc(4 * n);
            if (e != hipSuccess) return finish(e);
            hipLaunchKernelGGL(lk_ord_keys, grid(n), dim3(bs), 0, s, pall + off, n, a0, l0, i0);
            size_t tb = 0, tb2 = 0;
            (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tb, l0, l1, i0, i1, n, 0, 64);
            (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tb2, a0, a1, i1, ord + off, n, 0, 64);
            void *tmp = dalloc(std::max(tb, tb2));
            if (e != hipSuccess) return finish(e);
            if ((e = hipcub::DeviceRadixSort::SortPairs(tmp, tb, l0, l1, i0, i1, n, 0, 64, s)) != hipSuccess)
                return finish(e);
            // the (qb, tb) pass keyed by the positions the first pass left
            hipLaunchKernelGGL(lk_gather_keys, grid(n), dim3(bs), 0, s, a0, i1, n, a1);
            if ((e = hipcub::DeviceRadixSort::SortPairs(tmp, tb2, a1, a0, i1, ord + off, n, 0, 64, s)) != hipSuccess)
                return finish(e);
            // the te window: (te, DP position) ascending
            hipLaunchKernelGGL(lk_te_keys, grid(n), dim3(bs), 0, s, pall + off, ord + off, n, l0, tv0);
            if ((e = hipcub::DeviceRadixSort::SortPairs(tmp, tb, l0, tes + off, tv0, tev + off, n, 0, 64, s)) != hipSuccess)
                return finish(e);
        }
        // chains, one wave per strand
        const int nmax = std::max(nparts[0], nparts[1]);
        const int64_t wb = (((int64_t)8 * nmax + L + 64) * 4 + 64 + (int64_t)8 * (nmax + 2) + (int64_t)8 * (nmax / 64 + 2) +
                            255) & ~(int64_t)255;
        uint8_t *wk = (uint8_t *)dalloc(2 * wb);
        const int64_t rows_cap = 1 << 16, blk_cap = 1 << 22;
        RowsL R;
        R.rows = (af_psl *)dalloc(sizeof(af_psl) * rows_cap);
        R.seq = (int32_t *)dalloc(sizeof(int32_t) * rows_cap);
        R.boff = (int64_t *)dalloc(sizeof(int64_t) * rows_cap);
        R.blk = (Blk *)dalloc(sizeof(Blk) * blk_cap);
        R.n_rows = (int32_t *)dalloc(sizeof(int32_t) * 2);
        R.overflow = R.n_rows + 1;
        R.n_blk = (unsigned long long *)dalloc(sizeof(unsigned long long));
        R.rows_cap = rows_cap; R.blk_cap = blk_cap; R.caps = caps;
        if (e != hipSuccess) return finish(e);
        if ((e = hipMemsetAsync(R.n_rows, 0, 2 * sizeof(int32_t), s)) != hipSuccess ||
            (e = hipMemsetAsync(R.n_blk, 0, sizeof(unsigned long long), s)) != hipSuccess)
            return finish(e);
        hipLaunchKernelGGL(lk_chain, dim3(2), dim3(64), 0, s, X, d_q2, L, bp, pall, ord, tes, tev, d_np, (int64_t)nparts[0],
                           wk, wb, R, capped_mask);
        int32_t nr2[2] = {0, 0};
        unsigned long long nblk = 0;
        if ((e = hipGetLastError()) != hipSuccess || !d2h(nr2, R.n_rows, sizeof nr2) || !d2h(&nblk, R.n_blk, 8))
            return finish(e);
        if (nr2[1]) {
            *overflow = 1;
            return finish(hipSuccess);
        }
        const int32_t nrows = nr2[0];
        rows.resize(nrows);
        seq.resize(nrows);
        boff.resize(nrows);
        std::vector<Blk> hb(nblk);
        if ((nrows && (!d2h(rows.data(), R.rows, sizeof(af_psl) * nrows) || !d2h(seq.data(), R.seq, 4 * nrows) ||
                       !d2h(boff.data(), R.boff, 8 * nrows))) ||
            (nblk && !d2h(hb.data(), R.blk, sizeof(Blk) * nblk)))
            return finish(e);
        blocks.resize(nblk);
        for (size_t k = 0; k < nblk; ++k) blocks[k] = af_psl_block{hb[k].sz, hb[k].q, hb[k].t};
    }
    if (host_caps[0] || host_caps[1] || host_caps[2]) {
        int32_t cur[3];
        if (!d2h(cur, caps, sizeof cur)) return finish(e);
        for (int k = 0; k < 3; ++k) cur[k] += host_caps[k];
        if ((e = hipMemcpyAsync(caps, cur, sizeof cur, hipMemcpyHostToDevice, s)) != hipSuccess) return finish(e);
    }
    return finish(hipGetLastError());
}
