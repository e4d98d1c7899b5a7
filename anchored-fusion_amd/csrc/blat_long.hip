// blat_long.hip -- one long BLAT query searched whole on the GPU (af_blat_long): the anchor
// transcript, kilobases long, that functions.py:341 (`Find_homo_genes`, homologs vs the genome) and
// fn:966 (`Build_candidate_fasta`, the anchor vs the candidate blocks) hand BLAT as one query.
//
// The algorithm is k_blat's (blat.hip; contract oracle/blat.c afo_blat_long, bit-exact): every
// 11-mer of the query and of its reverse complement looked up, hits sorted by diagonal, clumps of
// >= min_match hits, one part per clump (ordered by hits, then diagonal) whose seed lies in no
// earlier part -- ksw_extend2 both ways from the seed tile (match 1, mismatch 1, gap 3 + 1, band
// 16, z-drop 20) and a banded global alignment for its blocks -- then the chain DP over the parts
// and every chain passing -minScore / -minIdentity as a row.  What differs is the size: a query
// of up to AF_BLAT_LONG_MAX bases, so
//   - the hits of a strand (up to 4 M: 1.7 M for a 6.8 kb anchor against hg38 at step 3) are
//     listed by a thread per hit and sorted by hipCUB, the clumps made a thread per run;
//   - every clump is aligned at once, one wave per clump (lk_align): the DPs keep their cells in
//     lanes sliding along the band (a row's <= 2w + 1 columns), their (h, e) state and traceback in
//     the wave's global scratch, so no row of the query needs to fit a wave; the parts the serial
//     rule then skips (a seed inside an earlier part) are discarded by lk_keep, which walks the
//     clumps in order as k_blat does;
//   - a part holds up to AF_BLAT_LONG_PART_BLOCKS blocks and a row any number (a 23-exon anchor's
//     locus is one row with 23 blocks), kept in a block arena.
// Rows come back unsorted with their strand and emission order; the host orders them (score desc,
// strand, tStart, qStart, tEnd, qEnd; then emission) -- a handful per gene.
#include <algorithm>
#include <vector>

#include <hipcub/hipcub.hpp>

#pragma clang diagnostic ignored "-Wunneeded-internal-declaration"  // ksw_dp.h's DPs this file does not use
#include "ksw_dp.h"

namespace {

constexpr int TILE = AF_TILE;
constexpr int QBITS = 17;                       // query offsets < 2^17 (AF_BLAT_LONG_MAX)
constexpr int64_t DIAG0 = (int64_t)1 << QBITS;  // diagonal + DIAG0 >= 0
constexpr int LPB = AF_BLAT_LONG_PART_BLOCKS;
constexpr int CIG_CAP = 2 * LPB + 1;
constexpr int64_t STITCH_WORK = 1 << 24;        // blat.hip / oracle/blat.c: the same budget
constexpr int NEG = -0x40000000;
static_assert(AF_BLAT_LONG_MAX <= (1 << QBITS), "query offsets in the hit keys");

struct Blk { int32_t sz, q; int64_t t; };
// one part: fields as blat.hip's Reg, blocks in the part pool (b0 = its first block, trimmed by chains)
struct RegL {
    int32_t qb, qe, score, matches, mismatches, ncount, qni, qbi, tni, tbi, nb, ok;
    int64_t tb, te;
};

__device__ __forceinline__ int sc_blat(uint8_t x, uint8_t y) { return (x > 3 || y > 3) ? -1 : (x == y ? 1 : -1); }

// exclusive prefix max over the lanes, `carry` below lane 0
__device__ __forceinline__ int excl_max(int v, int carry) {
    const int inc = wave_incl_max(v);
    return max(carry, wave_shr1(kMaxId, inc));
}

// ---- hits, clumps -------------------------------------------------------------------------------
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

__device__ __forceinline__ int64_t key_diag(uint64_t k) { return (int64_t)(k >> QBITS) - DIAG0; }

// run starts over the diagonal-sorted keys (a diagonal step > max_gap + 2 starts a run)
__global__ void lk_run_flags(const uint64_t *__restrict__ keys, int64_t nh, int64_t drift, uint8_t *__restrict__ flag) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nh) return;
    flag[i] = (i == 0 || key_diag(keys[i]) - key_diag(keys[i - 1]) > drift) ? 1 : 0;
}

struct ClumpL { int32_t cnt, q; int64_t t; };
// run r -> a clump when it holds >= min_match hits: its hit count and least (offset, position) hit
__global__ void lk_clumps(const uint64_t *__restrict__ keys, int64_t nh, const int64_t *__restrict__ starts,
                          int64_t nrun, int32_t min_match, ClumpL *__restrict__ cl, uint8_t *__restrict__ keep) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nrun) return;
    const int64_t s0 = starts[r], e0 = r + 1 < nrun ? starts[r + 1] : nh;
    ClumpL c{};
    keep[r] = e0 - s0 >= min_match ? 1 : 0;
    if (keep[r]) {
        int32_t bq = 1 << 30;
        int64_t bt = 0;
        for (int64_t i = s0; i < e0; ++i) {
            const int32_t q = (int32_t)(keys[i] & ((1u << QBITS) - 1));
            const int64_t t = key_diag(keys[i]) + q;
            if (q < bq || (q == bq && t < bt)) { bq = q; bt = t; }
        }
        c.cnt = (int32_t)(e0 - s0); c.q = bq; c.t = bt;
    }
    cl[r] = c;
}

// the low 32 bits of keys (a sort's values)
__global__ void lk_low_words(const uint64_t *__restrict__ k, int64_t n, int32_t *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = (int32_t)(uint32_t)k[i];
}
// out[p] = keys[perm[p]]
__global__ void lk_gather_keys(const uint64_t *__restrict__ keys, const int32_t *__restrict__ perm, int n,
                               uint64_t *__restrict__ out) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < n) out[p] = keys[perm[p]];
}
// ord[k] = the part index of kept entry perm[k]
__global__ void lk_map_ord(const int32_t *__restrict__ kept, const int32_t *__restrict__ perm, int n,
                           int32_t *__restrict__ ord) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n) ord[k] = kept[perm[k]];
}

// clump order keys: hits desc, then diagonal (= the clump's index in diagonal order)
__global__ void lk_clump_keys(const ClumpL *__restrict__ cl, int64_t ncl, uint64_t *__restrict__ k) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ncl) return;
    k[i] = ((uint64_t)(0xFFFFFFu - (uint32_t)min(cl[i].cnt, 0xFFFFFF)) << 32) | (uint64_t)i;
}

// ---- the DPs of one part on one wave --------------------------------------------------------------
// per-wave scratch for a query of length L (bytes): reversed query / target, (h, e) row, traceback,
// CIGAR ops
struct DpMem {
    uint8_t *qs, *ts, *z;
    int2 *eh;
    uint32_t *ops;
    int64_t z_cap;
};
__host__ __device__ inline int64_t dp_mem_bytes(int L) {
    const int64_t zc = (int64_t)(L + 160) * 160;
    return ((int64_t)L + 64 + 256) + ((int64_t)L + 256 + 64) + 8 * ((int64_t)L + 8) + zc + 4 * (2 * (int64_t)L + 512) + 512;
}
__device__ DpMem dp_mem(uint8_t *base, int L) {
    DpMem m;
    m.qs = base;
    m.ts = m.qs + (L + 64 + 256);
    m.eh = reinterpret_cast<int2 *>(((uintptr_t)(m.ts + L + 256 + 64) + 15) & ~(uintptr_t)15);
    m.z = reinterpret_cast<uint8_t *>(m.eh + L + 8);
    m.z_cap = (int64_t)(L + 160) * 160;
    m.ops = reinterpret_cast<uint32_t *>(((uintptr_t)(m.z + m.z_cap) + 15) & ~(uintptr_t)15);
    return m;
}

struct ExtL { int max, qle, tle, gtle, gscore; };

// ksw_extend2 (oracle afo_ext_dp) with match 1, mismatch 1, gap o + e (del and ins alike): target
// rows i, query columns j; lanes over the row's columns [beg, end) (chunks of 64), the (h, e) row in
// eh (columns above hw never written: their first-row values)
__device__ ExtL ext_band(int qlen, const uint8_t *query, int tlen, const uint8_t *target, int o, int e, int w, int zdrop,
                         int h0, int2 *eh, int lane) {
    const int oe = o + e;
    {   // band adjustment: the longest gap that can still score
        int mi = (int)((double)(qlen * 1 - o) / e + 1.);
        mi = mi > 1 ? mi : 1;
        w = w < mi ? w : mi;
    }
    const int h1_0 = h0 > oe ? h0 - oe : 0;
    int hw = -1;  // eh[0, hw] written
    int best = h0, max_i = -1, max_j = -1, max_ie = -1, gscore = -1;
    int beg = 0, end = qlen;
    for (int i = 0; i < tlen; ++i) {
        const uint8_t ti = target[i];
        if (beg < i - w) beg = i - w;
        if (end > i + w + 1) end = i + w + 1;
        if (end > qlen) end = qlen;
        int h1 = 0;
        if (beg == 0) { h1 = h0 - (o + e * (i + 1)); if (h1 < 0) h1 = 0; }
        int m = 0, mj = -1, hlast = h1;
        int fcarry = e * beg;  // F scan: max over u_k = g_k + e (k + 1), from e beg
        int hcarry = h1;       // H of the column before the chunk
        int first_nz = -1, last_nz = -1;  // columns in [beg, end) whose (h, e) after the row is non-zero
        for (int c0 = beg; c0 < end; c0 += 64) {
            const int j = c0 + lane;
            const bool v = j < end;
            int2 s = make_int2(0, 0);
            if (v) {
                if (j <= hw) s = eh[j];
                else s = make_int2(j == 0 ? h0 : (j == 1 ? h1_0 : max(h1_0 - e * (j - 1), 0)), 0);
            }
            int M = s.x ? s.x + sc_blat(ti, query[j]) : 0;
            const int g = max(M - oe, 0);
            const int u = v ? g + e * (j + 1) : kMaxId;
            const int fin = excl_max(u, fcarry) - e * j;
            int h = max(max(M, s.y), v ? fin : 0);
            int en = max(s.y - e, max(M - oe, 0));
            // row max (h >= 0 here: M >= 0 as mismatches cost 1) and the last column holding it
            const int cm = wave_max(v ? h : -1);
            if (cm >= m) {
                m = cm;
                mj = c0 + 63 - (int)__builtin_clzll(__ballot(v && h == cm));
            }
            // eh[j].h = H(i, j - 1): the lane below's h (the chunk's first: the carry)
            const int hprev = max(wave_shr1(kMaxId, h), lane == 0 ? hcarry : kMaxId);
            if (v) eh[j] = make_int2(hprev, en);
            const uint64_t nzb = __ballot(v && (hprev != 0 || en != 0));
            if (nzb) {
                if (first_nz < 0) first_nz = c0 + (int)__builtin_ctzll(nzb);
                last_nz = c0 + 63 - (int)__builtin_clzll(nzb);
            }
            const int top = min(63, end - 1 - c0);
            hcarry = __builtin_amdgcn_readlane(h, top);
            hlast = hcarry;
            fcarry = max(fcarry, wave_max(u));
        }
        wave_sync();
        if (lane == 0) eh[end] = make_int2(hlast, 0);
        if (end > hw) hw = end;
        wave_sync();
        if ((beg < end ? end : beg) == qlen) {  // the loop's j == qlen
            max_ie = gscore > hlast ? max_ie : i;
            gscore = gscore > hlast ? gscore : hlast;
        }
        if (m == 0) break;
        if (m > best) {
            best = m; max_i = i; max_j = mj;
        } else if (zdrop > 0) {
            if (i - max_i > mj - max_j) {
                if (best - m - ((i - max_i) - (mj - max_j)) * e > zdrop) break;
            } else {
                if (best - m - ((mj - max_j) - (i - max_i)) * e > zdrop) break;
            }
        }
        // beg: the first column in [beg, end) with a non-zero (h, e); end: the last one in [beg, end] + 2
        const bool end_nz = hlast != 0;  // eh[end] = (hlast, 0)
        beg = first_nz >= 0 ? first_nz : end;
        const int jl = end_nz ? end : (last_nz >= 0 ? last_nz : beg - 1);
        end = jl + 2 < qlen ? jl + 2 : qlen;
    }
    ExtL r;
    r.max = best; r.qle = max_j + 1; r.tle = max_i + 1; r.gtle = max_ie + 1; r.gscore = gscore;
    return r;
}

// ksw_global2 (oracle afo_global_dp) with traceback bits in z (row i at z[i * ncol]); returns the
// CIGAR ops in forward order at ops, their count (all of them; at most cap kept) in *n_ops
__device__ int global_band(int qlen, const uint8_t *query, int tlen, const uint8_t *target, int o, int e, int w,
                           int2 *eh, uint8_t *z, uint32_t *ops, int cap, int *n_ops, int lane) {
    const int oe = o + e;
    const int ncol = qlen < 2 * w + 1 ? qlen : 2 * w + 1;
    int hw = -1;
    for (int i = 0; i < tlen; ++i) {
        const uint8_t ti = target[i];
        const int beg = i > w ? i - w : 0;
        const int end = i + w + 1 < qlen ? i + w + 1 : qlen;
        const int h1 = beg == 0 ? -(o + e * (i + 1)) : NEG;
        int fcarry = NEG + e * beg, hcarry = h1, hlast = h1;
        uint8_t *zi = z + (int64_t)i * ncol;
        for (int c0 = beg; c0 < end; c0 += 64) {
            const int j = c0 + lane;
            const bool v = j < end;
            int2 s = make_int2(NEG, NEG);
            if (v) {
                if (j <= hw) s = eh[j];
                else if (j == 0) s = make_int2(0, NEG);
                else if (j <= w) s = make_int2(-(o + e * j), NEG);
            }
            const int m = s.x + sc_blat(ti, query[j]);
            const int u = v ? m - oe + e * (j + 1) : kMaxId;
            const int f = excl_max(u, fcarry) - e * j;
            uint8_t d = m >= s.y ? 0 : 1;
            int h = m >= s.y ? m : s.y;
            d = h >= f ? d : 2;
            h = h >= f ? h : f;
            int t = m - oe;
            int en = s.y - e;
            d |= en > t ? 1 << 2 : 0;
            en = en > t ? en : t;
            t = m - oe;
            d |= (f - e) > t ? 2 << 4 : 0;
            const int hprev = max(wave_shr1(kMaxId, h), lane == 0 ? hcarry : kMaxId);
            if (v) {
                eh[j] = make_int2(hprev, en);
                zi[j - beg] = d;
            }
            const int top = min(63, end - 1 - c0);
            hcarry = __builtin_amdgcn_readlane(h, top);
            hlast = hcarry;
            fcarry = max(fcarry, wave_max(u));
        }
        wave_sync();
        if (lane == 0) eh[end] = make_int2(hlast, NEG);
        if (end > hw) hw = end;
        wave_sync();
    }
    int score = 0;
    if (lane == 0) {
        int2 s = make_int2(NEG, NEG);
        if (qlen <= hw) s = eh[qlen];
        else if (qlen == 0) s = make_int2(0, NEG);
        else if (qlen <= w) s = make_int2(-(o + e * qlen), NEG);
        score = s.x;
        // backtrack from the last cell; ops pushed in reverse at ops[0..], then flipped
        int nc = 0, which = 0, i = tlen - 1;
        int k = (i + w + 1 < qlen ? i + w + 1 : qlen) - 1;
        auto push = [&](int op, int len) {
            if (nc > 0 && (int)(ops[nc - 1] & 0xf) == op) ops[nc - 1] += (uint32_t)len << 4;
            else ops[nc++] = (uint32_t)len << 4 | (uint32_t)op;
        };
        while (i >= 0 && k >= 0) {
            which = z[(int64_t)i * ncol + (k - (i > w ? i - w : 0))] >> (which << 1) & 3;
            if (which == 0) { push(0, 1); --i; --k; }
            else if (which == 1) { push(2, 1); --i; }
            else { push(1, 1); --k; }
        }
        if (i >= 0) push(2, i + 1);
        if (k >= 0) push(1, k + 1);
        for (int a = 0, b = nc - 1; a < b; ++a, --b) { const uint32_t x = ops[a]; ops[a] = ops[b]; ops[b] = x; }
        *n_ops = nc;
        (void)cap;
    }
    score = __builtin_amdgcn_readfirstlane(score);
    wave_sync();
    return score;
}

__device__ __forceinline__ int infer_bw_l(int l1, int l2, int score, int q, int r) {
    if (l1 == l2 && l1 - score < (q + r - 1) << 1) return 0;
    int w = (int)((double)((l1 < l2 ? l1 : l2) - score - q) / r + 2.);
    const int d = l1 - l2 < 0 ? l2 - l1 : l1 - l2;
    return w < d ? d : w;
}

// one clump seed (q, t) of the strand's codes Q (length L) -> part P with its blocks at B[0, LPB)
__device__ void align_part(const DevTile &X, const uint8_t *Q, int L, int32_t q, int64_t t, RegL *P, Blk *B,
                           const DpMem &M, int lane) {
    const int o = 3, e = 1, w = 16, zdrop = 20;
    int score, truesc, qb, qe;
    int64_t tb, te;
    if (q > 0) {
        const int tl = (int)(t < q + w ? t : q + w);
        for (int x = lane; x < q; x += 64) M.qs[x] = Q[q - 1 - x];
        for (int x = lane; x < tl; x += 64) M.ts[x] = X.T[t - 1 - x];
        wave_sync();
        const ExtL r = ext_band(q, M.qs, tl, M.ts, o, e, w, zdrop, TILE, M.eh, lane);
        score = r.max;
        if (r.gscore <= 0 || r.gscore <= score) { qb = q - r.qle; tb = t - r.tle; truesc = score; }
        else { qb = 0; tb = t - r.gtle; truesc = r.gscore; }
    } else {
        score = truesc = TILE; qb = 0; tb = t;
    }
    if (q + TILE < L) {
        const int qs0 = q + TILE;
        const int64_t t0 = t + TILE, room = X.n - t0;
        const int tl = (int)(room < (L - qs0) + w ? room : (int64_t)(L - qs0) + w);
        const int sc0 = score;
        const ExtL r = ext_band(L - qs0, Q + qs0, tl, X.T + t0, o, e, w, zdrop, sc0, M.eh, lane);
        score = r.max;
        if (r.gscore <= 0 || r.gscore <= score) { qe = qs0 + r.qle; te = t0 + r.tle; truesc += score - sc0; }
        else { qe = L; te = t0 + r.gtle; truesc += r.gscore - sc0; }
    } else {
        qe = L; te = t + TILE;
    }
    RegL out{};
    const int lq = qe - qb, rl = (int)(te - tb);
    if (lq <= 0 || rl <= 0) {
        if (lane == 0) *P = out;
        return;
    }
    int w2 = infer_bw_l(lq, rl, truesc, o, e);
    w2 = w2 < 64 ? w2 : 64;
    // bwa_gen_cigar2 (no reversal: the text is not doubled)
    int nc = 0;
    if (lq == rl && w2 == 0) {
        nc = 1;
        if (lane == 0) M.ops[0] = (uint32_t)lq << 4;
    } else {
        int max_gap = (int)((double)(((lq + 1) >> 1) - o) / e + 1.);
        max_gap = max_gap > 1 ? max_gap : 1;
        const int d = rl - lq < 0 ? lq - rl : rl - lq;
        int wg = (max_gap + d + 1) >> 1;
        wg = wg < w2 ? wg : w2;
        wg = wg > d + 3 ? wg : d + 3;
        int n = 0;
        if ((int64_t)rl * (lq < 2 * wg + 1 ? lq : 2 * wg + 1) > M.z_cap) {  // never at band 64 (scratch sized for it)
            if (lane == 0) *P = out;
            return;
        }
        global_band(lq, Q + qb, rl, X.T + tb, o, e, wg, M.eh, M.z, M.ops, CIG_CAP, &n, lane);
        nc = __builtin_amdgcn_readfirstlane(n);
    }
    wave_sync();
    if (nc > CIG_CAP) {
        if (lane == 0) *P = out;
        return;
    }
    // blocks: leading / trailing D trimmed from the target span; per block the match counts
    int xs = 0, xe = nc;
    const uint32_t f0 = M.ops[0], fl = M.ops[nc - 1];
    if (nc > 0 && (f0 & 0xf) == 2) { tb += f0 >> 4; xs = 1; }
    else if (nc > 0 && (fl & 0xf) == 2) { te -= fl >> 4; xe = nc - 1; }
    int32_t x = qb;
    int64_t y = tb;
    bool ok = true;
    for (int k = xs; k < xe && ok; ++k) {
        const uint32_t op4 = M.ops[k];
        const int len = (int)(op4 >> 4), op = (int)(op4 & 0xf);
        if (op == 0) {
            if (out.nb >= LPB) { ok = false; break; }
            if (lane == 0) B[out.nb] = Blk{len, x, y};
            ++out.nb;
            int mt = 0, mm = 0, nn = 0;
            for (int u = lane; u < len; u += 64) {
                const uint8_t a = Q[x + u], b = X.T[y + u];
                if (a > 3 || b > 3) ++nn;
                else if (a == b) ++mt;
                else ++mm;
            }
            out.matches += wave_sum(mt); out.mismatches += wave_sum(mm); out.ncount += wave_sum(nn);
            x += len; y += len;
        } else if (op == 1) {
            ++out.qni; out.qbi += len; x += len;
        } else {
            ++out.tni; out.tbi += len; y += len;
        }
    }
    if (out.nb == 0) ok = false;
    out.qb = qb; out.qe = qe; out.tb = tb; out.te = te;
    out.score = out.matches - out.mismatches - out.qni - out.tni;
    out.ok = ok ? 1 : 0;
    if (lane == 0) *P = out;
    wave_sync();
}

// every clump (clump order co) of both strands: one wave per clump (grid-stride)
__global__ __launch_bounds__(64) void lk_align(DevTile X, const uint8_t *__restrict__ Q2, int L,
                                                const ClumpL *__restrict__ cl0, const ClumpL *__restrict__ cl1,
                                                const int32_t *__restrict__ co0, const int32_t *__restrict__ co1,
                                                int64_t n0, int64_t n1, RegL *__restrict__ parts, Blk *__restrict__ pblk,
                                                uint8_t *__restrict__ scratch, int64_t mem_bytes) {
    const int lane = threadIdx.x;
    const DpMem M = dp_mem(scratch + (int64_t)blockIdx.x * mem_bytes, L);
    for (int64_t c = blockIdx.x; c < n0 + n1; c += gridDim.x) {
        const int s = c < n0 ? 0 : 1;
        const int64_t k = s ? c - n0 : c;
        const ClumpL cc = s ? cl1[co1[k]] : cl0[co0[k]];
        align_part(X, Q2 + (int64_t)s * L, L, cc.q, cc.t, parts + c, pblk + c * LPB, M, lane);
    }
}

// the parts the serial rule keeps, per strand (one wave each): clumps in order, a clump whose seed
// lies inside an earlier kept part skipped; kept[s][0, *n_kept[s]) = part indices (creation order)
__global__ __launch_bounds__(64) void lk_keep(const ClumpL *__restrict__ cl0, const ClumpL *__restrict__ cl1,
                                               const int32_t *__restrict__ co0, const int32_t *__restrict__ co1,
                                               int64_t n0, int64_t n1, const RegL *__restrict__ parts,
                                               int32_t *__restrict__ kept, int32_t *__restrict__ n_kept) {
    const int lane = threadIdx.x, s = blockIdx.x;
    const int64_t base = s ? n0 : 0, n = s ? n1 : n0;
    int32_t *K = kept + base;
    int nr = 0;
    for (int64_t c = 0; c < n; ++c) {
        const ClumpL cc = s ? cl1[co1[c]] : cl0[co0[c]];
        bool inside = false;
        for (int r0 = 0; r0 < nr && !inside; r0 += 64) {
            const int r = r0 + lane;
            bool in = false;
            if (r < nr) {
                const RegL &g = parts[K[r]];
                in = g.qb <= cc.q && cc.q + TILE <= g.qe && g.tb <= cc.t && cc.t + TILE <= g.te;
            }
            inside = __ballot(in) != 0;
        }
        if (inside || !parts[base + c].ok) continue;
        if (lane == 0) K[nr] = (int32_t)(base + c);
        ++nr;
        __threadfence_block();
        wave_sync();
    }
    if (lane == 0) n_kept[s] = nr;
}

// the chain DP's sort keys of the kept parts: (qb, tb) and (qe, creation order), for two stable passes
__global__ void lk_ord_keys(const RegL *__restrict__ parts, const int32_t *__restrict__ kept, int n,
                            uint64_t *__restrict__ k_hi, uint64_t *__restrict__ k_lo, int32_t *__restrict__ idx) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const RegL &g = parts[kept[r]];
    k_hi[r] = ((uint64_t)g.qb << 40) | (uint64_t)g.tb;
    k_lo[r] = ((uint64_t)g.qe << 32) | (uint32_t)r;
    idx[r] = r;
}

// ---- chains and rows ---------------------------------------------------------------------------
struct ChainL {
    const RegL *parts;
    const Blk *pblk;
    const int32_t *ord;   // part index at sorted position k
    int32_t *best, *prev, *fl, *ch, *pre;
    int32_t *qe;          // -1 once used
    int64_t *te;
    uint32_t *nxt;        // first N of the target at or after te (0xFFFFFFFF: none)
};

__device__ __forceinline__ uint32_t first_n_l(const DevTile &X, int64_t p) {
    const int64_t b = p >> 6;
    const uint64_t m = X.nmask[b] >> (p & 63);
    return m ? (uint32_t)(p + __builtin_ctzll(m)) : X.nnext[b + 1];
}

// best / prev of sorted part i over the unused parts before it (oracle chain_node)
__device__ void chain_node_l(const DevTile &X, const uint8_t *Q, const ChainL &C, int i, int64_t max_intron, int lane) {
    const RegL &ri = C.parts[C.ord[i]];
    const Blk b0 = C.pblk[(int64_t)C.ord[i] * LPB];
    int carry = 0;
    for (int u0 = 0; u0 < b0.sz; u0 += 64) {
        const int u = u0 + lane;
        int m = 0;
        if (u < b0.sz) {
            const uint8_t a = Q[b0.q + u], b = X.T[b0.t + u];
            m = (a > 3 || b > 3) ? 0 : (a == b ? 1 : -1);
        }
        int inc = m;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int v = __shfl_up(inc, d);
            if (lane >= d) inc += v;
        }
        if (u < b0.sz) C.pre[u] = carry + inc - m;
        carry += __builtin_amdgcn_readlane(inc, 63);
    }
    wave_sync();
    int best = ri.score, prev = -1;
    for (int j0 = 0; j0 < i; j0 += 64) {
        const int j = j0 + lane;
        int v = INT_MIN;
        if (j < i) {
            const int aqe = C.qe[j];
            const int64_t ate = C.te[j];
            if (aqe >= 0 && ri.qe > aqe && ri.te > ate) {
                int64_t kk = aqe - ri.qb;
                if (ate - ri.tb > kk) kk = ate - ri.tb;
                const int k = kk > 0 ? (int)kk : 0;
                const int64_t btb = ri.tb + k;
                if (!(k > 0 && k >= b0.sz) && btb - ate <= max_intron && (int64_t)C.nxt[j] >= btb)
                    v = C.best[j] + (ri.score - (k > 0 ? C.pre[k] : 0)) - (ri.qb + k > aqe) - (btb > ate);
            }
        }
        const int mx = wave_max(v);
        if (mx > best) { best = mx; prev = j0 + (int)__builtin_ctzll(__ballot(v == mx)); }
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
    int32_t *caps;  // the context's af_blat_caps counters
};

// one wave per strand: the chain DP over its kept parts in sorted order, chains best first as rows
__global__ __launch_bounds__(64) void lk_chain(DevTile X, const uint8_t *__restrict__ Q2, int L, af_blat_params bp,
                                                const RegL *__restrict__ parts, const Blk *__restrict__ pblk,
                                                const int32_t *__restrict__ ord_all, const int32_t *__restrict__ n_kept,
                                                int64_t n0, uint8_t *__restrict__ work_all, int64_t work_bytes,
                                                RowsL R) {
    const int lane = threadIdx.x, strand = blockIdx.x;
    const int nr = n_kept[strand];
    const uint8_t *Q = Q2 + (int64_t)strand * L;
    const int32_t *ord = ord_all + (strand ? n0 : 0);
    uint8_t *wk = work_all + strand * work_bytes;
    ChainL C;
    C.parts = parts; C.pblk = pblk; C.ord = ord;
    int32_t *w32 = reinterpret_cast<int32_t *>(wk);
    C.best = w32; C.prev = w32 + nr; C.fl = w32 + 2 * nr; C.ch = w32 + 3 * nr; C.qe = w32 + 4 * nr;
    C.nxt = reinterpret_cast<uint32_t *>(w32 + 5 * nr);
    C.pre = w32 + 6 * nr;
    C.te = reinterpret_cast<int64_t *>(((uintptr_t)(C.pre + L + 64) + 15) & ~(uintptr_t)15);
    for (int r = lane; r < nr; r += 64) {
        const RegL &g = parts[ord[r]];
        C.fl[r] = 0; C.qe[r] = g.qe; C.te[r] = g.te; C.nxt[r] = first_n_l(X, g.te);
    }
    __threadfence_block();
    wave_sync();
    for (int i = 0; i < nr; ++i) chain_node_l(X, Q, C, i, bp.max_intron, lane);
    int64_t work = 0;
    int emitted = 0;
    for (;;) {
        if (work > STITCH_WORK) {
            if (lane == 0) atomicAdd(&R.caps[AF_BLAT_CAP_PARTS], 1);
            break;
        }
        int bv = INT_MIN, bi = -1;
        for (int i0 = 0; i0 < nr; i0 += 64) {
            const int i = i0 + lane;
            const bool free_ = i < nr && !(C.fl[i] & 1);
            if (!__ballot(free_)) continue;
            const int v = free_ ? C.best[i] : INT_MIN;
            const int mx = wave_max(v);
            if (bi < 0 || mx > bv) { bv = mx; bi = i0 + (int)__builtin_ctzll(__ballot(free_ && v == mx)); }
        }
        if (bi < 0) break;
        int first = bi;
        if (lane == 0) {
            int m = 0;
            for (int i = bi; i >= 0; i = C.prev[i]) C.ch[m++] = i;
            first = C.ch[m - 1];
            af_psl o{};
            o.query = 0; o.strand = strand; o.q_size = L;
            // the row's blocks go to a fresh stretch of the arena (count them first)
            int nb = 0;
            for (int c = m - 1; c >= 0; --c) nb += parts[ord[C.ch[c]]].nb;
            const int64_t b0 = (int64_t)atomicAdd(R.n_blk, (unsigned long long)nb);
            int32_t pqe = 0;
            int64_t pte = 0;
            int32_t fqb = 0, lqe = 0;
            int64_t ftb = 0, lte = 0;
            int64_t bo = b0;
            for (int c = m - 1; c >= 0; --c) {
                const int k = C.ch[c];
                C.fl[k] |= 1;
                C.qe[k] = -1;
                const RegL &src = parts[ord[k]];
                const Blk *sb = pblk + (int64_t)ord[k] * LPB;
                int trim = 0;
                if (c < m - 1) {
                    int64_t kk = pqe - src.qb;
                    if (pte - src.tb > kk) kk = pte - src.tb;
                    trim = kk > 0 ? (int)kk : 0;
                    if (trim >= sb[0].sz) trim = 0;  // trim_front refuses; the oracle keeps the part whole
                }
                int mt = src.matches, mm = src.mismatches, nn = src.ncount;
                for (int u = 0; u < trim; ++u) {
                    const uint8_t a = Q[sb[0].q + u], b = X.T[sb[0].t + u];
                    if (a > 3 || b > 3) --nn;
                    else if (a == b) --mt;
                    else --mm;
                }
                // trim_front: the trimmed part starts at its first block's trimmed start
                const int32_t qb_c = trim ? sb[0].q + trim : src.qb;
                const int64_t tb_c = trim ? sb[0].t + trim : src.tb;
                if (c < m - 1) {
                    if (qb_c > pqe) { ++o.q_num_insert; o.q_base_insert += qb_c - pqe; }
                    if (tb_c > pte) { ++o.t_num_insert; o.t_base_insert += (int32_t)(tb_c - pte); }
                }
                o.matches += mt; o.mismatches += mm; o.n_count += nn;
                o.q_num_insert += src.qni; o.q_base_insert += src.qbi;
                o.t_num_insert += src.tni; o.t_base_insert += src.tbi;
                for (int b = 0; b < src.nb; ++b) {
                    Blk bk = sb[b];
                    if (b == 0 && trim) { bk.sz -= trim; bk.q += trim; bk.t += trim; }
                    if (o.block_count < AF_PSL_MAX_BLOCKS) {
                        o.block_sizes[o.block_count] = bk.sz; o.q_starts[o.block_count] = bk.q;
                        o.t_starts[o.block_count] = bk.t;
                    }
                    if (bo < R.blk_cap) R.blk[bo] = bk;
                    ++bo;
                    ++o.block_count;
                }
                if (c == m - 1) { fqb = qb_c; ftb = tb_c; }
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
                const int r = atomicAdd(R.n_rows, 1);
                if (r < R.rows_cap) { R.rows[r] = o; R.seq[r] = emitted; R.boff[r] = b0; }
                ++emitted;
            }
        }
        emitted = __builtin_amdgcn_readfirstlane(emitted);
        first = __builtin_amdgcn_readfirstlane(first);
        __threadfence_block();
        wave_sync();
        // parts after the chain's first whose predecessor is used or recomputed: recomputed in order
        for (int i = first + 1; i < nr; ++i) {
            const int f = C.fl[i];
            if (f & 1) continue;
            const int pv = C.prev[i];
            if (pv >= 0 && C.fl[pv]) {
                chain_node_l(X, Q, C, i, bp.max_intron, lane);
                work += i;
                if (lane == 0) C.fl[i] = 2;
                __threadfence_block();
                wave_sync();
            }
        }
        for (int i = lane; i < nr; i += 64) C.fl[i] &= 1;
        __threadfence_block();
        wave_sync();
    }
}

}  // namespace

// Host-driven search of one long query (codes of both strands in d_q2: strand s at d_q2 + s L).
// Returns hipSuccess or an error; *rc_cap = AF_E_CAPACITY when the row lists overflowed.
hipError_t af_blat_long_run(const DevTile &X, const uint8_t *d_q2, int L, const af_blat_params &bp, int32_t *caps,
                            std::vector<af_psl> &rows, std::vector<int32_t> &seq, std::vector<int64_t> &boff,
                            std::vector<af_psl_block> &blocks, int n_cu, hipStream_t s) {
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
    const int bs = 256;
    const int64_t maxh = AF_BLAT_LONG_HITS, maxcl = AF_BLAT_LONG_CLUMPS;
    ClumpL *cl[2] = {nullptr, nullptr};
    int32_t *co[2] = {nullptr, nullptr};
    int64_t ncl[2] = {0, 0};
    int32_t host_caps[3] = {0, 0, 0};
    for (int st = 0; st < 2; ++st) {
        const uint8_t *Q = d_q2 + (int64_t)st * L;
        uint32_t *lo = (uint32_t *)dalloc(sizeof(uint32_t) * (L + 1));
        int64_t *cnt = (int64_t *)dalloc(sizeof(int64_t) * (L + 1));
        int64_t *base = (int64_t *)dalloc(sizeof(int64_t) * (L + 1));
        if (e != hipSuccess) return finish(e);
        hipLaunchKernelGGL(lk_count, dim3((L + 1 + bs - 1) / bs), dim3(bs), 0, s, X, Q, L, bp.rep_match, lo, cnt);
        size_t tb = 0;
        (void)hipcub::DeviceScan::ExclusiveSum(nullptr, tb, cnt, base, L + 1);
        void *tmp = dalloc(tb);
        if (e != hipSuccess) return finish(e);
        if ((e = hipcub::DeviceScan::ExclusiveSum(tmp, tb, cnt, base, L + 1, s)) != hipSuccess) return finish(e);
        int64_t all = 0;
        if ((e = hipMemcpyAsync(&all, base + L, sizeof(int64_t), hipMemcpyDeviceToHost, s)) != hipSuccess ||
            (e = hipStreamSynchronize(s)) != hipSuccess)
            return finish(e);
        if (all > maxh) host_caps[0] += 1;
        const int64_t nh = std::min(all, maxh);
        if (nh == 0) continue;
        uint64_t *k0 = (uint64_t *)dalloc(sizeof(uint64_t) * nh), *k1 = (uint64_t *)dalloc(sizeof(uint64_t) * nh);
        if (e != hipSuccess) return finish(e);
        hipLaunchKernelGGL(lk_hits, dim3((unsigned)((nh + bs - 1) / bs)), dim3(bs), 0, s, X, L, lo, base, nh, k0);
        const int dbits = 64 - __builtin_clzll((unsigned long long)(X.n + DIAG0));
        tb = 0;
        (void)hipcub::DeviceRadixSort::SortKeys(nullptr, tb, k0, k1, (int)nh, 0, QBITS + dbits);
        void *tmp2 = dalloc(tb);
        if (e != hipSuccess) return finish(e);
        if ((e = hipcub::DeviceRadixSort::SortKeys(tmp2, tb, k0, k1, (int)nh, 0, QBITS + dbits, s)) != hipSuccess)
            return finish(e);
        // runs, then clumps (the first maxcl in diagonal order)
        uint8_t *flag = (uint8_t *)dalloc(nh);
        int64_t *starts = (int64_t *)dalloc(sizeof(int64_t) * nh);
        int64_t *nsel = (int64_t *)dalloc(sizeof(int64_t));
        if (e != hipSuccess) return finish(e);
        hipLaunchKernelGGL(lk_run_flags, dim3((unsigned)((nh + bs - 1) / bs)), dim3(bs), 0, s, k1, nh,
                           (int64_t)bp.max_gap + 2, flag);
        tb = 0;
        (void)hipcub::DeviceSelect::Flagged(nullptr, tb, hipcub::CountingInputIterator<int64_t>(0), flag, starts, nsel, nh);
        void *tmp3 = dalloc(tb);
        if (e != hipSuccess) return finish(e);
        if ((e = hipcub::DeviceSelect::Flagged(tmp3, tb, hipcub::CountingInputIterator<int64_t>(0), flag, starts, nsel,
                                               nh, s)) != hipSuccess)
            return finish(e);
        int64_t nrun = 0;
        if ((e = hipMemcpyAsync(&nrun, nsel, sizeof(int64_t), hipMemcpyDeviceToHost, s)) != hipSuccess ||
            (e = hipStreamSynchronize(s)) != hipSuccess)
            return finish(e);
        ClumpL *all_cl = (ClumpL *)dalloc(sizeof(ClumpL) * nrun);
        uint8_t *keep = (uint8_t *)dalloc(nrun);
        cl[st] = (ClumpL *)dalloc(sizeof(ClumpL) * nrun);
        if (e != hipSuccess) return finish(e);
        hipLaunchKernelGGL(lk_clumps, dim3((unsigned)((nrun + bs - 1) / bs)), dim3(bs), 0, s, k1, nh, starts, nrun,
                           bp.min_match, all_cl, keep);
        tb = 0;
        (void)hipcub::DeviceSelect::Flagged(nullptr, tb, all_cl, keep, cl[st], nsel, nrun);
        void *tmp4 = dalloc(tb);
        if (e != hipSuccess) return finish(e);
        if ((e = hipcub::DeviceSelect::Flagged(tmp4, tb, all_cl, keep, cl[st], nsel, nrun, s)) != hipSuccess)
            return finish(e);
        int64_t nk = 0;
        if ((e = hipMemcpyAsync(&nk, nsel, sizeof(int64_t), hipMemcpyDeviceToHost, s)) != hipSuccess ||
            (e = hipStreamSynchronize(s)) != hipSuccess)
            return finish(e);
        if (nk >= maxcl) host_caps[1] += 1;  // oracle: the clump loop stops at maxcl
        ncl[st] = std::min(nk, maxcl);
        if (ncl[st] == 0) continue;
        uint64_t *ck0 = (uint64_t *)dalloc(sizeof(uint64_t) * ncl[st]), *ck1 = (uint64_t *)dalloc(sizeof(uint64_t) * ncl[st]);
        int32_t *iv0 = (int32_t *)dalloc(sizeof(int32_t) * ncl[st]);
        co[st] = (int32_t *)dalloc(sizeof(int32_t) * ncl[st]);
        if (e != hipSuccess) return finish(e);
        hipLaunchKernelGGL(lk_clump_keys, dim3((unsigned)((ncl[st] + bs - 1) / bs)), dim3(bs), 0, s, cl[st], ncl[st], ck0);
        // values = the clump index (the low 32 bits of the key)
        hipLaunchKernelGGL(lk_low_words, dim3((unsigned)((ncl[st] + bs - 1) / bs)), dim3(bs), 0, s, ck0, ncl[st], iv0);
        tb = 0;
        (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tb, ck0, ck1, iv0, co[st], (int)ncl[st], 0, 64);
        void *tmp5 = dalloc(tb);
        if (e != hipSuccess) return finish(e);
        if ((e = hipcub::DeviceRadixSort::SortPairs(tmp5, tb, ck0, ck1, iv0, co[st], (int)ncl[st], 0, 64, s)) !=
            hipSuccess)
            return finish(e);
    }
    const int64_t np = ncl[0] + ncl[1];
    if (np > 0) {
        // every clump aligned (one wave per clump, a grid of at most 8 waves per CU)
        RegL *parts = (RegL *)dalloc(sizeof(RegL) * np);
        Blk *pblk = (Blk *)dalloc(sizeof(Blk) * LPB * np);
        const int64_t mb = (dp_mem_bytes(L) + 255) & ~(int64_t)255;
        const int64_t nw = std::min<int64_t>(np, (int64_t)n_cu * 8);
        uint8_t *scr = (uint8_t *)dalloc(mb * nw);
        int32_t *kept = (int32_t *)dalloc(sizeof(int32_t) * np), *nkept = (int32_t *)dalloc(sizeof(int32_t) * 2);
        if (e != hipSuccess) return finish(e);
        hipLaunchKernelGGL(lk_align, dim3((unsigned)nw), dim3(64), 0, s, X, d_q2, L, cl[0], cl[1], co[0], co[1], ncl[0],
                           ncl[1], parts, pblk, scr, mb);
        hipLaunchKernelGGL(lk_keep, dim3(2), dim3(64), 0, s, cl[0], cl[1], co[0], co[1], ncl[0], ncl[1], parts, kept,
                           nkept);
        int32_t nk[2] = {0, 0};
        if ((e = hipGetLastError()) != hipSuccess ||
            (e = hipMemcpyAsync(nk, nkept, sizeof nk, hipMemcpyDeviceToHost, s)) != hipSuccess ||
            (e = hipStreamSynchronize(s)) != hipSuccess)
            return finish(e);
        // sorted order of each strand's kept parts: (qb, tb, qe), ties in creation order (two stable passes)
        int32_t *ord = (int32_t *)dalloc(sizeof(int32_t) * np);
        if (e != hipSuccess) return finish(e);
        for (int st = 0; st < 2; ++st) {
            const int n = nk[st];
            if (n == 0) continue;
            uint64_t *a0 = (uint64_t *)dalloc(8 * n), *a1 = (uint64_t *)dalloc(8 * n), *l0 = (uint64_t *)dalloc(8 * n),
                     *l1 = (uint64_t *)dalloc(8 * n);
            int32_t *i0 = (int32_t *)dalloc(4 * n), *i1 = (int32_t *)dalloc(4 * n), *i2 = (int32_t *)dalloc(4 * n);
            if (e != hipSuccess) return finish(e);
            const int32_t *K = kept + (st ? ncl[0] : 0);
            hipLaunchKernelGGL(lk_ord_keys, dim3((n + bs - 1) / bs), dim3(bs), 0, s, parts, K, n, a0, l0, i0);
            size_t tb = 0, tb2 = 0;
            (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tb, l0, l1, i0, i1, n, 0, 64);
            (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tb2, a0, a1, i1, i2, n, 0, 64);
            void *tmp = dalloc(std::max(tb, tb2));
            if (e != hipSuccess) return finish(e);
            if ((e = hipcub::DeviceRadixSort::SortPairs(tmp, tb, l0, l1, i0, i1, n, 0, 64, s)) != hipSuccess)
                return finish(e);
            // the (qb, tb) pass keyed by the positions the first pass left
            hipLaunchKernelGGL(lk_gather_keys, dim3((n + bs - 1) / bs), dim3(bs), 0, s, a0, i1, n, a1);
            if ((e = hipcub::DeviceRadixSort::SortPairs(tmp, tb2, a1, a0, i1, i2, n, 0, 64, s)) != hipSuccess)
                return finish(e);
            hipLaunchKernelGGL(lk_map_ord, dim3((n + bs - 1) / bs), dim3(bs), 0, s, K, i2, n, ord + (st ? ncl[0] : 0));
        }
        // chains, one wave per strand
        const int nmax = std::max(nk[0], nk[1]);
        const int64_t wb = (((int64_t)6 * nmax + L + 64) * 4 + 64 + (int64_t)8 * nmax + 255) & ~(int64_t)255;
        uint8_t *wk = (uint8_t *)dalloc(2 * wb);
        const int64_t rows_cap = 1 << 16, blk_cap = 1 << 22;
        RowsL R;
        R.rows = (af_psl *)dalloc(sizeof(af_psl) * rows_cap);
        R.seq = (int32_t *)dalloc(sizeof(int32_t) * rows_cap);
        R.boff = (int64_t *)dalloc(sizeof(int64_t) * rows_cap);
        R.blk = (Blk *)dalloc(sizeof(Blk) * blk_cap);
        R.n_rows = (int32_t *)dalloc(sizeof(int32_t));
        R.n_blk = (unsigned long long *)dalloc(sizeof(unsigned long long));
        R.rows_cap = rows_cap; R.blk_cap = blk_cap; R.caps = caps;
        if (e != hipSuccess) return finish(e);
        if ((e = hipMemsetAsync(R.n_rows, 0, sizeof(int32_t), s)) != hipSuccess ||
            (e = hipMemsetAsync(R.n_blk, 0, sizeof(unsigned long long), s)) != hipSuccess)
            return finish(e);
        hipLaunchKernelGGL(lk_chain, dim3(2), dim3(64), 0, s, X, d_q2, L, bp, parts, pblk, ord, nkept, ncl[0], wk, wb, R);
        int32_t nrows = 0;
        unsigned long long nblk = 0;
        if ((e = hipGetLastError()) != hipSuccess ||
            (e = hipMemcpyAsync(&nrows, R.n_rows, 4, hipMemcpyDeviceToHost, s)) != hipSuccess ||
            (e = hipMemcpyAsync(&nblk, R.n_blk, 8, hipMemcpyDeviceToHost, s)) != hipSuccess ||
            (e = hipStreamSynchronize(s)) != hipSuccess)
            return finish(e);
        if (nrows > rows_cap || (int64_t)nblk > blk_cap) return finish(hipErrorOutOfMemory);
        rows.resize(nrows);
        seq.resize(nrows);
        boff.resize(nrows);
        std::vector<Blk> hb(nblk);
        if ((nrows && ((e = hipMemcpyAsync(rows.data(), R.rows, sizeof(af_psl) * nrows, hipMemcpyDeviceToHost, s)) !=
                           hipSuccess ||
                       (e = hipMemcpyAsync(seq.data(), R.seq, 4 * nrows, hipMemcpyDeviceToHost, s)) != hipSuccess ||
                       (e = hipMemcpyAsync(boff.data(), R.boff, 8 * nrows, hipMemcpyDeviceToHost, s)) != hipSuccess)) ||
            (nblk && (e = hipMemcpyAsync(hb.data(), R.blk, sizeof(Blk) * nblk, hipMemcpyDeviceToHost, s)) != hipSuccess) ||
            (e = hipStreamSynchronize(s)) != hipSuccess)
            return finish(e);
        blocks.resize(nblk);
        for (size_t k = 0; k < nblk; ++k) blocks[k] = af_psl_block{hb[k].sz, hb[k].q, hb[k].t};
    }
    if (host_caps[0] || host_caps[1]) {
        int32_t cur[2];
        if ((e = hipMemcpyAsync(cur, caps, sizeof cur, hipMemcpyDeviceToHost, s)) != hipSuccess ||
            (e = hipStreamSynchronize(s)) != hipSuccess)
            return finish(e);
        cur[0] += host_caps[0]; cur[1] += host_caps[1];
        if ((e = hipMemcpyAsync(caps, cur, sizeof cur, hipMemcpyHostToDevice, s)) != hipSuccess) return finish(e);
    }
    return finish(hipGetLastError());
}
