// s2.hip -- S2 on the GPU: `bwa mem -M -t T <anchor.fa> fq1 fq2` (Anchored_Fusion.py:182) as
// bwa 0.7.17 computes it in paired-end mode.  oracle/bwa_pe.c is the bit-exact contract; each
// device routine names the bwa routine (and oracle function) it restates.
//
// Kernels, one launch each per batch, all on the caller's stream (after K1, seed_filter.hip):
//   K2  k_s2_regions   one wave per candidate read (K1 list, per-XCD dequeue heads): SMEM
//                      seeds (mem_collect_intv's three passes, from the read's MEMs against the
//                      bwa text) -> mem_chain (klib kbtree) -> mem_chain_flt -> mem_chain2aln
//                      (ksw_extend2 on the wave, ksw_dp.h) -> mem_sort_dedup_patch; the regions
//                      go to a pool, one atomic per read
//   K3a k_s2_classify  one thread per pair: pairs without a candidate read get their unmapped
//                      records here (the bulk of the batch, 16 B/pair of nontemporal stores);
//                      the rest are listed; unique pairs add an insert size to their chunk
//   K3b k_s2_pestat    one workgroup per bwa chunk: mem_pestat from an LDS histogram
//   K3c k_s2_pairs     one wave per listed pair: mate rescue (mem_matesw, ksw_align2 with the
//                      striped-SW semantics), mem_mark_primary_se (hash tie-break), mem_pair,
//                      mem_sam_pe's record choice, mem_reg2aln (bwa_gen_cigar2 on the wave) and
//                      mem_aln2sam's flags; split-read tails for the partner search
//
// Serial parts of bwa (kbtree, klib introsort, the chain and pair loops) run on lane 0 over
// per-wave LDS state; the DP and the list scans run on the whole wave.  Double-precision
// arithmetic (pestat, patching, pair scores) is kept unfused so it rounds as the C oracle does.
#include "bwa_dev.h"

#pragma clang fp contract(off)

namespace {

#ifndef AF_S2_WPS
#define AF_S2_WPS 5  // k_s2_regions waves per SIMD (LDS: ~7 KB per wave)
#endif

struct S2Pm { int16_t s, t; int32_t r; };          // a MEM: query [s, t), text position r
struct S2Si { int16_t qb, qe, cnt, occ0; };        // a seed interval and its occurrences
struct S2Seed { int32_t rbeg; int16_t qbeg, len; };  // mem_seed_t (score = len)
struct S2Chain { int16_t n, first, kept, seed0; int32_t w, pos; };  // mem_chain_t
constexpr int KB_T = 5, KB_MAXK = 2 * KB_T - 1, KB_NODES = 2 * AF_S2_MAX_CHAIN + 4;
struct S2Kb { uint8_t n, internal, key[KB_MAXK], ptr[KB_MAXK + 1]; };

struct __attribute__((aligned(16))) S2Lds {
    union {
        S2Pm pm[AF_S2_MAX_PMEM];          // seeding: the read's MEMs
        S2Kb kb[KB_NODES];                // chaining: the kbtree
        S2Chain chtmp[AF_S2_MAX_CHAIN];   // chain reordering
        S2Reg reg[AF_S2_MAX_REG];         // extension: regions
    } x;
    union {
        struct { S2Si si[AF_S2_MAX_SEED]; int32_t occ[AF_S2_MAX_OCC]; int32_t tmp[AF_S2_MAX_OCC]; } a;
        struct { S2Seed seed[AF_S2_MAX_OCC]; int16_t srt[AF_S2_MAX_OCC]; } c;
    } y;
    S2Seed pool[AF_S2_MAX_OCC];
    int16_t next[AF_S2_MAX_OCC];
    S2Chain ch[AF_S2_MAX_CHAIN];
    int16_t last_of[AF_S2_MAX_CHAIN];
    uint8_t order[AF_S2_MAX_CHAIN];
    int32_t cnt[8];   // [0] MEMs [1] intervals [2] occurrences [3] overflow [4] chains [5] kb root [6] kb nodes [7] regions
    int64_t rmax[2];
    int32_t misc[4];
};
__shared__ S2Lds g_s2;

#ifdef AF_K2_PROF
// profiling build only (make prof): per-item phase cycles of K2 and K3c (scripts/s2_prof.py)
__device__ int32_t *g_s2prof = nullptr;  // K2 items at [item * 16], K3c items at [S2PROF_K3 + item * 16] (1 M items each)
constexpr int64_t S2PROF_K3 = (int64_t)1 << 24;
#define SPROF(...) __VA_ARGS__
__shared__ int64_t g_sub[5];  // K2 seeding sub-phase marks (pmems, pass 1, pass 2, pass 3)
__shared__ int32_t g_ext[2];  // K2 extension rows and ksw_extend2 calls of the read
#else
#define SPROF(...)
#endif

// ---- small wave helpers --------------------------------------------------------------------
__device__ __forceinline__ uint32_t getT16(const DevText &X, int64_t pos) {
    const int64_t wi = pos >> 4;
    const int sh = (int)(pos & 15) * 2;
    const uint32_t lo = X.T2[wi], hi = X.T2[wi + 1];
    return sh ? (lo >> sh) | (hi << (32 - sh)) : lo;
}

// debug build only (make dbg): progress prints of K2 (one wave; S2DBGL: bwa_dev.h)
#ifdef AF_S2_DEBUG
#define S2DBG(...) do { if (threadIdx.x == 0) printf(__VA_ARGS__); } while (0)
#else
#define S2DBG(...) do { } while (0)
#endif
// =========================================================================== K2: seeds
// MEMs >= min_seed_len of the read (L.q / L.pk / L.nm) against the bwa text T (oracle
// find_pmems).  Lanes over query offsets probe the 16-mer hash (in L2) and test left-maximality
// of each occurrence; every left-maximal (s, r0) is then extended by the whole wave at once:
// lane j compares the 16 bases at s + 16 (j + 1) with T, and the first lane short of 16 equal
// bases ends the match -- one round of loads instead of one per 16 bases.
__device__ void s2_pmems(const DevText &X, int l, int msl, int lane) {
    DpLds &L = g_dp;
    S2Lds &S = g_s2;
    const int64_t N = 2 * X.n;
    const uint32_t hm = (1u << X.hbits) - 1u;
    for (int s0 = 0; s0 + AF_K <= l; s0 += 64) {
        const int s = s0 + lane;
        int cnt = 0, st = 0, pos0 = 0;
        if (s + AF_K <= l) {
            const int wq = s >> 4, sq = s & 15;
            const uint32_t k = __builtin_amdgcn_alignbit(L.pk[wq + 1], L.pk[wq], 2 * sq);
            if (!(((L.nm[wq] | (L.nm[wq + 1] << 16)) >> sq) & 0xFFFFu)) {
                uint32_t sl = af_fmix(k) & hm;
                for (;;) {
                    const int4 e = X.hslot[sl];
                    if (e.z == 0) break;
                    if ((uint32_t)e.x == k) { cnt = e.z; st = e.y; pos0 = e.w; break; }
                    sl = (sl + 1) & hm;
                }
            }
        }
        const int qcl = s > 0 && s + AF_K <= l ? L.q[s - 1] : 4;
        const int ocnt = wave_max(cnt);
        for (int o = 0; o < ocnt; ++o) {
            bool lm = false;
            int64_t r0 = 0;
            if (o < cnt) {
                r0 = o == 0 ? (int64_t)pos0 : (int64_t)X.kpos[st + o];
                lm = !(qcl < 4 && r0 > 0 && X.T[r0 - 1] == qcl);
            }
            uint64_t msk = __ballot(lm);
            while (msk) {
                const int ln = __builtin_ctzll(msk);
                msk &= msk - 1;
                const int cs = __builtin_amdgcn_readlane(s, ln);
                const int cr = __builtin_amdgcn_readlane((int)r0, ln);
                // word lane + 1 of the match: query [cs + 16 (lane + 1), +16) vs T at cr + same
                const int qp = cs + AF_K + 16 * lane;
                const int64_t rp = (int64_t)cr + AF_K + 16 * lane;
                const int64_t room64 = min((int64_t)(l - qp), N - rp);
                int step = 0;
                if (room64 > 0) {
                    const int room = (int)min(room64, (int64_t)16);
                    const int wp = qp >> 4, sp = qp & 15;
                    const uint32_t qk = __builtin_amdgcn_alignbit(L.pk[wp + 1], L.pk[wp], 2 * sp);
                    const int qn = __builtin_ctz((((L.nm[wp] | (L.nm[wp + 1] << 16)) >> sp) & 0xFFFFu) | 0x10000u);
                    const uint32_t x = qk ^ getT16(X, rp);
                    const int eq = x ? (__builtin_ctz(x) >> 1) : 16;
                    step = min(min(eq, room), qn);
                }
                const uint64_t stop = __ballot(step < 16);  // lanes past the read's end stop too
                const int js = stop ? (int)__builtin_ctzll(stop) : 63;
                const int len = AF_K + 16 * js + __builtin_amdgcn_readlane(step, js);
                if (len >= msl) {
                    if (lane == 0) {
                        const int slot = S.cnt[0];
                        if (slot < AF_S2_MAX_PMEM) S.x.pm[slot] = S2Pm{(int16_t)cs, (int16_t)(cs + len), (int32_t)cr};
                        S.cnt[0] = slot + 1;
                    }
                    wave_sync();
                }
            }
        }
    }
}

// occurrences of q[b, e) (e - b >= min_seed_len) = the MEMs covering it (oracle count_cov)
__device__ __forceinline__ int s2_count_cov(int npm, int b, int e, int lane) {
    int c = 0;
    for (int k0 = 0; k0 < npm; k0 += 64) {
        const int k = k0 + lane;
        bool v = false;
        if (k < npm) {
            const S2Pm m = g_s2.x.pm[k];
            v = m.s <= b && e <= m.t;
        }
        c += __builtin_popcountll(__ballot(v));
    }
    return c;
}

// push seed interval [b, e) with its occurrences in suffix-rank (bwt_sa) order (oracle
// push_intv).  cnt0 >= 0 forces an occurrence-free interval (bwt_smem1 on an absent base).
__device__ void s2_push_intv(const DevText &X, int npm, int b, int e, int lane, bool empty = false) {
    S2Lds &S = g_s2;
    if (S.cnt[3]) return;
    const int si = S.cnt[1], occ0 = S.cnt[2];
    if (si >= AF_S2_MAX_SEED) {
        wave_sync();
        if (lane == 0) S.cnt[3] = 1;
        wave_sync();
        return;
    }
    int c = 0;
    if (!empty) {
        for (int k0 = 0; k0 < npm; k0 += 64) {
            const int k = k0 + lane;
            bool v = false;
            S2Pm m{};
            if (k < npm) {
                m = S.x.pm[k];
                v = m.s <= b && e <= m.t;
            }
            const uint64_t msk = __ballot(v);
            if (v) {
                const int idx = occ0 + c + lanes_below(msk, lane);
                if (idx < AF_S2_MAX_OCC) S.y.a.occ[idx] = m.r + (b - m.s);
            }
            c += __builtin_popcountll(msk);
        }
    }
    wave_sync();
    if (occ0 + c > AF_S2_MAX_OCC) {
        if (lane == 0) S.cnt[3] = 1;
        wave_sync();
        return;
    }
    // rank sort of occ[occ0, occ0 + c): each lane takes up to two entries (c <= 128); a single
    // occurrence needs no rank
    int pa = 0, ra = 0, pb = 0, rb = 0, da = -1, db = -1;
    if (c > 1) {
        if (lane < c) { pa = S.y.a.occ[occ0 + lane]; ra = X.rank[pa]; S.y.a.tmp[occ0 + lane] = ra; }
        if (lane + 64 < c) { pb = S.y.a.occ[occ0 + lane + 64]; rb = X.rank[pb]; S.y.a.tmp[occ0 + lane + 64] = rb; }
        wave_sync();
    }
    if (c > 1 && (lane < c || lane + 64 < c)) {
        int ca = 0, cb = 0;
        for (int j = 0; j < c; ++j) {
            const int rj = S.y.a.tmp[occ0 + j];
            ca += rj < ra;
            cb += rj < rb;
        }
        if (lane < c) da = ca;
        if (lane + 64 < c) db = cb;
    }
    wave_sync();
    if (da >= 0) S.y.a.occ[occ0 + da] = pa;
    if (db >= 0) S.y.a.occ[occ0 + db] = pb;
    if (lane == 0) {
        S.y.a.si[si] = S2Si{(int16_t)b, (int16_t)e, (int16_t)c, (int16_t)occ0};
        S.cnt[1] = si + 1;
        S.cnt[2] = occ0 + c;
    }
    wave_sync();
}

// bwt_smem1(x, min_intv = m) restricted to outputs >= min_seed_len (oracle smem_at)
__device__ void s2_smem_at(const DevText &X, int npm, int l, int msl, int x, int m, int lane) {
    DpLds &L = g_dp;
    S2Lds &S = g_s2;
    const int bx = __builtin_amdgcn_readfirstlane((int)L.q[x]);  // < 4 (callers skip N)
    const int c0 = bx == 0 ? X.base_cnt[0] : bx == 1 ? X.base_cnt[1] : bx == 2 ? X.base_cnt[2] : X.base_cnt[3];
    if (c0 < m) {  // degenerate: the single base occurs fewer than m times
        if (x + msl > l) return;
        for (int i = x + 1; i < x + msl; ++i) if (L.q[i] > 3) return;
        if (s2_count_cov(npm, x, x + msl, lane) != c0) return;
        int e1 = x + msl;
        while (e1 < l && L.q[e1] < 4 && s2_count_cov(npm, x, e1 + 1, lane) == c0) ++e1;
        s2_push_intv(X, npm, x, e1, lane, c0 == 0);
        return;
    }
    int prev_b = -1, prev_e = -1;
    for (;;) {
        // the next distinct start among MEMs holding x
        int bmin = 1 << 30;
        for (int k0 = 0; k0 < npm; k0 += 64) {
            const int k = k0 + lane;
            if (k < npm) {
                const S2Pm mm = S.x.pm[k];
                if (mm.s <= x && x < mm.t && mm.s > prev_b) bmin = min(bmin, (int)mm.s);
            }
        }
        const int b = wave_min(bmin);
        if (b >= (1 << 30)) break;
        // e(b): the largest end t_j (MEMs holding x, s <= b) with >= m such MEMs ending at or after t_j
        int cand = -1;
        for (int k0 = 0; k0 < npm; k0 += 64) {
            const int j = k0 + lane;
            if (j < npm) {
                const S2Pm mj = S.x.pm[j];
                if (mj.s <= b && x < mj.t) {
                    int cj = 0;
                    for (int u = 0; u < npm; ++u) {
                        const S2Pm mu = S.x.pm[u];
                        cj += mu.s <= b && x < mu.t && mu.t >= mj.t;
                    }
                    if (cj >= m) cand = max(cand, (int)mj.t);
                }
            }
        }
        const int e = wave_max(cand);
        if (e >= 0 && e > prev_e) {
            if (e - b >= msl) s2_push_intv(X, npm, b, e, lane);
            prev_e = e;
        }
        prev_b = b;
    }
}

// mem_collect_intv (oracle collect_intv): pass 1 SMEMs, pass 2 re-seeding, pass 3
// bwt_seed_strategy1; then the intervals sorted by (qb, qe).  Sets S.cnt[3] on overflow.
__device__ void s2_collect_intv(const DevText &X, const af_params &p, const S2Opt &o, int l, int lane) {
    DpLds &L = g_dp;
    S2Lds &S = g_s2;
    const int msl = p.min_seed_len;
    SPROF(if (lane == 0) g_sub[0] = clock64();)
    S2DBG("k2 pmems start\n");
    s2_pmems(X, l, msl, lane);
    wave_sync();
    S2DBG("k2 pmems %d\n", S.cnt[0]);
    SPROF(if (lane == 0) g_sub[1] = g_sub[2] = g_sub[3] = g_sub[4] = clock64();)
    const int npm_all = S.cnt[0];
    if (npm_all > AF_S2_MAX_PMEM) {
        if (lane == 0) S.cnt[3] = 1;
        wave_sync();
        return;
    }
    const int npm = npm_all;
    // pass 1: maximal MEM query intervals, each once (keep the lowest index of equal ones)
    for (int k0 = 0; k0 < npm; k0 += 64) {
        const int k = k0 + lane;
        bool keep = false;
        int s = 0, t = 0;
        if (k < npm) {
            s = S.x.pm[k].s; t = S.x.pm[k].t;
            keep = true;
            for (int j = 0; j < npm && keep; ++j) {
                const S2Pm mj = S.x.pm[j];
                if (mj.s == s && mj.t == t) { if (j < k) keep = false; continue; }
                if (mj.s <= s && t <= mj.t) keep = false;
            }
        }
        uint64_t msk = __ballot(keep);
        while (msk) {
            const int ln = __builtin_ctzll(msk);
            msk &= msk - 1;
            const int bs = __builtin_amdgcn_readlane(s, ln), bt = __builtin_amdgcn_readlane(t, ln);
            s2_push_intv(X, npm, bs, bt, lane);
        }
    }
    SPROF(if (lane == 0) g_sub[2] = g_sub[3] = g_sub[4] = clock64();)
    S2DBG("k2 pass1 seeds %d ovf %d\n", S.cnt[1], S.cnt[3]);
    if (S.cnt[3]) return;
    // pass 2
    const int split_len = (int)((float)msl * 1.5f + .499);
    const int n1 = S.cnt[1];
    for (int k = 0; k < n1 && !S.cnt[3]; ++k) {
        const S2Si v = S.y.a.si[k];
        if (v.qe - v.qb < split_len || v.cnt > o.split_width) continue;
        s2_smem_at(X, npm, l, msl, (v.qb + v.qe) >> 1, v.cnt + 1, lane);
    }
    SPROF(if (lane == 0) g_sub[3] = g_sub[4] = clock64();)
    S2DBG("k2 pass2 seeds %d ovf %d\n", S.cnt[1], S.cnt[3]);
    // pass 3 (bwt_seed_strategy1 with min_len = min_seed_len, max_intv = max_mem_intv)
    if (o.max_mem_intv > 0) {
        const int mi = o.max_mem_intv;
        int x = 0;
        while (x < l && !S.cnt[3]) {
            if (L.q[x] > 3) { ++x; continue; }
            // e* = the first end >= x + msl + 1 at which q[x, e) occurs < max_mem_intv times
            int na = 0;
            for (int k0 = 0; k0 < npm; k0 += 64) {
                const int k = k0 + lane;
                na += __builtin_popcountll(__ballot(k < npm && S.x.pm[k].s <= x && S.x.pm[k].t > x + msl));
            }
            int em = -1;
            if (na >= mi) {
                int cand = -1;
                for (int k0 = 0; k0 < npm; k0 += 64) {
                    const int j = k0 + lane;
                    if (j < npm && S.x.pm[j].s <= x) {
                        const int tj = S.x.pm[j].t;
                        int cj = 0;
                        for (int u = 0; u < npm; ++u) cj += S.x.pm[u].s <= x && S.x.pm[u].t >= tj;
                        if (cj >= mi) cand = max(cand, tj);
                    }
                }
                em = wave_max(cand);
            }
            const int es = max(x + msl + 1, em + 1);
            int pn = l;  // first N after x
            for (int i = x + 1 + lane; i < min(es, l); i += 64)
                if (L.q[i] > 3) { pn = min(pn, i); }
            pn = wave_min(pn);
            if (pn < min(es, l)) { x = pn + 1; continue; }
            if (es > l) { x = l; continue; }
            const int c = s2_count_cov(npm, x, es, lane);
            if (c > 0) s2_push_intv(X, npm, x, es, lane);
            x = es;
        }
    }
    SPROF(if (lane == 0) g_sub[4] = clock64();)
    S2DBG("k2 pass3 seeds %d ovf %d\n", S.cnt[1], S.cnt[3]);
    if (S.cnt[3]) return;
    // sort by (qb, qe): equal intervals are identical, any order among them
    const int ns = S.cnt[1];
    S2Si mine{};
    int dest = -1;
    if (lane < ns) {
        mine = S.y.a.si[lane];
        const int key = (int)mine.qb << 16 | (int)mine.qe;
        int d = 0;
        for (int j = 0; j < ns; ++j) {
            const S2Si sj = S.y.a.si[j];
            const int kj = (int)sj.qb << 16 | (int)sj.qe;
            d += kj < key || (kj == key && j < lane);
        }
        dest = d;
    }
    wave_sync();
    if (dest >= 0) S.y.a.si[dest] = mine;
    wave_sync();
}

// =========================================================================== K2: chains
// klib kbtree (t = 5) over chain indices keyed by chain pos; lane 0 only (oracle kb_*)
__device__ __forceinline__ int kb_cmp(int x, int32_t kpos) {
    const int32_t a = g_s2.ch[x].pos;
    return (kpos < a) - (a < kpos);
}
__device__ int kb_getp_aux(const S2Kb &x, int32_t kpos, int *r) {
    int tr, *rr, begin = 0, end = x.n;
    if (x.n == 0) return -1;
    rr = r ? r : &tr;
    while (begin < end) {
        const int mid = (begin + end) >> 1;
        if (kb_cmp(x.key[mid], kpos) < 0) begin = mid + 1;
        else end = mid;
    }
    if (begin == x.n) { *rr = 1; return x.n - 1; }
    if ((*rr = -kb_cmp(x.key[begin], kpos)) < 0) --begin;
    return begin;
}
__device__ int kb_new(int internal) {
    S2Lds &S = g_s2;
    const int zi = S.cnt[6]++;
    S2Kb &z = S.x.kb[zi];
    z.n = 0; z.internal = (uint8_t)internal;
    return zi;
}
__device__ int kb_lower(int32_t kpos) {
    S2Lds &S = g_s2;
    int r = 0, lower = -1, xi = S.cnt[5];
    while (xi >= 0) {
        const S2Kb &x = S.x.kb[xi];
        const int i = kb_getp_aux(x, kpos, &r);
        if (i >= 0 && r == 0) return x.key[i];
        if (i >= 0) lower = x.key[i];
        if (!x.internal) return lower;
        xi = x.ptr[i + 1];
    }
    return lower;
}
__device__ void kb_split(int xi, int i, int yi) {
    S2Lds &S = g_s2;
    const int zi = kb_new(S.x.kb[yi].internal);
    S2Kb &x = S.x.kb[xi], &y = S.x.kb[yi], &z = S.x.kb[zi];
    z.n = KB_T - 1;
    for (int u = 0; u < KB_T - 1; ++u) z.key[u] = y.key[KB_T + u];
    if (y.internal)
        for (int u = 0; u < KB_T; ++u) z.ptr[u] = y.ptr[KB_T + u];
    y.n = KB_T - 1;
    for (int u = x.n; u >= i + 1; --u) x.ptr[u + 1] = x.ptr[u];
    x.ptr[i + 1] = (uint8_t)zi;
    for (int u = x.n - 1; u >= i; --u) x.key[u + 1] = x.key[u];
    x.key[i] = y.key[KB_T - 1];
    ++x.n;
}
__device__ void kb_putp(int k) {
    S2Lds &S = g_s2;
    const int32_t kpos = S.ch[k].pos;
    int xi = S.cnt[5];
    if (S.x.kb[xi].n == KB_MAXK) {
        const int si = kb_new(1);
        S.x.kb[si].ptr[0] = (uint8_t)xi;
        S.cnt[5] = si;
        kb_split(si, 0, xi);
        xi = si;
    }
    for (;;) {  // __kb_putp_aux, iteratively
        S2Kb &x = S.x.kb[xi];
        if (!x.internal) {
            const int i = kb_getp_aux(x, kpos, nullptr);
            for (int u = x.n - 1; u >= i + 1; --u) x.key[u + 1] = x.key[u];
            x.key[i + 1] = (uint8_t)k;
            ++x.n;
            return;
        }
        int i = kb_getp_aux(x, kpos, nullptr) + 1;
        if (S.x.kb[x.ptr[i]].n == KB_MAXK) {
            kb_split(xi, i, x.ptr[i]);
            if (kb_cmp(S.x.kb[xi].key[i], kpos) < 0) ++i;  // klib: cmp(*k, key[i]) > 0, k past the promoted key
        }
        xi = S.x.kb[xi].ptr[i];
    }
}
__device__ int kb_traverse() {
    S2Lds &S = g_s2;
    int stk_node[8], stk_i[8], top = 0, n = 0;
    stk_node[0] = S.cnt[5]; stk_i[0] = 0;
    // in-order: for a node, child[i] then key[i] for i < n, then child[n]
    if (!S.x.kb[stk_node[0]].internal) {
        const S2Kb &x = S.x.kb[stk_node[0]];
        for (int i = 0; i < x.n; ++i) S.order[n++] = x.key[i];
        return n;
    }
    top = 1;
    while (top > 0) {
        const int xi = stk_node[top - 1];
        const int i = stk_i[top - 1];
        const S2Kb &x = S.x.kb[xi];
        if (!x.internal) {
            for (int u = 0; u < x.n; ++u) S.order[n++] = x.key[u];
            --top;
            continue;
        }
        if (i > x.n) { --top; continue; }
        stk_i[top - 1] = i + 1;
        if (i > 0) S.order[n++] = x.key[i - 1];
        stk_node[top] = x.ptr[i]; stk_i[top] = 0; ++top;
    }
    return n;
}

// test_and_merge (lane 0; oracle test_and_merge)
__device__ int s2_test_and_merge(int ci, const S2Seed &p, int64_t l_pac, int w, int max_chain_gap) {
    S2Lds &S = g_s2;
    S2Chain &c = S.ch[ci];
    const S2Seed first = S.pool[c.seed0], last = S.pool[S.last_of[ci]];
    const int64_t qend = (int64_t)last.qbeg + last.len, rend = (int64_t)last.rbeg + last.len;
    if (p.qbeg >= first.qbeg && p.qbeg + p.len <= qend && p.rbeg >= first.rbeg && (int64_t)p.rbeg + p.len <= rend)
        return 1;
    if ((last.rbeg < l_pac || first.rbeg < l_pac) && p.rbeg >= l_pac) return 0;
    const int64_t x = p.qbeg - last.qbeg, y = (int64_t)p.rbeg - last.rbeg;
    if (y >= 0 && x - y <= w && y - x <= w && x - last.len < max_chain_gap && y - last.len < max_chain_gap) {
        if (S.cnt[2] >= AF_S2_MAX_OCC) return -1;
        const int k = S.cnt[2]++;
        S.pool[k] = p;
        S.next[k] = -1;
        S.next[S.last_of[ci]] = (int16_t)k;
        S.last_of[ci] = (int16_t)k;
        ++c.n;
        return 1;
    }
    return 0;
}

// mem_chain (lane 0; oracle mem_chain): returns the chain count, -1 on overflow.  On return the
// chains are in S.ch in tree order, their seeds contiguous in S.y.c.seed.
__device__ int s2_mem_chain(const DevText &X, const af_params &p, const S2Opt &o) {
    S2Lds &S = g_s2;
    const int64_t l_pac = X.n;
    const int nsi = S.cnt[1];
    // the interval list (si/occ) stays in S.y.a while the pool fills; the pool count reuses cnt[2]
    int nocc_used = 0;
    (void)nocc_used;
    S.cnt[2] = 0;
    S.cnt[4] = 0;
    S.cnt[5] = -1;
    S.cnt[6] = 0;
    S.cnt[5] = kb_new(0);
    for (int i = 0; i < nsi; ++i) {
        const S2Si v = S.y.a.si[i];
        const int slen = v.qe - v.qb;
        const int step = v.cnt > p.max_occ ? v.cnt / p.max_occ : 1;
        for (int k = 0, count = 0; k < v.cnt && count < p.max_occ; k += step, ++count) {
            S2Seed s;
            s.rbeg = S.y.a.occ[v.occ0 + k];
            s.qbeg = v.qb;
            s.len = (int16_t)slen;
            if (s.rbeg < l_pac && (int64_t)s.rbeg + s.len > l_pac) continue;  // bns_intv2rid < 0
            bool to_add = false;
            if (S.cnt[4]) {
                const int lower = kb_lower(s.rbeg);
                if (lower < 0) to_add = true;
                else {
                    const int r = s2_test_and_merge(lower, s, l_pac, p.w, o.max_chain_gap);
                    if (r < 0) return -1;
                    if (!r) to_add = true;
                }
            } else to_add = true;
            if (to_add) {
                if (S.cnt[4] >= AF_S2_MAX_CHAIN || S.cnt[2] >= AF_S2_MAX_OCC) return -1;
                const int kk = S.cnt[2]++;
                S.pool[kk] = s;
                S.next[kk] = -1;
                const int nc = S.cnt[4];
                S.ch[nc] = S2Chain{1, -1, 0, (int16_t)kk, 0, s.rbeg};
                S.last_of[nc] = (int16_t)kk;
                kb_putp(nc);
                S.cnt[4] = nc + 1;
            }
        }
    }
    const int no = kb_traverse();
    // reorder the chains (tree order) and compact their seeds
    for (int a = 0; a < no; ++a) S.x.chtmp[a] = S.ch[S.order[a]];
    int ns = 0;
    for (int a = 0; a < no; ++a) {
        S2Chain c = S.x.chtmp[a];
        const int s0 = ns;
        for (int k = c.seed0; k >= 0; k = S.next[k]) S.y.c.seed[ns++] = S.pool[k];
        c.seed0 = (int16_t)s0;
        S.ch[a] = c;
    }
    return no;
}

__device__ int s2_chain_weight(const S2Chain &c) {
    const S2Seed *sd = g_s2.y.c.seed + c.seed0;
    int64_t end = 0;
    int w = 0, tmp;
    for (int j = 0; j < c.n; ++j) {
        const S2Seed s = sd[j];
        if (s.qbeg >= end) w += s.len;
        else if (s.qbeg + s.len > end) w += (int)(s.qbeg + s.len - end);
        end = end > s.qbeg + s.len ? end : s.qbeg + s.len;
    }
    tmp = w; w = 0; end = 0;
    for (int j = 0; j < c.n; ++j) {
        const S2Seed s = sd[j];
        if (s.rbeg >= end) w += s.len;
        else if ((int64_t)s.rbeg + s.len > end) w += (int)((int64_t)s.rbeg + s.len - end);
        end = end > (int64_t)s.rbeg + s.len ? end : (int64_t)s.rbeg + s.len;
    }
    w = w < tmp ? w : tmp;
    return w < 1 << 30 ? w : (1 << 30) - 1;
}

struct LtFlt {
    __device__ bool operator()(const S2Chain &a, const S2Chain &b) const { return a.w > b.w; }
};

// mem_chain_flt (lane 0; oracle mem_chain_flt): returns the kept chain count
__device__ int s2_chain_flt(int n_chn, const af_params &p, const S2Opt &o) {
    S2Lds &S = g_s2;
    S2Chain *a = S.ch;
    if (n_chn == 0) return 0;
    for (int i = 0; i < n_chn; ++i) { a[i].first = -1; a[i].kept = 0; a[i].w = s2_chain_weight(a[i]); }
    ks_introsort(a, n_chn, LtFlt());
    auto beg = [&](const S2Chain &c) { return (int)S.y.c.seed[c.seed0].qbeg; };
    auto endq = [&](const S2Chain &c) {
        const S2Seed t = S.y.c.seed[c.seed0 + c.n - 1];
        return (int)t.qbeg + t.len;
    };
    uint8_t chains[AF_S2_MAX_CHAIN];
    int nc = 0;
    a[0].kept = 3;
    chains[nc++] = 0;
    for (int i = 1; i < n_chn; ++i) {
        int large_ovlp = 0, k;
        for (k = 0; k < nc; ++k) {
            const int j = chains[k];
            const int b_max = beg(a[j]) > beg(a[i]) ? beg(a[j]) : beg(a[i]);
            const int e_min = endq(a[j]) < endq(a[i]) ? endq(a[j]) : endq(a[i]);
            if (e_min > b_max) {
                const int li = endq(a[i]) - beg(a[i]), lj = endq(a[j]) - beg(a[j]);
                const int min_l = li < lj ? li : lj;
                if ((float)(e_min - b_max) >= (float)min_l * 0.5f && min_l < o.max_chain_gap) {
                    large_ovlp = 1;
                    if (a[j].first < 0) a[j].first = (int16_t)i;
                    if ((float)a[i].w < (float)a[j].w * 0.5f && a[j].w - a[i].w >= p.min_seed_len << 1) break;
                }
            }
        }
        if (k == nc) {
            chains[nc++] = (uint8_t)i;
            a[i].kept = (int16_t)(large_ovlp ? 2 : 3);
        }
    }
    for (int i = 0; i < nc; ++i) {
        const S2Chain &c = a[chains[i]];
        if (c.first >= 0) a[c.first].kept = 1;
    }
    int k = 0;
    for (int i = 0; i < n_chn; ++i)
        if (a[i].kept != 0) a[k++] = a[i];
    return k;
}

// ====================================================================== K2: extension
// mem_chain2aln (oracle mem_chain2aln) for chain ci; regions appended to S.x.reg (S.cnt[7])
template <int CPL>
__device__ void s2_chain2aln(const DevText &X, const af_params &p, int l, int ci, int lane) {
    DpLds &L = g_dp;
    S2Lds &S = g_s2;
    const int64_t l_pac = X.n;
    const S2Chain c = S.ch[ci];
    const S2Seed *sd = S.y.c.seed + c.seed0;
    if (lane == 0) {
        int64_t r0 = l_pac << 1, r1 = 0;
        for (int i = 0; i < c.n; ++i) {
            const S2Seed t = sd[i];
            const int64_t b = t.rbeg - (t.qbeg + cal_max_gap(p, t.qbeg));
            const int rem = l - t.qbeg - t.len;
            const int64_t e = (int64_t)t.rbeg + t.len + (rem + cal_max_gap(p, rem));
            r0 = r0 < b ? r0 : b;
            r1 = r1 > e ? r1 : e;
        }
        r0 = r0 > 0 ? r0 : 0;
        r1 = r1 < l_pac << 1 ? r1 : l_pac << 1;
        if (r0 < l_pac && l_pac < r1) {
            if (sd[0].rbeg < l_pac) r1 = l_pac;
            else r0 = l_pac;
        }
        const int64_t fb = sd[0].rbeg < l_pac ? 0 : l_pac, fe = sd[0].rbeg < l_pac ? l_pac : l_pac << 1;
        S.rmax[0] = r0 > fb ? r0 : fb;
        S.rmax[1] = r1 < fe ? r1 : fe;
        // srt: seed indices by (score << 32 | i) ascending
        for (int i = 0; i < c.n; ++i) S.y.c.srt[i] = (int16_t)i;
        for (int i = 1; i < c.n; ++i)
            for (int j = i; j > 0; --j) {
                const S2Seed u = sd[S.y.c.srt[j]], v = sd[S.y.c.srt[j - 1]];
                const bool lt = u.len < v.len || (u.len == v.len && S.y.c.srt[j] < S.y.c.srt[j - 1]);
                if (!lt) break;
                const int16_t t = S.y.c.srt[j]; S.y.c.srt[j] = S.y.c.srt[j - 1]; S.y.c.srt[j - 1] = t;
            }
    }
    wave_sync();
    const int64_t rmax0 = S.rmax[0], rmax1 = S.rmax[1];
    for (int k = c.n - 1; k >= 0; --k) {
        const int si = S.y.c.srt[k];
        const S2Seed s = sd[si];
        const int nreg = S.cnt[7];
        // test whether extension has been made before (any region satisfying)
        bool hit = false;
        if (lane < nreg) {
            const S2Reg pr = S.x.reg[lane];
            if (!(s.rbeg < pr.rb || (int64_t)s.rbeg + s.len > pr.re || s.qbeg < pr.qb || s.qbeg + s.len > pr.qe) &&
                !((double)(s.len - pr.seedlen0) > .1 * l)) {
                int qd = s.qbeg - pr.qb;
                int64_t rd = s.rbeg - pr.rb;
                int mg = cal_max_gap(p, (int)(qd < rd ? (int64_t)qd : rd));
                int ww = mg < pr.w ? mg : pr.w;
                if (qd - rd < ww && rd - qd < ww) hit = true;
                else {
                    qd = pr.qe - (s.qbeg + s.len);
                    rd = pr.re - ((int64_t)s.rbeg + s.len);
                    mg = cal_max_gap(p, (int)(qd < rd ? (int64_t)qd : rd));
                    ww = mg < pr.w ? mg : pr.w;
                    if (qd - rd < ww && rd - qd < ww) hit = true;
                }
            }
        }
        if (__ballot(hit)) {
            // contained: extend only if a long overlapping seed on another diagonal follows
            bool ov = false;
            for (int i = k + 1 + lane; i < c.n; i += 64) {
                const int ti = S.y.c.srt[i];
                if (ti < 0) continue;
                const S2Seed t = sd[ti];
                if ((double)t.len < s.len * .95) continue;
                if (s.qbeg <= t.qbeg && s.qbeg + s.len - t.qbeg >= s.len >> 2 &&
                    (int64_t)(t.qbeg - s.qbeg) != (int64_t)t.rbeg - s.rbeg) ov = true;
                if (t.qbeg <= s.qbeg && t.qbeg + t.len - s.qbeg >= s.len >> 2 &&
                    (int64_t)(s.qbeg - t.qbeg) != (int64_t)s.rbeg - t.rbeg) ov = true;
            }
            if (!__ballot(ov)) {
                wave_sync();
                if (lane == 0) S.y.c.srt[k] = -1;
                wave_sync();
                continue;
            }
        }
        if (nreg >= AF_S2_MAX_REG) {
            wave_sync();
            if (lane == 0) S.cnt[3] = 1;
            wave_sync();
            return;
        }
        int a_score = -1, a_truesc = -1, a_qb = 0, a_qe = 0;
        int64_t a_rb = 0, a_re = 0;
        int aw0 = p.w, aw1 = p.w;
        if (s.qbeg) {  // left extension
            const int64_t tmp = s.rbeg - rmax0;
            const int tl = (int)min(tmp, (int64_t)(s.qbeg + 2 * p.w + 1));
            for (int x = lane; x < s.qbeg; x += 64) L.qs[x] = L.q[s.qbeg - 1 - x];
            for (int x = lane; x < tl; x += 64) L.t[x] = X.T[s.rbeg - 1 - x];
            wave_sync();
            ExtRes er;
            for (int it = 0; it < 2; ++it) {
                const int prev = a_score;
                aw0 = p.w << it;
                er = ext_dp<CPL>(s.qbeg, L.qs, tl, L.t, p, aw0, p.pen_clip5, p.zdrop, s.len * p.a, lane);
                SPROF(if (lane == 0) { g_ext[0] += er.rows; g_ext[1] += 1; })
                a_score = er.max;
                if (a_score == prev || er.max_off < (aw0 >> 1) + (aw0 >> 2)) break;
            }
            if (er.gscore <= 0 || er.gscore <= a_score - p.pen_clip5) {
                a_qb = s.qbeg - er.qle; a_rb = s.rbeg - er.tle; a_truesc = a_score;
            } else {
                a_qb = 0; a_rb = s.rbeg - er.gtle; a_truesc = er.gscore;
            }
            wave_sync();
        } else {
            a_score = a_truesc = s.len * p.a; a_qb = 0; a_rb = s.rbeg;
        }
        if (s.qbeg + s.len != l) {  // right extension
            const int qe = s.qbeg + s.len;
            const int64_t re = (int64_t)s.rbeg + s.len - rmax0;
            const int sc0 = a_score;
            const int tl = (int)min(rmax1 - rmax0 - re, (int64_t)((l - qe) + 2 * p.w + 1));
            for (int x = lane; x < tl; x += 64) L.t[x] = X.T[rmax0 + re + x];
            wave_sync();
            ExtRes er;
            for (int it = 0; it < 2; ++it) {
                const int prev = a_score;
                aw1 = p.w << it;
                er = ext_dp<CPL>(l - qe, L.q + qe, tl, L.t, p, aw1, p.pen_clip3, p.zdrop, sc0, lane);
                SPROF(if (lane == 0) { g_ext[0] += er.rows; g_ext[1] += 1; })
                a_score = er.max;
                if (a_score == prev || er.max_off < (aw1 >> 1) + (aw1 >> 2)) break;
            }
            if (er.gscore <= 0 || er.gscore <= a_score - p.pen_clip3) {
                a_qe = qe + er.qle; a_re = rmax0 + re + er.tle; a_truesc += a_score - sc0;
            } else {
                a_qe = l; a_re = rmax0 + re + er.gtle; a_truesc += er.gscore - sc0;
            }
            wave_sync();
        } else {
            a_qe = l; a_re = (int64_t)s.rbeg + s.len;
        }
        if (lane == 0) {
            S2Reg &a = S.x.reg[nreg];
            a.rb = a_rb; a.re = a_re; a.qb = a_qb; a.qe = a_qe; a.score = a_score; a.truesc = a_truesc;
            a.w = aw0 > aw1 ? aw0 : aw1; a.seedlen0 = s.len;
            S.cnt[7] = nreg + 1;
        }
        wave_sync();
    }
}

// mem_patch_reg (oracle mem_patch_reg): the merged score, 0 if not merged; *w_out its band
template <int CPL>
__device__ int s2_patch_reg(const DevText &X, const af_params &p, const S2Reg &a, const S2Reg &b, int *w_out,
                            uint8_t *zg, int lane) {
    const int64_t l_pac = X.n;
    if (a.rb < l_pac && b.rb >= l_pac) return 0;
    if (a.qb >= b.qb || a.qe >= b.qe || a.re >= b.re) return 0;
    if (b.re - a.rb > AF_S2_MAX_TSPAN) return 0;  // the oracle's AFO_PE_MAX_TSPAN (L.t holds 1 KiB)
    int w = (int)((a.re - b.rb) - (a.qe - b.qb));
    w = w > 0 ? w : -w;
    double r = (double)(a.re - b.rb) / (double)(b.re - a.rb) - (double)(a.qe - b.qb) / (double)(b.qe - a.qb);
    r = r > 0. ? r : -r;
    if (a.re < b.rb || a.qe < b.qb) {
        if (w > p.w << 1 || r >= (double)0.05f) return 0;
    } else if (w > p.w << 2 || r >= (double)(0.05f * 2)) return 0;
    w += a.w + b.w;
    w = w < p.w << 2 ? w : p.w << 2;
    const int lq = b.qe - a.qb;
    const int score = gen_cigar_wave<CPL, false>(X.T, l_pac, p, w, lq, a.qb, a.rb, b.re, g_dp, zg, lane);
    const int q_s = (int)((double)(b.qe - a.qb) / (double)((b.qe - b.qb) + (a.qe - a.qb)) * (double)(b.score + a.score) + .499);
    const int r_s = (int)((double)(b.re - a.rb) / (double)((b.re - b.rb) + (a.re - a.rb)) * (double)(b.score + a.score) + .499);
    if ((double)score / (double)(q_s > r_s ? q_s : r_s) < (double)0.90f) return 0;
    *w_out = w;
    return score;
}

struct LtArs2 {
    __device__ bool operator()(const S2Reg &a, const S2Reg &b) const { return a.re < b.re; }
};
struct LtArs {
    __device__ bool operator()(const S2Reg &a, const S2Reg &b) const {
        return a.score > b.score || (a.score == b.score && (a.rb < b.rb || (a.rb == b.rb && a.qb < b.qb)));
    }
};

// mem_sort_dedup_patch with patching (oracle mem_sort_dedup_patch, patch = 1) over S.x.reg
template <int CPL>
__device__ int s2_dedup_patch(const DevText &X, const af_params &p, const S2Opt &o, int n, uint8_t *zg, int lane) {
    S2Lds &S = g_s2;
    S2Reg *a = S.x.reg;
    if (n <= 1) return n;
    S2DBG("dedup n %d\n", n);
    if (lane == 0) ks_introsort(a, n, LtArs2());
    wave_sync();
    S2DBG("dedup sorted\n");
    for (int i = 1; i < n; ++i) {
        if (a[i].rb >= a[i - 1].re + o.max_chain_gap) continue;
        for (int j = i - 1; j >= 0 && a[i].rb < a[j].re + o.max_chain_gap; --j) {
            const S2Reg q = a[j], pp = a[i];
            if (q.qe == q.qb) continue;
            const int64_t or_ = q.re - pp.rb;
            const int64_t oq = q.qb < pp.qb ? q.qe - pp.qb : pp.qe - q.qb;
            const int64_t mr = q.re - q.rb < pp.re - pp.rb ? q.re - q.rb : pp.re - pp.rb;
            const int64_t mq = q.qe - q.qb < pp.qe - pp.qb ? q.qe - q.qb : pp.qe - pp.qb;
            S2DBG("dedup i %d j %d q [%d,%d) r [%ld,%ld) s %d | pp [%d,%d) r [%ld,%ld) s %d\n", i, j, q.qb, q.qe,
                  (long)q.rb, (long)q.re, q.score, pp.qb, pp.qe, (long)pp.rb, (long)pp.re, pp.score);
            if ((float)or_ > 0.95f * (float)mr && (float)oq > 0.95f * (float)mq) {
                const bool drop_p = pp.score < q.score;
                wave_sync();
                if (lane == 0) {
                    if (drop_p) a[i].qe = a[i].qb;
                    else a[j].qe = a[j].qb;
                }
                wave_sync();
                if (drop_p) break;
            } else if (q.rb < pp.rb) {
                int w = 0;
                S2DBG("patch i %d j %d q [%d,%d) r [%ld,%ld) w %d | pp [%d,%d) r [%ld,%ld) w %d\n", i, j, q.qb, q.qe,
                      (long)q.rb, (long)q.re, q.w, pp.qb, pp.qe, (long)pp.rb, (long)pp.re, pp.w);
                const int score = s2_patch_reg<CPL>(X, p, q, pp, &w, zg, lane);
                S2DBG("patch score %d\n", score);
                if (score > 0) {
                    wave_sync();
                    if (lane == 0) {
                        a[i].qb = q.qb; a[i].rb = q.rb;
                        a[i].truesc = a[i].score = score;
                        a[i].w = w;
                        a[j].qb = a[j].qe;
                    }
                    wave_sync();
                }
            }
        }
    }
    int m = 0;
    S2DBG("dedup final\n");
    if (lane == 0) {
        for (int i = 0; i < n; ++i)
            if (a[i].qe > a[i].qb) a[m++] = a[i];
        S2DBG("dedup final m %d\n", m);
        ks_introsort(a, m, LtArs());
        S2DBG("dedup final sorted\n");
        for (int i = 1; i < m; ++i)
            if (a[i].score == a[i - 1].score && a[i].rb == a[i - 1].rb && a[i].qb == a[i - 1].qb) a[i].qe = a[i].qb;
        int mm = 1;
        for (int i = 1; i < m; ++i)
            if (a[i].qe > a[i].qb) a[mm++] = a[i];
        S.misc[0] = mm;  // (bwa returns 1 for an emptied list, which cannot occur)
    }
    wave_sync();
    return S.misc[0];
}

// K2: mem_align1_core for every candidate read (one wave per read)
template <int CPL>
__global__ __launch_bounds__(64, AF_S2_WPS) void k_s2_regions(DevText X, const uint8_t *__restrict__ reads,
                                                             int32_t stride, const int32_t *__restrict__ lens,
                                                             af_params p, S2Opt o, const int32_t *__restrict__ cand,
                                                             const int32_t *__restrict__ n_cand, S2Work w,
                                                             uint8_t *__restrict__ zscratch, size_t zstride) {
    DpLds &L = g_dp;
    S2Lds &S = g_s2;
    const int lane = threadIdx.x;
    const int ncand = *n_cand;
    uint8_t *zg = zscratch + (size_t)blockIdx.x * zstride;
    int head = (int)(blockIdx.x & 7), heads_left = 8;
    for (;;) {
        int item = ncand;
        while (heads_left > 0) {
            int v = 0;
            if (lane == 0) v = atomicAdd(&w.heads_k2[AF_HEAD_STRIDE * head], 1);
            v = __builtin_amdgcn_readfirstlane(v);
            const int64_t it = head + 8 * (int64_t)v;
            if (it < ncand) { item = (int)it; break; }
            head = (head + 1) & 7;
            --heads_left;
        }
        if (item >= ncand) break;
        const int64_t r = cand[item];
        SPROF(const int64_t t0 = clock64(); int64_t t1 = t0, t2 = t0, t3 = t0, t4 = t0;
              if (lane == 0) g_ext[0] = g_ext[1] = 0;)
        int l = lens ? lens[r] : stride;
        if (l > stride) l = stride;
        if (l > AF_MAX_READ) l = AF_MAX_READ;
        if (l < 0) l = 0;
        const uint8_t *rd = reads + r * (int64_t)stride;
        for (int x = lane; x < l; x += 64) {
            const uint8_t ch = rd[x];
            uint8_t v = 4;
            switch (ch) {
            case 'A': case 'a': v = 0; break;
            case 'C': case 'c': v = 1; break;
            case 'G': case 'g': v = 2; break;
            case 'T': case 't': v = 3; break;
            default: v = 4;
            }
            L.q[x] = v;
        }
        if (lane < 8) S.cnt[lane] = 0;
        wave_sync();
        if (lane < AF_MAX_READ / 16 + 2) {
            const int b0 = lane * 16;
            uint32_t pw = 0, nw = 0;
            if (b0 < l) {
                const uint4 cc = *reinterpret_cast<const uint4 *>(&L.q[b0]);
                const uint32_t cw[4] = {cc.x, cc.y, cc.z, cc.w};
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const uint32_t y = cw[u] & 0x03030303u, t = y | (y >> 6);
                    pw |= ((t & 0xFu) | ((t >> 12) & 0xF0u)) << (8 * u);
                    nw |= ((((cw[u] >> 2) & 0x01010101u) * 0x01020408u) >> 24 & 0xFu) << (4 * u);
                }
            }
            const int valid = l - b0;
            if (valid < 16) nw |= valid <= 0 ? 0xFFFFu : (0xFFFFu << valid) & 0xFFFFu;
            L.pk[lane] = pw;
            L.nm[lane] = nw;
        }
        wave_sync();
        int n_reg = 0;
        SPROF(int pr_npm = 0, pr_nsi = 0, pr_nch = 0, pr_nreg0 = 0;)
        if (l >= p.min_seed_len) {
            s2_collect_intv(X, p, o, l, lane);
            SPROF(t1 = clock64(); pr_npm = S.cnt[0]; pr_nsi = S.cnt[1];)
            int n_chn = 0;
            if (!S.cnt[3]) {
                if (lane == 0) {
                    int nc = s2_mem_chain(X, p, o);
                    if (nc < 0) S.cnt[3] = 1;
                    else nc = s2_chain_flt(nc, p, o);
                    S.misc[1] = nc;
                    S.cnt[7] = 0;
                }
                wave_sync();
                n_chn = S.misc[1];
            }
            SPROF(t2 = clock64(); pr_nch = n_chn;)
            S2DBG("k2 read %d chains %d ovf %d\n", (int)r, n_chn, S.cnt[3]);
            for (int ci = 0; ci < n_chn && !S.cnt[3]; ++ci) s2_chain2aln<CPL>(X, p, l, ci, lane);
            SPROF(t3 = clock64(); pr_nreg0 = S.cnt[7];)
            S2DBG("k2 read %d regions %d\n", (int)r, S.cnt[7]);
            if (!S.cnt[3]) n_reg = s2_dedup_patch<CPL>(X, p, o, S.cnt[7], zg, lane);
            SPROF(t4 = clock64();)
            S2DBG("k2 read %d dedup %d\n", (int)r, n_reg);
        }
        const bool ovf = S.cnt[3] != 0;
        int off = 0;
        if (!ovf && n_reg > 0) {
            if (lane == 0) S.misc[2] = atomicAdd(w.pool_n, n_reg);
            wave_sync();
            off = S.misc[2];
        }
        const bool pool_ovf = !ovf && n_reg > 0 && (int64_t)off + n_reg > w.pool_cap;
        if (!ovf && !pool_ovf)
            for (int k = lane; k < n_reg; k += 64) w.pool[off + k] = S.x.reg[k];
        if (lane == 0) w.rmap[r] = (ovf || pool_ovf) ? int2{0, -1} : int2{off, n_reg};
        SPROF(if (lane == 0 && g_s2prof) {
            int32_t *pf = g_s2prof + (int64_t)item * 16;
            const int64_t t5 = clock64();
            pf[0] = (int32_t)r; pf[1] = (int32_t)(t5 - t0); pf[2] = (int32_t)(t1 - t0); pf[3] = (int32_t)(t2 - t1);
            pf[4] = (int32_t)(t3 - t2); pf[5] = (int32_t)(t4 - t3); pf[6] = pr_npm; pf[7] = pr_nsi; pf[8] = pr_nch;
            pf[9] = pr_nreg0; pf[10] = n_reg; pf[11] = g_ext[0] << 8 | min(g_ext[1], 255);
            pf[12] = (int32_t)(g_sub[0] - t0); pf[13] = (int32_t)(g_sub[1] - g_sub[0]);
            pf[14] = (int32_t)(g_sub[2] - g_sub[1]); pf[15] = (int32_t)(g_sub[3] - g_sub[2]);
            pf[6] |= (int32_t)min(g_sub[4] - g_sub[3], (int64_t)0x7FFFFF) << 8;
        })
        wave_sync();
    }
}

// ============================================================================ K3a
__device__ __forceinline__ int s2_chunk_of(const S2Work &w, int64_t pp) {
    if (w.ppc) return (int)(pp / w.ppc);
    int lo = 0, hi = *w.n_chunks;  // cstart[lo] <= pp < cstart[hi]
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (w.cstart[mid] <= pp) lo = mid;
        else hi = mid;
    }
    return lo;
}

__device__ __forceinline__ int s2_infer_dir(int64_t l_pac, int64_t b1, int64_t b2, int64_t *dist) {
    const int r1 = b1 >= l_pac, r2 = b2 >= l_pac;
    const int64_t p2 = r1 == r2 ? b2 : (l_pac << 1) - 1 - b2;
    *dist = p2 > b1 ? p2 - b1 : b1 - p2;
    return (r1 == r2 ? 0 : 1) ^ (p2 > b1 ? 0 : 3);
}

// cal_sub (oracle cal_sub) over a pool region list
__device__ int s2_cal_sub(const S2Reg *a, int n, int msl, int asc) {
    const S2Reg a0 = a[0];
    int j;
    for (j = 1; j < n; ++j) {
        const S2Reg aj = a[j];
        const int b_max = aj.qb > a0.qb ? aj.qb : a0.qb;
        const int e_min = aj.qe < a0.qe ? aj.qe : a0.qe;
        if (e_min > b_max) {
            const int min_l = aj.qe - aj.qb < a0.qe - a0.qb ? aj.qe - aj.qb : a0.qe - a0.qb;
            if ((float)(e_min - b_max) >= (float)min_l * 0.5f) break;
        }
    }
    return j < n ? a[j].score : msl * asc;
}

// One workgroup per AF_S2_CLS_PAIRS consecutive pairs: the listed pairs are gathered in LDS and
// appended with one atomic per workgroup; insert sizes go to the chunk histograms.
constexpr int CLS_THREADS = 256, CLS_PER = 16, AF_S2_CLS_PAIRS = CLS_THREADS * CLS_PER;
__global__ __launch_bounds__(CLS_THREADS) void k_s2_classify(int64_t n_pairs, int64_t l_pac,
                                                             const int32_t *__restrict__ hits, af_params p, S2Opt o,
                                                             S2Work w, af_aln_out out) {
    __shared__ int32_t lst[AF_S2_CLS_PAIRS];
    __shared__ int32_t nl, base;
    const int tid = threadIdx.x;
    if (blockIdx.x == 0 && tid < 8) {  // K2 ran; the previous call's K3c ran
        w.heads_k2[AF_HEAD_STRIDE * tid] = 0;
        w.heads_k3[AF_HEAD_STRIDE * tid] = 0;
        if (tid < 5 && w.sp.cnt) w.sp.cnt[tid] = tid == 4 ? 1ull << 62 : 0;  // K3c's heavy-pair counters
    }
    if (tid == 0) nl = 0;
    __syncthreads();
    const int64_t b0 = (int64_t)blockIdx.x * AF_S2_CLS_PAIRS;
    typedef int i32x2 __attribute__((ext_vector_type(2)));
    for (int k = 0; k < CLS_PER; ++k) {
        const int64_t pp = b0 + k * CLS_THREADS + tid;
        if (pp >= n_pairs) break;
        const i32x2 h = __builtin_nontemporal_load(reinterpret_cast<const i32x2 *>(hits) + pp);
        if (h.x == 0 && h.y == 0) {
            // both reads unmapped: flags 0x1|0x4|0x8|0x40 / 0x80, no position (bwa prints 0 and '*')
            __builtin_nontemporal_store(i32x2{0x4D, 0x8D}, reinterpret_cast<i32x2 *>(out.flag) + pp);
            __builtin_nontemporal_store(i32x2{-1, -1}, reinterpret_cast<i32x2 *>(out.pos) + pp);
            __builtin_nontemporal_store(i32x2{0, 0}, reinterpret_cast<i32x2 *>(out.score) + pp);
            __builtin_nontemporal_store(i32x2{0, 0}, reinterpret_cast<i32x2 *>(out.n_cigar) + pp);
            continue;
        }
        lst[atomicAdd(&nl, 1)] = (int32_t)pp;
        const int2 m0 = h.x > 0 ? w.rmap[2 * pp] : int2{0, 0};
        const int2 m1 = h.y > 0 ? w.rmap[2 * pp + 1] : int2{0, 0};
        if (m0.y > 0 && m1.y > 0) {  // mem_pestat's candidate unique pairs
            const S2Reg *a0 = w.pool + m0.x, *a1 = w.pool + m1.x;
            const int s0 = a0[0].score, s1 = a1[0].score;
            if (!((double)s2_cal_sub(a0, m0.y, p.min_seed_len, p.a) > 0.8 * s0) &&
                !((double)s2_cal_sub(a1, m1.y, p.min_seed_len, p.a) > 0.8 * s1)) {
                int64_t is;
                const int dir = s2_infer_dir(l_pac, a0[0].rb, a1[0].rb, &is);
                if (is && is <= o.max_ins) {
                    const int c = s2_chunk_of(w, pp);
                    atomicAdd(&w.ghist[((int64_t)c * 4 + dir) * (o.max_ins + 1) + is], 1);
                }
            }
        }
    }
    __syncthreads();
    if (tid == 0) base = nl ? atomicAdd(w.n_plist, nl) : 0;
    __syncthreads();
    for (int i = tid; i < nl; i += CLS_THREADS) w.plist[base + i] = lst[i];
}

// ============================================================================ K3b
// mem_pestat (oracle mem_pestat) for one chunk: per orientation, the chunk's insert-size
// histogram (counted by K3a) gives the percentiles by a block scan and the mean / standard
// deviation in bwa's summation order (sizes ascending); the histogram is zeroed for the next call
__global__ __launch_bounds__(256) void k_s2_pestat(S2Work w, int32_t max_ins) {
    __shared__ int part[256];
    __shared__ int nn[4], pv[3];
    const int c = blockIdx.x, tid = threadIdx.x;
    const int nch = w.ppc ? w.n_chunks_u : *w.n_chunks;
    if (c >= nch) return;
    const int nb = max_ins + 1;
    const int per = (nb + 255) / 256;
    S2Pes res[4];
    for (int d = 0; d < 4; ++d) {
        int *hist = w.ghist + ((int64_t)c * 4 + d) * nb;
        // this thread's bins [tid * per, (tid + 1) * per): its count, then an exclusive block scan
        int cnt = 0;
        for (int v = tid * per; v < min(nb, (tid + 1) * per); ++v) cnt += hist[v];
        part[tid] = cnt;
        __syncthreads();
        if (tid == 0) {
            int acc = 0;
            for (int t = 0; t < 256; ++t) { const int x = part[t]; part[t] = acc; acc += x; }
            nn[d] = acc;
        }
        __syncthreads();
        const int nd = nn[d];
        S2Pes &r = res[d];
        r.low = r.high = 0; r.failed = 0; r.pad = 0; r.avg = 0; r.std = 0;
        if (nd < 10) {  // MIN_DIR_CNT (the histogram may still hold a few sizes)
            r.failed = 1;
        } else {
            // percentiles q[(int)(f * n + .499)] of the sorted sizes
            const int kk[3] = {(int)(.25 * nd + .499), (int)(.50 * nd + .499), (int)(.75 * nd + .499)};
            int cum = part[tid];
            for (int v = tid * per; v < min(nb, (tid + 1) * per); ++v) {
                const int h = hist[v];
                for (int q = 0; q < 3; ++q)
                    if (cum <= kk[q] && kk[q] < cum + h) pv[q] = v;
                cum += h;
            }
            __syncthreads();
            if (tid == 0) {
                const int p25 = pv[0], p75 = pv[2];
                r.low = (int)(p25 - 2.0 * (p75 - p25) + .499);
                if (r.low < 1) r.low = 1;
                r.high = (int)(p75 + 2.0 * (p75 - p25) + .499);
                long long sum = 0;
                int x = 0;
                for (int v = r.low; v <= r.high && v < nb; ++v) { sum += (long long)v * hist[v]; x += hist[v]; }
                // bwa adds the sizes in sorted order in double: integers, exact below 2^53
                double avg = (double)sum;
                avg /= x;
                double sd = 0;
                for (int v = r.low; v <= r.high && v < nb; ++v)
                    for (int k = 0, h = hist[v]; k < h; ++k) sd += ((double)v - avg) * ((double)v - avg);
                sd = sqrt(sd / x);
                r.avg = avg; r.std = sd;
                r.low = (int)(p25 - 3.0 * (p75 - p25) + .499);
                r.high = (int)(p75 + 3.0 * (p75 - p25) + .499);
                if (r.low > avg - 4.0 * sd) r.low = (int)(avg - 4.0 * sd + .499);
                if (r.high < avg + 4.0 * sd) r.high = (int)(avg + 4.0 * sd + .499);
                if (r.low < 1) r.low = 1;
            }
        }
        __syncthreads();
        if (nd > 0)
            for (int v = tid * per; v < min(nb, (tid + 1) * per); ++v) hist[v] = 0;
    }
    if (tid == 0) {
        int mx = 0;
        for (int d = 0; d < 4; ++d) mx = mx > nn[d] ? mx : nn[d];
        for (int d = 0; d < 4; ++d) {
            if (res[d].failed == 0 && (double)nn[d] < mx * 0.05) res[d].failed = 1;
            w.pes[(int64_t)c * 4 + d] = res[d];
        }
    }
}

// ============================================================================ K3c
struct PeReg {
    S2Reg r;
    uint64_t hash;
    int32_t secondary, pad;
};
struct P64 { uint64_t x, y; };
constexpr int PE_TW = 2048;  // rescue windows up to this many bases are staged in LDS
struct __attribute__((aligned(16))) PeLds {
    PeReg a[2][AF_S2_MAX_REG];
    int64_t brb[2][AF_S2_MAX_REG];
    P64 v[2 * AF_S2_MAX_REG];          // mem_pair's hit list
    int32_t zz[AF_S2_MAX_REG];         // mem_mark_primary_se_core's kept hits
    uint8_t q[2][AF_MAX_READ + 16];
    uint8_t rq[AF_MAX_READ + 16];      // the rescue query (mate, maybe reverse-complemented)
    uint8_t rq2[AF_MAX_READ + 16];     // its reversed prefix (ksw_align2's start pass)
    uint8_t tw[PE_TW];                 // the rescue window of the reference
    S2Pes pes[4];
    int32_t na[2], nb[2], ovf[2], len[2];
    int32_t which[2], extra, misc[8];
};
__shared__ PeLds g_pe;

// the decision K3c hands to the record kernel K3d, per listed pair
struct S2Plan {
    S2Reg r[2];
    int32_t which[2], sec[2], extra, ovf;
};

// ksw_align2 with KSW_XSUBO | KSW_XSTART (oracle ksw_align2): score, te, qe and the start (tb, qb)
__device__ void s2_ksw_align2(const uint8_t *q, int qlen, const uint8_t *target, int tlen, int P, int minsc,
                              const af_params &p, int &score, int &te, int &qe, int &tb, int &qb, int lane) {
    PeLds &E = g_pe;
    const SwRes r = ksw_pass_any(q, qlen, target, tlen, -1, P, p, 0x10000, lane);
    score = r.score; te = r.te; qe = r.qe; tb = -1; qb = -1;
    if (r.score < minsc || r.qe < 0) return;
    for (int x = lane; x <= r.qe; x += 64) E.rq2[x] = q[r.qe - x];
    wave_sync();
    const SwRes rr = ksw_pass_any(E.rq2, r.qe + 1, target, tlen, r.te, P, p, r.score, lane);
    wave_sync();
    if (r.score == rr.score) { tb = r.te - rr.te; qb = r.qe - rr.qe; }
}

// mem_sort_dedup_patch without patching (mate-SW context) on the wave.  The two sorts run over
// keys (re | index; rb, score, qb | index): by rank on the wave when no two keys tie, else klib's
// introsort on lane 0 -- its swaps depend only on the comparator's answers, so the order, ties
// included, is the one the introsort over the regions gives.  Without patching, a[i]'s walk only
// drops, and a[i] itself does not change along it: every overlapping q below a[i] (all of them
// fit one wave, n <= 32) is known at once; they drop in walk order until one outscores a[i],
// which drops a[i] instead and ends its walk.
constexpr int PE_W8 = (int)(sizeof(PeReg) / 8);  // a region moves as this many 8-byte words
static_assert(AF_S2_MAX_REG <= 32 && sizeof(PeReg) % 8 == 0 && sizeof(P64) * 2 * AF_S2_MAX_REG >= 32 * AF_S2_MAX_REG,
              "the dedup moves <= 32 regions through registers; its keys fit E.v");
struct S2KeyRe {  // re << 6 | index
    __device__ bool operator()(uint64_t a, uint64_t b) const { return (a >> 6) < (b >> 6); }
};
struct S2Key16 { int64_t x; int32_t y; int32_t z; };
struct S2KeyArs {  // x = rb, y = score, z = qb << 8 | index: score desc, rb, qb (LtArs)
    __device__ bool operator()(const S2Key16 &a, const S2Key16 &b) const {
        return a.y > b.y || (a.y == b.y && (a.x < b.x || (a.x == b.x && (a.z >> 8) < (b.z >> 8))));
    }
};
// a[k] = old a[from(k)] for k < m <= 64 (wave; through registers)
template <class F>
__device__ __forceinline__ void s2_regs_gather(PeReg *a, int m, F from, int lane) {
    uint2 t[PE_W8];
    const int f = lane < m ? from(lane) : 0;
    if (lane < m)
        for (int c = 0; c < PE_W8; ++c) t[c] = reinterpret_cast<const uint2 *>(a + f)[c];
    __threadfence_block();
    wave_sync();
    if (lane < m)
        for (int c = 0; c < PE_W8; ++c) reinterpret_cast<uint2 *>(a + lane)[c] = t[c];
    __threadfence_block();
    wave_sync();
}

__device__ int s2_dedup_nopatch(PeReg *a, int n, int max_chain_gap, int lane) {
    if (n <= 1) return n;
    PeLds &E = g_pe;
    uint64_t *k1 = reinterpret_cast<uint64_t *>(E.v), *t1 = k1 + AF_S2_MAX_REG;
    if (lane < n) k1[lane] = (uint64_t)a[lane].r.re << 6 | (uint64_t)lane;
    wave_sync();
    if (!wave_rank_sort(k1, n, S2KeyRe(), t1, lane)) {
        if (lane == 0) ks_introsort(k1, n, S2KeyRe());
        wave_sync();
    }
    s2_regs_gather(a, n, [&](int k) { return (int)(k1[k] & 63); }, lane);
    for (int i = 1; i < n; ++i) {
        const S2Reg pp = a[i].r;
        const int jj = i - 1 - lane;
        bool cont = false, ev = false, win = false;
        if (jj >= 0) {
            const S2Reg q = a[jj].r;
            cont = pp.rb < q.re + max_chain_gap;
            if (cont && q.qe != q.qb) {
                const int64_t or_ = q.re - pp.rb;
                const int64_t oq = q.qb < pp.qb ? q.qe - pp.qb : pp.qe - q.qb;
                const int64_t mr = q.re - q.rb < pp.re - pp.rb ? q.re - q.rb : pp.re - pp.rb;
                const int64_t mq = q.qe - q.qb < pp.qe - pp.qb ? q.qe - q.qb : pp.qe - pp.qb;
                ev = (float)or_ > 0.95f * (float)mr && (float)oq > 0.95f * (float)mq;
                win = ev && pp.score < q.score;
            }
        }
        // the walk reaches lanes below the first that leaves the window
        const uint64_t stop = __ballot(!cont);
        const uint64_t reach = stop ? (stop & (0ull - stop)) - 1 : ~0ull;
        const uint64_t wm = __ballot(win) & reach;
        // events before the first q that outscores a[i] drop their q; that q drops a[i]
        const uint64_t before = wm ? (wm & (0ull - wm)) - 1 : reach;
        if (ev && ((1ull << lane) & before)) a[jj].r.qe = a[jj].r.qb;
        if (wm && lane == 0) a[i].r.qe = a[i].r.qb;
        __threadfence_block();
        wave_sync();
    }
    // the live regions (in order) sorted by LtArs; equal neighbours dropped
    const bool live = lane < n && a[lane].r.qe > a[lane].r.qb;
    const uint64_t lm = __ballot(live);
    const int m = __popcll(lm);
    S2Key16 *k2 = reinterpret_cast<S2Key16 *>(E.v), *t2 = k2 + AF_S2_MAX_REG;
    if (live) {
        const int pos = __popcll(lm & ((1ull << lane) - 1));
        const S2Reg &r = a[lane].r;
        k2[pos] = S2Key16{r.rb, r.score, r.qb << 8 | lane};
    }
    wave_sync();
    if (m == 0) return 0;
    if (!wave_rank_sort(k2, m, S2KeyArs(), t2, lane)) {
        if (lane == 0) ks_introsort(k2, m, S2KeyArs());
        wave_sync();
    }
    bool keep = false;
    if (lane < m) {
        const S2Key16 x = k2[lane];
        keep = lane == 0;
        if (lane > 0) {
            const S2Key16 y = k2[lane - 1];
            keep = !(x.y == y.y && x.x == y.x && (x.z >> 8) == (y.z >> 8));
        }
    }
    const uint64_t km = __ballot(keep);
    const int mm = __popcll(km);
    // surviving key k goes to slot popc(km below k); gather by the inverse map
    int *src = reinterpret_cast<int *>(t2);
    if (keep) src[__popcll(km & ((1ull << lane) - 1))] = k2[lane].z & 255;
    __threadfence_block();
    wave_sync();
    s2_regs_gather(a, mm, [&](int k) { return src[k]; }, lane);
    return mm;
}

// mem_matesw's window of direction r for a mate region starting at a_rb (the rescued read l_ms
// long): [rb, re) clipped to the strand's half of the doubled text; true when bwa runs its SW there
__device__ __forceinline__ bool s2_mate_window(int64_t l_pac, const af_params &p, const S2Pes &pe, int r,
                                               int64_t a_rb, int l_ms, int64_t &rb, int64_t &re, int &rid) {
    const bool is_rev = (r >> 1) != (r & 1);
    const bool is_larger = !(r >> 1);
    if (!is_rev) {
        rb = is_larger ? a_rb + pe.low : a_rb - pe.high;
        re = (is_larger ? a_rb + pe.high : a_rb - pe.low) + l_ms;
    } else {
        rb = (is_larger ? a_rb + pe.low : a_rb - pe.high) - l_ms;
        re = is_larger ? a_rb + pe.high : a_rb - pe.low;
    }
    if (rb < 0) rb = 0;
    if (re > l_pac << 1) re = l_pac << 1;
    if (rb < re) {
        const int64_t mid = (rb + re) >> 1;
        const int64_t fb = mid < l_pac ? 0 : l_pac, fe = mid < l_pac ? l_pac : l_pac << 1;
        rb = rb > fb ? rb : fb;
        re = re < fe ? re : fe;
        rid = 0;
    }
    // (rb >= re keeps rid from an earlier direction, as bwa does; re - rb < min_seed_len then)
    return rid == 0 && re - rb >= p.min_seed_len;
}

// that window's ksw_align2 for the rescued read's codes qc (strand of direction r)
__device__ __forceinline__ void s2_mate_ksw(const DevText &X, const af_params &p, const uint8_t *qc, int l_ms, int r,
                                            int64_t rb, int64_t re, int &sc, int &te, int &qe, int &tb, int &qb,
                                            int lane) {
    PeLds &E = g_pe;
    const bool is_rev = (r >> 1) != (r & 1);
    for (int x = lane; x < l_ms; x += 64) {
        const int c = qc[is_rev ? l_ms - 1 - x : x];
        E.rq[x] = (uint8_t)(is_rev ? (c < 4 ? 3 - c : 4) : c);
    }
    const bool staged = re - rb <= PE_TW;
    if (staged)
        for (int x = lane; x < (int)(re - rb); x += 64) E.tw[x] = X.T[rb + x];
    wave_sync();
    const int P = l_ms * p.a < 250 ? 16 : 8;
    SPROF(if (lane == 0) E.misc[7] += (int)(re - rb);)
    s2_ksw_align2(E.rq, l_ms, staged ? E.tw : X.T + rb, (int)(re - rb), P, p.min_seed_len * p.a, p, sc, te, qe, tb, qb,
                  lane);
}

// mem_matesw (oracle mem_matesw): rescue read mi in the insert-size window of a region at a_rb
// of its mate.  sr: the windows' SW results computed ahead (k_s2_pe_jobs; 4 directions x
// AF_G_PE_RES_W ints) or null.  Returns false on a region-cap overflow of read mi.
template <bool SPEC>
__device__ bool s2_matesw(const DevText &X, const af_params &p, const S2Opt &o, int mi, int64_t a_rb,
                          const int32_t *sr, int lane) {
    PeLds &E = g_pe;
    const int64_t l_pac = X.n;
    const int l_ms = E.len[mi];
    int skip[4];
    for (int r = 0; r < 4; ++r) skip[r] = E.pes[r].failed ? 1 : 0;
    for (int i = 0; i < E.na[mi]; ++i) {
        int64_t dist;
        const int r = s2_infer_dir(l_pac, a_rb, E.a[mi][i].r.rb, &dist);
        if (dist >= E.pes[r].low && dist <= E.pes[r].high) skip[r] = 1;
    }
    if (skip[0] + skip[1] + skip[2] + skip[3] == 4) return true;
    int n = 0, rid = -1;
    // bwa sorts and dedups the list after every searched direction once one has been searched;
    // the dedup is idempotent on its own output (its walk drops nothing more, its final order is by
    // unique keys), so it runs only when a rescued region went in since the last one
    bool deduped = false, dirty = false;
    for (int r = 0; r < 4; ++r) {
        if (skip[r]) continue;
        const bool is_rev = (r >> 1) != (r & 1);
        int64_t rb, re;
        if (s2_mate_window(l_pac, p, E.pes[r], r, a_rb, l_ms, rb, re, rid)) {
            int sc, te, qe, tb, qb;
            const int32_t *res = SPEC && sr ? sr + r * AF_G_PE_RES_W : nullptr;
            if (SPEC && res && res[5]) {
                sc = res[0]; te = res[1]; qe = res[2]; tb = res[3]; qb = res[4];
            } else {
                s2_mate_ksw(X, p, E.q[mi], l_ms, r, rb, re, sc, te, qe, tb, qb, lane);
            }
            if (sc >= p.min_seed_len && qb >= 0) {
                // into the list before the first region scoring less (regions move up on the wave)
                const int na = E.na[mi];
                if (na >= AF_S2_MAX_REG) return false;
                PeReg *ma = E.a[mi];
                const uint64_t lt = __ballot(lane < na && ma[lane].r.score < sc);
                const int i = lt ? __builtin_ctzll(lt) : na;
                uint2 t[PE_W8];
                const bool mv = lane >= i && lane < na;
                if (mv)
                    for (int c = 0; c < PE_W8; ++c) t[c] = reinterpret_cast<const uint2 *>(ma + lane)[c];
                __threadfence_block();
                wave_sync();
                if (mv)
                    for (int c = 0; c < PE_W8; ++c) reinterpret_cast<uint2 *>(ma + lane + 1)[c] = t[c];
                if (lane == 0) {
                    PeReg b{};
                    b.r.qb = is_rev ? l_ms - (qe + 1) : qb;
                    b.r.qe = is_rev ? l_ms - qb : qe + 1;
                    b.r.rb = is_rev ? (l_pac << 1) - (rb + te + 1) : rb + tb;
                    b.r.re = is_rev ? (l_pac << 1) - (rb + tb) : rb + te + 1;
                    b.r.score = sc;
                    b.r.truesc = 0; b.r.w = 0; b.r.seedlen0 = 0;
                    b.secondary = -1;
                    ma[i] = b;
                    E.na[mi] = na + 1;
                }
                __threadfence_block();
                wave_sync();
                dirty = true;
            }
            ++n;
        }
        if (n && (!deduped || dirty)) {
            {
                const int m = s2_dedup_nopatch(E.a[mi], E.na[mi], o.max_chain_gap, lane);
                if (lane == 0) E.na[mi] = m;
            }
            wave_sync();
            deduped = true;
            dirty = false;
        }
    }
    return true;
}

// mem_mark_primary_se (no ALT contigs) on the wave: the sort by (score desc, hash) over keys as in
// s2_dedup_nopatch, the kept-hit walk on lane 0
struct S2KeyHash {  // x = hash, y = score, z = index
    __device__ bool operator()(const S2Key16 &a, const S2Key16 &b) const {
        return a.y > b.y || (a.y == b.y && (uint64_t)a.x < (uint64_t)b.x);
    }
};
__device__ void s2_mark_primary(PeReg *a, int n, int64_t id, const af_params &p, int lane) {
    if (n == 0) return;
    PeLds &E = g_pe;
    S2Key16 *k = reinterpret_cast<S2Key16 *>(E.v), *t = k + AF_S2_MAX_REG;
    if (lane < n) {
        a[lane].secondary = -1;
        a[lane].hash = hash_64((uint64_t)(id + lane));
        k[lane] = S2Key16{(int64_t)a[lane].hash, a[lane].r.score, lane};
    }
    __threadfence_block();
    wave_sync();
    if (n > 1) {
        if (!wave_rank_sort(k, n, S2KeyHash(), t, lane)) {
            if (lane == 0) ks_introsort(k, n, S2KeyHash());
            wave_sync();
        }
        s2_regs_gather(a, n, [&](int x) { return k[x].z; }, lane);
    }
    if (lane == 0) {
        int32_t *z = E.zz;
        int nz = 0;
        z[nz++] = 0;
        for (int i = 1; i < n; ++i) {
            int kk;
            for (kk = 0; kk < nz; ++kk) {
                const int j = z[kk];
                const int b_max = a[j].r.qb > a[i].r.qb ? a[j].r.qb : a[i].r.qb;
                const int e_min = a[j].r.qe < a[i].r.qe ? a[j].r.qe : a[i].r.qe;
                if (e_min > b_max) {
                    const int min_l = a[i].r.qe - a[i].r.qb < a[j].r.qe - a[j].r.qb ? a[i].r.qe - a[i].r.qb : a[j].r.qe - a[j].r.qb;
                    if ((float)(e_min - b_max) >= (float)min_l * 0.5f) break;
                }
            }
            if (kk == nz) z[nz++] = i;
            else a[i].secondary = z[kk];
        }
    }
    __threadfence_block();
    wave_sync();
}

struct LtP64 {
    __device__ bool operator()(const P64 &a, const P64 &b) const { return a.x < b.x || (a.x == b.x && a.y < b.y); }
};

// mem_pair (oracle mem_pair), lane 0: the best pair's score (0 if none) and z[]
__device__ int s2_mem_pair(int64_t l_pac, const af_params &p, const S2Pes *pes, int id, int z[2]) {
    PeLds &E = g_pe;
    P64 *v = E.v;
    int nv = 0;
    for (int r = 0; r < 2; ++r)
        for (int i = 0; i < E.na[r]; ++i) {
            const S2Reg &e = E.a[r][i].r;
            P64 key;
            key.x = (uint64_t)(e.rb < l_pac ? e.rb : (l_pac << 1) - 1 - e.rb);
            key.y = (uint64_t)(uint32_t)e.score << 32 | (uint64_t)i << 2 | (uint64_t)(e.rb >= l_pac) << 1 | (uint64_t)r;
            v[nv++] = key;
        }
    ks_introsort(v, nv, LtP64());
    int y[4] = {-1, -1, -1, -1};
    bool have = false;
    P64 best{0, 0};
    for (int i = 0; i < nv; ++i) {
        for (int r = 0; r < 2; ++r) {
            const int dir = r << 1 | (int)(v[i].y >> 1 & 1);
            if (pes[dir].failed) continue;
            const int which = r << 1 | (int)((v[i].y & 1) ^ 1);
            if (y[which] < 0) continue;
            for (int k = y[which]; k >= 0; --k) {
                if ((int)(v[k].y & 3) != which) continue;
                const int64_t dist = (int64_t)v[i].x - (int64_t)v[k].x;
                if (dist > pes[dir].high) break;
                if (dist < pes[dir].low) continue;
                const double ns = ((double)dist - pes[dir].avg) / pes[dir].std;
                int q = (int)((double)((v[i].y >> 32) + (v[k].y >> 32)) + .721 * log(2. * erfc(fabs(ns) * 0.70710678118654752440)) * p.a + .499);
                if (q < 0) q = 0;
                P64 u;
                u.y = (uint64_t)k << 32 | (uint64_t)i;
                u.x = (uint64_t)q << 32 | (hash_64(u.y ^ (uint64_t)(int64_t)(int32_t)((uint32_t)id << 8)) & 0xffffffffU);
                if (!have || LtP64()(best, u)) { best = u; have = true; }
            }
        }
        y[v[i].y & 3] = i;
    }
    if (!have) return 0;
    const int i = (int)(best.y >> 32), k = (int)(best.y << 32 >> 32);
    z[v[i].y & 1] = (int)(v[i].y << 32 >> 34);
    z[v[k].y & 1] = (int)(v[k].y << 32 >> 34);
    return (int)(best.x >> 32);
}

// K3c: mem_sam_pe up to the record choice for every listed pair (one wave per pair): mate
// rescue, primary marking, pairing; the choice (S2Plan) goes to K3d
// mode 0: every listed pair; 1: every listed pair, those with at least w.sp.min_windows rescue
// windows left to k_s2_pe_jobs (their SWs) and mode 2 (the rest, with those SWs' results)
template <int mode>
__global__ __launch_bounds__(64, 4) void k_s2_pairs(DevText X, const uint8_t *__restrict__ reads, int32_t stride,
                                                 const int32_t *__restrict__ lens, af_params p, S2Opt o,
                                                 const int32_t *__restrict__ hits, S2Work w,
                                                 S2Plan *__restrict__ plan) {
    PeLds &E = g_pe;
    const int lane = threadIdx.x;
    const int64_t l_pac = X.n;
    const int npl = *w.n_plist;
    const GPeSpec &Y = w.sp;
    int64_t nh = 0;
    if constexpr (mode == 2) {
        nh = (int64_t)Y.cnt[0];
        if (nh > Y.cap_pairs) nh = Y.cap_pairs;
    }
    int head = (int)(blockIdx.x & 7), heads_left = 8;
    for (;;) {
        int item = npl;
        const int32_t *sres = nullptr;  // mode 2: the pair's precomputed SW results
        int nj0 = 0;
        if constexpr (mode == 2) {
            int64_t hp = 0;
            if (lane == 0) hp = (int64_t)atomicAdd(&Y.cnt[3], 1ull);
            hp = (int64_t)__builtin_amdgcn_readfirstlane((int)hp);
            if (hp >= nh) break;
            item = Y.pair[hp];
            if (item < 0) continue;  // reservation failed: mode 1 finished the pair
            sres = Y.res + (int64_t)Y.off[hp] * 4 * AF_G_PE_RES_W;
            nj0 = Y.nj[hp] & 0xffff;
        } else {
            while (heads_left > 0) {
                int v = 0;
                if (lane == 0) v = atomicAdd(&w.heads_k3[AF_HEAD_STRIDE * head], 1);
                v = __builtin_amdgcn_readfirstlane(v);
                const int64_t it = head + 8 * (int64_t)v;
                if (it < npl) { item = (int)it; break; }
                head = (head + 1) & 7;
                --heads_left;
            }
            if (item >= npl) break;
        }
        const int64_t pp = w.plist[item];
        S2DBG("k3c pair %d start\n", (int)pp);
        SPROF(const int64_t c0 = clock64(); int64_t c1 = c0, c2 = c0, c3 = c0; int nsw = 0;)
        // reads and their regions
        for (int m = 0; m < 2; ++m) {
            const int64_t r = 2 * pp + m;
            int l = lens ? lens[r] : stride;
            if (l > stride) l = stride;
            if (l > AF_MAX_READ) l = AF_MAX_READ;
            if (l < 0) l = 0;
            const uint8_t *rd = reads + r * (int64_t)stride;
            for (int x = lane; x < l; x += 64) {
                const uint8_t ch = rd[x];
                uint8_t v = 4;
                switch (ch) {
                case 'A': case 'a': v = 0; break;
                case 'C': case 'c': v = 1; break;
                case 'G': case 'g': v = 2; break;
                case 'T': case 't': v = 3; break;
                default: v = 4;
                }
                E.q[m][x] = v;
            }
            const int h = hits[r];
            const int2 mp = h > 0 ? w.rmap[r] : int2{0, 0};
            const int na = mp.y > 0 ? mp.y : 0;
            for (int k = lane; k < na; k += 64) E.a[m][k].r = w.pool[mp.x + k];
            if (lane == 0) { E.len[m] = l; E.na[m] = na; E.ovf[m] = mp.y < 0; }
        }
        if (lane < 4) E.pes[lane] = w.pes[(int64_t)s2_chunk_of(w, pp) * 4 + lane];
        wave_sync();
        // mate rescue for the top hits of each end
        if (lane == 0) {
            for (int i = 0; i < 2; ++i) {
                int nb = 0;
                for (int j = 0; j < E.na[i]; ++j)
                    if (E.a[i][j].r.score >= E.a[i][0].r.score - o.pen_unpaired) E.brb[i][nb++] = E.a[i][j].r.rb;
                E.nb[i] = nb;
            }
        }
        wave_sync();
        if constexpr (mode == 1) {
            // a heavy pair's windows to the job list (slot k: end i, its j-th top region); the pair
            // is finished by mode 2
            const int n0 = E.nb[0] < o.max_matesw ? E.nb[0] : o.max_matesw;
            const int n1 = E.nb[1] < o.max_matesw ? E.nb[1] : o.max_matesw;
            const int nwin = (E.ovf[1] ? 0 : n0) + (E.ovf[0] ? 0 : n1);
            if (nwin >= Y.min_windows) {
                int hp = -1, off = 0;
                if (lane == 0) {
                    const int64_t h = (int64_t)atomicAdd(&Y.cnt[0], 1ull);
                    if (h < Y.cap_pairs) {
                        const int64_t o0 = (int64_t)atomicAdd(&Y.cnt[1], (unsigned long long)(n0 + n1));
                        if (o0 + n0 + n1 <= Y.cap_jobs) {
                            hp = (int)h; off = (int)o0;
                            Y.pair[h] = item; Y.off[h] = off; Y.nj[h] = n0 | n1 << 16;
                        } else {
                            Y.pair[h] = -1;
                            atomicMin(&Y.cnt[4], (unsigned long long)o0);  // slots from o0 on are unwritten
                        }
                    }
                }
                hp = __builtin_amdgcn_readfirstlane(hp);
                off = __builtin_amdgcn_readfirstlane(off);
                if (hp >= 0) {
                    for (int k = lane; k < n0 + n1; k += 64) {
                        const int i = k >= n0, j = k - (i ? n0 : 0);
                        Y.job[off + k] = make_int2(hp, E.ovf[!i] ? -1 : (i << 16 | j));
                    }
                    wave_sync();
                    continue;
                }
            }
        }
        SPROF(c1 = clock64(); if (lane == 0) E.misc[7] = 0;)
        for (int i = 0; i < 2; ++i)
            for (int j = 0; j < E.nb[i] && j < o.max_matesw; ++j) {
                if (E.ovf[!i]) continue;
                const int32_t *sr = sres ? sres + (int64_t)((i ? nj0 : 0) + j) * 4 * AF_G_PE_RES_W : nullptr;
                if (!s2_matesw<mode == 2>(X, p, o, !i, E.brb[i][j], sr, lane)) {
                    wave_sync();
                    if (lane == 0) { E.ovf[!i] = 1; E.na[!i] = 0; }
                    wave_sync();
                }
            }
        SPROF(c2 = clock64(); nsw = E.misc[7];)
        // primary marking, pairing and the record choice (mem_sam_pe)
        const uint64_t id = (uint64_t)(o.pair_base + pp);
        s2_mark_primary(E.a[0], E.na[0], (int64_t)(id << 1 | 0), p, lane);
        s2_mark_primary(E.a[1], E.na[1], (int64_t)(id << 1 | 1), p, lane);
        if (lane == 0) {
            int z[2] = {0, 0}, extra = 1, which[2] = {-1, -1};
            bool paired = false;
            int o_sc = 0;
            if (E.na[0] && E.na[1] && (o_sc = s2_mem_pair(l_pac, p, E.pes, (int)(uint32_t)id, z)) > 0) {
                int is_multi = 0;
                for (int i = 0; i < 2; ++i) {
                    int j;
                    for (j = 1; j < E.na[i]; ++j)
                        if (E.a[i][j].secondary < 0 && E.a[i][j].r.score >= p.T) break;
                    is_multi |= j < E.na[i];
                }
                if (!is_multi) {
                    const int score_un = E.a[0][0].r.score + E.a[1][0].r.score - o.pen_unpaired;
                    if (o_sc > score_un) {
                        for (int i = 0; i < 2; ++i)
                            if (E.a[i][z[i]].secondary >= 0) E.a[i][z[i]].secondary = -2;
                        extra |= 2;
                    } else {
                        z[0] = z[1] = 0;
                    }
                    which[0] = z[0]; which[1] = z[1];
                    paired = true;
                }
            }
            if (!paired) {
                for (int i = 0; i < 2; ++i) which[i] = (E.na[i] && E.a[i][0].r.score >= p.T) ? 0 : -1;
                if (which[0] >= 0 && which[1] >= 0) {
                    int64_t dist;
                    const int d = s2_infer_dir(l_pac, E.a[0][0].r.rb, E.a[1][0].r.rb, &dist);
                    if (!E.pes[d].failed && dist >= E.pes[d].low && dist <= E.pes[d].high) extra |= 2;
                }
            }
            E.which[0] = which[0]; E.which[1] = which[1]; E.extra = extra;
        }
        wave_sync();
        SPROF(c3 = clock64();)
        if (lane == 0) {
            S2Plan &pl = plan[item];
            for (int m = 0; m < 2; ++m) {
                pl.which[m] = E.which[m];
                if (E.which[m] >= 0) {
                    pl.r[m] = E.a[m][E.which[m]].r;
                    pl.sec[m] = E.a[m][E.which[m]].secondary;
                }
            }
            pl.extra = E.extra;
            pl.ovf = E.ovf[0] | E.ovf[1] << 1;
        }
        SPROF(if (lane == 0 && g_s2prof) {
            int32_t *pf = g_s2prof + S2PROF_K3 + (int64_t)item * 16;
            const int64_t c4 = clock64();
            pf[0] = (int32_t)pp; pf[1] = (int32_t)(c4 - c0); pf[2] = (int32_t)(c1 - c0); pf[3] = (int32_t)(c2 - c1);
            pf[4] = (int32_t)(c3 - c2); pf[6] = nsw; pf[7] = E.na[0]; pf[8] = E.na[1];
        })
        wave_sync();
    }
}

// one rescue window of a heavy pair per wave (k_s2_pairs mode 1's job list): for each direction
// bwa may search, the window and its ksw_align2 as mem_matesw computes them (results ahead of the
// pair's own walk, which decides per window whether to use them)
__global__ __launch_bounds__(64, 4) void k_s2_pe_jobs(DevText X, const uint8_t *__restrict__ reads, int32_t stride,
                                                    const int32_t *__restrict__ lens, af_params p, S2Opt o,
                                                    const int32_t *__restrict__ hits, S2Work w) {
    PeLds &E = g_pe;
    const int lane = threadIdx.x;
    const GPeSpec &Y = w.sp;
    int64_t n = (int64_t)Y.cnt[1];
    if (n > Y.cap_jobs) n = Y.cap_jobs;
    if (n > (int64_t)Y.cnt[4]) n = (int64_t)Y.cnt[4];
    for (;;) {
        int64_t k = 0;
        if (lane == 0) k = (int64_t)atomicAdd(&Y.cnt[2], 1ull);
        k = (int64_t)__builtin_amdgcn_readfirstlane((int)k);
        if (k >= n) break;
        const int2 jb = Y.job[k];
        if (jb.y < 0) continue;
        const int i = jb.y >> 16, j = jb.y & 0xffff;
        const int64_t pp = w.plist[Y.pair[jb.x]];
        int32_t *out = Y.res + k * 4 * AF_G_PE_RES_W;
        // the rescued read (the other end) and its codes
        const int64_t rm = 2 * pp + !i;
        int l_ms = lens ? lens[rm] : stride;
        if (l_ms > stride) l_ms = stride;
        if (l_ms > AF_MAX_READ) l_ms = AF_MAX_READ;
        if (l_ms < 0) l_ms = 0;
        for (int x = lane; x < l_ms; x += 64) {
            const uint8_t ch = reads[rm * (int64_t)stride + x];
            E.q[0][x] = ch == 'A' || ch == 'a' ? 0 : ch == 'C' || ch == 'c' ? 1 : ch == 'G' || ch == 'g' ? 2
                      : ch == 'T' || ch == 't' ? 3 : 4;
        }
        if (lane < 4) E.pes[lane] = w.pes[(int64_t)s2_chunk_of(w, pp) * 4 + lane];
        // a_rb: end i's j-th region scoring within pen_unpaired of its best (K3c's list)
        const int64_t ri = 2 * pp + i;
        const int h = hits[ri];
        const int2 mp = h > 0 ? w.rmap[ri] : int2{0, 0};
        const int na = mp.y > 0 ? mp.y : 0;
        const S2Reg *ai = w.pool + mp.x;
        const int top = na ? ai[0].score : 0;
        int seen = 0, at = -1;
        for (int c0 = 0; c0 < na && at < 0; c0 += 64) {
            const bool q = c0 + lane < na && ai[c0 + lane].score >= top - o.pen_unpaired;
            const uint64_t m = __ballot(q);
            const int cnt = __builtin_popcountll(m);
            if (seen + cnt > j) {
                uint64_t mm = m;
                for (int t = 0; t < j - seen; ++t) mm &= mm - 1;
                at = c0 + __builtin_ctzll(mm);
            }
            seen += cnt;
        }
        wave_sync();
        if (at < 0) {  // (no such region: never used)
            if (lane < 4) out[lane * AF_G_PE_RES_W + 5] = 0;
            continue;
        }
        const int64_t a_rb = ai[at].rb;
        int rid = -1;
        for (int r = 0; r < 4; ++r) {
            int64_t rb, re;
            int ran = 0, sc = 0, te = 0, qe = 0, tb = 0, qb = 0;
            if (!E.pes[r].failed && s2_mate_window(X.n, p, E.pes[r], r, a_rb, l_ms, rb, re, rid)) {
                s2_mate_ksw(X, p, E.q[0], l_ms, r, rb, re, sc, te, qe, tb, qb, lane);
                ran = 1;
            }
            if (lane == 0) {
                int32_t *o_ = out + r * AF_G_PE_RES_W;
                o_[0] = sc; o_[1] = te; o_[2] = qe; o_[3] = tb; o_[4] = qb; o_[5] = ran;
            }
            wave_sync();
        }
    }
}

// K3d: mem_reg2aln + mem_aln2sam for both reads of every listed pair (one wave per pair): the
// CIGAR of each chosen region (bwa_gen_cigar2 with bwa's band retries), flags, split-read tails
struct __attribute__((aligned(16))) RecLds {
    int32_t o_rid[2], o_rev[2], o_flag[2], o_score[2], o_nc[2];
    int64_t o_pos[2];
};
__shared__ RecLds g_rec;

template <int CPL>
__global__ __launch_bounds__(64, 6) void k_s2_records(DevText X, const uint8_t *__restrict__ reads, int32_t stride,
                                                      const int32_t *__restrict__ lens, af_params p, S2Work w,
                                                      const S2Plan *__restrict__ plan, af_aln_out out,
                                                      uint8_t *__restrict__ zscratch, size_t zstride, AfTails tails,
                                                      int use_tails) {
    DpLds &L = g_dp;
    RecLds &E = g_rec;
    const int lane = threadIdx.x;
    const int64_t l_pac = X.n;
    const int npl = *w.n_plist;
    uint8_t *zg = zscratch + (size_t)blockIdx.x * zstride;
    for (int item = blockIdx.x; item < npl; item += gridDim.x) {
        const int64_t pp = w.plist[item];
        const S2Plan &pl = plan[item];
        S2DBG("k3d pair %d start\n", (int)pp);
        SPROF(const int64_t c0 = clock64();)
        // mem_reg2aln of each read's record
        for (int m = 0; m < 2; ++m) {
            const int wi = pl.which[m];
            const int64_t r = 2 * pp + m;
            if (wi < 0) {
                if (lane == 0) { E.o_rid[m] = -1; E.o_pos[m] = -1; E.o_rev[m] = 0; E.o_flag[m] = 0x4; E.o_score[m] = 0; E.o_nc[m] = 0; }
                wave_sync();
                continue;
            }
            const S2Reg ar = pl.r[m];
            const int secondary = pl.sec[m];
            int l = lens ? lens[r] : stride;
            if (l > stride) l = stride;
            if (l > AF_MAX_READ) l = AF_MAX_READ;
            if (l < 0) l = 0;
            const uint8_t *rd = reads + r * (int64_t)stride;
            for (int x = lane; x < l; x += 64) {
                const uint8_t ch = rd[x];
                L.q[x] = ch == 'A' || ch == 'a' ? 0 : ch == 'C' || ch == 'c' ? 1 : ch == 'G' || ch == 'g' ? 2
                       : ch == 'T' || ch == 't' ? 3 : 4;
            }
            wave_sync();
            const bool is_rev = ar.rb >= l_pac;
            const int lq = ar.qe - ar.qb;
            const int tmpw = infer_bw(lq, (int)(ar.re - ar.rb), ar.truesc, p.a, p.o_del, p.e_del);
            int w2 = infer_bw(lq, (int)(ar.re - ar.rb), ar.truesc, p.a, p.o_ins, p.e_ins);
            w2 = w2 > tmpw ? w2 : tmpw;
            if (w2 > p.w) w2 = w2 < ar.w ? w2 : ar.w;
            int score = 0, last_sc = -(1 << 30), it = 0;
            do {
                w2 = w2 < p.w << 2 ? w2 : p.w << 2;
                score = gen_cigar_wave<CPL>(X.T, l_pac, p, w2, lq, ar.qb, ar.rb, ar.re, L, zg, lane);
                if (score == last_sc || w2 == p.w << 2) break;
                last_sc = score;
                w2 <<= 1;
            } while (++it < 3 && score < ar.truesc - p.a);
            if (lane == 0) {
                uint32_t *co = out.cigar + r * AF_MAX_CIGAR;
                const int nc = L.misc[2];
                const int ncap = nc < AF_MAX_CIGAR ? nc : AF_MAX_CIGAR;
                bool of = nc > AF_MAX_CIGAR;
                int64_t pos = is_rev ? (l_pac << 1) - ar.re : ar.rb;
                int xs = 0, xe = ncap;
                const uint32_t first = L.ring[(nc - 1) & 63];
                const uint32_t last = L.ring[(nc - ncap) & 63];
                if (ncap > 0) {
                    if ((first & 0xf) == 2) { pos += first >> 4; xs = 1; }
                    else if ((last & 0xf) == 2) xe = ncap - 1;
                }
                const int clip5 = is_rev ? l - ar.qe : ar.qb;
                const int clip3 = is_rev ? ar.qb : l - ar.qe;
                int nf = 0;
                if (clip5) co[nf++] = (uint32_t)clip5 << 4 | 4;
                for (int x = xs; x < xe; ++x) {
                    if (nf < AF_MAX_CIGAR) co[nf] = L.ring[(nc - 1 - x) & 63];
                    ++nf;
                }
                if (clip3) {
                    if (nf < AF_MAX_CIGAR) co[nf] = (uint32_t)clip3 << 4 | 4;
                    ++nf;
                }
                if (nf > AF_MAX_CIGAR) { of = true; nf = AF_MAX_CIGAR; }
                E.o_rid[m] = 0; E.o_pos[m] = pos; E.o_rev[m] = is_rev;
                E.o_flag[m] = (secondary >= 0 ? 0x100 : 0) | (of ? AF_FLAG_CIGAR_OVERFLOW : 0);
                E.o_score[m] = ar.score; E.o_nc[m] = nf;
            }
            wave_sync();
        }
        // mem_aln2sam's flags and the mate copy rules
        if (lane == 0) {
            for (int m = 0; m < 2; ++m) {
                const int mm = m ^ 1;
                int prid = E.o_rid[m], mrid = E.o_rid[mm];
                int64_t ppos = E.o_pos[m];
                int prev = E.o_rev[m], mrev = E.o_rev[mm];
                int flag = E.o_flag[m] | (m ? 0x80 : 0x40) | pl.extra | 0x1;
                flag |= prid < 0 ? 0x4 : 0;
                flag |= mrid < 0 ? 0x8 : 0;
                if (prid < 0 && mrid >= 0) { ppos = E.o_pos[mm]; prev = mrev; }
                if (mrid < 0 && prid >= 0) mrev = prev;
                flag |= prev ? 0x10 : 0;
                flag |= mrev ? 0x20 : 0;
                if ((pl.ovf >> m) & 1) flag |= AF_FLAG_MEM_OVERFLOW;
                const int64_t r = 2 * pp + m;
                out.flag[r] = flag;
                out.pos[r] = (prid >= 0 || mrid >= 0) ? (int32_t)ppos : -1;
                out.score[r] = prid >= 0 ? E.o_score[m] : 0;
                out.n_cigar[r] = prid >= 0 ? E.o_nc[m] : 0;
                if (use_tails && prid >= 0 && E.o_nc[m] == 2)
                    af_emit_tail(tails, reads, stride, lens, r, flag, out.cigar + r * AF_MAX_CIGAR);
            }
        }
        SPROF(if (lane == 0 && g_s2prof) g_s2prof[S2PROF_K3 + (int64_t)item * 16 + 5] = (int32_t)(clock64() - c0);)
        wave_sync();
    }
}

// chunk boundaries of a ragged batch (bseq_read: a chunk ends after the pair that brings its
// bases to >= chunk_bases): prefix sums of pair lengths, then one binary search per chunk
__global__ __launch_bounds__(1024) void k_s2_chunks(int64_t n_pairs, int32_t stride, const int32_t *__restrict__ lens,
                                                     int64_t chunk_bases, int64_t *__restrict__ cstart,
                                                     int64_t *__restrict__ S, int32_t max_chunks,
                                                     int32_t *__restrict__ n_chunks) {
    __shared__ int64_t part[1024];
    const int tid = threadIdx.x;
    const int64_t per = (n_pairs + 1023) / 1024;
    const int64_t b0 = tid * per, b1 = min(n_pairs, b0 + per);
    int64_t s = 0;
    for (int64_t q = b0; q < b1; ++q) {
        const int64_t l0 = min(lens[2 * q], stride), l1 = min(lens[2 * q + 1], stride);
        s += max(l0, (int64_t)0) + max(l1, (int64_t)0);
    }
    part[tid] = s;
    __syncthreads();
    if (tid == 0) {
        int64_t acc = 0;
        for (int t = 0; t < 1024; ++t) { const int64_t v = part[t]; part[t] = acc; acc += v; }
    }
    __syncthreads();
    s = part[tid];
    for (int64_t q = b0; q < b1; ++q) {
        const int64_t l0 = min(lens[2 * q], stride), l1 = min(lens[2 * q + 1], stride);
        s += max(l0, (int64_t)0) + max(l1, (int64_t)0);
        S[q] = s;  // bases of pairs [0, q]
    }
    __syncthreads();
    if (tid == 0) {
        int nc = 0;
        int64_t c0 = 0;
        while (c0 < n_pairs && nc < max_chunks) {
            cstart[nc++] = c0;
            const int64_t before = c0 > 0 ? S[c0 - 1] : 0;
            int64_t lo = c0, hi = n_pairs - 1;  // first q >= c0 with S[q] - before >= chunk_bases
            if (S[hi] - before < chunk_bases) { c0 = n_pairs; break; }
            while (lo < hi) {
                const int64_t mid = (lo + hi) >> 1;
                if (S[mid] - before >= chunk_bases) hi = mid;
                else lo = mid + 1;
            }
            c0 = lo + 1;
        }
        cstart[nc] = n_pairs;
        *n_chunks = nc;
    }
}

}  // namespace

#ifdef AF_K2_PROF
extern "C" int af_debug_s2_prof_enable() {
    int32_t *d = nullptr;
    const size_t n = (size_t)2 << 24;
    if (hipMalloc(&d, sizeof(int32_t) * n) != hipSuccess) return -1;
    (void)hipMemset(d, 0, sizeof(int32_t) * n);
    return hipMemcpyToSymbol(HIP_SYMBOL(g_s2prof), &d, sizeof d) == hipSuccess ? 16 : -1;
}
extern "C" int af_debug_s2_prof_read(int32_t *host, int64_t n_k2, int64_t n_k3) {
    int32_t *d = nullptr;
    if (hipMemcpyFromSymbol(&d, HIP_SYMBOL(g_s2prof), sizeof d) != hipSuccess || !d) return -1;
    if (hipMemcpy(host, d, sizeof(int32_t) * 16 * n_k2, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    return hipMemcpy(host + 16 * n_k2, d + S2PROF_K3, sizeof(int32_t) * 16 * n_k3, hipMemcpyDeviceToHost) == hipSuccess
               ? 0 : -1;
}
#endif

size_t af_s2_plan_bytes() { return sizeof(S2Plan); }

// mem_pestat per chunk (K3b) for callers with their own insert-size histograms (the genome S4)
hipError_t af_launch_s2_pestat(const S2Work &w, int32_t max_ins, hipStream_t s) {
    hipLaunchKernelGGL(k_s2_pestat, dim3((unsigned)(w.ppc ? w.n_chunks_u : w.max_chunks)), dim3(256), 0, s, w, max_ins);
    return hipGetLastError();
}

hipError_t af_launch_s2_chunks(int64_t n_pairs, int32_t stride, const int32_t *lens, int64_t chunk_bases,
                               int64_t *cstart, int64_t *scan_tmp, int32_t max_chunks, int32_t *n_chunks_dev,
                               hipStream_t s) {
    hipLaunchKernelGGL(k_s2_chunks, dim3(1), dim3(1024), 0, s, n_pairs, stride, lens, chunk_bases, cstart, scan_tmp,
                       max_chunks, n_chunks_dev);
    return hipGetLastError();
}

hipError_t af_launch_s2(const DevText &X, const uint8_t *reads, int64_t n_pairs, int32_t stride, const int32_t *lens,
                        const af_params &p, const S2Opt &o, const int32_t *hits, const int32_t *cand,
                        const int32_t *n_cand, const S2Work &w, af_aln_out out, uint8_t *zscratch, int32_t n_slots,
                        int32_t n_cu, const AfTails *tails, hipStream_t s) {
    // zscratch holds n_slots = n_cu * 4 * AF_K2_WPS per-block slots (api.hip ensure_zscratch),
    // indexed by blockIdx in k_s2_regions and k_s2_records: a build with fewer slots than either
    // grid is refused at compile time, and a context whose slot count does not cover the grids
    // (a runtime change of either) is refused here instead of faulting
    static_assert(AF_S2_WPS <= AF_K2_WPS && 6 <= AF_K2_WPS,
                  "k_s2_regions / k_s2_records grids exceed the n_cu * 4 * AF_K2_WPS zscratch slots");
    const size_t zstride = (size_t)(AF_MAX_READ + 1) * 1024;
    const int cpl = (stride + 1 + 63) / 64;
    dim3 g(n_cu * 4 * AF_S2_WPS), g3(n_cu * 16), g4(n_cu * 4 * 6), b(64);
    if ((int64_t)g.x > n_slots || (int64_t)g4.x > n_slots) return hipErrorInvalidConfiguration;
#define AF_GO(C) hipLaunchKernelGGL((k_s2_regions<C>), g, b, 0, s, X, reads, stride, lens, p, o, cand, n_cand, w, \
                                    zscratch, zstride)
    if (cpl <= 2) AF_GO(2);
    else if (cpl <= 3) AF_GO(3);
    else if (cpl <= 4) AF_GO(4);
    else AF_GO(AF_CPL);
#undef AF_GO
    const int64_t nb = n_pairs > 0 ? (n_pairs + AF_S2_CLS_PAIRS - 1) / AF_S2_CLS_PAIRS : 1;
    hipLaunchKernelGGL(k_s2_classify, dim3((unsigned)nb), dim3(CLS_THREADS), 0, s, n_pairs, X.n, hits, p, o, w, out);
    hipLaunchKernelGGL(k_s2_pestat, dim3((unsigned)(w.ppc ? w.n_chunks_u : w.max_chunks)), dim3(256), 0, s, w,
                       o.max_ins);
    const AfTails t = tails ? *tails : AfTails{};
    S2Plan *plan = static_cast<S2Plan *>(w.plan);
    if (w.sp.min_windows > 0) {
        hipLaunchKernelGGL(k_s2_pairs<1>, g3, b, 0, s, X, reads, stride, lens, p, o, hits, w, plan);
        hipLaunchKernelGGL(k_s2_pe_jobs, dim3(2 * g3.x), b, 0, s, X, reads, stride, lens, p, o, hits, w);
        hipLaunchKernelGGL(k_s2_pairs<2>, g3, b, 0, s, X, reads, stride, lens, p, o, hits, w, plan);
    } else {
        hipLaunchKernelGGL(k_s2_pairs<0>, g3, b, 0, s, X, reads, stride, lens, p, o, hits, w, plan);
    }
#define AF_GO(C) hipLaunchKernelGGL((k_s2_records<C>), g4, b, 0, s, X, reads, stride, lens, p, w, plan, out, zscratch, \
                                    zstride, t, tails ? 1 : 0)
    if (cpl <= 2) AF_GO(2);
    else if (cpl <= 3) AF_GO(3);
    else if (cpl <= 4) AF_GO(4);
    else AF_GO(AF_CPL);
#undef AF_GO
    return hipGetLastError();
}
