// bwa_genome.hip -- the genome calls of the reference on the GPU, as bwa 0.7.17 computes them:
//     S4  bwa mem -M -t T <genome.fa> tmp1.fq tmp2.fq   (Anchored_Fusion.py:188), paired-end
//     S5  bwa mem -M -t T <genome.fa> split_reads.fa    (functions.py:716), single-end
// over the genome index of fmindex.hip.  oracle/bwa_pe.c (FM mode) is the bit-exact contract;
// each device routine names the bwa routine it restates.
//
// Kernels (one launch each per call, on the caller's stream):
//   G1 k_g_seeds     one LANE per read (the FM walk is a chain of dependent lookups, so a wave
//                    keeps 64 reads' lookups in flight): mem_collect_intv -- bwt_smem1 passes 1
//                    and 2, bwt_seed_strategy1 -- on the bidirectional FM index; the read's
//                    intervals (SA row range, size, query span) sorted by (qb, qe) into a pool
//   G2 k_g_regions   one wave per read: mem_chain (occurrences sampled at max_occ in SA order,
//                    64 SA rows gathered per step; klib kbtree on lane 0), mem_chain_flt,
//                    mem_chain2aln (ksw_extend2 on the wave, ksw_dp.h, windows clipped to the
//                    seed's contig: bns_fetch_seq), mem_sort_dedup_patch (same contig only) ->
//                    the read's regions into a pool
//   G3 k_g_se        one wave per read (S5): mem_mark_primary_se (hash_64 tie-break on the read
//                    id), mem_reg2sam with -M (mem_reg2aln: band inference + ksw_global2 on the
//                    wave; -M parts as 0x100 with hard clips) -> af_grec records
//   PE               k_g_pe_hist (one lane per pair: mem_pestat's insert sizes per bwa chunk),
//                    k_s2_pestat (s2.hip), k_g_pe (one wave per pair: mem_matesw with ksw_align2
//                    on the wave, mem_mark_primary_se, mem_pair, mem_sam_pe's branches and
//                    mem_reg2sam / mem_aln2sam for every record of both ends)
//
// Per-read state that can grow with repeats (seed lists, chains, the kbtree, regions) lives in
// per-wave global scratch (L2 / Infinity Cache resident for the common short lists); the DP
// rows, query and target windows in LDS (ksw_dp.h g_dp).  Caps equal the oracle's AFO_G_MAX_*;
// a read past one is reported unmapped with AF_FLAG_MEM_OVERFLOW, counted in the call's stats.
#include "bwa_dev.h"

#pragma clang fp contract(off)

namespace {

#ifdef AF_G_PROF
// profiling build only (make gprof -> libafgpu_gprof.so, scripts/g_prof.py): per-read timings of
// the genome calls, [call][read][GP_W]
__device__ int32_t *g_gprof = nullptr;
__device__ int64_t g_gprof_cap = 0;
__device__ int32_t g_gprof_call = 0;
// [0, 27) G1 (lane path) and G2, [27, 32) G1's wave path, [32, 40) k_g_pe's phases on the pair's
// first read: disjoint, so a read of both paths (or an S4 pair's first read) keeps every field
constexpr int GP_W = 44;
__device__ __forceinline__ int32_t *gp_row(int64_t r) {
    return g_gprof && r < g_gprof_cap ? g_gprof + ((int64_t)g_gprof_call * g_gprof_cap + r) * GP_W : nullptr;
}
__device__ __forceinline__ uint32_t gp_rt() { return (uint32_t)wall_clock64(); }
#define GPROF(...) __VA_ARGS__
#else
#define GPROF(...)
#endif

constexpr int G_KB_T = 5, G_KB_MAXK = 2 * G_KB_T - 1;
constexpr int G_KB_NODES = AF_G_MAX_CHAIN / 2 + 64;  // t = 5: >= 4 keys per non-root node

struct GSeed { int64_t rbeg; int32_t qbeg, len; };   // mem_seed_t (score = len)
struct GChain { int64_t pos; int32_t n, first, rid, w, kept, seed0; };  // mem_chain_t
struct GKb { int16_t n, internal; int16_t key[G_KB_MAXK]; int16_t ptr[G_KB_MAXK + 1]; };

// ================================================================== FM index (bwt.c)
// bwt_occ4: occurrences of A/C/G/T in the BWT rows [0, i).  A 128-row block holds its four
// counts and 128 2-bit symbols (symbol t of a 32-bit word at bits 2t, 2t + 1); the symbols
// below row i are counted for all four bases at once from three popcounts per word (low bits,
// high bits, both): T = both, G = high - T, C = low - T, A = the rest.
struct OccBlk { uint4 c01, c23, w01, w23; };
__device__ __forceinline__ OccBlk fm_blk(const DevGenome &G, int64_t b) {
    const uint4 *blk = reinterpret_cast<const uint4 *>(G.occ + b * 8);
    return OccBlk{blk[0], blk[1], blk[2], blk[3]};
}
// occ of row i from its (loaded) block
__device__ __forceinline__ void fm_occ4b(const DevGenome &G, const OccBlk &B, int64_t i, int64_t o[4]) {
    const int64_t b = i >> 7;
    const int r = (int)(i & 127);
    const uint4 c01 = B.c01, c23 = B.c23, w01 = B.w01, w23 = B.w23;
    const uint32_t wv[8] = {w01.x, w01.y, w01.z, w01.w, w23.x, w23.y, w23.z, w23.w};
    uint32_t nlo = 0, nhi = 0, n11 = 0;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        const int m = r - 16 * u;  // symbols of word u below row i
        const uint32_t mask = m >= 16 ? 0xffffffffu : m <= 0 ? 0u : (1u << (2 * m)) - 1u;
        const uint32_t x = wv[u] & mask;
        const uint32_t lo = x & 0x55555555u, hi = (x >> 1) & 0x55555555u;
        nlo += __builtin_popcount(lo);
        nhi += __builtin_popcount(hi);
        n11 += __builtin_popcount(lo & hi);
    }
    o[0] = (int64_t)((uint64_t)c01.x | (uint64_t)c01.y << 32) + r - (int)(nlo + nhi - n11);
    o[1] = (int64_t)((uint64_t)c01.z | (uint64_t)c01.w << 32) + (int)(nlo - n11);
    o[2] = (int64_t)((uint64_t)c23.x | (uint64_t)c23.y << 32) + (int)(nhi - n11);
    o[3] = (int64_t)((uint64_t)c23.z | (uint64_t)c23.w << 32) + (int)n11;
    if (G.primary >= (b << 7) && G.primary < i) o[0] -= 1;  // the '$' row is stored as A
}
__device__ __forceinline__ void fm_occ4(const DevGenome &G, int64_t i, int64_t o[4]) {
    fm_occ4b(G, fm_blk(G, i >> 7), i, o);
}
__device__ __forceinline__ int64_t sel4(const int64_t v[4], int c) {
    return c == 0 ? v[0] : c == 1 ? v[1] : c == 2 ? v[2] : v[3];
}
// bwt_extend restricted to one base (oracle fm_back4 / fm_fwd4, the c'th output): backward, the
// bi-interval of cW from W = (k, l, s); forward (fwd, W -> W comp(c') with c = 3 - c'), the same
// on the swapped interval, swapped back
__device__ __forceinline__ void fm_ext1(const DevGenome &G, int64_t k, int64_t l, int64_t s, int c, bool fwd,
                                       int64_t &ok, int64_t &ol, int64_t &os) {
    if (fwd) { const int64_t t = k; k = l; l = t; }
    int64_t a[4], b[4];
    // rows k and k + s: one 64-B block when both fall in it (a narrow interval), else two
    if (((k + s) >> 7) == (k >> 7)) {
        const OccBlk B = fm_blk(G, k >> 7);
        fm_occ4b(G, B, k, a);
        fm_occ4b(G, B, k + s, b);
    } else {
        fm_occ4(G, k, a);
        fm_occ4(G, k + s, b);
    }
    int64_t lo = l + (k <= G.primary && k + s - 1 >= G.primary);
#pragma unroll
    for (int d = 3; d > 0; --d)
        if (d > c) lo += b[d] - a[d];
    const int64_t Cc = c == 0 ? G.C[0] : c == 1 ? G.C[1] : c == 2 ? G.C[2] : G.C[3];
    const int64_t kk = Cc + sel4(a, c);
    os = sel4(b, c) - sel4(a, c);
    if (fwd) { ok = lo; ol = kk; }
    else { ok = kk; ol = lo; }
}

// the bi-interval of one base (oracle fm_set)
__device__ __forceinline__ void fm_set(const DevGenome &G, int c, int64_t &k, int64_t &l, int64_t &s) {
    k = c == 0 ? G.C[0] : c == 1 ? G.C[1] : c == 2 ? G.C[2] : G.C[3];
    l = c == 0 ? G.C[3] : c == 1 ? G.C[2] : c == 2 ? G.C[1] : G.C[0];
    s = c == 0 ? G.base_cnt[0] : c == 1 ? G.base_cnt[1] : c == 2 ? G.base_cnt[2] : G.base_cnt[3];
}

__device__ __forceinline__ uint8_t nt4(uint8_t ch) {
    return ch == 'A' || ch == 'a' ? 0 : ch == 'C' || ch == 'c' ? 1 : ch == 'G' || ch == 'g' ? 2
         : ch == 'T' || ch == 't' ? 3 : 4;
}
__device__ __forceinline__ int read_len(const int32_t *lens, int64_t r, int32_t stride) {
    int l = lens ? lens[r] : stride;
    if (l > stride) l = stride;
    if (l > AF_MAX_READ) l = AF_MAX_READ;
    return l < 0 ? 0 : l;
}

// ============================================================= G1: mem_collect_intv
// One lane per read, as a state machine whose every trip makes at most one FM extension per lane
// (bwt_extend of one interval by one base: two 64-B occurrence blocks), so the 64 lanes of a wave
// issue their dependent lookups together whatever phase each read is in: bwt_smem1's forward
// scan, its backward scan (one list entry per trip), or bwt_seed_strategy1.  Between extensions a
// lane runs its list bookkeeping; a lane whose read is done takes the next read (one atomic per
// wave).  The three passes of mem_collect_intv (oracle fm_collect: SMEMs, re-seeding of long
// SMEMs with few occurrences, bwt_seed_strategy1) and their list orders are bwa's.
//
// Per-lane lists in global scratch, lane-major (a lane's walk reads its lists sequentially),
// one 16-byte packed interval each: k, l, s (33 bits each: at most 2 l_pac + 1 rows < 2^33,
// checked when the index is built) and qb, qe (9 bits each).
constexpr int G1_LIST = AF_MAX_READ + 2;              // prev / curr / mem lists of bwt_smem1
constexpr int64_t G1_SLOT = 3 * G1_LIST + AF_G_MAX_INTV;  // + the read's interval list (uint4)
struct G1Iv { int64_t k, l, s; int qb, qe; };
__device__ __forceinline__ uint4 g1_pack(int64_t k, int64_t l, int64_t s, int qb, int qe) {
    return make_uint4((uint32_t)k, (uint32_t)l, (uint32_t)s,
                      (uint32_t)(k >> 32 & 1) | (uint32_t)(l >> 32 & 1) << 1 | (uint32_t)(s >> 32 & 1) << 2 |
                          (uint32_t)qb << 3 | (uint32_t)qe << 12);
}
__device__ __forceinline__ G1Iv g1_unpack(uint4 v) {
    G1Iv r;
    r.k = (int64_t)v.x | (int64_t)(v.w & 1) << 32;
    r.l = (int64_t)v.y | (int64_t)(v.w >> 1 & 1) << 32;
    r.s = (int64_t)v.z | (int64_t)(v.w >> 2 & 1) << 32;
    r.qb = (int)(v.w >> 3 & 511);
    r.qe = (int)(v.w >> 12 & 511);
    return r;
}
#ifndef G1_PC
#define G1_PC 1  // prev entries the backward scan holds in registers
#endif
enum : int { G1_IDLE, G1_P1, G1_FWD, G1_BWD, G1_P2, G1_P3, G1_SS, G1_DONE, G1_EXIT };

__global__ __launch_bounds__(64, AF_G1_WPS) void k_g_seeds(DevGenome G, const uint8_t *__restrict__ reads,
                                                          int32_t stride, const int32_t *__restrict__ lens,
                                                          const int32_t *__restrict__ n_ptr, int64_t cap,
                                                          int64_t read0, af_params p, GOpt o,
                                                          uint4 *__restrict__ scratch, GWork w) {
    const int lane = threadIdx.x;
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + lane;
    int64_t n = n_ptr ? (int64_t)*n_ptr : cap;
    if (n > cap) n = cap;
    uint4 *const base = scratch + tid * G1_SLOT;
    int lsel = 0;  // bwt_smem1's prev / curr: base + lsel G1_LIST / the other (swapped by the bit)
#define Lp (base + lsel * G1_LIST)
#define Lc (base + (lsel ^ 1) * G1_LIST)
    uint4 *const Lf = base + 3 * G1_LIST;  // the read's list (base + 2 G1_LIST: k_g_seeds_wave's mems)
    const int msl = p.min_seed_len;
    const int split_len = (int)((float)msl * 1.5f + .499);
    // lane state
    int st = G1_IDLE, len = 0, x = 0, i = 0, j = 0, np = 0, nc = 0, nm = 0, ret = 0, ni = 0, k2 = 0, old_n = 0;
    int pass = 1, sx = 0, last_mem_qb = 0, ik_qe = 0, p_qe = 0;
    bool ovf = false, rev = false;
    int64_t rr = -1, min_intv = 1, ik_k = 0, ik_l = 0, ik_s = 0, last_s = 0;
    const uint8_t *rd = nullptr;
    // bwt_smem1's backward scan reads prev's entries in order: entry pf_j of the scan is in pf,
    // loaded during the trip that extends entry pf_j - 1 (its wait overlaps that trip's FM
    // lookup); at a new position prev's first entry is curr's first (or, after the forward scan,
    // last) push, kept in registers (c_first / c_last): no list load waits on the critical path
    uint4 pf = make_uint4(0, 0, 0, 0), c_first = pf, c_last = pf;
    int pf_j = -1;
    // pass 1's intervals that pass 2 re-seeds (long, few occurrences, a base at the middle), for
    // the first 64 of the list: pass 2 reads only those
    uint64_t elig = 0;
    int ne = 0;  // the read's FM extensions so far (past w.g1_max_ext: handed to k_g_seeds_wave)
    GPROF(uint64_t gp_c0 = 0; uint32_t gp_t0 = 0; int gp_fwd = 0, gp_bwd = 0, gp_ss = 0;
          uint64_t gp_loop = 0, gp_ext = 0; int gp_trips = 0, gp_iters = 0;)
    // each lane's read as codes in LDS, two per byte, lane-interleaved (byte (t / 2) * 64 + lane):
    // the state machine's base reads stay off the memory path that every trip already waits on
    __shared__ uint8_t g1_rd[(AF_MAX_READ / 2) * 64];
    auto code = [&](int t) -> int { return (g1_rd[(t >> 1) * 64 + lane] >> ((t & 1) << 2)) & 15; };
    auto push_curr = [&](int64_t k, int64_t l, int64_t s, int qb, int qe) {
        const uint4 e = g1_pack(k, l, s, qb, qe);
        if (nc == 0) c_first = e;
        c_last = e;
        Lc[nc++] = e;
    };
    auto smem_start = [&](int x0, int64_t mi, int ps) {
        const int c = code(x0);
        sx = x0; min_intv = mi < 1 ? 1 : mi; pass = ps;
        fm_set(G, c, ik_k, ik_l, ik_s);
        ik_qe = x0 + 1; i = x0 + 1; nc = 0; nm = 0;
        st = G1_FWD;
    };
    auto fwd_end = [&]() {  // curr holds the forward intervals in push order (bwa reverses them)
        ret = (int)g1_unpack(c_last).qe;
        lsel ^= 1;
        np = nc; nc = 0; rev = true; i = sx - 1; j = 0;
        pf = c_last; pf_j = 0;  // prev in reverse push order: entry 0 is the last push
        st = G1_BWD;
    };
    auto take = [&](const G1Iv &m) -> bool {  // an interval into the read's list
        if (ni >= AF_G_MAX_INTV) { ovf = true; st = G1_DONE; return false; }
        Lf[ni++] = g1_pack(m.k, m.l, m.s, m.qb, m.qe);
        return true;
    };
    auto smem_end = [&]() {
        if (pass == 1) { x = ret; st = G1_P1; }
        else { ++k2; st = G1_P2; }
    };
    // a prev entry that cannot extend becomes a mem; those of >= min_seed_len go straight to the
    // read's list (bwa collects a smem's mems and appends them reversed: the list's order is
    // immaterial, k_g_regions sorts it by (qb, qe) and equal keys are identical intervals)
    auto mem_push = [&](const G1Iv &pv, int qb) {
        if (nc == 0 && (nm == 0 || qb < last_mem_qb)) {
            ++nm;
            last_mem_qb = qb;
            if (pv.qe - qb >= msl) {
                if (pass == 1 && ni < 64 && pv.qe - qb >= split_len && pv.s <= o.split_width &&
                    code((qb + pv.qe) >> 1) <= 3)
                    elig |= 1ull << ni;
                take(G1Iv{pv.k, pv.l, pv.s, qb, pv.qe});
            }
        }
    };
    for (;;) {
        // idle lanes take the next reads (one atomic per wave)
        const uint64_t im = __ballot(st == G1_IDLE);
        if (im) {
            uint64_t b0 = 0;
            if (lane == 0) b0 = atomicAdd(w.g1_next, (unsigned long long)__builtin_popcountll(im));
            b0 = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)b0) |
                 (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(b0 >> 32)) << 32;
            if (st == G1_IDLE) {
                rr = read0 + (int64_t)b0 + lanes_below(im, lane);
                if (rr >= n) st = G1_EXIT;
                else {
                    len = read_len(lens, rr, stride);
                    rd = reads + rr * (int64_t)stride;
                    for (int t = 0; t < len; t += 2)
                        g1_rd[(t >> 1) * 64 + lane] = (uint8_t)(nt4(rd[t]) | (t + 1 < len ? nt4(rd[t + 1]) : 4) << 4);
                    ni = 0; ovf = false; x = 0; ne = 0; elig = 0;
                    st = len >= msl ? G1_P1 : G1_DONE;
                    GPROF(gp_c0 = clock64(); gp_t0 = gp_rt(); gp_fwd = gp_bwd = gp_ss = 0;
                          gp_loop = gp_ext = 0; gp_trips = gp_iters = 0;)
                }
            }
        }
        if (__ballot(st != G1_EXIT) == 0) break;
        // advance each lane to its next FM extension
        bool need = false;
        int64_t ek = 0, el = 0, es = 0;
        int ec = 0;
        bool efwd = false;
        GPROF(const uint64_t gp_l0 = clock64(); ++gp_trips;)
        while (!need && st != G1_IDLE && st != G1_EXIT) {
            GPROF(++gp_iters;)
            if (st == G1_P1) {  // pass 1: SMEMs covering each position
                if (x >= len) { old_n = ni; k2 = 0; st = G1_P2; continue; }
                if (code(x) > 3) { ++x; continue; }
                smem_start(x, 1, 1);
            } else if (st == G1_FWD) {  // bwt_smem1 forward search
                if (i == len) { push_curr(ik_k, ik_l, ik_s, 0, ik_qe); fwd_end(); continue; }
                const int c = code(i);
                if (c > 3) { push_curr(ik_k, ik_l, ik_s, 0, ik_qe); fwd_end(); continue; }
                need = true; ek = ik_k; el = ik_l; es = ik_s; ec = 3 - c; efwd = true;
            } else if (st == G1_BWD) {  // backward search for MEMs: entry j of prev at position i
                if (j == np) {
                    if (nc == 0) { smem_end(); continue; }
                    lsel ^= 1;
                    np = nc; nc = 0; rev = false; --i; j = 0;
                    pf = c_first; pf_j = 0;  // prev in push order: entry 0 is the first push
                    continue;
                }
                if (pf_j != j) { pf = Lp[rev ? np - 1 - j : j]; pf_j = j; }
                const G1Iv pv = g1_unpack(pf);
                const int c = i < 0 ? -1 : code(i);
                if (c < 0 || c > 3) {
                    // no entry extends past the read's start or an N: each would become a mem at the
                    // same qb, and only the first can (mem_push needs qb < last_mem_qb after it, and
                    // curr stays as it is) -- the rest of prev is skipped unread
                    mem_push(pv, i + 1);
                    j = np;
                    continue;
                }
                need = true; ek = pv.k; el = pv.l; es = pv.s; ec = c; efwd = false; p_qe = pv.qe;
                if (j + 1 < np) { pf = Lp[rev ? np - 2 - j : j + 1]; pf_j = j + 1; }  // next trip's entry
            } else if (st == G1_P2) {  // pass 2: re-seed long SMEMs with few occurrences
                if (k2 < 64 && k2 < old_n) {  // the next interval pass 2 re-seeds, from the mask
                    const uint64_t m = elig & (~0ull << k2);
                    k2 = m ? (int)__builtin_ctzll(m) : (old_n < 64 ? old_n : 64);
                }
                if (k2 >= old_n) {
                    if (o.max_mem_intv > 0) { x = 0; st = G1_P3; }
                    else st = G1_DONE;
                    continue;
                }
                const G1Iv pk = g1_unpack(Lf[k2]);
                if (pk.qe - pk.qb < split_len || pk.s > o.split_width) { ++k2; continue; }
                const int mid = (pk.qb + pk.qe) >> 1;
                if (code(mid) > 3) { ++k2; continue; }
                smem_start(mid, pk.s + 1, 2);
            } else if (st == G1_P3) {  // pass 3: bwt_seed_strategy1 from each position
                if (x >= len) { st = G1_DONE; continue; }
                const int c = code(x);
                if (c > 3) { ++x; continue; }
                sx = x; i = x + 1;
                fm_set(G, c, ik_k, ik_l, ik_s);
                st = G1_SS;
            } else if (st == G1_SS) {
                if (i >= len) { x = len; st = G1_P3; continue; }
                const int c = code(i);
                if (c > 3) { x = i + 1; st = G1_P3; continue; }
                need = true; ek = ik_k; el = ik_l; es = ik_s; ec = 3 - c; efwd = true;
            } else {  // G1_DONE: the list into the call's pool (k_g_regions sorts it by (qb, qe))
                bool hv = false;  // G2 takes it first
                if (ovf) w.iv_n[rr] = -1;
                else {
                    const int64_t off = ni ? (int64_t)atomicAdd(w.iv_fill, (unsigned long long)ni) : 0;
                    if (ni && off + ni > w.iv_cap) {  // the pool is sized from the call's read count
                        atomicAdd(&w.stats[AF_GSTAT_POOL], 1);
                        w.iv_n[rr] = -1;
                    } else {
                        int64_t occ = 0;
                        // four list entries loaded before any store: one memory wait per four
                        for (int a0 = 0; a0 < ni; a0 += 4) {
                            uint4 e4[4];
#pragma unroll
                            for (int u = 0; u < 4; ++u) e4[u] = Lf[a0 + u < ni ? a0 + u : a0];
#pragma unroll
                            for (int u = 0; u < 4; ++u)
                                if (a0 + u < ni) {
                                    const G1Iv m = g1_unpack(e4[u]);
                                    w.iv[off + a0 + u] = GIv{m.k, m.s, m.qb, m.qe};
                                    occ += m.s > p.max_occ ? p.max_occ : m.s;
                                }
                        }
                        w.iv_off[rr] = off;
                        w.iv_n[rr] = ni;
                        hv = w.g2_first_occ > 0 && occ >= w.g2_first_occ;
                    }
                }
                if (w.g2_first_occ > 0) {
                    w.g2_flag[rr] = hv;
                    if (hv) w.g2_list[atomicAdd(w.g2_list_n, 1ull)] = (int32_t)rr;
                }
                GPROF({ int32_t *g = gp_row(rr); if (g) { g[0] = (int32_t)(clock64() - gp_c0); g[1] = ovf ? -1 : ni;
                        g[17] = (int32_t)gp_t0; g[18] = (int32_t)gp_rt(); g[20] = (int32_t)tid;
                        g[19] = gp_fwd; g[21] = gp_bwd; g[22] = gp_ss;
                        g[23] = (int32_t)(gp_loop >> 4); g[24] = (int32_t)(gp_ext >> 4); g[25] = gp_trips;
                        g[26] = gp_iters; } })
                st = G1_IDLE;
            }
        }
        GPROF(const uint64_t gp_l1 = clock64(); gp_loop += gp_l1 - gp_l0;)
        if (__ballot(need) == 0) continue;
        // the extensions of this trip: every lane that needs one at once
        int64_t rk = 0, rl = 0, rs = 0;
        if (need) fm_ext1(G, ek, el, es, ec, efwd, rk, rl, rs);
        GPROF(gp_ext += clock64() - gp_l1;)
        if (!need) continue;
        if (w.g1_max_ext > 0 && ++ne > w.g1_max_ext) {  // a heavy read: restarted by k_g_seeds_wave
            w.g1_hv[atomicAdd(w.g1_hv_n, 1ull)] = rr;
            st = G1_IDLE;
            continue;
        }
        GPROF(if (st == G1_FWD) ++gp_fwd; else if (st == G1_BWD) ++gp_bwd; else ++gp_ss;)
        if (st == G1_FWD) {
            if (rs != ik_s) {
                push_curr(ik_k, ik_l, ik_s, 0, ik_qe);
                if (rs < min_intv) { fwd_end(); continue; }
            }
            ik_k = rk; ik_l = rl; ik_s = rs; ik_qe = i + 1; ++i;
        } else if (st == G1_BWD) {
            if (rs < min_intv) mem_push(G1Iv{ek, el, es, 0, p_qe}, i + 1);
            else if (nc == 0 || rs != last_s) { push_curr(rk, rl, rs, 0, p_qe); last_s = rs; }
            ++j;
        } else {  // G1_SS
            if (rs < o.max_mem_intv && i - sx >= msl) {  // the caller keeps a non-empty interval
                if (rs > 0) take(G1Iv{rk, rl, rs, sx, i + 1});
                if (st != G1_DONE) { x = i + 1; st = G1_P3; }
            } else { ik_k = rk; ik_l = rl; ik_s = rs; ++i; }
        }
    }
}

#undef Lp
#undef Lc

// G1 for the reads k_g_seeds handed off (more than w.g1_max_ext FM extensions: repeat-rich reads
// whose backward scans hold many entries per position): one WAVE per read, restarted from the
// read's first pass.  Forward scans and the seed strategy run on the whole wave (every lane makes
// the same lookup); the backward scan extends all of a position's prev entries at once (lanes
// over entries) and applies bwt_smem1's ordered rules from ballots -- an entry joins curr when its
// interval survives and its size differs from the previous surviving entry's; only entry 0 can
// become a mem (no entry before it survived).  Lists in the wave's slot of the G1 scratch (prev,
// curr, mems, the read's intervals), written by the lanes that own the entries.  The intervals and
// their pool layout are those of k_g_seeds.
__device__ __forceinline__ void g1w_sync() {
    __threadfence_block();
    wave_sync();
}
__device__ __forceinline__ int64_t shfl64(int64_t v, int l) {
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, l), hi = (uint32_t)__shfl((int)(uint32_t)((uint64_t)v >> 32), l);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
struct G1W {
    uint4 *prev, *curr, *mem, *lst;
    const uint8_t *q;
    int len, ni, msl;
    bool ovf;
    int gp_f = 0, gp_bp = 0, gp_be = 0;  // profiling build: forward steps, backward positions / entries
};
// an interval into the read's list (uniform)
__device__ __forceinline__ bool g1w_take(G1W &R, const G1Iv &m, int lane) {
    if (R.ni >= AF_G_MAX_INTV) { R.ovf = true; return false; }
    if (lane == 0) R.lst[R.ni] = g1_pack(m.k, m.l, m.s, m.qb, m.qe);
    ++R.ni;
    return true;
}
// bwt_smem1 from x0 with min_intv (oracle fm_smem1), its mems of >= min_seed_len into the list in
// bwa's (reversed) order; returns the position the pass continues from
__device__ __forceinline__ int g1w_smem(const DevGenome &G, G1W &R, int x0, int64_t min_intv, int lane) {
    if (min_intv < 1) min_intv = 1;
    int64_t ik_k, ik_l, ik_s;
    fm_set(G, R.q[x0], ik_k, ik_l, ik_s);
    int ik_qe = x0 + 1, nc = 0, ret = 0;
    // forward: the wave as one lane
    for (int i = x0 + 1;; ++i) {
        bool push = false, stop = false;
        int64_t rk = 0, rl = 0, rs = 0;
        if (i == R.len || R.q[i] > 3) push = stop = true;
        else {
            GPROF(++R.gp_f;)
            fm_ext1(G, ik_k, ik_l, ik_s, 3 - R.q[i], true, rk, rl, rs);
            if (rs != ik_s) { push = true; stop = rs < min_intv; }
        }
        if (push) {
            if (lane == 0) R.curr[nc] = g1_pack(ik_k, ik_l, ik_s, 0, ik_qe);
            ++nc;
            ret = ik_qe;
        }
        if (stop) break;
        ik_k = rk; ik_l = rl; ik_s = rs; ik_qe = i + 1;
    }
    g1w_sync();
    // prev = curr reversed (bwa reverses the forward intervals)
    int np = nc;
    for (int j = lane; j < np; j += 64) R.prev[j] = R.curr[np - 1 - j];
    g1w_sync();
    int nm = 0, last_mem_qb = 0;
    for (int i = x0 - 1;; --i) {
        const int c = i < 0 ? -1 : (R.q[i] > 3 ? -1 : (int)R.q[i]);
        GPROF(++R.gp_bp; R.gp_be += np;)
        int ncur = 0;
        bool any = false;       // a surviving entry in an earlier chunk
        int64_t carry = 0;      // its size
        for (int j0 = 0; j0 < np; j0 += 64) {
            const int j = j0 + lane;
            const bool live = j < np;
            G1Iv pv{};
            if (live) pv = g1_unpack(R.prev[j]);
            int64_t rk = 0, rl = 0, rs = 0;
            bool valid = false;
            if (live && c >= 0) {
                fm_ext1(G, pv.k, pv.l, pv.s, c, false, rk, rl, rs);
                valid = rs >= min_intv;
            }
            const uint64_t vm = __ballot(valid);
            if (j0 == 0 && !(vm & 1ull) && (nm == 0 || i + 1 < last_mem_qb)) {  // entry 0 fails: a mem
                if (lane == 0) R.mem[nm] = g1_pack(pv.k, pv.l, pv.s, i + 1, pv.qe);
                ++nm;
                last_mem_qb = i + 1;
            }
            const uint64_t below = vm & ((1ull << lane) - 1ull);
            const int pl = below ? 63 - __builtin_clzll(below) : -1;
            const int64_t ps = shfl64(rs, pl < 0 ? 0 : pl);
            const bool push = valid && (pl >= 0 ? rs != ps : (!any || rs != carry));
            const uint64_t pm = __ballot(push);
            if (push) R.curr[ncur + __builtin_popcountll(pm & ((1ull << lane) - 1ull))] = g1_pack(rk, rl, rs, 0, pv.qe);
            ncur += __builtin_popcountll(pm);
            if (vm) { carry = shfl64(rs, 63 - __builtin_clzll(vm)); any = true; }
        }
        g1w_sync();
        if (ncur == 0) break;
        uint4 *t = R.prev; R.prev = R.curr; R.curr = t;
        np = ncur;
    }
    // bwa reverses the mems; the caller keeps those of >= min_seed_len
    for (int t = nm - 1; t >= 0; --t) {
        const G1Iv m = g1_unpack(R.mem[t]);
        if (m.qe - m.qb >= R.msl && !g1w_take(R, m, lane)) break;
    }
    g1w_sync();
    return ret;
}

__global__ __launch_bounds__(64, AF_G1W_WPS) void k_g_seeds_wave(DevGenome G, const uint8_t *__restrict__ reads, int32_t stride,
                                                     const int32_t *__restrict__ lens, int64_t cap, af_params p,
                                                     GOpt o, uint4 *__restrict__ scratch, GWork w) {
    __shared__ uint8_t qs[AF_MAX_READ + 16];
    const int lane = threadIdx.x;
    uint4 *const base = scratch + (int64_t)blockIdx.x * G1_SLOT;
    const int64_t nh = min((int64_t)*(volatile unsigned long long *)w.g1_hv_n, cap);
    const int msl = p.min_seed_len;
    const int split_len = (int)((float)msl * 1.5f + .499);
    for (;;) {
        int64_t h = 0;
        if (lane == 0) h = (int64_t)atomicAdd(w.g1_hv_next, 1ull);
        h = (int64_t)__builtin_amdgcn_readfirstlane((int)h);
        if (h >= nh) break;
        const int64_t rr = w.g1_hv[h];
        G1W R{base, base + G1_LIST, base + 2 * G1_LIST, base + 3 * G1_LIST, qs, read_len(lens, rr, stride), 0, msl, false};
        GPROF(const uint64_t gp_w0 = clock64(); int gp_ssn = 0;)
        const uint8_t *rd = reads + rr * (int64_t)stride;
        for (int t = lane; t < R.len; t += 64) qs[t] = nt4(rd[t]);
        wave_sync();
        // pass 1: SMEMs covering each position
        for (int x = 0; x < R.len && !R.ovf;) {
            if (R.q[x] > 3) { ++x; continue; }
            x = g1w_smem(G, R, x, 1, lane);
        }
        // pass 2: re-seeding of long SMEMs with few occurrences
        const int old_n = R.ni;
        for (int k2 = 0; k2 < old_n && !R.ovf; ++k2) {
            const G1Iv pk = g1_unpack(R.lst[k2]);
            if (pk.qe - pk.qb < split_len || pk.s > o.split_width) continue;
            const int mid = (pk.qb + pk.qe) >> 1;
            if (R.q[mid] > 3) continue;
            g1w_smem(G, R, mid, pk.s + 1, lane);
        }
        // pass 3: bwt_seed_strategy1 from each position
        if (o.max_mem_intv > 0)
            for (int x = 0; x < R.len && !R.ovf;) {
                const int c0 = R.q[x];
                if (c0 > 3) { ++x; continue; }
                int64_t ik_k, ik_l, ik_s;
                fm_set(G, c0, ik_k, ik_l, ik_s);
                const int sx = x;
                for (int i = x + 1;; ++i) {
                    if (i >= R.len) { x = R.len; break; }
                    const int c = R.q[i];
                    if (c > 3) { x = i + 1; break; }
                    int64_t rk, rl, rs;
                    GPROF(++gp_ssn;)
                    fm_ext1(G, ik_k, ik_l, ik_s, 3 - c, true, rk, rl, rs);
                    if (rs < o.max_mem_intv && i - sx >= msl) {
                        if (rs > 0) g1w_take(R, G1Iv{rk, rl, rs, sx, i + 1}, lane);
                        x = i + 1;
                        break;
                    }
                    ik_k = rk; ik_l = rl; ik_s = rs;
                }
            }
        g1w_sync();
        GPROF(if (lane == 0) { int32_t *g = gp_row(rr); if (g) { g[27] = -(int32_t)((clock64() - gp_w0) >> 4) - 1;
              g[28] = R.gp_f; g[29] = R.gp_bp; g[30] = R.gp_be; g[31] = gp_ssn; } })
        // the list into the call's pool (k_g_seeds' G1_DONE; k_g_regions sorts it)
        if (lane == 0) {
            const int ni = R.ni;
            uint4 *Lf = R.lst;
            bool hv = false;  // G2 takes it first
            if (R.ovf) w.iv_n[rr] = -1;
            else {
                const int64_t off = ni ? (int64_t)atomicAdd(w.iv_fill, (unsigned long long)ni) : 0;
                if (ni && off + ni > w.iv_cap) {
                    atomicAdd(&w.stats[AF_GSTAT_POOL], 1);
                    w.iv_n[rr] = -1;
                } else {
                    int64_t occ = 0;
                    for (int a = 0; a < ni; ++a) {
                        const G1Iv m = g1_unpack(Lf[a]);
                        w.iv[off + a] = GIv{m.k, m.s, m.qb, m.qe};
                        occ += m.s > p.max_occ ? p.max_occ : m.s;
                    }
                    w.iv_off[rr] = off;
                    w.iv_n[rr] = ni;
                    hv = w.g2_first_occ > 0 && occ >= w.g2_first_occ;
                }
            }
            if (w.g2_first_occ > 0) {
                w.g2_flag[rr] = hv;
                if (hv) w.g2_list[atomicAdd(w.g2_list_n, 1ull)] = (int32_t)rr;
            }
        }
        g1w_sync();
    }
}

// ============================================================= G2: mem_align1_core
struct G2Scr {           // one wave's scratch (global memory)
    GSeed *pool;         // chain seeds, linked per chain (next)
    int32_t *next;
    GChain *ch, *ch2;    // chains (mem_chain), then in tree order
    int32_t *last_of;
    int32_t *order;
    GKb *kb;
    GSeed *seed;         // compacted: each chain's seeds contiguous
    uint64_t *srt;
    GReg *reg;
    int32_t *kept;
};
constexpr size_t g2_slot_bytes() {
    return ((size_t)AF_G_MAX_OCC * sizeof(GSeed) + (size_t)AF_G_MAX_OCC * 4 + 2 * (size_t)AF_G_MAX_CHAIN * sizeof(GChain) +
            3 * (size_t)AF_G_MAX_CHAIN * 4 + (size_t)G_KB_NODES * sizeof(GKb) + (size_t)AF_G_MAX_OCC * sizeof(GSeed) +
            (size_t)AF_G_MAX_OCC * 8 + (size_t)AF_G_MAX_REG * sizeof(GReg) + 1024) & ~(size_t)255;
}
__device__ G2Scr g2_scr(uint8_t *base) {
    G2Scr s;
    uint8_t *p = base;
    auto take = [&](size_t b) { uint8_t *r = p; p += (b + 15) & ~(size_t)15; return r; };
    s.pool = (GSeed *)take((size_t)AF_G_MAX_OCC * sizeof(GSeed));
    s.next = (int32_t *)take((size_t)AF_G_MAX_OCC * 4);
    s.ch = (GChain *)take((size_t)AF_G_MAX_CHAIN * sizeof(GChain));
    s.ch2 = (GChain *)take((size_t)AF_G_MAX_CHAIN * sizeof(GChain));
    s.last_of = (int32_t *)take((size_t)AF_G_MAX_CHAIN * 4);
    s.order = (int32_t *)take((size_t)AF_G_MAX_CHAIN * 4);
    s.kept = (int32_t *)take((size_t)AF_G_MAX_CHAIN * 4);
    s.kb = (GKb *)take((size_t)G_KB_NODES * sizeof(GKb));
    s.seed = (GSeed *)take((size_t)AF_G_MAX_OCC * sizeof(GSeed));
    s.srt = (uint64_t *)take((size_t)AF_G_MAX_OCC * 8);
    s.reg = (GReg *)take((size_t)AF_G_MAX_REG * sizeof(GReg));
    return s;
}

struct G2Lds {
    int64_t occ[64];      // a batch of sampled occurrences (SA rows gathered by the wave)
    int32_t misc[8];
    int64_t rmax[2];
};
__shared__ G2Lds g_g2;
// the containment boxes of a read's first regions (mem_chain2aln's "extension made before" test
// reads them per seed: LDS instead of the region records in global scratch)
constexpr int G2_BOXES = 512;
struct G2Box {
    int64_t rb, re;
    int32_t qb, qe, w, seedlen0;
};
__shared__ G2Box g_box[G2_BOXES];
GPROF(__shared__ int64_t g_gp_flt;)  // mem_chain_flt's sort cycles of the current read (profiling build)

// ---- bntseq.c on the device
__device__ __forceinline__ int g_pos2rid(const DevGenome &G, int64_t pos_f) {
    if (pos_f >= G.l_pac) return -1;
    if (G.ctg_bkt) {  // the bucket's contig; past a boundary inside it, the next ones in turn
        const int32_t e = G.ctg_bkt[pos_f >> AF_CTG_BKT_SHIFT];
        int rid = e & 0x7fffffff;
        if (e < 0)
            while (rid + 1 < G.n_ctg && pos_f >= G.ctg_off_d[rid + 1]) ++rid;
        return rid;
    }
    int left = 0, mid = 0, right = G.n_ctg;
    while (left < right) {
        mid = (left + right) >> 1;
        if (pos_f >= G.ctg_off_d[mid]) {
            if (mid == G.n_ctg - 1) break;
            if (pos_f < G.ctg_off_d[mid + 1]) break;
            left = mid + 1;
        } else right = mid;
    }
    return mid;
}
__device__ __forceinline__ int64_t g_depos(const DevGenome &G, int64_t pos, int *is_rev) {
    return (*is_rev = (pos >= G.l_pac)) ? (G.l_pac << 1) - 1 - pos : pos;
}
__device__ __forceinline__ int g_intv2rid(const DevGenome &G, int64_t rb, int64_t re) {
    int is_rev;
    if (rb < G.l_pac && re > G.l_pac) return -2;
    const int rid_b = g_pos2rid(G, g_depos(G, rb, &is_rev));
    const int rid_e = rb < re ? g_pos2rid(G, g_depos(G, re - 1, &is_rev)) : rid_b;
    return rid_b == rid_e ? rid_b : -1;
}
__device__ __forceinline__ void g_fetch_clip(const DevGenome &G, int64_t *beg, int64_t mid, int64_t *end, int *rid) {
    int is_rev;
    if (*end < *beg) { const int64_t t = *end; *end = *beg; *beg = t; }
    *rid = g_pos2rid(G, g_depos(G, mid, &is_rev));
    int64_t fb = G.ctg_off_d[*rid], fe = fb + G.ctg_len_d[*rid];
    if (is_rev) { const int64_t t = fb; fb = (G.l_pac << 1) - fe; fe = (G.l_pac << 1) - t; }
    *beg = *beg > fb ? *beg : fb;
    *end = *end < fe ? *end : fe;
}

// ---- mem_chain's working set in LDS (the G2 boxes' space, free until chain2aln): the first
// G_POS_LDS chains' keys (the kbtree's comparisons read only these), its first G_KB_LDS nodes and
// the first G_CH_LDS chains' end seeds (test_and_merge's one read per seed); the rest stays in the
// wave's global scratch.  Lane 0's walk then reads LDS for the lists of up to ~a thousand chains
// instead of chasing scratch lines through L2.
constexpr int G_POS_LDS = 1024, G_KB_LDS = 96, G_CH_LDS = 120;
struct GChainHot {             // a chain's last seed, contig, seed count and first seed's query span
    int64_t r_last;
    int32_t rid, n;
    int16_t q_first, len_first, q_last, len_last, last, pad;
};
static_assert(AF_MAX_READ < 32768 && AF_G_MAX_OCC <= 32768, "16-bit query spans and pool indices");
struct GChainLds {
    int64_t pos[G_POS_LDS];
    GChainHot ch[G_CH_LDS];
    GKb node[G_KB_LDS];
    int32_t rid[64];           // the wave's batch of occurrences: each one's contig (g_intv2rid)
};

static_assert(sizeof(GChainLds) <= sizeof(G2Box) * G2_BOXES, "mem_chain's LDS set fits the boxes");

// ---- klib kbtree (t = 5) over chain indices keyed by chain pos; lane 0 (oracle kb_*)
struct GTree {
    GKb *node_l, *node_g;
    int nn, root;
    const GChain *ch;
    const int64_t *pos_l;
    __device__ GKb &nd(int i) const { return i < G_KB_LDS ? node_l[i] : node_g[i]; }
    __device__ int64_t pos(int x) const { return x < G_POS_LDS ? pos_l[x] : ch[x].pos; }
};
__device__ __forceinline__ int gkb_cmp(const GTree &b, int x, int64_t kpos) {
    const int64_t a = b.pos(x);
    return (kpos < a) - (a < kpos);
}
__device__ int gkb_getp_aux(const GTree &b, const GKb &x, int64_t kpos, int *r) {
    int tr, *rr, begin = 0, end = x.n;
    if (x.n == 0) return -1;
    rr = r ? r : &tr;
    while (begin < end) {
        const int mid = (begin + end) >> 1;
        if (gkb_cmp(b, x.key[mid], kpos) < 0) begin = mid + 1;
        else end = mid;
    }
    if (begin == x.n) { *rr = 1; return x.n - 1; }
    if ((*rr = -gkb_cmp(b, x.key[begin], kpos)) < 0) --begin;
    return begin;
}
__device__ int gkb_new(GTree &b, int internal) {
    GKb &z = b.nd(b.nn);
    z.n = 0; z.internal = (int16_t)internal;
    return b.nn++;
}
__device__ int gkb_lower(const GTree &b, int64_t kpos) {
    int r = 0, lower = -1, xi = b.root;
    while (xi >= 0) {
        const GKb &x = b.nd(xi);
        const int i = gkb_getp_aux(b, x, kpos, &r);
        if (i >= 0 && r == 0) return x.key[i];
        if (i >= 0) lower = x.key[i];
        if (!x.internal) return lower;
        xi = x.ptr[i + 1];
    }
    return lower;
}
__device__ void gkb_split(GTree &b, int xi, int i, int yi) {
    const int zi = gkb_new(b, b.nd(yi).internal);
    GKb &x = b.nd(xi), &y = b.nd(yi), &z = b.nd(zi);
    z.n = G_KB_T - 1;
    for (int u = 0; u < G_KB_T - 1; ++u) z.key[u] = y.key[G_KB_T + u];
    if (y.internal)
        for (int u = 0; u < G_KB_T; ++u) z.ptr[u] = y.ptr[G_KB_T + u];
    y.n = G_KB_T - 1;
    for (int u = x.n; u >= i + 1; --u) x.ptr[u + 1] = x.ptr[u];
    x.ptr[i + 1] = (int16_t)zi;
    for (int u = x.n - 1; u >= i; --u) x.key[u + 1] = x.key[u];
    x.key[i] = y.key[G_KB_T - 1];
    ++x.n;
}
__device__ bool gkb_putp(GTree &b, int k) {
    const int64_t kpos = b.pos(k);
    int xi = b.root;
    if (b.nn + 16 >= G_KB_NODES) return false;  // one insertion adds at most depth + 1 nodes
    if (b.nd(xi).n == G_KB_MAXK) {
        const int si = gkb_new(b, 1);
        b.nd(si).ptr[0] = (int16_t)xi;
        b.root = si;
        gkb_split(b, si, 0, xi);
        xi = si;
    }
    for (;;) {  // __kb_putp_aux, iteratively
        GKb &x = b.nd(xi);
        if (!x.internal) {
            const int i = gkb_getp_aux(b, x, kpos, nullptr);
            for (int u = x.n - 1; u >= i + 1; --u) x.key[u + 1] = x.key[u];
            x.key[i + 1] = (int16_t)k;
            ++x.n;
            return true;
        }
        int i = gkb_getp_aux(b, x, kpos, nullptr) + 1;
        if (b.nd(x.ptr[i]).n == G_KB_MAXK) {
            gkb_split(b, xi, i, x.ptr[i]);
            if (gkb_cmp(b, b.nd(xi).key[i], kpos) < 0) ++i;  // klib: cmp(*k, key[i]) > 0, k past the promoted key
        }
        xi = b.nd(xi).ptr[i];
    }
}
// in-order traversal into order[] (iterative; depth <= 8 for 8192 keys at t = 5)
__device__ int gkb_traverse(const GTree &b, int32_t *order) {
    int stk_node[16], stk_i[16], top = 1, n = 0;
    stk_node[0] = b.root; stk_i[0] = 0;
    while (top > 0) {
        const int xi = stk_node[top - 1];
        const int i = stk_i[top - 1];
        const GKb &x = b.nd(xi);
        if (!x.internal) {
            for (int u = 0; u < x.n; ++u) order[n++] = x.key[u];
            --top;
            continue;
        }
        if (i > x.n) { --top; continue; }
        stk_i[top - 1] = i + 1;
        if (i > 0) order[n++] = x.key[i - 1];
        stk_node[top] = x.ptr[i]; stk_i[top] = 0; ++top;
    }
    return n;
}

// test_and_merge (oracle test_and_merge), lane 0: 1 merged / contained, 0 not, -1 overflow
// (hot: the first nhot chains' end seeds in LDS; r_first: chain ci's pos, its first seed's rbeg)
__device__ int g_test_and_merge(const G2Scr &S, GChainHot *hot, int nhot, int ci, int64_t r_first, const GSeed &p,
                                int rid, int64_t l_pac, int w, int max_chain_gap, int *npool) {
    int64_t r_last;
    int q_first, len_first, q_last, len_last, crid, cn, clast;
    if (ci < nhot) {
        const GChainHot h = hot[ci];
        r_last = h.r_last;
        q_first = h.q_first; len_first = h.len_first; q_last = h.q_last; len_last = h.len_last;
        crid = h.rid; cn = h.n; clast = h.last;
    } else {
        const GChain c = S.ch[ci];
        clast = S.last_of[ci];
        const GSeed first = S.pool[c.seed0], last = S.pool[clast];
        r_last = last.rbeg;
        q_first = first.qbeg; len_first = first.len; q_last = last.qbeg; len_last = last.len;
        crid = c.rid; cn = c.n;
    }
    (void)len_first;
    const int64_t qend = (int64_t)q_last + len_last, rend = r_last + len_last;
    if (rid != crid) return 0;
    if (p.qbeg >= q_first && p.qbeg + p.len <= qend && p.rbeg >= r_first && p.rbeg + p.len <= rend) return 1;
    if ((r_last < l_pac || r_first < l_pac) && p.rbeg >= l_pac) return 0;
    const int64_t x = p.qbeg - q_last, y = p.rbeg - r_last;
    if (y >= 0 && x - y <= w && y - x <= w && x - len_last < max_chain_gap && y - len_last < max_chain_gap) {
        if (*npool >= AF_G_MAX_OCC) return -1;
        const int k = (*npool)++;
        S.pool[k] = p;
        S.next[k] = -1;
        S.next[clast] = k;
        S.last_of[ci] = k;
        S.ch[ci].n = cn + 1;
        if (ci < nhot) {
            GChainHot &g = hot[ci];
            g.r_last = p.rbeg; g.q_last = (int16_t)p.qbeg; g.len_last = (int16_t)p.len; g.n = cn + 1; g.last = (int16_t)k;
        }
        return 1;
    }
    return 0;
}

// ---- mem_chain's chains as a sorted array in LDS (the same space): while no two chains share a
// pos and there are at most G_ARR of them, the kbtree holds distinct keys, so its lookups (the
// largest key <= the seed's rbeg) and its in-order traversal are those of a sorted array -- the
// wave searches it (two ballots) and shifts it open for an insertion, instead of lane 0 walking
// tree nodes.  A second chain at an existing pos (whose place among the equal keys depends on the
// tree's shape) or chain G_ARR + 1 restarts the read on the kbtree.
constexpr int G_ARR = 1392, G_CH_ARR = 64;
// the array mode's chain limit (tests: env AF_G_CHAIN_ARR -- 0 every read on the kbtree, a small
// count most reads restarted there)
__device__ int g_chain_arr = G_ARR;
struct GChainArr {
    int64_t key[G_ARR];
    int16_t id[G_ARR];
    GChainHot ch[G_CH_ARR];
    int32_t rid[64];
};
static_assert(sizeof(GChainArr) <= sizeof(G2Box) * G2_BOXES, "the array mode's LDS set fits the boxes");
static_assert(G_ARR <= 64 * 32, "g_arr_rank covers 64 strides of 32 keys");
// the number of keys <= kpos among key[0, n) (ascending, n <= 2048): a ballot over the 64
// strides of 32, then one over the stride
__device__ __forceinline__ int g_arr_rank(const int64_t *key, int n, int64_t kpos, int lane) {
    const int i1 = lane << 5;
    const uint64_t m1 = __ballot(i1 < n && key[i1] <= kpos);
    if (!m1) return 0;
    const int b = __builtin_popcountll(m1) - 1;
    const int i2 = (b << 5) + (lane & 31);
    const uint64_t m2 = __ballot(lane < 32 && i2 < n && key[i2] <= kpos);
    return (b << 5) + __builtin_popcountll(m2);
}

// mem_chain over the read's intervals (oracle mem_chain): returns the chain count (tree order,
// seeds compacted in S.seed), -1 on overflow.  The wave gathers 64 SA rows at a time; the array
// mode takes each seed on the whole wave, the kbtree mode on lane 0.
__device__ int g_mem_chain(const DevGenome &G, const G2Scr &S, const GIv *iv, int niv, const af_params &p,
                           const GOpt &o, int lane) {
    G2Lds &E = g_g2;
    GChainLds &C = *reinterpret_cast<GChainLds *>(g_box);
    GChainArr &A = *reinterpret_cast<GChainArr *>(g_box);
    int nch = 0, npool = 0;
    bool ovf = false;
    GTree tree{C.node, S.kb, 0, 0, S.ch, C.pos};
    bool by_arr = true;
    for (int arr = 1; arr >= 0; --arr) {
        by_arr = arr;
        nch = 0; npool = 0; ovf = false;
        bool restart = false;
        tree.nn = 0; tree.root = 0;
        if (!arr && lane == 0) tree.root = gkb_new(tree, 0);
        int32_t *const ridv = arr ? A.rid : C.rid;
        for (int i = 0; i < niv && !ovf && !restart; ++i) {
            const GIv v = iv[i];
            const int slen = v.qe - v.qb;
            const int64_t step = v.s > p.max_occ ? v.s / p.max_occ : 1;
            const int64_t cnt = v.s > p.max_occ ? (int64_t)p.max_occ : v.s;  // k < s && count < max_occ
            for (int64_t c0 = 0; c0 < cnt && !ovf && !restart; c0 += 64) {
                const int64_t c = c0 + lane;
                const int nb = (int)min((int64_t)64, cnt - c0);
                wave_sync();
                if (c < cnt) {
                    const int64_t rb = G.sa[v.sa_k + c * step];
                    E.occ[lane] = rb;
                    ridv[lane] = g_intv2rid(G, rb, rb + slen);
                }
                wave_sync();
                if (arr) {
                    for (int u = 0; u < nb; ++u) {
                        GSeed s;
                        s.rbeg = E.occ[u];
                        s.qbeg = v.qb;
                        s.len = slen;
                        const int rid = A.rid[u];
                        if (rid < 0) continue;
                        const int at = g_arr_rank(A.key, nch, s.rbeg, lane);  // lower: entry at - 1
                        int r = 0;
                        if (at > 0) {
                            const int64_t kl = A.key[at - 1];
                            if (lane == 0)
                                r = g_test_and_merge(S, A.ch, G_CH_ARR, A.id[at - 1], kl, s, rid, G.l_pac, p.w,
                                                     o.max_chain_gap, &npool);
                            r = __builtin_amdgcn_readfirstlane(r);
                            npool = __builtin_amdgcn_readfirstlane(npool);
                            if (r < 0) { ovf = true; break; }
                            if (r == 0 && kl == s.rbeg) { restart = true; break; }  // a second chain at this pos
                        }
                        if (r) continue;
                        if (nch >= g_chain_arr) { restart = true; break; }
                        if (nch >= AF_G_MAX_CHAIN || npool >= AF_G_MAX_OCC) { ovf = true; break; }
                        // open entry `at`: move [at, nch) up by one, the top 64 first
                        for (int top = nch - 1; top >= at; top -= 64) {
                            const int e = top - lane;
                            int64_t kv = 0;
                            int16_t iv_ = 0;
                            if (e >= at) { kv = A.key[e]; iv_ = A.id[e]; }
                            wave_sync();
                            if (e >= at) { A.key[e + 1] = kv; A.id[e + 1] = iv_; }
                            wave_sync();
                        }
                        if (lane == 0) {
                            const int kk = npool;
                            S.pool[kk] = s;
                            S.next[kk] = -1;
                            S.ch[nch] = GChain{s.rbeg, 1, -1, rid, 0, 0, kk};
                            S.last_of[nch] = kk;
                            if (nch < G_CH_ARR)
                                A.ch[nch] = GChainHot{s.rbeg, rid, 1, (int16_t)s.qbeg, (int16_t)s.len, (int16_t)s.qbeg,
                                                      (int16_t)s.len, (int16_t)kk, 0};
                            A.key[at] = s.rbeg;
                            A.id[at] = (int16_t)nch;
                        }
                        ++npool;
                        ++nch;
                        wave_sync();
                    }
                } else if (lane == 0) {
                    for (int u = 0; u < nb && !ovf; ++u) {
                        GSeed s;
                        s.rbeg = E.occ[u];
                        s.qbeg = v.qb;
                        s.len = slen;
                        const int rid = C.rid[u];
                        if (rid < 0) continue;
                        bool to_add = false;
                        if (nch) {
                            const int lower = gkb_lower(tree, s.rbeg);
                            if (lower < 0) to_add = true;
                            else {
                                const int r = g_test_and_merge(S, C.ch, G_CH_LDS, lower, tree.pos(lower), s, rid, G.l_pac,
                                                               p.w, o.max_chain_gap, &npool);
                                if (r < 0) ovf = true;
                                else if (!r) to_add = true;
                            }
                        } else to_add = true;
                        if (to_add && !ovf) {
                            if (nch >= AF_G_MAX_CHAIN || npool >= AF_G_MAX_OCC) { ovf = true; break; }
                            const int kk = npool++;
                            S.pool[kk] = s;
                            S.next[kk] = -1;
                            S.ch[nch] = GChain{s.rbeg, 1, -1, rid, 0, 0, kk};
                            S.last_of[nch] = kk;
                            if (nch < G_POS_LDS) C.pos[nch] = s.rbeg;
                            if (nch < G_CH_LDS)
                                C.ch[nch] = GChainHot{s.rbeg, rid, 1, (int16_t)s.qbeg, (int16_t)s.len, (int16_t)s.qbeg,
                                                      (int16_t)s.len, (int16_t)kk, 0};
                            if (!gkb_putp(tree, nch)) { ovf = true; break; }
                            ++nch;
                        }
                    }
                    E.misc[0] = ovf;
                }
                wave_sync();
                if (!arr) ovf = E.misc[0] != 0;
            }
        }
        if (!restart) break;
    }
    int no = 0;
    if (!ovf) {
        // the chains in key order: the array's ids, or the tree's in-order traversal
        if (by_arr) {
            for (int a = lane; a < nch; a += 64) S.order[a] = A.id[a];
            no = nch;
            __threadfence_block();
            wave_sync();
        } else if (lane == 0) no = gkb_traverse(tree, S.order);
    }
    if (lane == 0 && !ovf) {
        int ns = 0;
        for (int a = 0; a < no; ++a) {
            GChain c = S.ch[S.order[a]];
            const int s0 = ns;
            for (int k = c.seed0; k >= 0; k = S.next[k]) S.seed[ns++] = S.pool[k];
            c.seed0 = s0;
            S.ch2[a] = c;
        }
        E.misc[1] = no;
    }
    wave_sync();
    return ovf ? -1 : E.misc[1];
}

__device__ int g_chain_weight(const G2Scr &S, const GChain &c) {
    const GSeed *sd = S.seed + c.seed0;
    int64_t end = 0;
    int w = 0, tmp;
    for (int j = 0; j < c.n; ++j) {
        const GSeed s = sd[j];
        if (s.qbeg >= end) w += s.len;
        else if (s.qbeg + s.len > end) w += (int)(s.qbeg + s.len - end);
        end = end > s.qbeg + s.len ? end : s.qbeg + s.len;
    }
    tmp = w; w = 0; end = 0;
    for (int j = 0; j < c.n; ++j) {
        const GSeed s = sd[j];
        if (s.rbeg >= end) w += s.len;
        else if (s.rbeg + s.len > end) w += (int)(s.rbeg + s.len - end);
        end = end > s.rbeg + s.len ? end : s.rbeg + s.len;
    }
    w = w < tmp ? w : tmp;
    return w < 1 << 30 ? w : (1 << 30) - 1;
}
struct GLtFlt {
    __device__ bool operator()(const GChain &a, const GChain &b) const { return a.w > b.w; }
};
struct GKeyFlt {  // w << 32 | index: GLtFlt on the keys
    __device__ bool operator()(uint64_t a, uint64_t b) const { return (a >> 32) > (b >> 32); }
};

// mem_chain_flt (oracle mem_chain_flt) over S.ch2 on the wave: returns the kept count.  The
// chains' weights, query spans and the overlap scan against the kept list are lane-parallel (the
// scan's first breaking chain found by a ballot, so `first` is set exactly for the overlapping
// kept chains the sequential scan visits); klib's introsort (its tie order is bwa's) and the
// order-preserving compaction run as in the oracle.
__device__ int g_chain_flt(const G2Scr &S, int n_chn, const af_params &p, const GOpt &o, int lane) {
    GChain *a = S.ch2;
    if (n_chn == 0) return 0;
    for (int i = lane; i < n_chn; i += 64) {
        GChain c = a[i];
        c.first = -1; c.kept = 0; c.w = g_chain_weight(S, c);
        a[i] = c;
    }
    wave_sync();
    GPROF(const int64_t gp_s0 = clock64();)
    static_assert(3 * AF_G_MAX_CHAIN >= 5 * (int)(sizeof(G2Box) * G2_BOXES / sizeof(uint64_t)),
                  "wave_introsort's scratch: S.last_of, S.order and S.kept (consecutive in g2_scr)");
    if (n_chn <= (int)(sizeof(G2Box) * G2_BOXES / sizeof(uint64_t))) {
        // lane 0's introsort over (w, index) keys in LDS (the boxes, free until chain2aln) instead
        // of 32-B chains in scratch: the swaps depend only on the comparator's answers, so the
        // order, ties included, is the one the introsort over the chains gives; the wave then
        // moves the chains in key order through S.ch (free after mem_chain)
        uint64_t *key = reinterpret_cast<uint64_t *>(g_box);
        for (int i = lane; i < n_chn; i += 64) key[i] = (uint64_t)(uint32_t)a[i].w << 32 | (uint32_t)i;
        __threadfence_block();
        wave_sync();
        // (weights tie, so the order is klib's introsort's: lane 0 for short lists, its exact wave
        // form past 64 keys, with the scratch free after mem_chain)
        if (n_chn >= 64) wave_introsort(key, n_chn, GKeyFlt(), S.last_of, lane);
        else if (lane == 0) ks_introsort(key, n_chn, GKeyFlt());
        __threadfence_block();
        wave_sync();
        for (int i = lane; i < n_chn; i += 64) S.ch[i] = a[(uint32_t)key[i]];
        __threadfence_block();
        wave_sync();
        for (int i = lane; i < n_chn; i += 64) a[i] = S.ch[i];
    } else if (lane == 0) {
        ks_introsort(a, n_chn, GLtFlt());
    }
    __threadfence_block();
    wave_sync();
    GPROF(if (lane == 0) g_gp_flt = clock64() - gp_s0;)
    // the overlap scan: the kept chains in kept order, each packed in one word (query begin / end
    // and weight, 9 bits each, and bit 31 once its `first` is set) with its `first` beside it, so a
    // lane tests one kept chain per LDS read; LDS (the boxes, free again after the sort) when the
    // lists fit, else the scratch free after mem_chain
    // In LDS the kept chains are also grouped by their packed word (a repeat-rich read's chains
    // come from a few intervals: hundreds of chains, a handful of distinct spans and weights), so a
    // chain is tested against the groups (a lane each) instead of every kept chain: members of a
    // group answer alike, the scan's first breaking chain is the first member of the earliest
    // breaking group, and the members whose `first` is still unset form a suffix of the group's
    // list (each member is set once).  Past NG groups the chunk scan takes over.
    static_assert(AF_MAX_READ < 512 && AF_G_MAX_CHAIN < 32768, "9-bit spans and weights, 16-bit chain indices");
    constexpr int NG = 64;
    constexpr int NL = (int)((sizeof(G2Box) * G2_BOXES - NG * 10) / 14) & ~1;
    const bool lds = n_chn <= NL;
    uint8_t *const lb = reinterpret_cast<uint8_t *>(g_box);
    uint32_t *kp = lds ? reinterpret_cast<uint32_t *>(lb) : reinterpret_cast<uint32_t *>(S.last_of);
    int16_t *kf = lds ? reinterpret_cast<int16_t *>(lb + 4 * NL) : reinterpret_cast<int16_t *>(S.order);
    static_assert(AF_G_MAX_OCC >= AF_G_MAX_CHAIN, "S.next holds two 16-bit lists of the chains");
    int16_t *cb = lds ? reinterpret_cast<int16_t *>(lb + 6 * NL) : reinterpret_cast<int16_t *>(S.next);
    int16_t *ce = lds ? cb + NL : cb + AF_G_MAX_CHAIN;
    int16_t *cw = lds ? ce + NL : reinterpret_cast<int16_t *>(S.kept);
    int16_t *nx = reinterpret_cast<int16_t *>(lb + 12 * NL);  // the next member of a kept chain's group
    uint32_t *gkey = reinterpret_cast<uint32_t *>(lb + 14 * NL);
    int16_t *gfirst = reinterpret_cast<int16_t *>(gkey + NG), *gpend = gfirst + NG, *gtail = gpend + NG;
    for (int i = lane; i < n_chn; i += 64) {
        const GChain c = a[i];
        const GSeed t = S.seed[c.seed0 + c.n - 1];
        cb[i] = (int16_t)S.seed[c.seed0].qbeg;
        ce[i] = (int16_t)(t.qbeg + t.len);
        cw[i] = (int16_t)(c.w < 511 ? c.w : 511);
    }
    __threadfence_block();
    wave_sync();
    auto pack = [&](int i) -> uint32_t { return (uint32_t)cb[i] | (uint32_t)ce[i] << 9 | (uint32_t)cw[i] << 18; };
    bool grp = lds && g_chain_arr > 0;  // (AF_G_CHAIN_ARR=0, a test mode: the kbtree and the chunk scan)
    int ng = 1;
    if (lane == 0) {
        a[0].kept = 3; kp[0] = pack(0); kf[0] = -1;
        if (grp) { nx[0] = -1; gkey[0] = kp[0]; gfirst[0] = 0; gpend[0] = 0; gtail[0] = 0; }
    }
    wave_sync();
    int nc = 1;
    // a chain whose span and weight equal the previous chain's, when that one broke off, breaks at
    // the same kept chain and finds every `first` up to it set: nothing to do
    uint32_t prev_key = 0xFFFFFFFFu;
    bool prev_brk = false;
    for (int i = 1; i < n_chn; ++i) {
        const int bi = cb[i], ei = ce[i], wi = cw[i], li = ei - bi;
        const uint32_t key_i = pack(i);
        if (prev_brk && key_i == prev_key) continue;
        prev_key = key_i;
        bool large_ovlp = false, brk = false;
        if (grp) {
            const uint32_t x = lane < ng ? gkey[lane] : 0u;
            const int gf = lane < ng ? gfirst[lane] : INT_MAX;
            bool ov = false, bk = false;
            if (lane < ng) {
                const int bj = (int)(x & 511), ej = (int)(x >> 9 & 511);
                const int b_max = bj > bi ? bj : bi, e_min = ej < ei ? ej : ei;
                if (e_min > b_max) {
                    const int lj = ej - bj, min_l = li < lj ? li : lj;
                    if ((float)(e_min - b_max) >= (float)min_l * 0.5f && min_l < o.max_chain_gap) {
                        ov = true;
                        const int wj = (int)(x >> 18 & 511);
                        bk = (float)wi < (float)wj * 0.5f && wj - wi >= p.min_seed_len << 1;
                    }
                }
            }
            int bp = bk ? gf : INT_MAX;  // the first breaking kept chain
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) bp = min(bp, __shfl_xor(bp, d));
            brk = bp != INT_MAX;
            large_ovlp = __ballot(ov && gf <= bp) != 0;
            if (ov) {  // the group's members up to bp whose `first` is unset
                int pos = gpend[lane];
                while (pos >= 0 && pos <= bp) {
                    kp[pos] |= 1u << 31;
                    kf[pos] = (int16_t)i;
                    pos = nx[pos];
                }
                gpend[lane] = (int16_t)pos;
            }
            prev_brk = brk;
            if (!brk) {
                const uint32_t key = key_i;
                const uint64_t gm = __ballot(lane < ng && x == key);
                if (lane == 0) {
                    kp[nc] = key; kf[nc] = -1; nx[nc] = -1; a[i].kept = large_ovlp ? 2 : 3;
                    if (gm) {
                        const int g = __builtin_ctzll(gm);
                        nx[gtail[g]] = (int16_t)nc;
                        gtail[g] = (int16_t)nc;
                        if (gpend[g] < 0) gpend[g] = (int16_t)nc;
                    } else if (ng < NG) {
                        gkey[ng] = key; gfirst[ng] = (int16_t)nc; gpend[ng] = (int16_t)nc; gtail[ng] = (int16_t)nc;
                    }
                }
                if (!gm) {
                    if (ng < NG) ++ng;
                    else grp = false;  // past NG groups: the chunk scan (kp / kf hold every kept chain)
                }
                ++nc;
            }
            __threadfence_block();
            wave_sync();
            continue;
        }
        // four chunks of 64 kept chains per round: their loads issued together, then taken in
        // kept order up to the first breaking chain
        for (int k0 = 0; k0 < nc && !brk; k0 += 256) {
            uint32_t x[4];
            uint64_t om[4], bm[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int k = k0 + 64 * u + lane;
                x[u] = k < nc ? kp[k] : 0u;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int k = k0 + 64 * u + lane;
                bool ov = false, bk = false;
                if (k < nc) {
                    const int bj = (int)(x[u] & 511), ej = (int)(x[u] >> 9 & 511);
                    const int b_max = bj > bi ? bj : bi, e_min = ej < ei ? ej : ei;
                    if (e_min > b_max) {
                        const int lj = ej - bj, min_l = li < lj ? li : lj;
                        if ((float)(e_min - b_max) >= (float)min_l * 0.5f && min_l < o.max_chain_gap) {
                            ov = true;
                            const int wj = (int)(x[u] >> 18 & 511);
                            bk = (float)wi < (float)wj * 0.5f && wj - wi >= p.min_seed_len << 1;
                        }
                    }
                }
                bm[u] = __ballot(bk);
                om[u] = __ballot(ov);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if (brk) break;
                uint64_t m = om[u];
                if (bm[u]) {
                    const int f = __builtin_ctzll(bm[u]);
                    if (f < 63) m &= (2ull << f) - 1ull;
                    brk = true;
                }
                if (m) large_ovlp = true;
                const int k = k0 + 64 * u + lane;
                if (((m >> lane) & 1ull) && !(x[u] >> 31)) { kp[k] = x[u] | 1u << 31; kf[k] = (int16_t)i; }
            }
        }
        prev_brk = brk;
        if (!brk) {
            if (lane == 0) { kp[nc] = key_i; kf[nc] = -1; a[i].kept = large_ovlp ? 2 : 3; }
            ++nc;
        }
        __threadfence_block();
        wave_sync();
    }
    for (int k = lane; k < nc; k += 64) {
        const int f = kf[k];
        if (f >= 0) a[f].kept = 1;
    }
    __threadfence_block();
    wave_sync();
    int m = 0;
    for (int i0 = 0; i0 < n_chn; i0 += 64) {
        const int i = i0 + lane;
        GChain c;
        bool keep = false;
        if (i < n_chn) { c = a[i]; keep = c.kept != 0; }
        const uint64_t km = __ballot(keep);
        if (keep) a[m + lanes_below(km, lane)] = c;
        m += __builtin_popcountll(km);
        wave_sync();
    }
    return m;
}

// mem_chain2aln's extension window of a chain (rmax; clipped to the seed's contig, one strand)
// into E.rmax (lane 0 computes it)
__device__ void g_chain_rmax(const DevGenome &G, const af_params &p, int l, const GSeed *sd, int n, int lane) {
    G2Lds &E = g_g2;
    const int64_t l_pac = G.l_pac;
    if (lane == 0) {
        int64_t r0 = l_pac << 1, r1 = 0;
        for (int i = 0; i < n; ++i) {
            const GSeed t = sd[i];
            const int64_t b = t.rbeg - (t.qbeg + cal_max_gap(p, t.qbeg));
            const int rem = l - t.qbeg - t.len;
            const int64_t e = t.rbeg + t.len + (rem + cal_max_gap(p, rem));
            r0 = r0 < b ? r0 : b;
            r1 = r1 > e ? r1 : e;
        }
        r0 = r0 > 0 ? r0 : 0;
        r1 = r1 < l_pac << 1 ? r1 : l_pac << 1;
        if (r0 < l_pac && l_pac < r1) {
            if (sd[0].rbeg < l_pac) r1 = l_pac;
            else r0 = l_pac;
        }
        int rid;
        g_fetch_clip(G, &r0, sd[0].rbeg, &r1, &rid);
        E.rmax[0] = r0; E.rmax[1] = r1;
    }
    wave_sync();
}

// mem_chain2aln's extension of seed s of a chain (seeds sd[0, n), contig rid): ksw_extend2 to
// the left and right of the seed inside the window [rmax0, rmax1) and the chain's seed coverage
// of the region; the read's codes in L.q.  The region on every lane.
template <int CPL>
__device__ GReg g_seed_region(const DevGenome &G, const af_params &p, int l, const GSeed *sd, int n, int rid,
                              const GSeed &s, int64_t rmax0, int64_t rmax1, int lane) {
    DpLds &L = g_dp;
    int a_score = -1, a_truesc = -1, a_qb = 0, a_qe = 0;
    int64_t a_rb = 0, a_re = 0;
    int aw0 = p.w, aw1 = p.w;
    if (s.qbeg) {  // left extension
        const int64_t tmp = s.rbeg - rmax0;
        const int tl = (int)min(tmp, (int64_t)(s.qbeg + 2 * p.w + 1));
        for (int x = lane; x < s.qbeg; x += 64) L.qs[x] = L.q[s.qbeg - 1 - x];
        for (int x = lane; x < tl; x += 64) L.t[x] = G.T[s.rbeg - 1 - x];
        wave_sync();
        ExtRes er;
        for (int it = 0; it < 2; ++it) {
            const int prev = a_score;
            aw0 = p.w << it;
            er = ext_dp<CPL>(s.qbeg, L.qs, tl, L.t, p, aw0, p.pen_clip5, p.zdrop, s.len * p.a, lane);
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
        const int64_t re = s.rbeg + s.len - rmax0;
        const int sc0 = a_score;
        const int tl = (int)min(rmax1 - rmax0 - re, (int64_t)((l - qe) + 2 * p.w + 1));
        for (int x = lane; x < tl; x += 64) L.t[x] = G.T[rmax0 + re + x];
        wave_sync();
        ExtRes er;
        for (int it = 0; it < 2; ++it) {
            const int prev = a_score;
            aw1 = p.w << it;
            er = ext_dp<CPL>(l - qe, L.q + qe, tl, L.t, p, aw1, p.pen_clip3, p.zdrop, sc0, lane);
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
        a_qe = l; a_re = s.rbeg + s.len;
    }
    // seedcov: the chain's seeds inside the region
    int cov = 0;
    for (int i = lane; i < n; i += 64) {
        const GSeed t = sd[i];
        if (t.qbeg >= a_qb && t.qbeg + t.len <= a_qe && t.rbeg >= a_rb && t.rbeg + t.len <= a_re) cov += t.len;
    }
    cov = wave_sum(cov);
    GReg a;
    a.rb = a_rb; a.re = a_re; a.qb = a_qb; a.qe = a_qe; a.rid = rid; a.score = a_score; a.truesc = a_truesc;
    a.w = aw0 > aw1 ? aw0 : aw1; a.seedlen0 = s.len; a.seedcov = cov; a.secondary = -1; a.sub = 0; a.hash = 0;
    return a;
}

// mem_chain2aln (oracle mem_chain2aln) for chain ci of S.ch2; regions appended to S.reg.  pre
// (heavy reads): the region of the chain's first seed in bwa's order (its longest) already
// extended by k_g_ext_jobs, at pre[seed0]; the other seeds the walk keeps (few: most lie inside
// the first one's region) are extended here.
// Returns false on a region-cap overflow.
template <int CPL>
__device__ bool g_chain2aln(const DevGenome &G, const G2Scr &S, const af_params &p, int l, int ci, int *nreg_io,
                            int lane, const GReg *pre = nullptr) {
    G2Lds &E = g_g2;
    G2Box *const box = g_box;
    const GChain c = S.ch2[ci];
    const GSeed *sd = S.seed + c.seed0;
    bool have_rmax = false;  // the chain's window, made when a seed is extended here (not for pre's)
    // srt: seed indices by (score << 32 | i) ascending (keys distinct): rank sort on the wave
    for (int i0 = 0; i0 < c.n; i0 += 64) {
        const int i = i0 + lane;
        if (i < c.n) {
            const uint64_t ki = (uint64_t)(uint32_t)sd[i].len << 32 | (uint32_t)i;
            int rk = 0;
            for (int j = 0; j < c.n; ++j) rk += ((uint64_t)(uint32_t)sd[j].len << 32 | (uint32_t)j) < ki;
            S.srt[rk] = ki;
        }
    }
    wave_sync();
    for (int k = c.n - 1; k >= 0; --k) {
        const uint64_t sk = S.srt[k];
        const GSeed s = sd[(uint32_t)sk];
        const int nreg = *nreg_io;
        // test whether extension has been made before (any region satisfying)
        bool hit = false;
        for (int i0 = 0; i0 < nreg && !hit; i0 += 64) {
            const int i = i0 + lane;
            bool h = false;
            if (i < nreg) {
                // the region's box: LDS for the first G2_BOXES regions of the read, else its record
                GReg pr;
                if (i < G2_BOXES) {
                    const G2Box &bx = box[i];
                    pr.rb = bx.rb; pr.re = bx.re; pr.qb = bx.qb; pr.qe = bx.qe; pr.w = bx.w; pr.seedlen0 = bx.seedlen0;
                } else {
                    pr = S.reg[i];
                }
                if (!(s.rbeg < pr.rb || s.rbeg + s.len > pr.re || s.qbeg < pr.qb || s.qbeg + s.len > pr.qe) &&
                    !((double)(s.len - pr.seedlen0) > .1 * l)) {
                    int qd = s.qbeg - pr.qb;
                    int64_t rd = s.rbeg - pr.rb;
                    int mg = cal_max_gap(p, (int)(qd < rd ? (int64_t)qd : rd));
                    int ww = mg < pr.w ? mg : pr.w;
                    if (qd - rd < ww && rd - qd < ww) h = true;
                    else {
                        qd = pr.qe - (s.qbeg + s.len);
                        rd = pr.re - (s.rbeg + s.len);
                        mg = cal_max_gap(p, (int)(qd < rd ? (int64_t)qd : rd));
                        ww = mg < pr.w ? mg : pr.w;
                        if (qd - rd < ww && rd - qd < ww) h = true;
                    }
                }
            }
            hit = __ballot(h) != 0;
        }
        if (hit) {
            // contained: extend only if a long overlapping seed on another diagonal follows
            bool ov = false;
            for (int i = k + 1 + lane; i < c.n; i += 64) {
                const uint64_t ti = S.srt[i];
                if (ti == 0) continue;
                const GSeed t = sd[(uint32_t)ti];
                if ((double)t.len < s.len * .95) continue;
                if (s.qbeg <= t.qbeg && s.qbeg + s.len - t.qbeg >= s.len >> 2 &&
                    (int64_t)(t.qbeg - s.qbeg) != t.rbeg - s.rbeg) ov = true;
                if (t.qbeg <= s.qbeg && t.qbeg + t.len - s.qbeg >= s.len >> 2 &&
                    (int64_t)(s.qbeg - t.qbeg) != s.rbeg - t.rbeg) ov = true;
            }
            if (!__ballot(ov)) {
                wave_sync();
                if (lane == 0) S.srt[k] = 0;
                wave_sync();
                continue;
            }
        }
        if (nreg >= AF_G_MAX_REG) return false;
        const bool use_pre = pre && k == c.n - 1;
        if (!use_pre && !have_rmax) { g_chain_rmax(G, p, l, sd, c.n, lane); have_rmax = true; }
        const GReg a = use_pre ? pre[c.seed0] : g_seed_region<CPL>(G, p, l, sd, c.n, c.rid, s, E.rmax[0], E.rmax[1], lane);
        if (lane == 0) {
            S.reg[nreg] = a;
            if (nreg < G2_BOXES) box[nreg] = G2Box{a.rb, a.re, a.qb, a.qe, a.w, a.seedlen0};
        }
        *nreg_io = nreg + 1;
        wave_sync();
    }
    return true;
}

// mem_patch_reg's tests before its alignment (oracle mem_patch_reg): false if a and b cannot
// merge; else *w_out the band
__device__ __forceinline__ bool g_patch_pre(int64_t l_pac, const af_params &p, const GReg &a, const GReg &b,
                                            int *w_out) {
    if (a.rb < l_pac && b.rb >= l_pac) return false;
    if (a.qb >= b.qb || a.qe >= b.qe || a.re >= b.re) return false;
    if (b.re - a.rb > AF_S2_MAX_TSPAN) return false;  // the oracle's AFO_PE_MAX_TSPAN (L.t holds 1 KiB)
    int w = (int)((a.re - b.rb) - (a.qe - b.qb));
    w = w > 0 ? w : -w;
    double r = (double)(a.re - b.rb) / (double)(b.re - a.rb) - (double)(a.qe - b.qb) / (double)(b.qe - a.qb);
    r = r > 0. ? r : -r;
    if (a.re < b.rb || a.qe < b.qb) {
        if (w > p.w << 1 || r >= (double)0.05f) return false;
    } else if (w > p.w << 2 || r >= (double)(0.05f * 2)) return false;
    w += a.w + b.w;
    *w_out = w < p.w << 2 ? w : p.w << 2;
    return true;
}

// mem_patch_reg (oracle mem_patch_reg): the merged score, 0 if not merged; *w_out its band
template <int CPL>
__device__ int g_patch_reg(const DevGenome &G, const af_params &p, const GReg &a, const GReg &b, int *w_out,
                           uint8_t *zg, int lane) {
    const int64_t l_pac = G.l_pac;
    int w;
    if (!g_patch_pre(l_pac, p, a, b, &w)) return 0;
    const int lq = b.qe - a.qb;
    const int score = gen_cigar_wave<CPL, false>(G.T, l_pac, p, w, lq, a.qb, a.rb, b.re, g_dp, zg, lane);
    const int q_s = (int)((double)(b.qe - a.qb) / (double)((b.qe - b.qb) + (a.qe - a.qb)) * (double)(b.score + a.score) + .499);
    const int r_s = (int)((double)(b.re - a.rb) / (double)((b.re - b.rb) + (a.re - a.rb)) * (double)(b.score + a.score) + .499);
    if ((double)score / (double)(q_s > r_s ? q_s : r_s) < (double)0.90f) return 0;
    *w_out = w;
    return score;
}

// ---- region lists sorted through keys in LDS: lane 0's introsort compares and swaps small keys
// (each region's index with the fields its comparator reads) in the G2 boxes' space, which is dead
// once a read's chains are extended; the wave then moves the 64-B regions in key order through tmp.
// The swaps depend only on the comparator's answers, so the order (ties included) is the one the
// introsort over the regions themselves gives.
static_assert(AF_G_MAX_REG <= 1024 && AF_MAX_READ < 32768, "region keys pack a 10-bit index and a 15-bit qb");
static_assert(sizeof(G2Box) * G2_BOXES >= 16 * AF_G_MAX_REG, "the boxes hold 16 B of key per region");
static_assert(sizeof(GReg) == 64, "regions move as 4 x 16 B");
// lists this long or longer are sorted on the wave by rank (wave_rank_sort), shorter by lane 0
constexpr int G_RANK_MIN = 24;
struct GKeyRe {  // re << 10 | index (mem_sort_dedup_patch's sort by re)
    __device__ bool operator()(uint64_t a, uint64_t b) const { return (a >> 10) < (b >> 10); }
};
struct GKey16 { int64_t x; int32_t y; int32_t z; };
struct GKeyArs {  // x = rb, y = score, z = qb << 16 | index: score desc, rb, qb
    __device__ bool operator()(const GKey16 &a, const GKey16 &b) const {
        return a.y > b.y || (a.y == b.y && (a.x < b.x || (a.x == b.x && (a.z >> 16) < (b.z >> 16))));
    }
};
struct GKeyHash {  // x = hash, y = score, z = index: score desc, hash (mark_primary_se)
    __device__ bool operator()(const GKey16 &a, const GKey16 &b) const {
        return a.y > b.y || (a.y == b.y && (uint64_t)a.x < (uint64_t)b.x);
    }
};
// a[k] = old a[from(k)] for k < m (wave)
template <class F>
__device__ __forceinline__ void g_regs_gather(GReg *a, GReg *tmp, int m, F from, int lane) {
    const uint4 *src = reinterpret_cast<const uint4 *>(a);
    uint4 *t = reinterpret_cast<uint4 *>(tmp);
    for (int k = lane; k < 4 * m; k += 64) t[k] = src[4 * from(k >> 2) + (k & 3)];
    wave_sync();
    uint4 *dst = reinterpret_cast<uint4 *>(a);
    for (int k = lane; k < 4 * m; k += 64) dst[k] = t[k];
    wave_sync();
}

// mem_sort_dedup_patch's overlap test of q = a[j] against p = a[i] (oracle mem_sort_dedup_patch)
__device__ __forceinline__ bool g_dd_overlap(const GReg &q, const GReg &pp) {
    const int64_t or_ = q.re - pp.rb;
    const int64_t oq = q.qb < pp.qb ? q.qe - pp.qb : pp.qe - q.qb;
    const int64_t mr = q.re - q.rb < pp.re - pp.rb ? q.re - q.rb : pp.re - pp.rb;
    const int64_t mq = q.qe - q.qb < pp.qe - pp.qb ? q.qe - q.qb : pp.qe - pp.qb;
    return (float)or_ > 0.95f * (float)mr && (float)oq > 0.95f * (float)mq;
}

// mem_sort_dedup_patch (oracle mem_sort_dedup_patch) over a[0, n); patch: merge colinear hits;
// tmp: n regions of scratch.  bwa's walk for a[i] visits j = i-1, i-2, ... while a[j] is on a[i]'s
// contig within max_chain_gap; the wave tests 64 of them at once and stops at the first that
// changes something (an overlap drop, or a patch candidate passing mem_patch_reg's cheap tests),
// which lane 0 applies before the walk resumes below it with a[i] as it now is.
template <int CPL>
__device__ int g_dedup_patch(const DevGenome &G, const af_params &p, const GOpt &o, GReg *a, int n, bool patch,
                             uint8_t *zg, int lane, GReg *tmp) {
    G2Lds &E = g_g2;
    if (n <= 1) return n;
    const int64_t l_pac = G.l_pac, gap = o.max_chain_gap;
    uint64_t *k1 = reinterpret_cast<uint64_t *>(g_box);
    for (int i = lane; i < n; i += 64) k1[i] = (uint64_t)a[i].re << 10 | (uint64_t)i;
    wave_sync();
    if (n < G_RANK_MIN || !wave_rank_sort(k1, n, GKeyRe(), reinterpret_cast<uint64_t *>(tmp), lane)) {
        if (lane == 0) ks_introsort(k1, n, GKeyRe());
        wave_sync();
    }
    g_regs_gather(a, tmp, n, [&](int k) { return (int)(k1[k] & 1023); }, lane);
    for (int i0 = 1; i0 < n; i0 += 64) {
        // a[i] is walked unless it starts a new contig or lies past a[i-1] + max_chain_gap (reads of
        // a[i].rb and a[i-1].re, which no earlier step of the walk changes)
        bool walk = false;
        if (i0 + lane < n) {
            const GReg &x = a[i0 + lane], &y = a[i0 + lane - 1];
            walk = !(x.rid != y.rid || x.rb >= y.re + gap);
        }
        uint64_t wm = __ballot(walk);
        while (wm) {
            const int i = i0 + __builtin_ctzll(wm);
            wm &= wm - 1;
            GReg pp = a[i];
            for (int j = i - 1; j >= 0;) {
                const int jj = j - lane;
                bool cont = false, ev = false;
                if (jj >= 0) {
                    const GReg q = a[jj];
                    // without patching only an overlap changes something, and it needs q.re > pp.rb:
                    // re ascends along the list, so the walk may stop at the first q ending at or
                    // before pp's start (the regions below it cannot overlap pp either)
                    cont = pp.rid == q.rid && pp.rb < q.re + gap && (patch || q.re > pp.rb);
                    if (cont && q.qe != q.qb) {
                        int w_;
                        ev = g_dd_overlap(q, pp) || (patch && q.rb < pp.rb && g_patch_pre(l_pac, p, q, pp, &w_));
                    }
                }
                const uint64_t stop = __ballot(!cont), em = __ballot(ev);
                const uint64_t e = em & (stop ? (stop & (0ull - stop)) - 1 : ~0ull);
                if (!e) {
                    if (stop) break;
                    j -= 64;
                    continue;
                }
                const int js = j - __builtin_ctzll(e);
                const GReg q = a[js];
                if (g_dd_overlap(q, pp)) {
                    const bool drop_p = pp.score < q.score;
                    if (lane == 0) {
                        if (drop_p) a[i].qe = a[i].qb;
                        else a[js].qe = a[js].qb;
                    }
                    wave_sync();
                    if (drop_p) break;
                } else {
                    int w = 0;
                    const int score = g_patch_reg<CPL>(G, p, q, pp, &w, zg, lane);
                    if (score > 0) {
                        wave_sync();
                        if (lane == 0) {
                            GReg &P = a[i];
                            P.seedcov = P.seedcov > q.seedcov ? P.seedcov : q.seedcov;
                            P.sub = P.sub > q.sub ? P.sub : q.sub;
                            P.qb = q.qb; P.rb = q.rb;
                            P.truesc = P.score = score;
                            P.w = w;
                            a[js].qb = a[js].qe;
                        }
                        wave_sync();
                        pp = a[i];
                    }
                }
                j = js - 1;
            }
        }
    }
    // the live regions (in order) sorted by (score desc, rb, qb); equal neighbours dropped
    GKey16 *k2 = reinterpret_cast<GKey16 *>(g_box);
    int m = 0;
    for (int i0 = 0; i0 < n; i0 += 64) {
        const int i = i0 + lane;
        GReg x;
        const bool live = i < n && ((x = a[i]), x.qe > x.qb);
        const uint64_t lm = __ballot(live);
        if (live) k2[m + lanes_below(lm, lane)] = GKey16{x.rb, x.score, x.qb << 16 | i};
        m += __builtin_popcountll(lm);
    }
    wave_sync();
    if (m < G_RANK_MIN || !wave_rank_sort(k2, m, GKeyArs(), reinterpret_cast<GKey16 *>(tmp), lane)) {
        if (lane == 0) ks_introsort(k2, m, GKeyArs());
        wave_sync();
    }
    // kept keys compacted in order: a kept key's z goes to slot mm + (kept before it) <= its own
    // slot, so the next chunk's first comparison (with this chunk's last key) still reads that
    // key's own z
    int mm = 0;
    for (int i0 = 0; i0 < m; i0 += 64) {
        const int i = i0 + lane;
        bool keep = false;
        GKey16 c{0, 0, 0};
        if (i < m) {
            c = k2[i];
            keep = i == 0;
            if (i > 0) {
                const GKey16 d = k2[i - 1];
                keep = !(c.y == d.y && c.x == d.x && (c.z >> 16) == (d.z >> 16));
            }
        }
        const uint64_t km = __ballot(keep);
        wave_sync();
        if (keep) k2[mm + lanes_below(km, lane)].z = c.z;
        mm += __builtin_popcountll(km);
        wave_sync();
    }
    g_regs_gather(a, tmp, mm, [&](int k) { return k2[k].z & 0xffff; }, lane);
    (void)E;
    return mm;
}

__device__ __forceinline__ void g_load_read(const uint8_t *reads, int64_t r, int32_t stride, int l, int lane) {
    DpLds &L = g_dp;
    const uint8_t *rd = reads + r * (int64_t)stride;
    for (int x = lane; x < l; x += 64) L.q[x] = nt4(rd[x]);
    wave_sync();
}

__device__ __forceinline__ int g_next_item(int32_t *heads, int &head, int &heads_left, int64_t n, int lane) {
    while (heads_left > 0) {
        int v = 0;
        if (lane == 0) v = atomicAdd(&heads[AF_HEAD_STRIDE * head], 1);
        v = __builtin_amdgcn_readfirstlane(v);
        const int64_t it = head + 8 * (int64_t)v;
        if (it < n) return (int)it;
        head = (head + 1) & 7;
        --heads_left;
    }
    return -1;
}

// the read's regions S.reg[0, nreg) into the call's pool (ovf: the read past a cap)
__device__ void g_put_regions(const GWork &w, const G2Scr &S, int64_t r, int nreg, bool ovf, int lane) {
    int off = 0;
    if (!ovf && nreg > 0) {
        if (lane == 0) g_g2.misc[4] = atomicAdd(w.reg_fill, nreg);
        wave_sync();
        off = g_g2.misc[4];
        if ((int64_t)off + nreg > w.reg_cap) {
            if (lane == 0) atomicAdd(&w.stats[AF_GSTAT_POOL], 1);
            ovf = true;
        }
    }
    if (!ovf)
        for (int k = lane; k < nreg; k += 64) w.reg[off + k] = S.reg[k];
    if (lane == 0) {
        w.reg_off[r] = off;
        w.reg_n[r] = ovf ? -1 : nreg;
        if (ovf) atomicAdd(&w.stats[AF_GSTAT_OVERFLOW], 1);
    }
    wave_sync();
}

// a heavy read's kept chains S.ch2[0, nch) and their seeds into the heavy pools (false: a pool is
// full -- the read is then extended by its own wave)
__device__ bool g_defer_heavy(const GWork &w, const G2Scr &S, int64_t r, int nch, int lane) {
    const GHeavy &h = w.hv;
    G2Lds &E = g_g2;
    int nsd = 0;
    for (int i = lane; i < nch; i += 64) nsd += S.ch2[i].n;
    nsd = wave_sum(nsd);
    if (lane == 0) {
        const int64_t hr = (int64_t)atomicAdd(&h.cnt[0], 1ull);
        const int64_t co = (int64_t)atomicAdd(&h.cnt[1], (unsigned long long)nch);
        const int64_t so = (int64_t)atomicAdd(&h.cnt[2], (unsigned long long)nsd);
        const bool ok = hr < h.cap_reads && co + nch <= h.cap_ch && so + nsd <= h.cap_sd;
        if (hr < h.cap_reads) {
            h.read[hr] = ok ? r : -1;
            h.nch[hr] = nch; h.ch_off[hr] = (int32_t)co; h.sd_off[hr] = (int32_t)so;
        }
        E.misc[5] = ok ? (int32_t)hr : -1;
        E.misc[6] = (int32_t)min(co, h.cap_ch);
        E.misc[7] = (int32_t)so;
    }
    wave_sync();
    const int hr = E.misc[5], co = E.misc[6], so = E.misc[7];
    if (hr < 0) {  // chain slots of a failed reservation hold no job
        for (int i = co + lane; i < h.cap_ch && i < co + nch; i += 64) h.ch_read[i] = -1;
        return false;
    }
    GChain *hch = reinterpret_cast<GChain *>(h.ch) + co;
    GSeed *hsd = reinterpret_cast<GSeed *>(h.sd) + so;
    int base = 0;  // each chain's seeds contiguous, in chain order
    for (int i0 = 0; i0 < nch; i0 += 64) {
        const int i = i0 + lane;
        GChain c{};
        int cn = 0;
        if (i < nch) { c = S.ch2[i]; cn = c.n; }
        // exclusive prefix of the chain sizes over the 64 lanes
        int inc = cn;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int t = __shfl_up(inc, d);
            if (lane >= d) inc += t;
        }
        const int s0 = base + inc - cn;
        if (i < nch) {
            for (int k = 0; k < cn; ++k) hsd[s0 + k] = S.seed[c.seed0 + k];
            c.seed0 = s0;
            hch[i] = c;
            h.ch_read[co + i] = hr;
        }
        base += __shfl(inc, 63);
    }
    return true;
}

// G2: mem_align1_core for every read (one wave per read); a read with at least hv.min_chains
// kept chains leaves their extensions to k_g_ext_jobs and its finish to k_g_heavy
// a read's intervals iv[0, n) into (qb, qe) order, as mem_collect_intv's ks_introsort leaves them
// (equal keys are identical intervals: any order among them is bwa's); G1 pools them in collection
// order.  Lanes rank the keys in LDS (the G2 boxes, free until mem_chain); the entries move
// through tmp (n of them).
static_assert(AF_G_MAX_INTV <= 1024 && AF_MAX_READ < 512, "interval keys pack qb, qe and a 10-bit index");
__device__ void g_iv_sort(GIv *iv, int n, GIv *tmp, int lane) {
    if (n <= 1) return;
    uint32_t *key = reinterpret_cast<uint32_t *>(g_box);
    for (int i = lane; i < n; i += 64) key[i] = (uint32_t)iv[i].qb << 19 | (uint32_t)iv[i].qe << 10 | (uint32_t)i;
    __threadfence_block();
    wave_sync();
    for (int i = lane; i < n; i += 64) {
        const uint32_t x = key[i];
        int r = 0;
        for (int j = 0; j < n; ++j) r += key[j] < x;
        tmp[r] = iv[i];
    }
    __threadfence_block();
    wave_sync();
    for (int i = lane; i < n; i += 64) iv[i] = tmp[i];
    __threadfence_block();
    wave_sync();
}

template <int CPL>
__global__ __launch_bounds__(64, 2) void k_g_regions(DevGenome G, const uint8_t *__restrict__ reads, int32_t stride,
                                                     const int32_t *__restrict__ lens, const int32_t *__restrict__ n_ptr,
                                                     int64_t cap, int64_t read0, af_params p, GOpt o, GWork w,
                                                     uint8_t *__restrict__ scr_base, size_t scr_stride,
                                                     uint8_t *__restrict__ zscratch, size_t zstride) {
    const int lane = threadIdx.x;
    int64_t n = n_ptr ? (int64_t)*n_ptr : cap;
    if (n > cap) n = cap;
    const G2Scr S = g2_scr(scr_base + (size_t)blockIdx.x * scr_stride);
    uint8_t *zg = zscratch + (size_t)blockIdx.x * zstride;
    int head = (int)(blockIdx.x & 7), heads_left = 8;
    // G1's list of the reads with the most seeds first, then the others in order
    bool first = w.g2_first_occ > 0;
    const int64_t n_first = first ? (int64_t)*(volatile unsigned long long *)w.g2_list_n : 0;
    for (;;) {
        int64_t r;
        if (first) {
            int h = 0;
            if (lane == 0) h = (int)atomicAdd(w.g2_list_next, 1ull);
            h = __builtin_amdgcn_readfirstlane(h);
            if (h >= n_first) { first = false; continue; }
            r = w.g2_list[h];
        } else {
            const int it = g_next_item(w.heads, head, heads_left, n - read0, lane);
            if (it < 0) break;
            r = read0 + it;
            if (w.g2_first_occ > 0 && w.g2_flag[r]) continue;
        }
        const int l = read_len(lens, r, stride);
        const int niv = w.iv_n[r];
        int nreg = 0;
        bool ovf = niv < 0, deferred = false;
        GPROF(uint64_t gp_c[5] = {(uint64_t)clock64(), 0, 0, 0, 0}; const uint32_t gp_t0 = gp_rt(); int gp_n[4] = {0, 0, 0, 0};
              int64_t gp_occ = 0; if (niv > 0) for (int i = 0; i < niv; ++i) { const int64_t s_ = w.iv[w.iv_off[r] + i].s;
                  gp_occ += s_ > p.max_occ ? p.max_occ : s_; })
        if (!ovf && l >= p.min_seed_len && niv > 0) {
            g_load_read(reads, r, stride, l, lane);
            g_iv_sort(w.iv + w.iv_off[r], niv, reinterpret_cast<GIv *>(S.seed), lane);
            const int nch0 = g_mem_chain(G, S, w.iv + w.iv_off[r], niv, p, o, lane);
            GPROF(gp_c[1] = clock64(); gp_n[0] = nch0;)
            if (nch0 < 0) ovf = true;
            else {
                const int nch = g_chain_flt(S, nch0, p, o, lane);
                GPROF(gp_c[2] = clock64(); gp_n[1] = nch;)
                if (w.hv.min_chains > 0 && nch >= w.hv.min_chains) deferred = g_defer_heavy(w, S, r, nch, lane);
                if (!deferred) {
                    for (int ci = 0; ci < nch && !ovf; ++ci)
                        if (!g_chain2aln<CPL>(G, S, p, l, ci, &nreg, lane)) ovf = true;
                    GPROF(gp_c[3] = clock64(); gp_n[2] = nreg;)
                    if (!ovf) nreg = g_dedup_patch<CPL>(G, p, o, S.reg, nreg, true, zg, lane, reinterpret_cast<GReg *>(S.seed));
                    GPROF(gp_c[4] = clock64(); gp_n[3] = nreg;)
                }
            }
        }
        GPROF(if (lane == 0) { int32_t *g = gp_row(r); if (g) { const uint64_t ce = clock64();
              g[3] = (int32_t)(ce - gp_c[0]);
              g[4] = gp_c[1] ? (int32_t)(gp_c[1] - gp_c[0]) : 0; g[5] = gp_c[2] ? (int32_t)(gp_c[2] - gp_c[1]) : 0;
              g[6] = gp_c[3] ? (int32_t)(gp_c[3] - gp_c[2]) : 0; g[7] = gp_c[4] ? (int32_t)(gp_c[4] - gp_c[3]) : 0;
              g[8] = (int32_t)gp_occ; g[10] = gp_n[0]; g[11] = gp_n[1]; g[12] = gp_n[2]; g[13] = gp_n[3];
              g[14] = (int32_t)blockIdx.x; g[15] = (int32_t)gp_t0; g[16] = (int32_t)gp_rt(); g[2] = l;
              g[9] = deferred; g[43] = gp_c[2] ? (int32_t)g_gp_flt : 0; } })
        if (!deferred) g_put_regions(w, S, r, nreg, ovf, lane);
    }
}

// G2, heavy reads: one job per pooled chain -- the region of the chain's first seed in bwa's walk
// (the longest; ties: the last), extended whether or not the walk keeps it; k_g_heavy decides.
template <int CPL>
__global__ __launch_bounds__(64, 2) void k_g_ext_jobs(DevGenome G, const uint8_t *__restrict__ reads, int32_t stride,
                                                      const int32_t *__restrict__ lens, af_params p, GWork w) {
    const int lane = threadIdx.x;
    const GHeavy &h = w.hv;
    const int64_t n_jobs = min((int64_t)*(volatile unsigned long long *)&h.cnt[1], h.cap_ch);
    const GChain *hch = reinterpret_cast<const GChain *>(h.ch);
    const GSeed *hsd = reinterpret_cast<const GSeed *>(h.sd);
    GReg *res = reinterpret_cast<GReg *>(h.res);
    for (;;) {
        int64_t j = 0;
        if (lane == 0) j = (int64_t)atomicAdd(&h.cnt[3], 1ull);
        j = (int64_t)__builtin_amdgcn_readfirstlane((int)j);
        if (j >= n_jobs) break;
        const int hr = h.ch_read[j];
        if (hr < 0) continue;
        const int64_t r = h.read[hr];
        if (r < 0) continue;
        const GChain c = hch[j];
        const GSeed *sd = hsd + h.sd_off[hr] + c.seed0;
        const int l = read_len(lens, r, stride);
        g_load_read(reads, r, stride, l, lane);
        g_chain_rmax(G, p, l, sd, c.n, lane);
        const int64_t rmax0 = g_g2.rmax[0], rmax1 = g_g2.rmax[1];
        uint64_t best = 0;  // max of (len << 32 | i): srt's last entry
        for (int i = lane; i < c.n; i += 64) {
            const uint64_t ki = (uint64_t)(uint32_t)sd[i].len << 32 | (uint32_t)i;
            best = ki > best ? ki : best;
        }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            const uint64_t t = (uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)best, d) |
                               (uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(best >> 32), d) << 32;
            best = t > best ? t : best;
        }
        const GReg a = g_seed_region<CPL>(G, p, l, sd, c.n, c.rid, sd[(uint32_t)best], rmax0, rmax1, lane);
        if (lane == 0) res[h.sd_off[hr] + c.seed0] = a;
        wave_sync();
    }
}

// G2, heavy reads: bwa's walk over the kept chains with the jobs' regions, dedup / patch, the
// read's regions into the pool
template <int CPL>
__global__ __launch_bounds__(64, 2) void k_g_heavy(DevGenome G, const uint8_t *__restrict__ reads, int32_t stride,
                                                   const int32_t *__restrict__ lens, af_params p, GOpt o, GWork w,
                                                   uint8_t *__restrict__ scr_base, size_t scr_stride,
                                                   uint8_t *__restrict__ zscratch, size_t zstride) {
    const int lane = threadIdx.x;
    const GHeavy &h = w.hv;
    const int64_t n_heavy = min((int64_t)*(volatile unsigned long long *)&h.cnt[0], h.cap_reads);
    const G2Scr S = g2_scr(scr_base + (size_t)blockIdx.x * scr_stride);
    uint8_t *zg = zscratch + (size_t)blockIdx.x * zstride;
    const GChain *hch = reinterpret_cast<const GChain *>(h.ch);
    const GSeed *hsd = reinterpret_cast<const GSeed *>(h.sd);
    const GReg *res = reinterpret_cast<const GReg *>(h.res);
    for (;;) {
        int64_t hr = 0;
        if (lane == 0) hr = (int64_t)atomicAdd(&h.cnt[4], 1ull);
        hr = (int64_t)__builtin_amdgcn_readfirstlane((int)hr);
        if (hr >= n_heavy) break;
        const int64_t r = h.read[hr];
        if (r < 0) continue;
        GPROF(const uint64_t gp_c0 = clock64(); const uint32_t gp_t0 = gp_rt();)
        const int nch = h.nch[hr], co = h.ch_off[hr], so = h.sd_off[hr];
        int nsd = 0;
        for (int i = lane; i < nch; i += 64) {
            const GChain c = hch[co + i];
            S.ch2[i] = c;
            nsd = max(nsd, c.seed0 + c.n);
        }
        nsd = wave_max(nsd);
        for (int k = lane; k < nsd; k += 64) S.seed[k] = hsd[so + k];
        wave_sync();
        const int l = read_len(lens, r, stride);
        g_load_read(reads, r, stride, l, lane);
        int nreg = 0;
        bool ovf = false;
        for (int ci = 0; ci < nch && !ovf; ++ci)
            if (!g_chain2aln<CPL>(G, S, p, l, ci, &nreg, lane, res + so)) ovf = true;
        GPROF(const uint64_t gp_c1 = clock64();)
        if (!ovf) nreg = g_dedup_patch<CPL>(G, p, o, S.reg, nreg, true, zg, lane, reinterpret_cast<GReg *>(S.seed));
        GPROF(if (lane == 0) { int32_t *g = gp_row(r); if (g) { g[6] = (int32_t)(gp_c1 - gp_c0);
              g[7] = (int32_t)(clock64() - gp_c1); g[12] = nreg; g[13] = nreg;
              g[40] = (int32_t)gp_t0; g[41] = (int32_t)gp_rt(); g[42] = (int32_t)blockIdx.x; } })
        g_put_regions(w, S, r, nreg, ovf, lane);
    }
}

// ==================================================================== records
// mem_mark_primary_se (oracle mark_primary_se) on the wave: the sort through keys in LDS, then lane 0's walk over the
// regions' query spans, scores and subs in LDS (the boxes' space); tmp: n regions of scratch
__device__ void g_mark_primary_w(GReg *a, int n, int64_t id, GReg *tmp, int lane) {
    if (n == 0) return;
    GKey16 *k = reinterpret_cast<GKey16 *>(g_box);
    for (int i = lane; i < n; i += 64) {
        const uint64_t h = hash_64((uint64_t)(id + i));
        a[i].sub = 0; a[i].secondary = -1; a[i].hash = h;
        k[i] = GKey16{(int64_t)h, a[i].score, i};
    }
    wave_sync();
    if (n < G_RANK_MIN || !wave_rank_sort(k, n, GKeyHash(), reinterpret_cast<GKey16 *>(tmp), lane)) {
        if (lane == 0) ks_introsort(k, n, GKeyHash());
        wave_sync();
    }
    g_regs_gather(a, tmp, n, [&](int j) { return k[j].z; }, lane);
    int32_t *span = reinterpret_cast<int32_t *>(g_box);  // qb << 16 | qe
    int32_t *score = span + AF_G_MAX_REG, *sub = score + AF_G_MAX_REG, *z = sub + AF_G_MAX_REG;
    for (int i = lane; i < n; i += 64) { span[i] = a[i].qb << 16 | a[i].qe; score[i] = a[i].score; sub[i] = 0; }
    wave_sync();
    if (lane == 0) {
        int nz = 0;
        z[nz++] = 0;
        for (int i = 1; i < n; ++i) {
            const int qbi = span[i] >> 16, qei = span[i] & 0xffff;
            int kk;
            for (kk = 0; kk < nz; ++kk) {
                const int j = z[kk];
                const int qbj = span[j] >> 16, qej = span[j] & 0xffff;
                const int b_max = qbj > qbi ? qbj : qbi;
                const int e_min = qej < qei ? qej : qei;
                if (e_min > b_max) {
                    const int min_l = qei - qbi < qej - qbj ? qei - qbi : qej - qbj;
                    if ((float)(e_min - b_max) >= (float)min_l * 0.5f) {
                        if (sub[j] == 0) sub[j] = score[i];
                        break;
                    }
                }
            }
            if (kk == nz) z[nz++] = i;
            else a[i].secondary = z[kk];
        }
    }
    wave_sync();
    for (int i = lane; i < n; i += 64) a[i].sub = sub[i];
    wave_sync();
}

// one mem_aln_t (oracle aln_t)
struct GAln { int rid; int64_t pos; int is_rev, flag, score, n_cigar, of; uint32_t cigar[AF_MAX_CIGAR]; };

// mem_reg2aln (oracle reg2aln) on the wave; the read's codes in L.q; result on lane 0
template <int CPL>
__device__ void g_reg2aln(const DevGenome &G, const af_params &p, int l, const GReg *ar, GAln &o, uint8_t *zg,
                          int lane) {
    DpLds &L = g_dp;
    const int64_t l_pac = G.l_pac;
    o.flag = 0; o.n_cigar = 0; o.of = 0; o.score = 0; o.is_rev = 0;
    if (!ar || ar->rb < 0 || ar->re < 0) { o.rid = -1; o.pos = -1; o.flag = 0x4; return; }
    const GReg a = *ar;
    if (a.secondary >= 0) o.flag |= 0x100;
    const int lq = a.qe - a.qb;
    const int tmpw = infer_bw(lq, (int)(a.re - a.rb), a.truesc, p.a, p.o_del, p.e_del);
    int w2 = infer_bw(lq, (int)(a.re - a.rb), a.truesc, p.a, p.o_ins, p.e_ins);
    w2 = w2 > tmpw ? w2 : tmpw;
    if (w2 > p.w) w2 = w2 < a.w ? w2 : a.w;
    int score = 0, last_sc = -(1 << 30), it = 0;
    do {
        w2 = w2 < p.w << 2 ? w2 : p.w << 2;
        score = gen_cigar_wave<CPL>(G.T, l_pac, p, w2, lq, a.qb, a.rb, a.re, L, zg, lane);
        if (score == last_sc || w2 == p.w << 2) break;
        last_sc = score;
        w2 <<= 1;
    } while (++it < 3 && score < a.truesc - p.a);
    (void)score;
    if (lane == 0) {
        const int nc = L.misc[2];
        const int ncap = nc < AF_MAX_CIGAR ? nc : AF_MAX_CIGAR;
        bool of = nc > AF_MAX_CIGAR;
        int is_rev;
        int64_t pos = g_depos(G, a.rb < l_pac ? a.rb : a.re - 1, &is_rev);
        int xs = 0, xe = ncap;
        const uint32_t first = L.ring[(nc - 1) & 63];
        const uint32_t last = L.ring[(nc - ncap) & 63];
        if (ncap > 0) {
            if ((first & 0xf) == 2) { pos += first >> 4; xs = 1; }
            else if ((last & 0xf) == 2) xe = ncap - 1;
        }
        const int clip5 = is_rev ? l - a.qe : a.qb;
        const int clip3 = is_rev ? a.qb : l - a.qe;
        int nf = 0;
        if (clip5) o.cigar[nf++] = (uint32_t)clip5 << 4 | 4;
        for (int x = xs; x < xe; ++x) {
            if (nf < AF_MAX_CIGAR) o.cigar[nf] = L.ring[(nc - 1 - x) & 63];
            ++nf;
        }
        if (clip3) {
            if (nf < AF_MAX_CIGAR) o.cigar[nf] = (uint32_t)clip3 << 4 | 4;
            ++nf;
        }
        if (nf > AF_MAX_CIGAR) { of = true; nf = AF_MAX_CIGAR; }
        o.n_cigar = nf;
        o.of = of;
        o.rid = g_pos2rid(G, pos);
        o.pos = pos - G.ctg_off_d[o.rid];
        o.is_rev = is_rev;
        o.score = a.score;
    }
}

// mem_aln2sam (oracle aln2grec), lane 0: record `which` of a read, mate m (nullptr: single-end)
__device__ void g_aln2rec(const GAln &p_, const GAln *m_, int which, int l_seq, int32_t read, af_grec &o) {
    GAln p = p_, m{};
    if (m_) m = *m_;
    p.flag |= m_ ? 0x1 : 0;
    p.flag |= p.rid < 0 ? 0x4 : 0;
    p.flag |= m_ && m.rid < 0 ? 0x8 : 0;
    if (p.rid < 0 && m_ && m.rid >= 0) { p.rid = m.rid; p.pos = m.pos; p.is_rev = m.is_rev; p.n_cigar = 0; }
    if (m_ && m.rid < 0 && p.rid >= 0) { m.rid = p.rid; m.pos = p.pos; m.is_rev = p.is_rev; m.n_cigar = 0; }
    p.flag |= p.is_rev ? 0x10 : 0;
    p.flag |= m_ && m.is_rev ? 0x20 : 0;
    o.read = read;
    o.flag = (p.flag & 0xffff) | ((p.flag & 0x10000) ? 0x100 : 0) | (p_.of ? AF_FLAG_CIGAR_OVERFLOW : 0);
    o.rid = p.rid;
    o.pos = p.rid >= 0 ? p.pos : -1;
    o.score = p.rid >= 0 && p_.rid >= 0 ? p.score : 0;
    o.n_cigar = p.n_cigar;
    for (int c = 0; c < AF_MAX_CIGAR; ++c) {
        uint32_t v = 0;
        if (c < p.n_cigar) {
            uint32_t op = p.cigar[c] & 0xf;
            if (op == 4 && which) op = 5;
            v = (p.cigar[c] & ~0xfu) | op;
        }
        o.cigar[c] = v;
    }
    o.mrid = m_ && m.rid >= 0 ? m.rid : -1;
    o.mpos = m_ && m.rid >= 0 ? m.pos : -1;
    o.seq_b = 0; o.seq_e = l_seq;
    if (p.n_cigar && which) {
        if ((p.cigar[0] & 0xf) == 4) o.seq_b = (int32_t)(p.cigar[0] >> 4);
        if ((p.cigar[p.n_cigar - 1] & 0xf) == 4) o.seq_e = l_seq - (int32_t)(p.cigar[p.n_cigar - 1] >> 4);
    }
}

struct G3Lds {
    GAln al;              // the record being built
    GAln mate[2];         // mem_sam_pe's h[]
    int32_t misc[8];
};
__shared__ G3Lds g_g3;

// mem_reg2sam (-M): records of one read from its marked regions a[0, n); returns the record
// count (more than AF_G_MAX_REC: the read is flagged by the caller)
template <int CPL>
__device__ int g_reg2sam(const DevGenome &G, const af_params &p, int l, const GReg *a, int n, int extra_flag,
                         const GAln *m, int32_t read, af_grec *out, uint8_t *zg, int lane) {
    G3Lds &E = g_g3;
    int na = 0;
    for (int k = 0; k < n; ++k) {
        if (a[k].score < p.T || a[k].secondary >= 0) continue;
        if (na < AF_G_MAX_REC) {
            g_reg2aln<CPL>(G, p, l, &a[k], E.al, zg, lane);
            if (lane == 0) {
                E.al.flag |= extra_flag;
                if (na) E.al.flag |= 0x10000;  // -M: supplementary -> 0x100
                g_aln2rec(E.al, m, na, l, read, out[na]);
            }
            wave_sync();
        }
        ++na;
    }
    if (na == 0) {
        if (lane == 0) {
            GAln t;
            t.rid = -1; t.pos = -1; t.flag = 0x4 | extra_flag; t.n_cigar = 0; t.of = 0; t.score = 0; t.is_rev = 0;
            g_aln2rec(t, m, 0, l, read, out[0]);
        }
        wave_sync();
        return 1;
    }
    return na;
}

// G3: S5 records (one wave per read): mark_primary_se + mem_reg2sam
template <int CPL>
__global__ __launch_bounds__(64, 2) void k_g_se(DevGenome G, const uint8_t *__restrict__ reads, int32_t stride,
                                                const int32_t *__restrict__ lens, const int32_t *__restrict__ n_ptr,
                                                int64_t cap, af_params p, int64_t id_base,
                                                const int64_t *__restrict__ ids, GWork w,
                                                uint8_t *__restrict__ scr_base, size_t scr_stride,
                                                uint8_t *__restrict__ zscratch, size_t zstride,
                                                af_grec *__restrict__ recs, int32_t *__restrict__ n_rec) {
    const int lane = threadIdx.x;
    int64_t n = n_ptr ? (int64_t)*n_ptr : cap;
    if (n > cap) n = cap;
    const G2Scr S = g2_scr(scr_base + (size_t)blockIdx.x * scr_stride);
    uint8_t *zg = zscratch + (size_t)blockIdx.x * zstride;
    for (;;) {  // reads dequeued one at a time (their costs vary by orders of magnitude)
        int64_t r = 0;
        if (lane == 0) r = (int64_t)atomicAdd(&w.hv.cnt[6], 1ull);
        r = (int64_t)__builtin_amdgcn_readfirstlane((int)r);
        if (r >= n) break;
        const int l = read_len(lens, r, stride);
        const int nr = w.reg_n[r];
        const bool ovf = nr < 0;
        const int na = ovf ? 0 : nr;
        for (int k = lane; k < na; k += 64) S.reg[k] = w.reg[w.reg_off[r] + k];
        wave_sync();
        g_mark_primary_w(S.reg, na, ids ? ids[r] : id_base + r, reinterpret_cast<GReg *>(S.seed), lane);
        g_load_read(reads, r, stride, l, lane);
        af_grec *out = recs + r * AF_G_MAX_REC;
        const int nrec = g_reg2sam<CPL>(G, p, l, S.reg, na, 0, nullptr, (int32_t)r, out, zg, lane);
        if (lane == 0) {
            n_rec[r] = nrec;
            if (ovf || nrec > AF_G_MAX_REC) {
                for (int j = 0; j < (nrec < AF_G_MAX_REC ? nrec : AF_G_MAX_REC); ++j) out[j].flag |= AF_FLAG_MEM_OVERFLOW;
                if (nrec > AF_G_MAX_REC) atomicAdd(&w.stats[AF_GSTAT_RECS], 1);
            }
        }
        wave_sync();
    }
}

// ==================================================================== paired end (S4)
__device__ __forceinline__ int g_infer_dir(int64_t l_pac, int64_t b1, int64_t b2, int64_t *dist) {
    const int r1 = b1 >= l_pac, r2 = b2 >= l_pac;
    const int64_t p2 = r1 == r2 ? b2 : (l_pac << 1) - 1 - b2;
    *dist = p2 > b1 ? p2 - b1 : b1 - p2;
    return (r1 == r2 ? 0 : 1) ^ (p2 > b1 ? 0 : 3);
}
__device__ int g_cal_sub(const GReg *a, int n, int msl, int asc) {
    int j;
    for (j = 1; j < n; ++j) {
        const int b_max = a[j].qb > a[0].qb ? a[j].qb : a[0].qb;
        const int e_min = a[j].qe < a[0].qe ? a[j].qe : a[0].qe;
        if (e_min > b_max) {
            const int min_l = a[j].qe - a[j].qb < a[0].qe - a[0].qb ? a[j].qe - a[j].qb : a[0].qe - a[0].qb;
            if ((float)(e_min - b_max) >= (float)min_l * 0.5f) break;
        }
    }
    return j < n ? a[j].score : msl * asc;
}
__device__ __forceinline__ int g_chunk_of(const S2Work &w, int64_t pp) {
    int lo = 0, hi = *w.n_chunks;  // cstart[lo] <= pp < cstart[hi]
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (w.cstart[mid] <= pp) lo = mid;
        else hi = mid;
    }
    return lo;
}

// mem_pestat's insert sizes (one lane per pair) into the chunks' histograms
__global__ void k_g_pe_hist(const int32_t *__restrict__ n_pairs_ptr, int64_t cap, int64_t l_pac, af_params p, GOpt o,
                            GWork w, S2Work sw) {
    int64_t n = n_pairs_ptr ? (int64_t)*n_pairs_ptr : cap;
    if (n > cap) n = cap;
    for (int64_t pp = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; pp < n; pp += (int64_t)gridDim.x * blockDim.x) {
        const int n0 = w.reg_n[2 * pp], n1 = w.reg_n[2 * pp + 1];
        if (n0 <= 0 || n1 <= 0) continue;
        const GReg *a0 = w.reg + w.reg_off[2 * pp], *a1 = w.reg + w.reg_off[2 * pp + 1];
        if ((double)g_cal_sub(a0, n0, p.min_seed_len, p.a) > 0.8 * a0[0].score) continue;
        if ((double)g_cal_sub(a1, n1, p.min_seed_len, p.a) > 0.8 * a1[0].score) continue;
        if (a0[0].rid != a1[0].rid) continue;
        int64_t is;
        const int dir = g_infer_dir(l_pac, a0[0].rb, a1[0].rb, &is);
        if (is && is <= o.max_ins) {
            const int c = g_chunk_of(sw, pp);
            atomicAdd(&sw.ghist[((int64_t)c * 4 + dir) * (o.max_ins + 1) + is], 1);
        }
    }
}

struct GPeLds {
    S2Pes pes[4];
    uint8_t q[2][AF_MAX_READ + 16];
    uint8_t rq[AF_MAX_READ + 16];
    uint8_t rq2[AF_MAX_READ + 16];
    uint8_t tw[2048];
    int32_t na[2], nb[2], ovf[2], len[2], misc[8];
};
__shared__ GPeLds g_gpe;

// ksw_align2 with KSW_XSUBO | KSW_XSTART (oracle ksw_align2)
__device__ void g_ksw_align2(const uint8_t *q, int qlen, const uint8_t *target, int tlen, int P, int minsc,
                             const af_params &p, int &score, int &te, int &qe, int &tb, int &qb, int lane) {
    GPeLds &E = g_gpe;
    const SwRes r = ksw_pass_any(q, qlen, target, tlen, -1, P, p, 0x10000, lane);
    score = r.score; te = r.te; qe = r.qe; tb = -1; qb = -1;
    if (r.score < minsc || r.qe < 0) return;
    for (int x = lane; x <= r.qe; x += 64) E.rq2[x] = q[r.qe - x];
    wave_sync();
    const SwRes rr = ksw_pass_any(E.rq2, r.qe + 1, target, tlen, r.te, P, p, r.score, lane);
    wave_sync();
    if (r.score == rr.score) { tb = r.te - rr.te; qb = r.qe - rr.qe; }
}

// mem_matesw's window of direction r for the mate region a (the rescued read l_ms long): [rb, re)
// clipped to one contig (rid); true when bwa runs its SW there
__device__ __forceinline__ bool g_mate_window(const DevGenome &G, const af_params &p, const S2Pes &pe, int r,
                                              const GReg &a, int l_ms, int64_t &rb, int64_t &re, int &rid) {
    const int64_t l_pac = G.l_pac;
    const bool is_rev = (r >> 1) != (r & 1);
    const bool is_larger = !(r >> 1);
    if (!is_rev) {
        rb = is_larger ? a.rb + pe.low : a.rb - pe.high;
        re = (is_larger ? a.rb + pe.high : a.rb - pe.low) + l_ms;
    } else {
        rb = (is_larger ? a.rb + pe.low : a.rb - pe.high) - l_ms;
        re = is_larger ? a.rb + pe.high : a.rb - pe.low;
    }
    if (rb < 0) rb = 0;
    if (re > l_pac << 1) re = l_pac << 1;
    if (rb < re) g_fetch_clip(G, &rb, (rb + re) >> 1, &re, &rid);
    // (rb >= re leaves rid from the previous direction, as bwa does; re - rb < min_seed_len then)
    return a.rid == rid && re - rb >= p.min_seed_len;
}

// that window's ksw_align2 for the rescued read's codes qc (strand of direction r)
__device__ __forceinline__ void g_mate_ksw(const DevGenome &G, const af_params &p, const uint8_t *qc, int l_ms, int r,
                                           int64_t rb, int64_t re, int &sc, int &te, int &qe, int &tb, int &qb,
                                           int lane) {
    GPeLds &E = g_gpe;
    const bool is_rev = (r >> 1) != (r & 1);
    for (int x = lane; x < l_ms; x += 64) {
        const int c = qc[is_rev ? l_ms - 1 - x : x];
        E.rq[x] = (uint8_t)(is_rev ? (c < 4 ? 3 - c : 4) : c);
    }
    const bool staged = re - rb <= (int64_t)sizeof(E.tw);
    if (staged)
        for (int x = lane; x < (int)(re - rb); x += 64) E.tw[x] = G.T[rb + x];
    wave_sync();
    const int P = l_ms * p.a < 250 ? 16 : 8;
    g_ksw_align2(E.rq, l_ms, staged ? E.tw : G.T + rb, (int)(re - rb), P, p.min_seed_len * p.a, p, sc, te, qe, tb, qb,
                 lane);
}

// mem_matesw (oracle mem_matesw): rescue read mi (regions ma[0, *na)) in the insert-size window
// of its mate's region a.  sr: the windows' SW results computed ahead (k_g_pe_jobs; 4 directions
// x AF_G_PE_RES_W ints) or null.  Returns false on a region-cap overflow.
__device__ bool g_matesw(const DevGenome &G, const af_params &p, const GOpt &o, const G2Scr &S, int mi, GReg *ma,
                         const GReg &a, uint8_t *zg, const int32_t *sr, int lane) {
    GPeLds &E = g_gpe;
    const int64_t l_pac = G.l_pac;
    const int l_ms = E.len[mi];
    int skip[4];
    for (int r = 0; r < 4; ++r) skip[r] = E.pes[r].failed ? 1 : 0;
    {  // a direction is skipped when some region already pairs with a in it: lanes over the regions
        int bits = 0;
        const int na0 = E.na[mi];
        for (int i = lane; i < na0; i += 64) {
            int64_t dist;
            const int r = g_infer_dir(l_pac, a.rb, ma[i].rb, &dist);
            if (dist >= E.pes[r].low && dist <= E.pes[r].high) bits |= 1 << r;
        }
        for (int r = 0; r < 4; ++r)
            if (__ballot((bits >> r) & 1)) skip[r] = 1;
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
        if (g_mate_window(G, p, E.pes[r], r, a, l_ms, rb, re, rid)) {
            int sc, te, qe, tb, qb;
            const int32_t *q = sr ? sr + r * AF_G_PE_RES_W : nullptr;
            if (q && q[5]) {
                sc = q[0]; te = q[1]; qe = q[2]; tb = q[3]; qb = q[4];
            } else {
                GPROF(if (lane == 0) ++E.misc[5];)
                g_mate_ksw(G, p, E.q[mi], l_ms, r, rb, re, sc, te, qe, tb, qb, lane);
            }
            if (sc >= p.min_seed_len && qb >= 0) {
                // the rescued region into the list, before the first region of a lower score (found
                // by ballots; the tail moves up one slot a lane per region, top chunk first)
                const int na = E.na[mi];
                if (na >= AF_G_MAX_REG) return false;
                int at = na;
                for (int i0 = 0; i0 < na; i0 += 64) {
                    const int i = i0 + lane;
                    const uint64_t m = __ballot(i < na && ma[i].score < sc);
                    if (m) { at = i0 + (int)__builtin_ctzll(m); break; }
                }
                for (int top = na - 1; top >= at; top -= 64) {
                    const int e = top - lane;
                    GReg x;
                    if (e >= at) x = ma[e];
                    __threadfence_block();
                    wave_sync();
                    if (e >= at) ma[e + 1] = x;
                    __threadfence_block();
                    wave_sync();
                }
                if (lane == 0) {
                    GReg b{};
                    b.rid = a.rid;
                    b.qb = is_rev ? l_ms - (qe + 1) : qb;
                    b.qe = is_rev ? l_ms - qb : qe + 1;
                    b.rb = is_rev ? (l_pac << 1) - (rb + te + 1) : rb + tb;
                    b.re = is_rev ? (l_pac << 1) - (rb + tb) : rb + te + 1;
                    b.score = sc;
                    b.secondary = -1;
                    b.seedcov = (int)((b.re - b.rb < b.qe - b.qb ? b.re - b.rb : b.qe - b.qb) >> 1);
                    ma[at] = b;
                    E.na[mi] = na + 1;
                }
                __threadfence_block();
                wave_sync();
                dirty = true;
            }
            ++n;
        }
        if (n && (!deduped || dirty)) {
            deduped = true;
            dirty = false;
            GPROF(const uint64_t gp_d0 = clock64();)
            const int m = g_dedup_patch<2>(G, p, o, ma, E.na[mi], false, zg, lane, reinterpret_cast<GReg *>(S.seed));
            if (lane == 0) E.na[mi] = m;
            GPROF(if (lane == 0) E.misc[6] += (int32_t)(clock64() - gp_d0);)
            wave_sync();
        }
    }
    return true;
}

struct P64g { uint64_t x, y; };
static_assert(sizeof(G2Box) * G2_BOXES >= sizeof(P64g) * AF_G_MAX_REG, "the boxes hold mem_pair's keys");
struct GLtP64 {
    __device__ bool operator()(const P64g &a, const P64g &b) const { return a.x < b.x || (a.x == b.x && a.y < b.y); }
};

// mem_pair (oracle mem_pair), lane 0: the best pair's score (0 if none) and z[]
__device__ int g_mem_pair(const DevGenome &G, const af_params &p, const S2Pes *pes, GReg *a0, int n0, GReg *a1, int n1,
                          int id, int z[2], P64g *v) {
    const int64_t l_pac = G.l_pac;
    int nv = 0;
    GReg *aa[2] = {a0, a1};
    const int nn[2] = {n0, n1};
    for (int r = 0; r < 2; ++r)
        for (int i = 0; i < nn[r]; ++i) {
            const GReg &e = aa[r][i];
            P64g key;
            const int64_t x = e.rb < l_pac ? e.rb : (l_pac << 1) - 1 - e.rb;
            key.x = (uint64_t)e.rid << 32 | (uint64_t)(x - G.ctg_off_d[e.rid]);
            key.y = (uint64_t)(uint32_t)e.score << 32 | (uint64_t)i << 2 | (uint64_t)(e.rb >= l_pac) << 1 | (uint64_t)r;
            v[nv++] = key;
        }
    ks_introsort(v, nv, GLtP64());
    int y[4] = {-1, -1, -1, -1};
    bool have = false;
    P64g best{0, 0};
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
                P64g u;
                u.y = (uint64_t)k << 32 | (uint64_t)i;
                u.x = (uint64_t)q << 32 | (hash_64(u.y ^ (uint64_t)(int64_t)(int32_t)((uint32_t)id << 8)) & 0xffffffffU);
                if (!have || GLtP64()(best, u)) { best = u; have = true; }
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

// mem_pair on the wave for long region lists (the same result as g_mem_pair: its keys are unique,
// so the rank sort gives klib's order, and the best pair is the maximum of keys that name their two
// entries, so it does not depend on the scan order).  Lanes build the keys; the scan keeps bwa's
// order over i, with lanes over the earlier entries k of the wanted kind, 64 at a time from y[which]
// down, stopping at the first (highest) k past the insert-size window as bwa's break does.  Every
// lane returns the score (0: none) and z.
__device__ int g_mem_pair_w(const DevGenome &G, const af_params &p, const S2Pes *pes, const GReg *a0, int n0,
                            const GReg *a1, int n1, int id, int z[2], P64g *v, P64g *tmp, int lane) {
    const int64_t l_pac = G.l_pac;
    const int nv = n0 + n1;
    for (int t = lane; t < nv; t += 64) {
        const int r = t >= n0, i = t - (r ? n0 : 0);
        const GReg &e = r ? a1[i] : a0[i];
        const int64_t x = e.rb < l_pac ? e.rb : (l_pac << 1) - 1 - e.rb;
        P64g key;
        key.x = (uint64_t)e.rid << 32 | (uint64_t)(x - G.ctg_off_d[e.rid]);
        key.y = (uint64_t)(uint32_t)e.score << 32 | (uint64_t)i << 2 | (uint64_t)(e.rb >= l_pac) << 1 | (uint64_t)r;
        v[t] = key;
    }
    __threadfence_block();
    wave_sync();
    if (!wave_rank_sort(v, nv, GLtP64(), tmp, lane)) {  // (keys name their entry: never taken)
        if (lane == 0) ks_introsort(v, nv, GLtP64());
        __threadfence_block();
        wave_sync();
    }
    int y[4] = {-1, -1, -1, -1};
    bool have = false;
    P64g best{0, 0};
    for (int i = 0; i < nv; ++i) {
        const P64g vi = v[i];
        for (int r = 0; r < 2; ++r) {
            const int dir = r << 1 | (int)(vi.y >> 1 & 1);
            if (pes[dir].failed) continue;
            const int which = r << 1 | (int)((vi.y & 1) ^ 1);
            if (y[which] < 0) continue;
            const int64_t lo = pes[dir].low, hi = pes[dir].high;
            for (int k0 = y[which]; k0 >= 0; k0 -= 64) {
                const int k = k0 - lane;
                bool valid = false, brk = false;
                int64_t dist = 0;
                P64g vk{0, 0};
                if (k >= 0) {
                    vk = v[k];
                    valid = (int)(vk.y & 3) == which;
                    dist = (int64_t)vi.x - (int64_t)vk.x;
                    brk = valid && dist > hi;
                }
                const uint64_t bm = __ballot(brk);
                const int first = bm ? (int)__builtin_ctzll(bm) : 64;  // lanes below it precede bwa's break
                if (valid && lane < first && dist >= lo) {
                    const double ns = ((double)dist - pes[dir].avg) / pes[dir].std;
                    int q = (int)((double)((vi.y >> 32) + (vk.y >> 32)) + .721 * log(2. * erfc(fabs(ns) * 0.70710678118654752440)) * p.a + .499);
                    if (q < 0) q = 0;
                    P64g u;
                    u.y = (uint64_t)k << 32 | (uint64_t)i;
                    u.x = (uint64_t)q << 32 | (hash_64(u.y ^ (uint64_t)(int64_t)(int32_t)((uint32_t)id << 8)) & 0xffffffffU);
                    if (!have || GLtP64()(best, u)) { best = u; have = true; }
                }
                if (bm) break;
            }
        }
        y[vi.y & 3] = i;
    }
    // the lanes' best to lane 0 through tmp (its sort copy is dead)
    tmp[lane] = have ? best : P64g{0, 0};
    reinterpret_cast<uint8_t *>(tmp + 64)[lane] = have ? 1 : 0;
    __threadfence_block();
    wave_sync();
    int res = 0;
    if (lane == 0) {
        bool any = false;
        P64g b{0, 0};
        for (int l = 0; l < 64; ++l)
            if (reinterpret_cast<const uint8_t *>(tmp + 64)[l] && (!any || GLtP64()(b, tmp[l]))) { b = tmp[l]; any = true; }
        if (any) {
            const int i = (int)(b.y >> 32), k = (int)(b.y << 32 >> 32);
            z[v[i].y & 1] = (int)(v[i].y << 32 >> 34);
            z[v[k].y & 1] = (int)(v[k].y << 32 >> 34);
            res = (int)(b.x >> 32);
        }
        tmp[0].x = (uint64_t)(uint32_t)res | (uint64_t)(uint32_t)z[0] << 32;
        tmp[0].y = (uint64_t)(uint32_t)z[1];
    }
    __threadfence_block();
    wave_sync();
    const P64g o = tmp[0];
    z[0] = (int)(o.x >> 32); z[1] = (int)(uint32_t)o.y;
    res = (int)(uint32_t)o.x;
    wave_sync();
    return res;
}

// G4: mem_sam_pe for every pair (one wave per pair); records of read 2pp + m at
// recs[(2 pp + m) * AF_G_MAX_REC ..], counts n_rec[2 pp + m]
template <int CPL>
__global__ __launch_bounds__(64, 2) void k_g_pe(DevGenome G, const uint8_t *__restrict__ reads, int32_t stride,
                                                const int32_t *__restrict__ lens, const int32_t *__restrict__ n_pairs_ptr,
                                                int64_t cap, af_params p, GOpt o, GWork w, S2Work sw,
                                                uint8_t *__restrict__ scr_base, size_t scr_stride,
                                                uint8_t *__restrict__ zscratch, size_t zstride,
                                                af_grec *__restrict__ recs, int32_t *__restrict__ n_rec, int mode) {
    GPeLds &E = g_gpe;
    G3Lds &H = g_g3;
    const int lane = threadIdx.x;
    int64_t n = n_pairs_ptr ? (int64_t)*n_pairs_ptr : cap;
    if (n > cap) n = cap;
    const G2Scr S = g2_scr(scr_base + (size_t)blockIdx.x * scr_stride);
    uint8_t *zg = zscratch + (size_t)blockIdx.x * zstride;
    // region lists of both ends (and the rescue copies) in the wave's scratch
    GReg *A[2] = {S.reg, reinterpret_cast<GReg *>(S.pool)};
    GReg *B = reinterpret_cast<GReg *>(S.ch);
    P64g *V = reinterpret_cast<P64g *>(S.seed);
    static_assert((size_t)AF_G_MAX_OCC * sizeof(GSeed) >= (size_t)(AF_G_MAX_REG + 1) * sizeof(GReg), "pool holds a region list");
    static_assert((size_t)AF_G_MAX_CHAIN * sizeof(GChain) >= 2 * (size_t)(AF_G_MAX_REG + 1) * sizeof(GReg), "ch holds 2 lists");
    static_assert((size_t)AF_G_MAX_OCC * sizeof(GSeed) >= 2 * (size_t)(AF_G_MAX_REG + 4) * sizeof(P64g), "seed holds v");
    // mode 0: every pair; 1: every pair, those with at least w.pe.min_windows rescue windows left
    // to k_g_pe_jobs (their SWs) and mode 2 (the rest, with those SWs' results)
    const GPeSpec &X = w.pe;
    int64_t nh = 0;
    if (mode == 2) {
        nh = (int64_t)X.cnt[0];
        if (nh > X.cap_pairs) nh = X.cap_pairs;
    }
    for (;;) {  // pairs dequeued one at a time (a pair with many rescue windows costs many others)
        int64_t pp = 0;
        const int32_t *sres = nullptr;  // mode 2: the pair's precomputed SW results
        int nj0 = 0;
        if (mode == 2) {
            int64_t hp = 0;
            if (lane == 0) hp = (int64_t)atomicAdd(&X.cnt[3], 1ull);
            hp = (int64_t)__builtin_amdgcn_readfirstlane((int)hp);
            if (hp >= nh) break;
            pp = X.pair[hp];
            if (pp < 0) continue;  // reservation failed: mode 1 finished the pair
            sres = X.res + (int64_t)X.off[hp] * 4 * AF_G_PE_RES_W;
            nj0 = X.nj[hp] & 0xffff;
        } else {
            if (lane == 0) pp = (int64_t)atomicAdd(&w.hv.cnt[5], 1ull);
            pp = (int64_t)__builtin_amdgcn_readfirstlane((int)pp);
            if (pp >= n) break;
        }
        GPROF(const uint64_t gp_c0 = clock64(); const uint32_t gp_t0 = gp_rt();
              if (lane == 0) { E.misc[5] = 0; E.misc[6] = 0; })
        for (int m = 0; m < 2; ++m) {
            const int64_t r = 2 * pp + m;
            const int l = read_len(lens, r, stride);
            const uint8_t *rd = reads + r * (int64_t)stride;
            for (int x = lane; x < l; x += 64) E.q[m][x] = nt4(rd[x]);
            const int nr = w.reg_n[r];
            const int na = nr > 0 ? nr : 0;
            for (int k = lane; k < na; k += 64) A[m][k] = w.reg[w.reg_off[r] + k];
            if (lane == 0) { E.len[m] = l; E.na[m] = na; E.ovf[m] = nr < 0; }
        }
        if (lane < 4) E.pes[lane] = sw.pes[(int64_t)g_chunk_of(sw, pp) * 4 + lane];
        wave_sync();
        // mate rescue for the top hits of each end (copies taken before any rescue)
        if (lane == 0) {
            for (int i = 0; i < 2; ++i) {
                int nb = 0;
                for (int j = 0; j < E.na[i]; ++j)
                    if (A[i][j].score >= A[i][0].score - o.pen_unpaired) B[i * (AF_G_MAX_REG + 1) + nb++] = A[i][j];
                E.nb[i] = nb;
            }
        }
        wave_sync();
        if (mode == 1 && X.min_windows > 0) {
            // a heavy pair's windows to the job list (slot k: end i, its j-th top hit); the
            // pair is finished by mode 2
            const int n0 = E.nb[0] < o.max_matesw ? E.nb[0] : o.max_matesw;
            const int n1 = E.nb[1] < o.max_matesw ? E.nb[1] : o.max_matesw;
            const int nwin = (E.ovf[1] ? 0 : n0) + (E.ovf[0] ? 0 : n1);
            if (nwin >= X.min_windows) {
                int hp = -1, off = 0;
                if (lane == 0) {
                    const int64_t h = (int64_t)atomicAdd(&X.cnt[0], 1ull);
                    if (h < X.cap_pairs) {
                        const int64_t o0 = (int64_t)atomicAdd(&X.cnt[1], (unsigned long long)(n0 + n1));
                        if (o0 + n0 + n1 <= X.cap_jobs) {
                            hp = (int)h; off = (int)o0;
                            X.pair[h] = (int32_t)pp; X.off[h] = off; X.nj[h] = n0 | n1 << 16;
                            atomicAdd(&w.stats[AF_GSTAT_PE_JOBS], 1);
                        } else {
                            X.pair[h] = -1;
                            atomicMin(&X.cnt[4], (unsigned long long)o0);  // slots from o0 on are unwritten
                        }
                    }
                }
                hp = __builtin_amdgcn_readfirstlane(hp);
                off = __builtin_amdgcn_readfirstlane(off);
                if (hp >= 0) {
                    for (int k = lane; k < n0 + n1; k += 64) {
                        const int i = k >= n0, j = k - (i ? n0 : 0);
                        X.job[off + k] = make_int2(hp, E.ovf[!i] ? -1 : (i << 16 | j));
                    }
                    wave_sync();
                    continue;
                }
            }
        }
        for (int i = 0; i < 2; ++i)
            for (int j = 0; j < E.nb[i] && j < o.max_matesw; ++j) {
                if (E.ovf[!i]) continue;
                const GReg bj = B[i * (AF_G_MAX_REG + 1) + j];
                const int32_t *sr = sres ? sres + (int64_t)((i ? nj0 : 0) + j) * 4 * AF_G_PE_RES_W : nullptr;
                if (!g_matesw(G, p, o, S, !i, A[!i], bj, zg, sr, lane)) {
                    wave_sync();
                    if (lane == 0) { E.ovf[!i] = 1; E.na[!i] = 0; }
                    wave_sync();
                }
            }
        GPROF(const uint64_t gp_c1 = clock64(); const int gp_na0 = E.na[0], gp_na1 = E.na[1];)
        // primary marking, pairing and the record choice (mem_sam_pe)
        g_mark_primary_w(A[0], E.na[0], (int64_t)((uint64_t)(o.pair_base + pp) << 1 | 0), reinterpret_cast<GReg *>(S.seed), lane);
        g_mark_primary_w(A[1], E.na[1], (int64_t)((uint64_t)(o.pair_base + pp) << 1 | 1), reinterpret_cast<GReg *>(S.seed), lane);
        // mem_pair of long region lists on the wave (lane 0's g_mem_pair below otherwise)
        int zw[2] = {0, 0}, o_sc_w = 0;
        const int npr = E.na[0] + E.na[1];
        const bool pair_w = E.na[0] && E.na[1] && npr >= G_RANK_MIN && npr <= AF_G_MAX_REG;
        if (pair_w)
            o_sc_w = g_mem_pair_w(G, p, E.pes, A[0], E.na[0], A[1], E.na[1], (int)(uint32_t)(o.pair_base + pp), zw,
                                  reinterpret_cast<P64g *>(g_box), V, lane);
        if (lane == 0) {
            const uint64_t id = (uint64_t)(o.pair_base + pp);
            int z[2] = {zw[0], zw[1]}, extra = 1, mode = 0;  // mode 1: paired records
            int o_sc = 0;
            // mem_pair's sort keys in LDS (the boxes' space) when they fit
            P64g *Vp = E.na[0] + E.na[1] <= AF_G_MAX_REG ? reinterpret_cast<P64g *>(g_box) : V;
            if (E.na[0] && E.na[1] &&
                (o_sc = pair_w ? o_sc_w : g_mem_pair(G, p, E.pes, A[0], E.na[0], A[1], E.na[1], (int)(uint32_t)id, z, Vp)) > 0) {
                int is_multi = 0;
                for (int i = 0; i < 2; ++i) {
                    int j;
                    for (j = 1; j < E.na[i]; ++j)
                        if (A[i][j].secondary < 0 && A[i][j].score >= p.T) break;
                    is_multi |= j < E.na[i];
                }
                if (!is_multi) {
                    const int score_un = A[0][0].score + A[1][0].score - o.pen_unpaired;
                    if (o_sc > score_un) {
                        for (int i = 0; i < 2; ++i) {
                            GReg &c = A[i][z[i]];
                            if (c.secondary >= 0) { c.sub = A[i][c.secondary].score; c.secondary = -2; }
                        }
                        extra |= 2;
                    } else {
                        z[0] = z[1] = 0;
                    }
                    mode = 1;
                }
            }
            E.misc[1] = mode; E.misc[2] = z[0]; E.misc[3] = z[1]; E.misc[4] = extra;
        }
        wave_sync();
        GPROF(const uint64_t gp_c2 = clock64();)
        const int mode = E.misc[1];
        int extra = E.misc[4];
        const int zz[2] = {E.misc[2], E.misc[3]};
        // h[i] = mem_reg2aln of each end's chosen region (paired) or top region >= T
        for (int i = 0; i < 2; ++i) {
            const int l = E.len[i];
            DpLds &L = g_dp;
            for (int x = lane; x < l; x += 64) L.q[x] = E.q[i][x];
            wave_sync();
            const GReg *ar = nullptr;
            if (mode == 1) ar = &A[i][zz[i]];
            else if (E.na[i] && A[i][0].score >= p.T) ar = &A[i][0];
            g_reg2aln<CPL>(G, p, l, ar, H.mate[i], zg, lane);
            wave_sync();
        }
        if (mode == 1) {
            if (lane == 0) {
                for (int i = 0; i < 2; ++i) {
                    H.mate[i].flag |= 0x40 << i | extra;
                }
                for (int i = 0; i < 2; ++i) {
                    const int64_t r = 2 * pp + i;
                    g_aln2rec(H.mate[i], &H.mate[!i], 0, E.len[i], (int32_t)r, recs[r * AF_G_MAX_REC]);
                    n_rec[r] = 1;
                }
            }
            wave_sync();
        } else {
            if (H.mate[0].rid == H.mate[1].rid && H.mate[0].rid >= 0) {
                int64_t dist;
                const int d = g_infer_dir(G.l_pac, A[0][0].rb, A[1][0].rb, &dist);
                if (!E.pes[d].failed && dist >= E.pes[d].low && dist <= E.pes[d].high) extra |= 2;
            }
            for (int i = 0; i < 2; ++i) {
                const int64_t r = 2 * pp + i;
                const int l = E.len[i];
                DpLds &L = g_dp;
                for (int x = lane; x < l; x += 64) L.q[x] = E.q[i][x];
                wave_sync();
                const GAln mate = H.mate[!i];
                const int nrec = g_reg2sam<CPL>(G, p, l, A[i], E.na[i], (0x40 << i) | extra, &mate, (int32_t)r,
                                                recs + r * AF_G_MAX_REC, zg, lane);
                if (lane == 0) n_rec[r] = nrec;
                wave_sync();
            }
        }
        if (lane == 0) {
            for (int i = 0; i < 2; ++i) {
                const int64_t r = 2 * pp + i;
                const int nr = n_rec[r];
                if (E.ovf[i] || nr > AF_G_MAX_REC) {
                    for (int j = 0; j < (nr < AF_G_MAX_REC ? nr : AF_G_MAX_REC); ++j)
                        recs[r * AF_G_MAX_REC + j].flag |= AF_FLAG_MEM_OVERFLOW;
                    if (nr > AF_G_MAX_REC) atomicAdd(&w.stats[AF_GSTAT_RECS], 1);
                }
            }
        }
        GPROF(if (lane == 0) { int32_t *g = gp_row(2 * pp); if (g) { const uint64_t ce = clock64();
              g[32] = (int32_t)(gp_c1 - gp_c0); g[33] = (int32_t)(gp_c2 - gp_c1); g[34] = (int32_t)(ce - gp_c2);
              g[35] = E.misc[5]; g[36] = E.misc[6]; g[37] = gp_na0 << 16 | gp_na1; g[38] = (int32_t)gp_t0;
              g[39] = (int32_t)gp_rt(); } })
        wave_sync();
    }
}

// one rescue window of a heavy pair per wave (k_g_pe mode 1's job list): for each direction bwa
// may search, the window and its ksw_align2 as mem_matesw computes them (results ahead of the
// pair's own walk, which decides per window whether to use them)
__global__ __launch_bounds__(64, 2) void k_g_pe_jobs(DevGenome G, const uint8_t *__restrict__ reads, int32_t stride,
                                                     const int32_t *__restrict__ lens, af_params p, GOpt o, GWork w,
                                                     S2Work sw) {
    GPeLds &E = g_gpe;
    const int lane = threadIdx.x;
    const GPeSpec &X = w.pe;
    int64_t n = (int64_t)X.cnt[1];
    if (n > X.cap_jobs) n = X.cap_jobs;
    if (n > (int64_t)X.cnt[4]) n = (int64_t)X.cnt[4];
    for (;;) {
        int64_t k = 0;
        if (lane == 0) k = (int64_t)atomicAdd(&X.cnt[2], 1ull);
        k = (int64_t)__builtin_amdgcn_readfirstlane((int)k);
        if (k >= n) break;
        const int2 jb = X.job[k];
        if (jb.y < 0) continue;
        const int i = jb.y >> 16, j = jb.y & 0xffff;
        const int64_t pp = X.pair[jb.x];
        int32_t *out = X.res + k * 4 * AF_G_PE_RES_W;
        // the rescued read (the other end) and its codes
        const int64_t rm = 2 * pp + !i;
        const int l_ms = read_len(lens, rm, stride);
        for (int x = lane; x < l_ms; x += 64) E.q[0][x] = nt4(reads[rm * (int64_t)stride + x]);
        if (lane < 4) E.pes[lane] = sw.pes[(int64_t)g_chunk_of(sw, pp) * 4 + lane];
        // bj: end i's j-th region scoring within pen_unpaired of its best (k_g_pe's copy list)
        const GReg *ai = w.reg + w.reg_off[2 * pp + i];
        const int na = w.reg_n[2 * pp + i] > 0 ? w.reg_n[2 * pp + i] : 0;
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
        const GReg bj = ai[at];
        int rid = -1;
        for (int r = 0; r < 4; ++r) {
            int64_t rb, re;
            int ran = 0, sc = 0, te = 0, qe = 0, tb = 0, qb = 0;
            if (!E.pes[r].failed && g_mate_window(G, p, E.pes[r], r, bj, l_ms, rb, re, rid)) {
                g_mate_ksw(G, p, E.q[0], l_ms, r, rb, re, sc, te, qe, tb, qb, lane);
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

__global__ void k_g_zero(GWork w, int64_t n_reads, int32_t *heads) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t == 0) { *w.iv_fill = 0; *w.reg_fill = 0; *w.g1_next = 0; }
    if (t == 1 && w.g1_hv_n) { *w.g1_hv_n = 0; *w.g1_hv_next = 0; }
    if (t == 2 && w.g2_list_n) { *w.g2_list_n = 0; *w.g2_list_next = 0; }
    if (t < 7 && w.hv.cnt) w.hv.cnt[t] = 0;  // [5] k_g_pe's and [6] k_g_se's dequeue counters too
    if (t < 5 && w.pe.cnt) w.pe.cnt[t] = t == 4 ? 1ull << 62 : 0;
    if (t < 8) heads[AF_HEAD_STRIDE * t] = 0;
    if (t < AF_GSTAT_N) w.stats[t] = 0;
    (void)n_reads;
}

}  // namespace

size_t af_g1_slot_bytes() { return (size_t)G1_SLOT * sizeof(uint4); }


// ---- test hook: wave_introsort (mem_chain_flt's sort, weights << 32 | index keys compared by
// weight only, descending) against klib's introsort on lane 0, on the same keys.  One wave per
// list; scratch 5 n ints.  tests/test_gpu_genome.py::test_wave_introsort_equals_klib.
__global__ __launch_bounds__(64) void k_debug_isort(uint64_t *__restrict__ a, uint64_t *__restrict__ b, int n,
                                                    int32_t *__restrict__ scr) {
    const int lane = threadIdx.x;
    if (blockIdx.x == 0) {
        if (lane == 0) ks_introsort(a, n, GKeyFlt());
    } else {
        wave_introsort(b, n, GKeyFlt(), scr, lane);
    }
}
extern "C" int af_debug_wave_introsort(const uint64_t *keys, int32_t n, uint64_t *out_klib, uint64_t *out_wave) {
    if (n < 0 || n > (1 << 16) || (n > 0 && (!keys || !out_klib || !out_wave))) return -1;
    if (n == 0) return 0;
    uint64_t *da = nullptr, *db = nullptr;
    int32_t *ds = nullptr;
    int rc = -1;
    const size_t nb = sizeof(uint64_t) * (size_t)n;
    if (hipMalloc(&da, nb) == hipSuccess && hipMalloc(&db, nb) == hipSuccess &&
        hipMalloc(&ds, sizeof(int32_t) * 5 * (size_t)n) == hipSuccess &&
        hipMemcpy(da, keys, nb, hipMemcpyHostToDevice) == hipSuccess &&
        hipMemcpy(db, keys, nb, hipMemcpyHostToDevice) == hipSuccess) {
        hipLaunchKernelGGL(k_debug_isort, dim3(2), dim3(64), 0, 0, da, db, n, ds);
        if (hipGetLastError() == hipSuccess && hipDeviceSynchronize() == hipSuccess &&
            hipMemcpy(out_klib, da, nb, hipMemcpyDeviceToHost) == hipSuccess &&
            hipMemcpy(out_wave, db, nb, hipMemcpyDeviceToHost) == hipSuccess)
            rc = 0;
    }
    (void)hipFree(da); (void)hipFree(db); (void)hipFree(ds);
    return rc;
}

#ifdef AF_G_PROF
static int32_t *h_gprof = nullptr;
static int64_t h_gprof_cap = 0;
static int32_t h_gprof_calls = 0, h_gprof_next = 0;
static int32_t h_gprof_ids[64];
extern "C" int af_debug_g_prof_enable(int64_t cap, int32_t calls) {
    if (h_gprof) { (void)hipFree(h_gprof); h_gprof = nullptr; }
    if (hipMalloc(&h_gprof, sizeof(int32_t) * GP_W * cap * calls) != hipSuccess) return -1;
    (void)hipMemset(h_gprof, 0, sizeof(int32_t) * GP_W * cap * calls);
    h_gprof_cap = cap; h_gprof_calls = calls > 64 ? 64 : calls; h_gprof_next = 0;
    for (int i = 0; i < 64; ++i) h_gprof_ids[i] = i;
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_gprof), &h_gprof, sizeof(h_gprof));
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_gprof_cap), &h_gprof_cap, sizeof(h_gprof_cap));
    return GP_W;
}
extern "C" int af_debug_g_prof_read(void *dst, int64_t n_ints) {
    (void)hipDeviceSynchronize();
    if (!h_gprof || n_ints > (int64_t)GP_W * h_gprof_cap * h_gprof_calls) return -1;
    return hipMemcpy(dst, h_gprof, sizeof(int32_t) * n_ints, hipMemcpyDeviceToHost) == hipSuccess ? h_gprof_next : -1;
}
// the next genome call's slot (calls past the last slot reuse it)
static void gprof_next(hipStream_t s) {
    if (!h_gprof) return;
    const int k = h_gprof_next < h_gprof_calls ? h_gprof_next : h_gprof_calls - 1;
    (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_gprof_call), &h_gprof_ids[k], sizeof(int32_t), 0, hipMemcpyHostToDevice, s);
    ++h_gprof_next;
}
#endif
size_t af_g2_slot_bytes() { return g2_slot_bytes(); }
size_t af_g_chain_bytes() { return sizeof(GChain); }
size_t af_g_seed_bytes() { return sizeof(GSeed); }

// S4 / S5 up to the regions: G1 + G2 over reads [0, *d_n) (or cap) of a call
hipError_t af_launch_genome_regions(const DevGenome &G, const uint8_t *reads, int32_t stride, const int32_t *lens,
                                    const int32_t *d_n, int64_t cap, const af_params &p, const GOpt &o, const GWork &w,
                                    uint8_t *g1_scratch, int n_g1_threads, uint8_t *g2_scratch, int n_g2_waves,
                                    uint8_t *zscratch, hipStream_t s) {
    GPROF(gprof_next(s);)
    {
        static int chain_arr = G_ARR;  // the value the symbol holds (read by the kernel at its launch)
        const char *e = getenv("AF_G_CHAIN_ARR");
        const int want = e ? std::max(0, std::min(G_ARR, atoi(e))) : G_ARR;
        if (want != chain_arr) {
            chain_arr = want;
            (void)hipMemcpyToSymbol(HIP_SYMBOL(g_chain_arr), &chain_arr, sizeof(int));
        }
    }
    hipLaunchKernelGGL(k_g_zero, dim3(1), dim3(64), 0, s, w, cap, w.heads);
    // one lane per read, at most the scratch's lanes (idle lanes refill from w.g1_next)
    const int64_t g1_waves = std::max<int64_t>(1, std::min<int64_t>(n_g1_threads / 64, (cap + 63) / 64));
    hipLaunchKernelGGL(k_g_seeds, dim3((unsigned)g1_waves), dim3(64), 0, s, G, reads, stride, lens, d_n, cap,
                       (int64_t)0, p, o, reinterpret_cast<uint4 *>(g1_scratch), w);
    // the heavy reads, one wave each, in the lane kernel's (finished) scratch: as many waves as the
    // scratch holds lanes' slots (their count is known on the device only; a call of few reads can
    // hand off thousands of repeat-rich ones, each 600+ dependent lookups long)
    if (w.g1_max_ext > 0)
        hipLaunchKernelGGL(k_g_seeds_wave, dim3((unsigned)std::max<int64_t>(1, n_g1_threads / 64 * AF_G1W_WPS / AF_G1_WPS)),
                           dim3(64), 0, s, G,
                           reads, stride, lens, cap, p, o, reinterpret_cast<uint4 *>(g1_scratch), w);
    const size_t zstride = (size_t)(AF_MAX_READ + 1) * 1024;
    const int cpl = (stride + 1 + 63) / 64;
#define AF_GO(C)                                                                                                       \
    do {                                                                                                               \
        hipLaunchKernelGGL((k_g_regions<C>), dim3(n_g2_waves), dim3(64), 0, s, G, reads, stride, lens, d_n, cap,       \
                           (int64_t)0, p, o, w, g2_scratch, g2_slot_bytes(), zscratch, zstride);                       \
        if (w.hv.min_chains > 0) {                                                                                     \
            hipLaunchKernelGGL((k_g_ext_jobs<C>), dim3(2 * n_g2_waves), dim3(64), 0, s, G, reads, stride, lens, p, w); \
            hipLaunchKernelGGL((k_g_heavy<C>), dim3(n_g2_waves), dim3(64), 0, s, G, reads, stride, lens, p, o, w,      \
                               g2_scratch, g2_slot_bytes(), zscratch, zstride);                                        \
        }                                                                                                              \
    } while (0)
    if (cpl <= 2) AF_GO(2);
    else if (cpl <= 3) AF_GO(3);
    else if (cpl <= 4) AF_GO(4);
    else AF_GO(AF_CPL);
#undef AF_GO
    return hipGetLastError();
}

// G1 alone (af_genome_intervals, parity tests)
hipError_t af_launch_genome_intervals(const DevGenome &G, const uint8_t *reads, int32_t stride, const int32_t *lens,
                                      int64_t cap, const af_params &p, const GOpt &o, const GWork &w,
                                      uint8_t *g1_scratch, int n_g1_threads, hipStream_t s) {
    hipLaunchKernelGGL(k_g_zero, dim3(1), dim3(64), 0, s, w, cap, w.heads);
    const int64_t g1_waves = std::max<int64_t>(1, std::min<int64_t>(n_g1_threads / 64, (cap + 63) / 64));
    hipLaunchKernelGGL(k_g_seeds, dim3((unsigned)g1_waves), dim3(64), 0, s, G, reads, stride, lens, nullptr, cap,
                       (int64_t)0, p, o, reinterpret_cast<uint4 *>(g1_scratch), w);
    if (w.g1_max_ext > 0)
        hipLaunchKernelGGL(k_g_seeds_wave, dim3((unsigned)std::max<int64_t>(1, n_g1_threads / 64 * AF_G1W_WPS / AF_G1_WPS)),
                           dim3(64), 0, s, G,
                           reads, stride, lens, cap, p, o, reinterpret_cast<uint4 *>(g1_scratch), w);
    return hipGetLastError();
}

hipError_t af_launch_genome_se(const DevGenome &G, const uint8_t *reads, int32_t stride, const int32_t *lens,
                               const int32_t *d_n, int64_t cap, const af_params &p, int64_t id_base, const int64_t *ids,
                               const GWork &w, uint8_t *g2_scratch, int n_waves, uint8_t *zscratch, af_grec *recs,
                               int32_t *n_rec, hipStream_t s) {
    const size_t zstride = (size_t)(AF_MAX_READ + 1) * 1024;
    const int cpl = (stride + 1 + 63) / 64;
#define AF_GO(C) hipLaunchKernelGGL((k_g_se<C>), dim3(n_waves), dim3(64), 0, s, G, reads, stride, lens, d_n, cap, p, \
                                    id_base, ids, w, g2_scratch, g2_slot_bytes(), zscratch, zstride, recs, n_rec)
    if (cpl <= 2) AF_GO(2);
    else if (cpl <= 3) AF_GO(3);
    else if (cpl <= 4) AF_GO(4);
    else AF_GO(AF_CPL);
#undef AF_GO
    return hipGetLastError();
}

hipError_t af_launch_genome_pe(const DevGenome &G, const uint8_t *reads, int32_t stride, const int32_t *lens,
                               const int32_t *d_npairs, int64_t cap_pairs, const af_params &p, const GOpt &o,
                               const GWork &w, const S2Work &sw, uint8_t *g2_scratch, int n_waves, uint8_t *zscratch,
                               af_grec *recs, int32_t *n_rec, hipStream_t s) {
    hipLaunchKernelGGL(k_g_pe_hist, dim3((unsigned)std::max<int64_t>(1, (cap_pairs + 255) / 256)), dim3(256), 0, s,
                       d_npairs, cap_pairs, G.l_pac, p, o, w, sw);
    hipError_t e = af_launch_s2_pestat(sw, o.max_ins, s);
    if (e != hipSuccess) return e;
    const size_t zstride = (size_t)(AF_MAX_READ + 1) * 1024;
    const int cpl = (stride + 1 + 63) / 64;
    const int mode = w.pe.min_windows > 0 ? 1 : 0;
#define AF_GO(C)                                                                                                      \
    do {                                                                                                              \
        hipLaunchKernelGGL((k_g_pe<C>), dim3(n_waves), dim3(64), 0, s, G, reads, stride, lens, d_npairs, cap_pairs, p, \
                           o, w, sw, g2_scratch, g2_slot_bytes(), zscratch, zstride, recs, n_rec, mode);               \
        if (mode) {                                                                                                   \
            hipLaunchKernelGGL(k_g_pe_jobs, dim3(2 * n_waves), dim3(64), 0, s, G, reads, stride, lens, p, o, w, sw);   \
            hipLaunchKernelGGL((k_g_pe<C>), dim3(n_waves), dim3(64), 0, s, G, reads, stride, lens, d_npairs,          \
                               cap_pairs, p, o, w, sw, g2_scratch, g2_slot_bytes(), zscratch, zstride, recs, n_rec, 2); \
        }                                                                                                             \
    } while (0)
    if (cpl <= 2) AF_GO(2);
    else if (cpl <= 3) AF_GO(3);
    else if (cpl <= 4) AF_GO(4);
    else AF_GO(AF_CPL);
#undef AF_GO
    return hipGetLastError();
}
