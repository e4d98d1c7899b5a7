// ksw_dp.h -- wave-level primitives and the ksw DP restatements shared by the alignment kernels
// (align.hip: placement; s2.hip: the bwa-mem paired-end S2 path).  Every function restates one
// bwa routine (ksw_extend2, ksw_global2, bwa_gen_cigar2) with the same recurrences and
// tie-breaks as oracle/af_oracle.c; lanes hold query columns (or, for bands that fit the wave,
// the band's diagonals: ext_dp_band, global_dp_band) and DPP scans carry the horizontal gap
// chain.  Header-only, anonymous namespace: each translation unit gets its own
// LDS slot (g_dp, g_z), referenced only by the kernels that use it.
#pragma once
#include "af_internal.h"

namespace {

#ifdef AF_K2_PROF
// profiling build only (make prof -> libafgpu_prof.so): per-candidate phase timings
__device__ int32_t *g_k2prof = nullptr;
constexpr int PROF_W = 20;  // [16] slot, [17]/[18] s_memrealtime (100 MHz) at item start/end
#define PROF(...) __VA_ARGS__
#else
#define PROF(...)
#endif

#ifndef AF_EXIT_MASK
#define AF_EXIT_MASK 3  // the exact early-exit test runs on rows i with (i & mask) == mask (every 4th row: 0.7 % faster step than every 2nd)
#endif

#ifndef AF_K2_ZLDS
#define AF_K2_ZLDS 2048
#endif
constexpr int ZLDS = AF_K2_ZLDS;  // traceback bytes per wave kept in LDS (larger DPs: global scratch)

// Per-wave LDS of the DP routines (one wave per workgroup).  The slot lives at namespace scope
// so that out-of-line helpers address it as LDS (ds_* instructions), not through generic
// pointers.  Traceback bytes are a separate variable so kernels without a traceback do not
// reserve them.
struct __attribute__((aligned(16))) DpLds {
    uint32_t ring[64];     // traceback CIGAR ring
    int32_t misc[8];       // [0] list counter of the caller, [2] n traceback ops
    uint32_t pk[AF_MAX_READ / 16 + 2];  // the read as 2-bit codes, 16 bases per word (base i at bits 2i)
    uint32_t nm[AF_MAX_READ / 16 + 2];  // N bits of the same bases (positions >= l set)
    uint8_t q[AF_MAX_READ + 16];
    uint8_t qs_pad[16];    // qs_pad[15] = qs[-1] (read as N by the band DP)
    uint8_t qs[AF_MAX_READ + 16];
    uint8_t t[1024];
};
__shared__ DpLds g_dp;
__shared__ __attribute__((aligned(16))) uint8_t g_z[ZLDS];

// ---- wave primitives (DPP; gfx9-family controls) ---------------------------------------
template <int CTRL, int ROWM = 0xf, int BANKM = 0xf>
__device__ __forceinline__ int dpp(int old, int v) {
    return __builtin_amdgcn_update_dpp(old, v, CTRL, ROWM, BANKM, false);
}
constexpr int kNeg = -(1 << 30) - (1 << 29);  // identity for max (below every DP value used)

// inclusive prefix max over lanes 0..63.  The DPP `old` operand is INT_MIN, the identity of
// max, so the compiler folds each step into one v_max_i32_dpp.
constexpr int kMaxId = (int)0x80000000;
__device__ __forceinline__ int wave_incl_max(int v) {
    v = max(v, dpp<0x111>(kMaxId, v));        // row_shr:1
    v = max(v, dpp<0x112>(kMaxId, v));        // row_shr:2
    v = max(v, dpp<0x114>(kMaxId, v));        // row_shr:4
    v = max(v, dpp<0x118>(kMaxId, v));        // row_shr:8
    v = max(v, dpp<0x142, 0xa>(kMaxId, v));   // row_bcast:15 -> rows 1, 3
    v = max(v, dpp<0x143, 0xc>(kMaxId, v));   // row_bcast:31 -> rows 2, 3
    return v;
}
// lane l receives lane l-1's value; lane 0 receives `old`
__device__ __forceinline__ int wave_shr1(int old, int v) { return dpp<0x138>(old, v); }
// inclusive prefix max over lanes 0..SPAN-1 (SPAN = 16, 32 or 64); lanes >= SPAN get partial values
template <int SPAN>
__device__ __forceinline__ int span_incl_max(int v) {
    v = max(v, dpp<0x111>(kMaxId, v));
    v = max(v, dpp<0x112>(kMaxId, v));
    v = max(v, dpp<0x114>(kMaxId, v));
    v = max(v, dpp<0x118>(kMaxId, v));
    if (SPAN > 16) v = max(v, dpp<0x142, 0xa>(kMaxId, v));
    if (SPAN > 32) v = max(v, dpp<0x143, 0xc>(kMaxId, v));
    return v;
}
template <int SPAN>
__device__ __forceinline__ int span_max(int v) { return __builtin_amdgcn_readlane(span_incl_max<SPAN>(v), SPAN - 1); }
__device__ __forceinline__ int bcast(int v, int lane) { return __builtin_amdgcn_readlane(v, lane); }
__device__ __forceinline__ int wave_max(int v) { return bcast(wave_incl_max(v), 63); }
__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
    return v;
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int scd(const af_params &p, int x, int y) {
    return (x > 3 || y > 3) ? -1 : (x == y ? p.a : -p.b);
}

// (int)((double)x / y + c) as bwa computes it (y >= 1): the default gap-extension cost 1 takes one add
// instead of a double-precision division
__device__ __forceinline__ int div_plus(int x, int y, int c) {
    if (y == 1) return x + c;
    return (int)((double)x / y + (double)c);
}

__device__ __forceinline__ int cal_max_gap(const af_params &p, int qlen) {
    int l_del = div_plus(qlen * p.a - p.o_del, p.e_del, 1);
    int l_ins = div_plus(qlen * p.a - p.o_ins, p.e_ins, 1);
    int l = l_del > l_ins ? l_del : l_ins;
    l = l > 1 ? l : 1;
    return l < p.w << 1 ? l : p.w << 1;
}

__device__ __forceinline__ int infer_bw(int l1, int l2, int score, int a, int q, int r) {
    if (l1 == l2 && l1 * a - score < (q + r - a) << 1) return 0;
    int w = div_plus((l1 < l2 ? l1 : l2) * a - score - q, r, 2);
    int d = l1 - l2 < 0 ? l2 - l1 : l1 - l2;
    return w < d ? d : w;
}

struct ExtRes { int max, qle, tle, gtle, gscore, max_off, rows; };

// select element c (runtime, < CPL) of a register array without scratch
template <int CPL>
__device__ __forceinline__ int pick(const int (&a)[CPL], int c) {
    int v = a[0];
#pragma unroll
    for (int x = 1; x < CPL; ++x)
        if (x == c) v = a[x];
    return v;
}

// ksw_extend2 semantics (see oracle ext_dp), row-parallel over query columns.
template <int CPL>
__device__ ExtRes ext_dp_wave(int qlen, const uint8_t *q, int tlen, const uint8_t *t, const af_params &p, int w,
                              int end_bonus, int zdrop, int h0, int lane) {
    const int oe_del = p.o_del + p.e_del, oe_ins = p.o_ins + p.e_ins;
    const int cpl = (qlen + 1 + 63) >> 6;
    const int j0 = lane * cpl;
    int eh_h[CPL], eh_e[CPL], qc[CPL];
    {
        const int v1 = h0 > oe_ins ? h0 - oe_ins : 0;
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            const int j = j0 + c;
            int v = 0;
            if (c < cpl && j <= qlen) {
                if (j == 0) v = h0;
                else {
                    const int vj = v1 - (j - 1) * p.e_ins;
                    v = j == 1 ? v1 : (vj > 0 ? vj : 0);
                }
            }
            eh_h[c] = v;
            eh_e[c] = 0;
            qc[c] = (c < cpl && j < qlen) ? q[j] : 4;
        }
    }
    {
        const int mx = p.a;
        int max_ins = div_plus(qlen * mx + end_bonus - p.o_ins, p.e_ins, 1);
        max_ins = max_ins > 1 ? max_ins : 1;
        w = w < max_ins ? w : max_ins;
        int max_del = div_plus(qlen * mx + end_bonus - p.o_del, p.e_del, 1);
        max_del = max_del > 1 ? max_del : 1;
        w = w < max_del ? w : max_del;
    }
    int mx = h0, max_i = -1, max_j = -1, max_ie = -1, gscore = -1, max_off = 0;
    int beg = 0, end = qlen;
    const int jq = qlen - 1, lq_lane = jq / cpl, lq_c = jq - lq_lane * cpl;
    int ti_next = tlen > 0 ? t[0] : 4;
    int rows = 0;
    for (int i = 0; i < tlen; ++i) {
        const int ti = ti_next;
        if (i + 1 < tlen) ti_next = t[i + 1];
        ++rows;
        if (beg < i - w) beg = i - w;
        if (end > i + w + 1) end = i + w + 1;
        if (end > qlen) end = qlen;
        int h1s = 0;
        if (beg == 0) {
            h1s = h0 - (p.o_del + p.e_del * (i + 1));
            if (h1s < 0) h1s = 0;
        }
        if (beg >= end) {  // empty row: bwa's loop body never runs, m == 0
            if (beg == qlen) {
                max_ie = gscore > h1s ? max_ie : i;
                gscore = gscore > h1s ? gscore : h1s;
            }
            break;
        }
        int Mv[CPL], bx[CPL], hv[CPL];
        int run = kNeg;
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            const int j = j0 + c;
            const bool in = c < cpl && j >= beg && j < end;
            const int d = eh_h[c];
            const int M = (in && d) ? d + scd(p, ti, qc[c]) : 0;
            Mv[c] = M;
            bx[c] = run;
            const int tk = M - oe_ins > 0 ? M - oe_ins : 0;
            if (in) run = max(run, tk + j * p.e_ins);
        }
        const int lex = wave_shr1(kNeg, wave_incl_max(run));
        int key = -1;
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            const int j = j0 + c;
            const bool in = c < cpl && j >= beg && j < end;
            const int P = max(lex, bx[c]);
            const int f = j > beg ? P - (j - 1) * p.e_ins : 0;
            const int e = eh_e[c], M = Mv[c];
            int h = M > e ? M : e;
            h = h > f ? h : f;
            hv[c] = h;
            if (in) {
                int tt = M - oe_del;
                tt = tt > 0 ? tt : 0;
                const int en = e - p.e_del;
                eh_e[c] = en > tt ? en : tt;
                key = max(key, (h << 10) | j);
            }
        }
        key = wave_max(key);
        const int m = key < 0 ? 0 : key >> 10;
        const int mj = key < 0 ? -1 : (key & 1023);
        const int hq = bcast(pick<CPL>(hv, lq_c), lq_lane);
        const int from_left = wave_shr1(0, pick<CPL>(hv, cpl - 1));
#pragma unroll
        for (int c = CPL - 1; c >= 0; --c) {
            const int j = j0 + c;
            if (c < cpl) {
                const int prevH = c == 0 ? from_left : hv[c > 0 ? c - 1 : 0];
                if (j == beg) eh_h[c] = h1s;
                else if (j > beg && j <= end) eh_h[c] = prevH;
                if (j == end) eh_e[c] = 0;
            }
        }
        if (end == qlen) {
            max_ie = gscore > hq ? max_ie : i;
            gscore = gscore > hq ? gscore : hq;
        }
        if (m == 0) break;
        if (m > mx) {
            mx = m; max_i = i; max_j = mj;
            const int off = mj - i < 0 ? i - mj : mj - i;
            max_off = max_off > off ? max_off : off;
        } else if (zdrop > 0) {
            if (i - max_i > mj - max_j) {
                if (mx - m - ((i - max_i) - (mj - max_j)) * p.e_del > zdrop) break;
            } else {
                if (mx - m - ((mj - max_j) - (i - max_i)) * p.e_ins > zdrop) break;
            }
        }
        // band trimming on the updated eh over [beg, end]
        int fnz = 1 << 30, lnz = -1;
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            const int j = j0 + c;
            if (c < cpl && (eh_h[c] != 0 || eh_e[c] != 0)) {
                if (j >= beg && j < end) fnz = min(fnz, j);
                if (j >= beg && j <= end) lnz = max(lnz, j);
            }
        }
        const uint64_t bf = __ballot(fnz < (1 << 30));
        const uint64_t bl = __ballot(lnz >= 0);
        const int FNZ = bf ? bcast(fnz, __ffsll((unsigned long long)bf) - 1) : (1 << 30);
        const int LNZ = bl ? bcast(lnz, 63 - __clzll((unsigned long long)bl)) : -1;
        const int beg_new = FNZ == (1 << 30) ? end : FNZ;
        const int jstar = LNZ >= beg_new ? LNZ : beg_new - 1;
        beg = beg_new;
        end = jstar + 2 < qlen ? jstar + 2 : qlen;
        // Early exit (exact): no later row can raise any cell above
        // U = max_j (max(eh[j].h, eh[j].e) + (qlen - j) * a) -- cells only grow along the
        // diagonal and a zero cell never restarts -- so once U <= max and U < gscore no later
        // row can change max/max_i/max_j/max_off (need m > max) or gscore/max_ie (need
        // H(i, qlen-1) >= gscore).  Checked every 4th row (AF_EXIT_MASK); the oracle runs every row.
        if ((i & AF_EXIT_MASK) == AF_EXIT_MASK && gscore > 0) {
            int u = 0;
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                const int j = j0 + c;
                if (c < cpl && j >= beg && j <= qlen) u = max(u, max(eh_h[c], eh_e[c]) + (qlen - j) * p.a);
            }
            const int U = wave_max(u);
            if (U <= mx && U < gscore) break;
        }
    }
    ExtRes r;
    r.max = mx; r.qle = max_j + 1; r.tle = max_i + 1; r.gtle = max_ie + 1; r.gscore = gscore; r.max_off = max_off; r.rows = rows;
    return r;
}

// ksw_extend2 for qlen <= 63: lane j owns query column j (and lane qlen the eh[qlen] slot).
// Same recurrences and tie-breaks as ext_dp_wave; the band bookkeeping is done on 64-bit lane
// masks (ballots + s_ff1/s_flbit) so that a row costs ~40 VALU and no readlane of an index.
// Kept out of line: inlined into k_align its loop ran out of SGPRs and spilled to VGPR lanes
// on every row; as a call it gets its own register allocation (one save/restore per call).
struct Sc { int a, b, o_del, e_del, o_ins, e_ins; };
// SPAN: the lanes the row's scans and maxima cover (qlen + 1 <= SPAN; lanes past qlen hold no
// band cell and never feed a lane to their left), so short flanks skip the cross-row DPP steps
template <int SPAN>
__device__ __noinline__ ExtRes ext_dp_w1(int qlen_, int qsel_, int qoff_, int tlen_, Sc p_, int w_, int end_bonus_,
                                         int zdrop_, int h0_) {
    // arguments of an out-of-line call arrive in VGPRs: re-assert wave uniformity
#define AF_U(x) __builtin_amdgcn_readfirstlane(x)
    const int qlen = AF_U(qlen_), tlen = AF_U(tlen_), end_bonus = AF_U(end_bonus_), zdrop = AF_U(zdrop_),
              h0 = AF_U(h0_), qoff = AF_U(qoff_);
    int w = AF_U(w_);
    const Sc p{AF_U(p_.a), AF_U(p_.b), AF_U(p_.o_del), AF_U(p_.e_del), AF_U(p_.o_ins), AF_U(p_.e_ins)};
    const uint8_t *q = (AF_U(qsel_) ? g_dp.q : g_dp.qs) + qoff;
    const uint8_t *t = g_dp.t;
#undef AF_U
    const int lane = threadIdx.x;
    const int oe_del = p.o_del + p.e_del, oe_ins = p.o_ins + p.e_ins;
    const int j = lane;
    int H, E = 0;
    {
        const int v1 = h0 > oe_ins ? h0 - oe_ins : 0;
        const int vj = v1 - (j - 1) * p.e_ins;
        H = j > qlen ? 0 : (j == 0 ? h0 : (j == 1 ? v1 : (vj > 0 ? vj : 0)));
    }
    const int qc = j < qlen ? q[j] : 4;
    const bool qn = qc > 3;
    // lane constants: run = max(M - oe_ins, 0) + jE = max(M + jEo, jE); f = P - jE1
    // (lane 0's f must lose to every M/E >= 0: the scan's shift brings 0 into lane 0, and its
    // jE1 is 2^30, so f = -2^30 there -- no -inf operand to rematerialise per row)
    const int jE = j * p.e_ins, jEo = jE - oe_ins, jE1 = j == 0 ? (1 << 30) : (j - 1) * p.e_ins,
              tailA = (qlen - j) * p.a;
    {
        int max_ins = div_plus(qlen * p.a + end_bonus - p.o_ins, p.e_ins, 1);
        max_ins = max_ins > 1 ? max_ins : 1;
        w = w < max_ins ? w : max_ins;
        int max_del = div_plus(qlen * p.a + end_bonus - p.o_del, p.e_del, 1);
        max_del = max_del > 1 ? max_del : 1;
        w = w < max_del ? w : max_del;
    }
    // Split of the per-row bookkeeping between the two issue ports.  The scalar unit is shared
    // by a CU's four SIMDs and bounds this loop, so the band (beg, end), the row index and the
    // target base stay in SGPRs while the maxima, z-drop, gscore and early-exit state are
    // wave-uniform values in VGPRs, updated with selects (`vz` is 0 but opaque to the
    // compiler's uniformity analysis) and tested through one readfirstlane per decision.
    const int vz = (int)__builtin_amdgcn_mbcnt_lo(0u, 0u);
    int mx = h0 + vz, max_i = vz - 1, max_j = vz - 1, max_ie = vz - 1, gscore = vz - 1, max_off = vz;
    int beg = 0, end = qlen, rows = 0;
    int ti_next = tlen > 0 ? t[0] : 4;
    for (int i = 0; i < tlen; ++i) {
        const int ti = ti_next;
        if (i + 1 < tlen) ti_next = t[i + 1];
        ++rows;
        beg = max(beg, i - w);
        end = min(min(end, i + w + 1), qlen);
        int h1s = 0;
        if (beg == 0) h1s = max(h0 - (p.o_del + p.e_del * (i + 1)), 0);
        if (beg >= end) {
            if (beg == qlen) {
                max_ie = gscore > h1s ? max_ie : i + vz;
                gscore = gscore > h1s ? gscore : h1s;
            }
            break;
        }
        // Lanes left of beg are never read again (beg only grows), so they may hold anything;
        // lanes right of end keep their H/E exactly as bwa's untouched eh[] entries.  Every
        // lane outside [beg, end) has M = 0, so its run term (jE) never wins the f scan over the
        // in-band term at j - 1 (>= 0), and at j == beg the scan gives f = 0 (beg > 0) or a
        // large negative (beg == 0), both below max(M, E) >= 0: no per-lane masking of f.
        const bool in = (unsigned)(j - beg) < (unsigned)(end - beg);
        // score: a / -b, -1 when either base is N (ti is wave-uniform: keep it in an SGPR)
        const int tiu = __builtin_amdgcn_readfirstlane(ti);
        const int s_eq = tiu > 3 ? -1 : p.a, s_ne = tiu > 3 ? -1 : -p.b;
        const int sc = qc == tiu ? s_eq : (qn ? -1 : s_ne);
        int M = H != 0 ? H + sc : 0;
        M = in ? M : 0;
        const int P = __builtin_amdgcn_mov_dpp(span_incl_max<SPAN>(max(M + jEo, jE)), 0x138, 0xf, 0xf, true);
        const int f = P - jE1;
        const int h = max(max(M, E), f);
        const int key = in ? ((h << 10) | j) : -1;
        const int kmax = span_max<SPAN>(key) + vz;
        const int m = max(kmax, 0) >> 10;
        const int mj = kmax < 0 ? -1 : (kmax & 1023);
        const int hq = bcast(h, qlen - 1) + vz;
        const int from_left = __builtin_amdgcn_mov_dpp(h, 0x138, 0xf, 0xf, true);  // wave_shr:1, lane 0 <- 0
        const int Eu = max(max(E - p.e_del, M - oe_del), 0);
        H = j <= end ? (j == beg ? h1s : from_left) : H;
        E = j < end ? Eu : (j == end ? 0 : E);
        if (end == qlen) {  // scalar test, vector update
            max_ie = gscore > hq ? max_ie : i + vz;
            gscore = max(gscore, hq);
        }
        // bwa: break on m == 0; else a new maximum, or the z-drop test against the old one
        const bool better = m > mx;
        const int di = i - max_i, dj = mj - max_j;
        // (24-bit multiplies: full-rate VALU; |di - dj| < 2^12 and the gap costs are small)
        const int zgap = di > dj ? mx - m - __mul24(di - dj, p.e_del) : mx - m - __mul24(dj - di, p.e_ins);
        const int zt = better ? INT_MIN : zgap;
        const int off = mj - i < 0 ? i - mj : mj - i;
        max_off = better ? max(max_off, off) : max_off;
        max_i = better ? i + vz : max_i;
        max_j = better ? mj : max_j;
        mx = better ? m : mx;
        const int stop = m == 0 ? 1 : (zt > zdrop ? zdrop : 0);  // zdrop > 0 for a z-drop break
        if (__builtin_amdgcn_readfirstlane(stop) > 0) break;
        // band trimming: first non-zero eh in [beg, end), last in [beg, end]
        const int x = (H | E) != 0 ? j - beg : 1 << 20;
        const uint64_t f_m = __ballot((unsigned)x < (unsigned)(end - beg));
        const uint64_t l_m = __ballot((unsigned)x <= (unsigned)(end - beg));
        const int beg_new = f_m ? (int)__builtin_ctzll(f_m) : end;
        const int lnz = l_m ? 63 - (int)__builtin_clzll(l_m) : -1;
        const int jstar = lnz >= beg_new ? lnz : beg_new - 1;
        beg = beg_new;
        end = jstar + 2 < qlen ? jstar + 2 : qlen;
        // exact early exit (see ext_dp_wave), every 4th row
        if ((i & AF_EXIT_MASK) == AF_EXIT_MASK) {
            const int u = (unsigned)(j - beg) <= (unsigned)(qlen - beg) ? max(H, E) + tailA : 0;
            const int U = span_max<SPAN>(u) + vz;
            const int g = U <= mx ? (U < gscore ? gscore : 0) : 0;  // > 0 iff gscore > 0, U <= max, U < gscore
            if (__builtin_amdgcn_readfirstlane(g) > 0) break;
        }
    }
    ExtRes r;
    r.max = mx; r.qle = max_j + 1; r.tle = max_i + 1; r.gtle = max_ie + 1; r.gscore = gscore; r.max_off = max_off;
    r.rows = rows;
    return r;
}

// ksw_extend2 for 64 <= qlen <= 127: lane l owns query columns 2l and 2l + 1 (column qlen is the
// eh[qlen] slot).  Same recurrences, tie-breaks and bookkeeping split as ext_dp_w1; the F chain
// takes one wave scan of the lane pairs' maxima (column 2l + 1 adds column 2l's term in-lane) and
// the band trimming two ballots per column parity.
__device__ __noinline__ ExtRes ext_dp_w2(int qlen_, int qsel_, int qoff_, int tlen_, Sc p_, int w_, int end_bonus_,
                                         int zdrop_, int h0_) {
#define AF_U(x) __builtin_amdgcn_readfirstlane(x)
    const int qlen = AF_U(qlen_), tlen = AF_U(tlen_), end_bonus = AF_U(end_bonus_), zdrop = AF_U(zdrop_),
              h0 = AF_U(h0_), qoff = AF_U(qoff_);
    int w = AF_U(w_);
    const Sc p{AF_U(p_.a), AF_U(p_.b), AF_U(p_.o_del), AF_U(p_.e_del), AF_U(p_.o_ins), AF_U(p_.e_ins)};
    const uint8_t *q = (AF_U(qsel_) ? g_dp.q : g_dp.qs) + qoff;
    const uint8_t *t = g_dp.t;
#undef AF_U
    const int lane = threadIdx.x;
    const int oe_del = p.o_del + p.e_del, oe_ins = p.o_ins + p.e_ins;
    const int j0 = 2 * lane, j1 = j0 + 1;
    int H0, H1, E0 = 0, E1 = 0;
    {
        const int v1 = h0 > oe_ins ? h0 - oe_ins : 0;
        const int va = v1 - (j0 - 1) * p.e_ins, vb = v1 - (j1 - 1) * p.e_ins;
        H0 = j0 > qlen ? 0 : (j0 == 0 ? h0 : (va > 0 ? va : 0));
        H1 = j1 > qlen ? 0 : (j1 == 1 ? v1 : (vb > 0 ? vb : 0));
    }
    const int qc0 = j0 < qlen ? q[j0] : 4, qc1 = j1 < qlen ? q[j1] : 4;
    const bool qn0 = qc0 > 3, qn1 = qc1 > 3;
    // per-column constants as in ext_dp_w1 (column 0's jE1 is 2^30: its f loses to M/E >= 0)
    const int jEa = j0 * p.e_ins, jEoa = jEa - oe_ins, jE1a = j0 == 0 ? (1 << 30) : (j0 - 1) * p.e_ins;
    const int jEb = j1 * p.e_ins, jEob = jEb - oe_ins, jE1b = j0 * p.e_ins;
    const int tailA0 = (qlen - j0) * p.a, tailA1 = (qlen - j1) * p.a;
    {
        int max_ins = div_plus(qlen * p.a + end_bonus - p.o_ins, p.e_ins, 1);
        max_ins = max_ins > 1 ? max_ins : 1;
        w = w < max_ins ? w : max_ins;
        int max_del = div_plus(qlen * p.a + end_bonus - p.o_del, p.e_del, 1);
        max_del = max_del > 1 ? max_del : 1;
        w = w < max_del ? w : max_del;
    }
    const int vz = (int)__builtin_amdgcn_mbcnt_lo(0u, 0u);
    int mx = h0 + vz, max_i = vz - 1, max_j = vz - 1, max_ie = vz - 1, gscore = vz - 1, max_off = vz;
    int beg = 0, end = qlen, rows = 0;
    const int lq_lane = (qlen - 1) >> 1, lq_odd = (qlen - 1) & 1;
    int ti_next = tlen > 0 ? t[0] : 4;
    for (int i = 0; i < tlen; ++i) {
        const int ti = ti_next;
        if (i + 1 < tlen) ti_next = t[i + 1];
        ++rows;
        beg = max(beg, i - w);
        end = min(min(end, i + w + 1), qlen);
        int h1s = 0;
        if (beg == 0) h1s = max(h0 - (p.o_del + p.e_del * (i + 1)), 0);
        if (beg >= end) {
            if (beg == qlen) {
                max_ie = gscore > h1s ? max_ie : i + vz;
                gscore = gscore > h1s ? gscore : h1s;
            }
            break;
        }
        const bool in0 = (unsigned)(j0 - beg) < (unsigned)(end - beg);
        const bool in1 = (unsigned)(j1 - beg) < (unsigned)(end - beg);
        const int tiu = __builtin_amdgcn_readfirstlane(ti);
        const int s_eq = tiu > 3 ? -1 : p.a, s_ne = tiu > 3 ? -1 : -p.b;
        const int sc0 = qc0 == tiu ? s_eq : (qn0 ? -1 : s_ne);
        const int sc1 = qc1 == tiu ? s_eq : (qn1 ? -1 : s_ne);
        const int M0 = (in0 && H0 != 0) ? H0 + sc0 : 0;
        const int M1 = (in1 && H1 != 0) ? H1 + sc1 : 0;
        const int va = max(M0 + jEoa, jEa), vb = max(M1 + jEob, jEb);
        // exclusive prefix over lanes of the pair maxima (0 into lane 0: every term is >= 0)
        const int X = __builtin_amdgcn_mov_dpp(wave_incl_max(max(va, vb)), 0x138, 0xf, 0xf, true);
        const int f0 = X - jE1a, f1 = max(X, va) - jE1b;
        const int hA = max(max(M0, E0), f0), hB = max(max(M1, E1), f1);
        const int key = max(in0 ? ((hA << 10) | j0) : -1, in1 ? ((hB << 10) | j1) : -1);
        const int kmax = wave_max(key) + vz;
        const int m = max(kmax, 0) >> 10;
        const int mj = kmax < 0 ? -1 : (kmax & 1023);
        const int hq = bcast(lq_odd ? hB : hA, lq_lane) + vz;
        const int from_left = __builtin_amdgcn_mov_dpp(hB, 0x138, 0xf, 0xf, true);  // column j0 - 1
        const int Eu0 = max(max(E0 - p.e_del, M0 - oe_del), 0);
        const int Eu1 = max(max(E1 - p.e_del, M1 - oe_del), 0);
        H0 = j0 <= end ? (j0 == beg ? h1s : from_left) : H0;
        H1 = j1 <= end ? (j1 == beg ? h1s : hA) : H1;
        E0 = j0 < end ? Eu0 : (j0 == end ? 0 : E0);
        E1 = j1 < end ? Eu1 : (j1 == end ? 0 : E1);
        if (end == qlen) {
            max_ie = gscore > hq ? max_ie : i + vz;
            gscore = max(gscore, hq);
        }
        const bool better = m > mx;
        const int di = i - max_i, dj = mj - max_j;
        const int zgap = di > dj ? mx - m - __mul24(di - dj, p.e_del) : mx - m - __mul24(dj - di, p.e_ins);
        const int zt = better ? INT_MIN : zgap;
        const int off = mj - i < 0 ? i - mj : mj - i;
        max_off = better ? max(max_off, off) : max_off;
        max_i = better ? i + vz : max_i;
        max_j = better ? mj : max_j;
        mx = better ? m : mx;
        const int stop = m == 0 ? 1 : (zt > zdrop ? zdrop : 0);
        if (__builtin_amdgcn_readfirstlane(stop) > 0) break;
        // band trimming: first non-zero eh in [beg, end), last in [beg, end]; even and odd
        // columns on separate ballots
        const int x0 = (H0 | E0) != 0 ? j0 - beg : 1 << 20, x1 = (H1 | E1) != 0 ? j1 - beg : 1 << 20;
        const uint32_t span = (uint32_t)(end - beg);
        const uint64_t fa = __ballot((unsigned)x0 < span), fb = __ballot((unsigned)x1 < span);
        const uint64_t la = __ballot((unsigned)x0 <= span), lb = __ballot((unsigned)x1 <= span);
        const int fza = fa ? 2 * (int)__builtin_ctzll(fa) : (1 << 20), fzb = fb ? 2 * (int)__builtin_ctzll(fb) + 1 : (1 << 20);
        const int fz = min(fza, fzb);
        const int beg_new = fz < (1 << 20) ? fz : end;
        const int lza = la ? 2 * (63 - (int)__builtin_clzll(la)) : -1, lzb = lb ? 2 * (63 - (int)__builtin_clzll(lb)) + 1 : -1;
        const int lnz = max(lza, lzb);
        const int jstar = lnz >= beg_new ? lnz : beg_new - 1;
        beg = beg_new;
        end = jstar + 2 < qlen ? jstar + 2 : qlen;
        if ((i & AF_EXIT_MASK) == AF_EXIT_MASK) {
            const int ua = (unsigned)(j0 - beg) <= (unsigned)(qlen - beg) ? max(H0, E0) + tailA0 : 0;
            const int ub = (unsigned)(j1 - beg) <= (unsigned)(qlen - beg) ? max(H1, E1) + tailA1 : 0;
            const int U = wave_max(max(ua, ub)) + vz;
            const int g = U <= mx ? (U < gscore ? gscore : 0) : 0;
            if (__builtin_amdgcn_readfirstlane(g) > 0) break;
        }
    }
    ExtRes r;
    r.max = mx; r.qle = max_j + 1; r.tle = max_i + 1; r.gtle = max_ie + 1; r.gscore = gscore; r.max_off = max_off;
    r.rows = rows;
    return r;
}

// ksw_extend2 when the band fits the wave (w <= 31 after the max_ins / max_del clamp): lane k
// holds column j = i - w + k of row i, one cell per lane whatever qlen is (BLAT's band-16
// extensions of 150-bp queries).  bwa's eh[j].h (H(i-1, j-1), the diagonal predecessor) of a
// column the row rewrites is the h this lane just computed; eh[j].e and the entries the row
// leaves alone move down one lane per row; lanes 2w+1.. hold the initial eh of their (untouched)
// columns.  Same recurrences, tie-breaks, band trimming and bookkeeping split as ext_dp_w1; the
// exact early exit bounds the columns later rows can read (>= i + 1 - w).
__device__ __noinline__ ExtRes ext_dp_band(int qlen_, int qsel_, int qoff_, int tlen_, Sc p_, int w_, int end_bonus_,
                                           int zdrop_, int h0_) {
#define AF_U(x) __builtin_amdgcn_readfirstlane(x)
    const int qlen = AF_U(qlen_), tlen = AF_U(tlen_), end_bonus = AF_U(end_bonus_), zdrop = AF_U(zdrop_),
              h0 = AF_U(h0_), qoff = AF_U(qoff_);
    int w = AF_U(w_);
    const Sc p{AF_U(p_.a), AF_U(p_.b), AF_U(p_.o_del), AF_U(p_.e_del), AF_U(p_.o_ins), AF_U(p_.e_ins)};
    const uint8_t *q = (AF_U(qsel_) ? g_dp.q : g_dp.qs) + qoff;
    const uint8_t *t = g_dp.t;
#undef AF_U
    const int lane = threadIdx.x;
    const int oe_del = p.o_del + p.e_del, oe_ins = p.o_ins + p.e_ins;
    {
        int max_ins = div_plus(qlen * p.a + end_bonus - p.o_ins, p.e_ins, 1);
        max_ins = max_ins > 1 ? max_ins : 1;
        w = w < max_ins ? w : max_ins;
        int max_del = div_plus(qlen * p.a + end_bonus - p.o_del, p.e_del, 1);
        max_del = max_del > 1 ? max_del : 1;
        w = w < max_del ? w : max_del;
    }
    const int v1 = h0 > oe_ins ? h0 - oe_ins : 0;
    int j = lane - w;  // this lane's column in row i
    int H = j < 0 || j > qlen ? 0 : (j == 0 ? h0 : max(v1 - (j - 1) * p.e_ins, 0));
    int E = 0;
    const bool tail = lane >= 2 * w + 1;  // lanes past the band: untouched columns
    const int vz = (int)__builtin_amdgcn_mbcnt_lo(0u, 0u);
    int mx = h0 + vz, max_i = vz - 1, max_j = vz - 1, max_ie = vz - 1, gscore = vz - 1, max_off = vz;
    int beg = 0, end = qlen, rows = 0;
    int ti_next = tlen > 0 ? t[0] : 4;
    int qv = q[min(max(j, 0), qlen - 1)];
    for (int i = 0; i < tlen; ++i, ++j) {
        const int ti = ti_next;
        if (i + 1 < tlen) ti_next = t[i + 1];
        const int qc = (unsigned)j < (unsigned)qlen ? qv : 4;
        qv = q[min(max(j + 1, 0), qlen - 1)];  // the next row's base of this lane
        ++rows;
        beg = max(beg, i - w);
        end = min(min(end, i + w + 1), qlen);
        int h1s = 0;
        if (beg == 0) h1s = max(h0 - (p.o_del + p.e_del * (i + 1)), 0);
        if (beg >= end) {
            if (beg == qlen) {
                max_ie = gscore > h1s ? max_ie : i + vz;
                gscore = gscore > h1s ? gscore : h1s;
            }
            break;
        }
        const bool in = (unsigned)(j - beg) < (unsigned)(end - beg);
        const int tiu = __builtin_amdgcn_readfirstlane(ti);
        const int s_eq = tiu > 3 ? -1 : p.a, s_ne = tiu > 3 ? -1 : -p.b;
        const int sc = qc == tiu ? s_eq : (qc > 3 ? -1 : s_ne);
        int M = H != 0 ? H + sc : 0;
        M = in ? M : 0;
        // f as in ext_dp_w1: lanes left of the band carry jE (M = 0), column 0 gets -2^30
        const int jE = j * p.e_ins, jEo = jE - oe_ins, jE1 = j <= 0 ? (1 << 30) : jE - p.e_ins;
        const int P = __builtin_amdgcn_mov_dpp(span_incl_max<64>(max(M + jEo, jE)), 0x138, 0xf, 0xf, true);
        const int f = P - jE1;
        const int h = max(max(M, E), f);
        const int key = in ? ((h << 10) | j) : -1;
        const int kmax = span_max<64>(key) + vz;
        const int m = max(kmax, 0) >> 10;
        const int mj = kmax < 0 ? -1 : (kmax & 1023);
        const int hq = bcast(h, min(max(qlen - 1 - i + w, 0), 63)) + vz;
        const int Eu = max(max(E - p.e_del, M - oe_del), 0);
        // the row's eh: E of column j (this layout), then both moved to the next row's layout
        // (lane k <- column j + 1)
        const int En = j < end ? Eu : (j == end ? 0 : E);
        const int e_beg = __builtin_amdgcn_readlane(En, 0);  // column i - w
        const int Hs = __builtin_amdgcn_mov_dpp(H, 0x130, 0xf, 0xf, true);  // wave_shl:1
        const int Es = __builtin_amdgcn_mov_dpp(En, 0x130, 0xf, 0xf, true);
        const int jn = j + 1;
        H = jn == beg ? h1s : (jn <= end ? h : Hs);
        E = Es;
        if (tail) { H = jn > qlen ? 0 : max(v1 - (jn - 1) * p.e_ins, 0); E = 0; }
        if (end == qlen) {
            max_ie = gscore > hq ? max_ie : i + vz;
            gscore = max(gscore, hq);
        }
        const bool better = m > mx;
        const int di = i - max_i, dj = mj - max_j;
        const int zgap = di > dj ? mx - m - __mul24(di - dj, p.e_del) : mx - m - __mul24(dj - di, p.e_ins);
        const int zt = better ? INT_MIN : zgap;
        const int off = mj - i < 0 ? i - mj : mj - i;
        max_off = better ? max(max_off, off) : max_off;
        max_i = better ? i + vz : max_i;
        max_j = better ? mj : max_j;
        mx = better ? m : mx;
        const int stop = m == 0 ? 1 : (zt > zdrop ? zdrop : 0);
        if (__builtin_amdgcn_readfirstlane(stop) > 0) break;
        // band trimming: first non-zero eh in [beg, end), last in [beg, end]; column i - w (no
        // lane in the next row's layout) is column beg when beg == i - w: eh = (h1s, e_beg)
        const int x = (H | E) != 0 ? jn - beg : 1 << 20;
        const uint64_t f_m = __ballot((unsigned)x < (unsigned)(end - beg));
        const uint64_t l_m = __ballot((unsigned)x <= (unsigned)(end - beg));
        const bool edge = beg == i - w && (h1s | e_beg) != 0;
        const int c0 = i + 1 - w;  // column of lane 0 in the next row
        const int beg_new = edge ? beg : (f_m ? c0 + (int)__builtin_ctzll(f_m) : end);
        const int lnz = l_m ? c0 + 63 - (int)__builtin_clzll(l_m) : (edge ? beg : -1);
        const int jstar = lnz >= beg_new ? lnz : beg_new - 1;
        beg = beg_new;
        end = jstar + 2 < qlen ? jstar + 2 : qlen;
        if ((i & AF_EXIT_MASK) == AF_EXIT_MASK) {
            const int u = (unsigned)(jn - beg) <= (unsigned)(qlen - beg) ? max(H, E) + (qlen - jn) * p.a : 0;
            const int U = span_max<64>(u) + vz;
            const int g = U <= mx ? (U < gscore ? gscore : 0) : 0;
            if (__builtin_amdgcn_readfirstlane(g) > 0) break;
        }
    }
    ExtRes r;
    r.max = mx; r.qle = max_j + 1; r.tle = max_i + 1; r.gtle = max_ie + 1; r.gscore = gscore; r.max_off = max_off;
    r.rows = rows;
    return r;
}

// the w ksw_extend2 uses for qlen (ext_dp_w1's clamp)
__device__ __forceinline__ int ext_band_w(int qlen, const af_params &p, int w, int end_bonus) {
    int max_ins = div_plus(qlen * p.a + end_bonus - p.o_ins, p.e_ins, 1);
    max_ins = max_ins > 1 ? max_ins : 1;
    int max_del = div_plus(qlen * p.a + end_bonus - p.o_del, p.e_del, 1);
    max_del = max_del > 1 ? max_del : 1;
    return min(w, min(max_ins, max_del));
}

// ext_dp_w1 at the narrowest scan span that covers the query (qlen + 1 <= 64)
__device__ __forceinline__ ExtRes ext_dp_w1s(int qlen, const uint8_t *q, int tlen, const af_params &p, int w,
                                             int end_bonus, int zdrop, int h0) {
    const int qsel = q == g_dp.qs ? 0 : 1, qoff = (int)(q - (q == g_dp.qs ? g_dp.qs : g_dp.q));
    const Sc sc{p.a, p.b, p.o_del, p.e_del, p.o_ins, p.e_ins};
    if (qlen + 1 <= 16) return ext_dp_w1<16>(qlen, qsel, qoff, tlen, sc, w, end_bonus, zdrop, h0);
    if (qlen + 1 <= 32) return ext_dp_w1<32>(qlen, qsel, qoff, tlen, sc, w, end_bonus, zdrop, h0);
    return ext_dp_w1<64>(qlen, qsel, qoff, tlen, sc, w, end_bonus, zdrop, h0);
}

// one column per lane when the query fits a wave (the common case: a 100-bp read's flanks),
// otherwise CPL columns per lane; the per-row VALU cost scales with the columns per lane
template <int CPL>
__device__ __forceinline__ ExtRes ext_dp(int qlen, const uint8_t *q, int tlen, const uint8_t *t, const af_params &p,
                                         int w, int end_bonus, int zdrop, int h0, int lane) {
#ifdef AF_K2_PROF
    const int64_t c0 = clock64();
    ExtRes r;
    const bool one = CPL == 1 || qlen + 1 <= 64;
    if (one)
        r = ext_dp_w1s(qlen, q, tlen, p, w, end_bonus, zdrop, h0);
    else if (ext_band_w(qlen, p, w, end_bonus) <= 31)
        r = ext_dp_band(qlen, q == g_dp.qs ? 0 : 1, (int)(q - (q == g_dp.qs ? g_dp.qs : g_dp.q)), tlen,
                        Sc{p.a, p.b, p.o_del, p.e_del, p.o_ins, p.e_ins}, w, end_bonus, zdrop, h0);
    else if (qlen + 1 <= 128)
        r = ext_dp_w2(qlen, q == g_dp.qs ? 0 : 1, (int)(q - (q == g_dp.qs ? g_dp.qs : g_dp.q)), tlen,
                      Sc{p.a, p.b, p.o_del, p.e_del, p.o_ins, p.e_ins}, w, end_bonus, zdrop, h0);
    else
        r = ext_dp_wave<CPL>(qlen, q, tlen, t, p, w, end_bonus, zdrop, h0, lane);
    const int dc = (int)(clock64() - c0);
    if (lane == 0) { g_dp.misc[one ? 4 : 6] += dc; g_dp.misc[one ? 5 : 7] += r.rows; }
    return r;
#endif
    if (CPL == 1 || qlen + 1 <= 64)
        return ext_dp_w1s(qlen, q, tlen, p, w, end_bonus, zdrop, h0);
    if (ext_band_w(qlen, p, w, end_bonus) <= 31)  // the band fits the wave: one cell per lane
        return ext_dp_band(qlen, q == g_dp.qs ? 0 : 1, (int)(q - (q == g_dp.qs ? g_dp.qs : g_dp.q)), tlen,
                           Sc{p.a, p.b, p.o_del, p.e_del, p.o_ins, p.e_ins}, w, end_bonus, zdrop, h0);
    if (qlen + 1 <= 128)
        return ext_dp_w2(qlen, q == g_dp.qs ? 0 : 1, (int)(q - (q == g_dp.qs ? g_dp.qs : g_dp.q)), tlen,
                         Sc{p.a, p.b, p.o_del, p.e_del, p.o_ins, p.e_ins}, w, end_bonus, zdrop, h0);
    return ext_dp_wave<CPL>(qlen, q, tlen, t, p, w, end_bonus, zdrop, h0, lane);
}

// Traceback of a filled ksw_global2 direction matrix z, leaving the CIGAR (reverse order) in
// L.ring with L.misc[2] ops.  Byte layout (global_dp_wave): n_col = min(qlen, 2w+1) bytes per
// row from column beg, codes which | E-extend << 2 | F-extend << 4.  BAND layout (global_dp_band):
// a nibble per band lane k = j - i + w, 2w + 2 nibbles per row, codes which | E << 2 | F << 3.
template <bool BAND>
__device__ __forceinline__ void global_traceback(int qlen, int tlen, int w, const uint8_t *z, DpLds &L, int lane) {
    const int n_col = qlen < 2 * w + 1 ? qlen : 2 * w + 1;
    wave_sync();
    PROF(const int64_t tb0 = clock64();)
    // Traceback, wave-parallel.  The serial walk (bwa ksw_global2) is
    //   which = z[i][k] >> (2 * which) & 3;  0: M (--i, --k)  1: D (--i)  2: I (--k)
    // While `which` keeps its value the walk moves in a straight line, so lane t reads the
    // cell t steps ahead on that line; the first lane whose code differs (or that leaves the
    // matrix) ends the run.  One LDS read per lane and a ballot per run instead of one
    // dependent read per step.
    {
        const int zsize = n_col * tlen;
        int i = tlen - 1;
        int k = (i + w + 1 < qlen ? i + w + 1 : qlen) - 1;
        int state = 0, nc = 0, cur_op = -1, cur_len = 0;
        auto push = [&](int op, int len) {
            if (len <= 0) return;
            if (op == cur_op) { cur_len += len; return; }
            if (cur_op >= 0) {
                if (lane == 0) L.ring[nc & 63] = (uint32_t)cur_len << 4 | (uint32_t)cur_op;
                ++nc;
            }
            cur_op = op; cur_len = len;
        };
        while (i >= 0 && k >= 0) {
            const int it = i - (state != 2 ? lane : 0), kt = k - (state != 1 ? lane : 0);
            int wt = -1;
            if (BAND) {
                const int kk = kt - it + w;
                if (it >= 0 && kt >= 0 && (unsigned)kk <= (unsigned)(2 * w)) {
                    const uint32_t nib = (uint32_t)it * (uint32_t)(2 * w + 2) + (uint32_t)kk;
                    const int v = (z[nib >> 1] >> ((nib & 1u) << 2)) & 15;
                    wt = state == 0 ? (v & 3) : (state == 1 ? ((v >> 2) & 1) : ((v >> 2) & 2));
                }
            } else if (it >= 0 && kt >= 0) {
                const int idx = it * n_col + (kt - (it > w ? it - w : 0));
                if (idx >= 0 && idx < zsize) wt = z[idx] >> (state << 1) & 3;
            }
            const uint64_t stop = __ballot(wt != state);
            const int r = stop ? __ffsll((unsigned long long)stop) - 1 : 64;
            const int op_state = state == 0 ? 0 : (state == 1 ? 2 : 1);
            push(op_state, r);
            if (state != 2) i -= r;
            if (state != 1) k -= r;
            if (r == 64) continue;
            if (i < 0 || k < 0) break;
            const int which = bcast(wt, r);
            if (which < 0) break;  // walked off the stored matrix (not reachable from a valid score)
            if (which == 0) { push(0, 1); --i; --k; }
            else if (which == 1) { push(2, 1); --i; }
            else { push(1, 1); --k; }
            state = which;
        }
        if (i >= 0) push(2, i + 1);
        if (k >= 0) push(1, k + 1);
        push(-2, 1);  // flush
        if (lane == 0) L.misc[2] = nc;
    }
    wave_sync();
    PROF(L.misc[3] += (int)(clock64() - tb0);)
}

// ksw_global2 semantics with traceback (see oracle global_dp).  z: n_col*tlen bytes.
// Returns the score; the CIGAR (reverse order) is left in L.ring with L.misc[2] ops.
template <int CPL, bool TB = true>
__device__ int global_dp_wave(int qlen, const uint8_t *q, int tlen, const uint8_t *t, const af_params &p, int w,
                              uint8_t *z, DpLds &L, int lane) {
    const int oe_del = p.o_del + p.e_del, oe_ins = p.o_ins + p.e_ins;
    const int n_col = qlen < 2 * w + 1 ? qlen : 2 * w + 1;
    const int cpl = (qlen + 1 + 63) >> 6;
    const int j0 = lane * cpl;
    int eh_h[CPL], eh_e[CPL], qc[CPL];
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
        const int j = j0 + c;
        eh_h[c] = AF_NEG_INF;
        eh_e[c] = AF_NEG_INF;
        if (c < cpl && j <= qlen) {
            if (j == 0) eh_h[c] = 0;
            else if (j <= w) eh_h[c] = -(p.o_ins + p.e_ins * j);
        }
        qc[c] = (c < cpl && j < qlen) ? q[j] : 4;
    }
    int ti_next = tlen > 0 ? t[0] : 4;
    for (int i = 0; i < tlen; ++i) {
        const int ti = ti_next;
        if (i + 1 < tlen) ti_next = t[i + 1];
        const int beg = i > w ? i - w : 0;
        const int end = i + w + 1 < qlen ? i + w + 1 : qlen;
        const int h1s = beg == 0 ? -(p.o_del + p.e_del * (i + 1)) : AF_NEG_INF;
        int Mv[CPL], bx[CPL], hv[CPL];
        const int seed = AF_NEG_INF + (beg - 1) * p.e_ins;  // the f = -inf chain entering at beg
        int run = seed;
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            const int j = j0 + c;
            const bool in = c < cpl && j >= beg && j < end;
            const int m = eh_h[c] + scd(p, ti, qc[c]);
            Mv[c] = m;
            bx[c] = run;
            if (in) run = max(run, m - oe_ins + j * p.e_ins);
        }
        const int lex = wave_shr1(seed, wave_incl_max(run));
        uint8_t *zi = z + (size_t)i * n_col;
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            const int j = j0 + c;
            const bool in = c < cpl && j >= beg && j < end;
            const int P = max(lex, bx[c]);
            const int f = P - (j - 1) * p.e_ins;
            const int m = Mv[c];
            const int e = eh_e[c];
            int d = m >= e ? 0 : 1;
            int h = m >= e ? m : e;
            d = h >= f ? d : 2;
            h = h >= f ? h : f;
            hv[c] = h;
            if (in) {
                const int tt = m - oe_del;
                const int ee = e - p.e_del;
                d |= ee > tt ? 1 << 2 : 0;
                eh_e[c] = ee > tt ? ee : tt;
                const int tf = m - oe_ins;
                const int ff = f - p.e_ins;
                d |= ff > tf ? 2 << 4 : 0;
                if (TB) zi[j - beg] = (uint8_t)d;
            }
        }
        const int from_left = wave_shr1(0, pick<CPL>(hv, cpl - 1));
#pragma unroll
        for (int c = CPL - 1; c >= 0; --c) {
            const int j = j0 + c;
            if (c < cpl) {
                const int prevH = c == 0 ? from_left : hv[c > 0 ? c - 1 : 0];
                if (j == beg) eh_h[c] = h1s;
                else if (j > beg && j <= end) eh_h[c] = prevH;
                if (j == end) eh_e[c] = AF_NEG_INF;
            }
        }
    }
    const int score = bcast(pick<CPL>(eh_h, qlen - (qlen / cpl) * cpl), qlen / cpl);
    if (TB) global_traceback<false>(qlen, tlen, w, z, L, lane);
    return score;
}

// ksw_global2 (as global_dp_wave) when the band is at most 64 columns wide (w <= 31): lane k
// holds column j = i - w + k of row i, so one cell per lane whatever qlen is.  H(i-1, j-1) stays
// in the lane, E(i, j) arrives from lane k + 1 (wave_shl:1) and the query base moves down one
// lane per row.  Lanes outside [beg, end) carry -inf, except the H(i, -1) boundary of rows with
// beg == 0.  Same recurrences, tie-breaks and direction codes as global_dp_wave.
// ZL: the traceback nibbles ((w + 1) * tlen bytes <= ZLDS) go to the wave's LDS slot g_z instead
// of its global scratch zg
template <bool TB = true, bool ZL = false>
__device__ int global_dp_band(int qlen, const uint8_t *q, int tlen, const uint8_t *t, const af_params &p, int w,
                              uint8_t *__restrict__ zg_, DpLds &L, int lane) {
    uint8_t *__restrict__ zg = ZL ? g_z : zg_;
    const int oe_del = p.o_del + p.e_del, oe_ins = p.o_ins + p.e_ins;
    const int k = lane;  // qlen >= 64 > 2w + 1: every band lane exists
    const bool band = k <= 2 * w;
    // q[-1] and q[qlen] read as N: the query base of any lane is one clamped LDS read
    if (lane == 0) { L.qs_pad[15] = 4; L.qs[qlen] = 4; }
    int Hd;  // H(i-1, j-1) for this lane's cell of row i; row 0 reads ksw_global2's initial eh[j].h
    {
        const int j = k - w;
        Hd = (band && j == 0) ? 0
                              : ((band && j >= 1 && j <= w && j <= qlen) ? -(p.o_ins + p.e_ins * j) : AF_NEG_INF);
    }
    int Eo = AF_NEG_INF;     // E(i+1, j) produced by this lane's cell of row i
    int j = k - w;           // this lane's column in row i (advances one per row)
    int jE1 = (j - 1) * p.e_ins, jEo = j * p.e_ins - oe_ins;
    wave_sync();
    int qc = q[min(max(j, -1), qlen)];
    int ti_next = tlen > 0 ? t[0] : 4;
    for (int i = 0; i < tlen; ++i) {
        const int ti = __builtin_amdgcn_readfirstlane(ti_next);
        if (i + 1 < tlen) ti_next = t[i + 1];
        const int beg = i > w ? i - w : 0;
        const bool in = band && (unsigned)j < (unsigned)qlen;
        const int qn = q[min(max(j + 1, -1), qlen)];  // next row's base for this lane
        const int s_eq = ti > 3 ? -1 : p.a, s_ne = ti > 3 ? -1 : -p.b;
        const int m = Hd + (qc == ti ? s_eq : (qc > 3 ? -1 : s_ne));
        const int e = dpp<0x130>(AF_NEG_INF, Eo);  // wave_shl:1: E(i, j) from lane k + 1
        const int seed = AF_NEG_INF + (beg - 1) * p.e_ins;
        const int run = in ? max(seed, m + jEo) : seed;
        const int f = wave_shr1(seed, wave_incl_max(run)) - jE1;
        int d = m >= e ? 0 : 1;
        int h = m >= e ? m : e;
        d = h >= f ? d : 2;
        h = h >= f ? h : f;
        const int tt = m - oe_del, ee = e - p.e_del;
        d |= ee > tt ? 1 << 2 : 0;
        const int tf = m - oe_ins, ff = f - p.e_ins;
        d |= ff > tf ? 1 << 3 : 0;
        // z row i: one nibble per band lane (2w + 2 per row), lanes 2m and 2m + 1 in one byte
        // written by the even lane (nibbles of lanes whose cell is outside the matrix are never
        // read by the traceback)
        const int dup = __builtin_amdgcn_mov_dpp(d, 0x130, 0xf, 0xf, true);  // wave_shl:1: lane k + 1
        if (TB && !(k & 1) && k <= 2 * w) zg[(uint32_t)i * (uint32_t)(w + 1) + (uint32_t)(k >> 1)] = (uint8_t)(d | (dup << 4));
        Eo = in ? (ee > tt ? ee : tt) : AF_NEG_INF;
        Hd = in ? h : ((j == -1 && beg == 0) ? -(p.o_del + p.e_del * (i + 1)) : AF_NEG_INF);
        qc = qn;
        ++j;
        jE1 += p.e_ins;
        jEo += p.e_ins;
    }
    const int score = bcast(Hd, qlen - tlen + w);  // eh[qlen].h = H(tlen-1, qlen-1)
    if (TB) global_traceback<true>(qlen, tlen, w, zg, L, lane);
    return score;
}

// 16 bases of the packed doubled reference starting at pos, plus its N mask (bit per base)
__device__ __forceinline__ void getD16(const DevIndex &ix, int64_t pos, uint32_t &bits, uint32_t &nmask) {
    const int64_t wi = pos >> 4;
    const int sh = (int)(pos & 15) * 2;
    const uint32_t lo = ix.D2[wi], hi = ix.D2[wi + 1];
    bits = sh ? (lo >> sh) | (hi << (32 - sh)) : lo;
    const int64_t ni = pos >> 5;
    const int nsh = (int)(pos & 31);
    const uint32_t nlo = ix.Dn[ni], nhi = ix.Dn[ni + 1];
    nmask = (nsh ? (nlo >> nsh) | (nhi << (32 - nsh)) : nlo) & 0xFFFFu;
}

// gen_cigar restated (bwa_gen_cigar2): returns score, cigar in L.ring/L.misc[2]
// TB = false: the score only (mem_patch_reg), no traceback bytes written
template <int CPL, bool TB = true>
__device__ __forceinline__ int gen_cigar_wave(const uint8_t *text, int64_t n, const af_params &p, int w_, int lq, int qb,
                                              int64_t rb, int64_t re, DpLds &L, uint8_t *zg, int lane) {
    const int rlen = (int)(re - rb);
    const bool rev = rb >= n;
    for (int x = lane; x < lq; x += 64) L.qs[x] = rev ? L.q[qb + lq - 1 - x] : L.q[qb + x];
    for (int x = lane; x < rlen; x += 64) L.t[x] = rev ? text[re - 1 - x] : text[rb + x];
    wave_sync();
    int score;
    if (lq == rlen && w_ == 0) {
        int s = 0;
        for (int x = lane; x < lq; x += 64) s += scd(p, L.t[x], L.qs[x]);
        score = wave_sum(s);
        if (TB && lane == 0) { L.ring[0] = (uint32_t)lq << 4; L.misc[2] = 1; }
        wave_sync();
    } else {
        int max_ins = div_plus(((lq + 1) >> 1) * p.a - p.o_ins, p.e_ins, 1);
        int max_del = div_plus(((lq + 1) >> 1) * p.a - p.o_del, p.e_del, 1);
        int max_gap = max_ins > max_del ? max_ins : max_del;
        max_gap = max_gap > 1 ? max_gap : 1;
        const int d = rlen - lq < 0 ? lq - rlen : rlen - lq;
        int w = (max_gap + d + 1) >> 1;
        w = w < w_ ? w : w_;
        const int min_w = d + 3;
        w = w > min_w ? w : min_w;
        const int n_col = lq < 2 * w + 1 ? lq : 2 * w + 1;
        uint8_t *z = (TB && (size_t)n_col * rlen <= ZLDS) ? g_z : zg;
        if (lq + 1 <= 64) score = global_dp_wave<1, TB>(lq, L.qs, rlen, L.t, p, w, z, L, lane);
        else if (w <= 31) {
            if (TB && (size_t)(w + 1) * rlen <= ZLDS) score = global_dp_band<TB, true>(lq, L.qs, rlen, L.t, p, w, zg, L, lane);
            else score = global_dp_band<TB, false>(lq, L.qs, rlen, L.t, p, w, zg, L, lane);
        }
        else score = global_dp_wave<CPL, TB>(lq, L.qs, rlen, L.t, p, w, z, L, lane);
    }
    return score;
}

}  // namespace
