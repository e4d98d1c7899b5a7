// align.hip -- K2 (candidate alignment) and K3 (pair flags) of the anchor alignment path
// (`bwa mem -M` at Anchored_Fusion.py:182; a3 record fields).
//
// K2 is a persistent kernel: one 64-thread workgroup (= one wave, one LDS slot) per
// resident slot pulls candidate reads from a device-side work counter.  Per read the wave
//   1. finds every MEM >= min_seed_len against the doubled anchor (16-mer position hash in
//      L2, right extension by 2-bit word compares),
//   2. sorts MEMs (len desc, qb, rb) with a wave rank sort in LDS,
//   3. extends seeds in order (skipping seeds contained in an earlier region) with a
//      row-parallel banded DP: lanes own contiguous query columns; the horizontal gap chain
//      is a DPP prefix-max scan, row max / band trimming are DPP scans, ballots and
//      readlanes (no LDS round trips on the per-row critical path),
//   4. runs band inference + the global DP with traceback bits in LDS (global scratch for
//      oversize matrices) to produce the CIGAR of the best region.
// The recurrences, tie-breaks and band bookkeeping are exactly those of oracle/af_oracle.c.
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

#ifndef AF_K2_STATIC_PCT
#define AF_K2_STATIC_PCT 0  // share of candidates assigned round-robin (rest: per-XCD dequeue)
#endif
constexpr int MEMCAP = 64;   // == max allowed af_params.max_mems
#ifndef AF_K2_ZLDS
#define AF_K2_ZLDS 2048
#endif
constexpr int ZLDS = AF_K2_ZLDS;  // traceback bytes per wave kept in LDS (larger DPs: global scratch)

struct __attribute__((aligned(16))) AlnLds {
    uint64_t mem[MEMCAP];
    uint64_t smem[MEMCAP];
    int32_t regs[16][8];   // score, truesc, qb, qe, -, -, seedlen0, w
    int64_t rpos[16][2];   // rb, re of the regions (genome-scale references exceed 2^31)
    uint32_t ring[64];     // traceback CIGAR ring
    int32_t misc[8];       // [0] nmem (total found), [2] n traceback ops
    uint32_t pk[AF_MAX_READ / 16 + 2];  // the read as 2-bit codes, 16 bases per word (base i at bits 2i)
    uint32_t nm[AF_MAX_READ / 16 + 2];  // N bits of the same bases (positions >= l set)
    uint8_t q[AF_MAX_READ + 16];
    uint8_t qs_pad[16];    // qs_pad[15] = qs[-1] (read as N by the band DP)
    uint8_t qs[AF_MAX_READ + 16];
    uint8_t t[1024];
    uint8_t z[ZLDS];
};

// One wave per workgroup: the per-wave LDS slot lives at namespace scope so that out-of-line
// helpers address it as LDS (ds_* instructions) rather than through generic pointers.
__shared__ AlnLds g_aln;

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
        // H(i, qlen-1) >= gscore).  Checked on odd rows; the oracle runs every row.
        if ((i & 1) && gscore > 0) {
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
    const uint8_t *q = (AF_U(qsel_) ? g_aln.q : g_aln.qs) + qoff;
    const uint8_t *t = g_aln.t;
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
        // exact early exit (see ext_dp_wave), on odd rows
        if (i & 1) {
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
    const uint8_t *q = (AF_U(qsel_) ? g_aln.q : g_aln.qs) + qoff;
    const uint8_t *t = g_aln.t;
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
        if (i & 1) {
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

// ext_dp_w1 at the narrowest scan span that covers the query (qlen + 1 <= 64)
__device__ __forceinline__ ExtRes ext_dp_w1s(int qlen, const uint8_t *q, int tlen, const af_params &p, int w,
                                             int end_bonus, int zdrop, int h0) {
    const int qsel = q == g_aln.qs ? 0 : 1, qoff = (int)(q - (q == g_aln.qs ? g_aln.qs : g_aln.q));
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
    else if (qlen + 1 <= 128)
        r = ext_dp_w2(qlen, q == g_aln.qs ? 0 : 1, (int)(q - (q == g_aln.qs ? g_aln.qs : g_aln.q)), tlen,
                      Sc{p.a, p.b, p.o_del, p.e_del, p.o_ins, p.e_ins}, w, end_bonus, zdrop, h0);
    else
        r = ext_dp_wave<CPL>(qlen, q, tlen, t, p, w, end_bonus, zdrop, h0, lane);
    const int dc = (int)(clock64() - c0);
    if (lane == 0) { g_aln.misc[one ? 4 : 6] += dc; g_aln.misc[one ? 5 : 7] += r.rows; }
    return r;
#endif
    if (CPL == 1 || qlen + 1 <= 64)
        return ext_dp_w1s(qlen, q, tlen, p, w, end_bonus, zdrop, h0);
    if (qlen + 1 <= 128)
        return ext_dp_w2(qlen, q == g_aln.qs ? 0 : 1, (int)(q - (q == g_aln.qs ? g_aln.qs : g_aln.q)), tlen,
                         Sc{p.a, p.b, p.o_del, p.e_del, p.o_ins, p.e_ins}, w, end_bonus, zdrop, h0);
    return ext_dp_wave<CPL>(qlen, q, tlen, t, p, w, end_bonus, zdrop, h0, lane);
}

// Traceback of a filled ksw_global2 direction matrix z, leaving the CIGAR (reverse order) in
// L.ring with L.misc[2] ops.  Byte layout (global_dp_wave): n_col = min(qlen, 2w+1) bytes per
// row from column beg, codes which | E-extend << 2 | F-extend << 4.  BAND layout (global_dp_band):
// a nibble per band lane k = j - i + w, 2w + 2 nibbles per row, codes which | E << 2 | F << 3.
template <bool BAND>
__device__ __forceinline__ void global_traceback(int qlen, int tlen, int w, const uint8_t *z, AlnLds &L, int lane) {
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
template <int CPL>
__device__ int global_dp_wave(int qlen, const uint8_t *q, int tlen, const uint8_t *t, const af_params &p, int w,
                              uint8_t *z, AlnLds &L, int lane) {
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
                zi[j - beg] = (uint8_t)d;
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
    global_traceback<false>(qlen, tlen, w, z, L, lane);
    return score;
}

// ksw_global2 (as global_dp_wave) when the band is at most 64 columns wide (w <= 31): lane k
// holds column j = i - w + k of row i, so one cell per lane whatever qlen is.  H(i-1, j-1) stays
// in the lane, E(i, j) arrives from lane k + 1 (wave_shl:1) and the query base moves down one
// lane per row.  Lanes outside [beg, end) carry -inf, except the H(i, -1) boundary of rows with
// beg == 0.  Same recurrences, tie-breaks and direction codes as global_dp_wave.
__device__ int global_dp_band(int qlen, const uint8_t *q, int tlen, const uint8_t *t, const af_params &p, int w,
                              uint8_t *__restrict__ zg, AlnLds &L, int lane) {
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
        if (!(k & 1) && k <= 2 * w) zg[(uint32_t)i * (uint32_t)(w + 1) + (uint32_t)(k >> 1)] = (uint8_t)(d | (dup << 4));
        Eo = in ? (ee > tt ? ee : tt) : AF_NEG_INF;
        Hd = in ? h : ((j == -1 && beg == 0) ? -(p.o_del + p.e_del * (i + 1)) : AF_NEG_INF);
        qc = qn;
        ++j;
        jE1 += p.e_ins;
        jEo += p.e_ins;
    }
    const int score = bcast(Hd, qlen - tlen + w);  // eh[qlen].h = H(tlen-1, qlen-1)
    global_traceback<true>(qlen, tlen, w, zg, L, lane);
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
template <int CPL>
__device__ __forceinline__ int gen_cigar_wave(const DevIndex &ix, const af_params &p, int w_, int lq, int qb, int64_t rb, int64_t re,
                              AlnLds &L, uint8_t *zg, int lane) {
    const int rlen = (int)(re - rb);
    const bool rev = rb >= ix.n;
    for (int x = lane; x < lq; x += 64) L.qs[x] = rev ? L.q[qb + lq - 1 - x] : L.q[qb + x];
    for (int x = lane; x < rlen; x += 64) L.t[x] = rev ? ix.D[re - 1 - x] : ix.D[rb + x];
    wave_sync();
    int score;
    if (lq == rlen && w_ == 0) {
        int s = 0;
        for (int x = lane; x < lq; x += 64) s += scd(p, L.t[x], L.qs[x]);
        score = wave_sum(s);
        if (lane == 0) { L.ring[0] = (uint32_t)lq << 4; L.misc[2] = 1; }
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
        uint8_t *z = ((size_t)n_col * rlen <= ZLDS) ? L.z : zg;
        if (lq + 1 <= 64) score = global_dp_wave<1>(lq, L.qs, rlen, L.t, p, w, z, L, lane);
        else if (w <= 31) score = global_dp_band(lq, L.qs, rlen, L.t, p, w, zg, L, lane);
        else score = global_dp_wave<CPL>(lq, L.qs, rlen, L.t, p, w, z, L, lane);
    }
    return score;
}

// MULTI = placement mode (af_place): every region scoring >= T becomes an af_hit (best first,
// at most max_hits per query); cand == nullptr means "all reads".
template <int CPL, bool MULTI>
__global__ __launch_bounds__(64, AF_K2_WPS) void k_align(DevIndex ix, const uint8_t *__restrict__ reads, int32_t stride,
                                              const int32_t *__restrict__ lens, af_params p,
                                              const int32_t *__restrict__ cand, const int32_t *__restrict__ n_cand,
                                              int32_t *__restrict__ work, ReadRec *__restrict__ recs,
                                              uint32_t *__restrict__ cigar, uint8_t *__restrict__ zscratch,
                                              size_t zstride, af_hit *__restrict__ hits, int32_t *__restrict__ n_hits,
                                              int32_t max_hits) {
    AlnLds &L = g_aln;
    const int lane = threadIdx.x;
    const int ncand = *n_cand;
    uint8_t *zg = zscratch + (size_t)blockIdx.x * zstride;
    const int64_t n = ix.n, n2 = 2 * ix.n;
    const int max_ext = p.max_ext < 16 ? p.max_ext : 16;
    const int max_mems = p.max_mems < MEMCAP ? p.max_mems : MEMCAP;
    const uint32_t hm = (1u << ix.hbits) - 1u;
    // Work split: the first AF_K2_STATIC_PCT % of the candidates go round-robin to slots (no atomics); the
    // tail is dequeued from 8 per-XCD heads (one 128-B line each) so that no single word
    // takes every dequeue (one device-scope word saturates near 88 dequeues/us).
    const int S = (int)gridDim.x;
    const int nstat = (int)(((int64_t)ncand * AF_K2_STATIC_PCT / 100) / S * S);
    int next_static = (int)blockIdx.x;
    int head = (int)(blockIdx.x & 7), heads_left = 8;
    for (;;) {
        int item;
        if (next_static < nstat) {
            item = next_static;
            next_static += S;
        } else {
            item = ncand;
            while (heads_left > 0) {
                int v = 0;
                if (lane == 0) v = atomicAdd(&work[AF_HEAD_STRIDE * head], 1);
                v = __builtin_amdgcn_readfirstlane(v);
                const int64_t it = (int64_t)nstat + head + 8 * (int64_t)v;
                if (it < ncand) { item = (int)it; break; }
                head = (head + 1) & 7;
                --heads_left;
            }
            if (item >= ncand) break;
        }
        const int64_t r = cand ? cand[item] : item;
        PROF(const uint64_t rt0 = __builtin_amdgcn_s_memrealtime();)
        PROF(const int64_t pt0 = clock64(); int64_t pt1 = pt0, pt2 = pt0; int p_ext_rows = 0, p_cig_rows = 0,
             p_ext_calls = 0, p_nreg = 0, p_ext_dp = 0;)
        int l = lens ? lens[r] : stride;
        if (l > stride) l = stride;  // a length past the row (device-side lens are unchecked)
        if (l > AF_MAX_READ) l = AF_MAX_READ;
        if (l < 0) l = 0;
        const uint8_t *rd = reads + r * (int64_t)stride;
        for (int x = lane; x < l; x += 64) {
            const uint8_t c = rd[x];
            uint8_t v = 4;
            switch (c) {
            case 'A': case 'a': v = 0; break;
            case 'C': case 'c': v = 1; break;
            case 'G': case 'g': v = 2; break;
            case 'T': case 't': v = 3; break;
            default: v = 4;
            }
            L.q[x] = v;
        }
        if (lane == 0) L.misc[0] = 0;
        PROF(if (lane < 8 && lane >= 3) L.misc[lane] = 0;)
        wave_sync();
        // pack the codes: lane w owns bases 16w..16w+15 (2-bit codes + an N mask that also
        // covers every position >= l), so any lane can form a 16-mer with one funnel shift
        if (lane < AF_MAX_READ / 16 + 2) {
            const int b0 = lane * 16;
            uint32_t pw = 0, nw = 0;
            if (b0 < l) {
                const uint4 c = *reinterpret_cast<const uint4 *>(&L.q[b0]);
                const uint32_t cw[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const uint32_t y = cw[u] & 0x03030303u, t = y | (y >> 6);
                    pw |= ((t & 0xFu) | ((t >> 12) & 0xF0u)) << (8 * u);
                    nw |= ((((cw[u] >> 2) & 0x01010101u) * 0x01020408u) >> 24 & 0xFu) << (4 * u);
                }
            }
            const int valid = l - b0;  // bases of this word inside the read
            if (valid < 16) nw |= valid <= 0 ? 0xFFFFu : (0xFFFFu << valid) & 0xFFFFu;
            L.pk[lane] = pw;
            L.nm[lane] = nw;
        }
        wave_sync();
        // ---- 1. MEMs ------------------------------------------------------------------
        // placement (MULTI) re-seeds with the minimum MEM length raised by AF_RESEED_STEP while
        // a query has more than max_mems MEMs (random 16-mer hits on a genome-scale reference)
        int seed_min = p.min_seed_len;
        int nm_total;
        for (;;) {
        for (int qb = lane; qb + AF_K <= l; qb += 64) {
            const int wq = qb >> 4, sq = qb & 15;
            const uint32_t k = __builtin_amdgcn_alignbit(L.pk[wq + 1], L.pk[wq], 2 * sq);
            if (((L.nm[wq] | (L.nm[wq + 1] << 16)) >> sq) & 0xFFFFu) continue;
            // occurrences in the doubled reference: a hash index holds both strands' 16-mers; a
            // direct (genome-scale) index holds the forward strand only, so k's occurrences are
            // its forward run plus the reverse-strand images n2 - 16 - q of rc(k)'s forward run
            int cnt = 0, st = 0, n_fwd = 0, pos0 = 0;
            uint32_t b_fwd = 0, b_rc = 0;
            if (ix.kend) {
                const uint32_t rk = af_rc16(k);
                b_fwd = k ? ix.kend[k - 1] : 0u;
                b_rc = rk ? ix.kend[rk - 1] : 0u;
                n_fwd = (int)(ix.kend[k] - b_fwd);
                cnt = n_fwd + (int)(ix.kend[rk] - b_rc);
            } else {
                uint32_t s = af_fmix(k) & hm;
                for (;;) {
                    const int4 e = ix.hslot[s];
                    if (e.z == 0) break;
                    if ((uint32_t)e.x == k) { cnt = e.z; st = e.y; pos0 = e.w; break; }
                    s = (s + 1) & hm;
                }
            }
            if (cnt == 0 || cnt > p.max_occ) continue;
            for (int o = 0; o < cnt; ++o) {
                const int64_t rb = !ix.kend ? (int64_t)(o == 0 ? pos0 : ix.kpos[st + o])
                                            : (o < n_fwd ? (int64_t)ix.kposu[b_fwd + o]
                                                         : n2 - AF_K - (int64_t)ix.kposu[b_rc + (o - n_fwd)]);
                if (qb > 0 && rb != 0 && rb != n) {
                    const int qc = L.q[qb - 1];
                    if (qc < 4 && qc == ix.D[rb - 1]) continue;
                }
                const int64_t lim = rb < n ? n : n2;
                int len = AF_K;
                for (;;) {
                    const int qp = qb + len;
                    const int64_t rp = rb + len;
                    const int64_t room64 = min((int64_t)(l - qp), lim - rp);
                    if (room64 <= 0) break;
                    const int room = (int)min(room64, (int64_t)16);
                    const int wp = qp >> 4, sp = qp & 15;
                    const uint32_t qk = __builtin_amdgcn_alignbit(L.pk[wp + 1], L.pk[wp], 2 * sp);
                    const int qn = __builtin_ctz((((L.nm[wp] | (L.nm[wp + 1] << 16)) >> sp) & 0xFFFFu) | 0x10000u);
                    uint32_t dk, dn;
                    getD16(ix, rp, dk, dn);
                    const uint32_t x = qk ^ dk;
                    const int eq = x ? (__builtin_ctz(x) >> 1) : 16;
                    const int dnf = dn ? __builtin_ctz(dn) : 16;
                    const int step = min(min(eq, room), min(qn, dnf));
                    len += step;
                    if (step < 16) break;
                }
                if (len < seed_min) continue;
                const int slot = atomicAdd(&L.misc[0], 1);
                if (slot < MEMCAP)
                    L.mem[slot] = ((uint64_t)(1023 - len) << 50) | ((uint64_t)qb << 40) | (uint64_t)rb;
            }
        }
        wave_sync();
        nm_total = L.misc[0];
        if constexpr (MULTI) {
            if (nm_total > max_mems && seed_min + AF_RESEED_STEP <= AF_RESEED_MAX) {
                seed_min += AF_RESEED_STEP;
                wave_sync();  // every lane has read the count
                if (lane == 0) L.misc[0] = 0;
                wave_sync();
                continue;
            }
        }
        break;
        }
        PROF(pt1 = clock64();)
        int flag = 0x4;
        int out_pos = 0, out_score = 0, out_nc = 0;
        if (nm_total > max_mems) {
            flag = 0x4 | AF_FLAG_MEM_OVERFLOW;
        } else {
            const int nm = nm_total;
            // ---- 2. rank sort --------------------------------------------------------
            if (lane < nm) {
                const uint64_t ka = L.mem[lane];
                int rank = 0;
                for (int b = 0; b < nm; ++b) rank += L.mem[b] < ka;
                L.smem[rank] = ka;
            }
            wave_sync();
            // ---- 3. seed extension ---------------------------------------------------
            int n_reg = 0;
            for (int si = 0; si < nm; ++si) {
                const uint64_t key = L.smem[si];
                const int slen = 1023 - (int)(key >> 50);
                const int sqb = (int)((key >> 40) & 1023);
                const int64_t srb = (int64_t)(key & 0xFFFFFFFFFFull);
                bool skip = false;
                for (int rr = 0; rr < n_reg; ++rr) {
                    const int *a = L.regs[rr];
                    const int aqb = a[2], aqe = a[3], asl = a[6], aw = a[7];
                    const int64_t arb = L.rpos[rr][0], are = L.rpos[rr][1];
                    if (srb < arb || srb + slen > are || sqb < aqb || sqb + slen > aqe) continue;
                    if (10 * (slen - asl) > l) continue;
                    int qd = sqb - aqb, rd = (int)(srb - arb);
                    int mg = cal_max_gap(p, qd < rd ? qd : rd);
                    int ww = mg < aw ? mg : aw;
                    if (qd - rd < ww && rd - qd < ww) { skip = true; break; }
                    qd = aqe - (sqb + slen); rd = (int)(are - (srb + slen));
                    mg = cal_max_gap(p, qd < rd ? qd : rd);
                    ww = mg < aw ? mg : aw;
                    if (qd - rd < ww && rd - qd < ww) { skip = true; break; }
                }
                if (skip) continue;
                if (n_reg >= max_ext) break;
                // extend_seed
                const int64_t bq = srb - (sqb + cal_max_gap(p, sqb));
                const int rem = l - sqb - slen;
                const int64_t eq = srb + slen + (rem + cal_max_gap(p, rem));
                int64_t rmax0 = bq > 0 ? bq : 0, rmax1 = eq < n2 ? eq : n2;
                if (rmax0 < n && n < rmax1) {
                    if (srb < n) rmax1 = n; else rmax0 = n;
                }
                int a_score = 0, a_truesc = 0, a_qb = 0, a_qe = 0;
                int64_t a_rb = 0, a_re = 0;
                int aw0 = p.w, aw1 = p.w;
                if (sqb) {
                    const int tmp = (int)(srb - rmax0);
                    for (int x = lane; x < sqb; x += 64) L.qs[x] = L.q[sqb - 1 - x];
                    for (int x = lane; x < tmp; x += 64) L.t[x] = ix.D[rmax0 + tmp - 1 - x];
                    wave_sync();
                    ExtRes er;
                    for (int it = 0; it < 2; ++it) {
                        const int prev = a_score;
                        aw0 = p.w << it;
                        PROF(const int64_t te0 = clock64();)
                        er = ext_dp<CPL>(sqb, L.qs, tmp, L.t, p, aw0, p.pen_clip5, p.zdrop, slen * p.a, lane);
                        PROF(p_ext_dp += (int)(clock64() - te0);)
                        PROF(p_ext_rows += er.rows; ++p_ext_calls;)
                        a_score = er.max;
                        if (a_score == prev || er.max_off < (aw0 >> 1) + (aw0 >> 2)) break;
                    }
                    if (er.gscore <= 0 || er.gscore <= a_score - p.pen_clip5) {
                        a_qb = sqb - er.qle; a_rb = srb - er.tle; a_truesc = a_score;
                    } else {
                        a_qb = 0; a_rb = srb - er.gtle; a_truesc = er.gscore;
                    }
                    wave_sync();
                } else {
                    a_score = a_truesc = slen * p.a; a_qb = 0; a_rb = srb;
                }
                if (sqb + slen != l) {
                    const int qe = sqb + slen;
                    const int re = (int)(srb + slen - rmax0);
                    const int sc0 = a_score;
                    const int tl = (int)(rmax1 - rmax0 - re);
                    for (int x = lane; x < tl; x += 64) L.t[x] = ix.D[rmax0 + re + x];
                    wave_sync();
                    ExtRes er;
                    for (int it = 0; it < 2; ++it) {
                        const int prev = a_score;
                        aw1 = p.w << it;
                        PROF(const int64_t te0 = clock64();)
                        er = ext_dp<CPL>(l - qe, L.q + qe, tl, L.t, p, aw1, p.pen_clip3, p.zdrop, sc0, lane);
                        PROF(p_ext_dp += (int)(clock64() - te0);)
                        PROF(p_ext_rows += er.rows; ++p_ext_calls;)
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
                    a_qe = l; a_re = srb + slen;
                }
                if (lane == 0) {
                    int *a = L.regs[n_reg];
                    a[0] = a_score; a[1] = a_truesc; a[2] = a_qb; a[3] = a_qe;
                    a[4] = 0; a[5] = 0; a[6] = slen; a[7] = aw0 > aw1 ? aw0 : aw1;
                    L.rpos[n_reg][0] = a_rb; L.rpos[n_reg][1] = a_re;
                }
                wave_sync();
                ++n_reg;
            }
            PROF(pt2 = clock64(); p_nreg = n_reg;)
            // ---- 4. CIGAR of a region (bwa_gen_cigar2 + the band retry loop) -------------
            // Lane 0 writes the assembled ops to `co` and the record fields; with `want_mt`
            // every lane also gets the identical-base count and reference span of the
            // alignment (the oracle's emit_region, over its first AF_MAX_CIGAR ops).
            auto emit = [&](int ri, uint32_t *co, int &o_flag, int64_t &o_pos, int &o_score, int &o_nc,
                            bool want_mt, int &o_mt, int &o_span) {
                const int *a = L.regs[ri];
                const int a_score = a[0], a_truesc = a[1], aqb = a[2], aqe = a[3], awb = a[7];
                const int64_t arb = L.rpos[ri][0], are = L.rpos[ri][1];
                const bool is_rev = arb >= n;
                const int lq = aqe - aqb;
                const int tmpw = infer_bw(lq, (int)(are - arb), a_truesc, p.a, p.o_del, p.e_del);
                int w2 = infer_bw(lq, (int)(are - arb), a_truesc, p.a, p.o_ins, p.e_ins);
                w2 = w2 > tmpw ? w2 : tmpw;
                if (w2 > p.w) w2 = w2 < awb ? w2 : awb;
                int score = 0, last_sc = -(1 << 30), it = 0;
                do {
                    w2 = w2 < p.w << 2 ? w2 : p.w << 2;
                    score = gen_cigar_wave<CPL>(ix, p, w2, lq, aqb, arb, are, L, zg, lane);
                    PROF(p_cig_rows += (int)(are - arb);)
                    if (score == last_sc || w2 == p.w << 2) break;
                    last_sc = score;
                    w2 <<= 1;
                } while (++it < 3 && score < a_truesc - p.a);
                const int nc = L.misc[2];
                const int ncap = nc < AF_MAX_CIGAR ? nc : AF_MAX_CIGAR;
                if (want_mt) {
                    int mt = 0, span = 0, x = 0, y = 0;
                    for (int k = 0; k < ncap; ++k) {
                        const uint32_t op = L.ring[(nc - 1 - k) & 63];
                        const int len = (int)(op >> 4), o = (int)(op & 0xf);
                        if (o == 0) {
                            for (int u = lane; u < len; u += 64) mt += (L.qs[x + u] < 4 && L.qs[x + u] == L.t[y + u]);
                            x += len; y += len; span += len;
                        } else if (o == 1) {
                            x += len;
                        } else {
                            y += len; span += len;
                        }
                    }
                    if (ncap > 0) {
                        const uint32_t f0 = L.ring[(nc - 1) & 63], fl = L.ring[(nc - ncap) & 63];
                        if ((f0 & 0xf) == 2) span -= (int)(f0 >> 4);
                        else if ((fl & 0xf) == 2) span -= (int)(fl >> 4);
                    }
                    o_mt = wave_sum(mt);
                    o_span = span;
                }
                // assemble: ring holds the traceback in reverse order (count misc[2])
                if (lane == 0) {
                    bool of = nc > AF_MAX_CIGAR;
                    int64_t pos = is_rev ? n2 - are : arb;
                    int xs = 0, xe = ncap;  // window of ring entries (forward order)
                    const uint32_t first = L.ring[(nc - 1) & 63];
                    const uint32_t last = L.ring[(nc - ncap) & 63];
                    if (ncap > 0) {
                        if ((first & 0xf) == 2) { pos += first >> 4; xs = 1; }
                        else if ((last & 0xf) == 2) xe = ncap - 1;
                    }
                    const int clip5 = is_rev ? l - aqe : aqb;
                    const int clip3 = is_rev ? aqb : l - aqe;
                    int nf = 0;
                    if (clip5) { co[nf++] = (uint32_t)clip5 << 4 | 4; }
                    for (int x = xs; x < xe; ++x) {
                        if (nf < AF_MAX_CIGAR) co[nf] = L.ring[(nc - 1 - x) & 63];
                        ++nf;
                    }
                    if (clip3) {
                        if (nf < AF_MAX_CIGAR) co[nf] = (uint32_t)clip3 << 4 | 4;
                        ++nf;
                    }
                    if (nf > AF_MAX_CIGAR) { of = true; nf = AF_MAX_CIGAR; }
                    o_flag = (is_rev ? 0x10 : 0) | (of ? AF_FLAG_CIGAR_OVERFLOW : 0);
                    o_pos = pos;
                    o_score = a_score;
                    o_nc = nf;
                }
                wave_sync();
            };
            if (!MULTI) {
                int best = -1;
                for (int rr = 0; rr < n_reg; ++rr)
                    if (best < 0 || L.regs[rr][0] > L.regs[best][0]) best = rr;
                if (best >= 0 && L.regs[best][0] >= p.T) {
                    int mt_unused = 0, span_unused = 0;
                    int64_t pos64 = 0;
                    emit(best, cigar + r * AF_MAX_CIGAR, flag, pos64, out_score, out_nc, false, mt_unused,
                         span_unused);
                    out_pos = (int)pos64;  // hash (anchor) indexes only: < 2^31 (af_align_* check)
                }
            } else {
                // every region scoring >= T, best first (ties: region order), at most max_hits
                int32_t *order = reinterpret_cast<int32_t *>(L.mem);
                if (lane < n_reg) {
                    const int me = L.regs[lane][0];
                    int rank = 0;
                    for (int u = 0; u < n_reg; ++u) {
                        const int su = L.regs[u][0];
                        rank += su > me || (su == me && u < lane);
                    }
                    order[rank] = lane;
                }
                wave_sync();
                int nh = 0;
                for (int k = 0; k < n_reg && nh < max_hits; ++k) {
                    const int *a = L.regs[order[k]];
                    if (a[0] < p.T) break;
                    af_hit *h = hits + r * max_hits + nh;
                    int hf = 0, hs = 0, hn = 0, mt = 0, span = 0;
                    int64_t hp = 0;
                    emit(order[k], h->cigar, hf, hp, hs, hn, true, mt, span);
                    if (lane == 0) {
                        h->query = (int32_t)r; h->flag = hf; h->score = hs;
                        h->q_start = a[2]; h->q_end = a[3]; h->q_size = l; h->matches = mt;
                        h->n_cigar = hn; h->t_start = hp; h->t_end = hp + span;
                        for (int c = hn; c < AF_MAX_CIGAR; ++c) h->cigar[c] = 0;
                    }
                    ++nh;
                }
                if (lane == 0) n_hits[r] = nh;
            }
        }
        if (MULTI && nm_total > max_mems && lane == 0) n_hits[r] = -1;
        if (!MULTI && lane == 0) {
            ReadRec rec;
            rec.flag = flag; rec.pos = out_pos; rec.score = out_score; rec.n_cigar = out_nc;
            recs[r] = rec;
        }
#ifdef AF_K2_PROF
        if (lane == 0 && g_k2prof) {
            const int64_t pt3 = clock64();
            int32_t *o = g_k2prof + (int64_t)item * PROF_W;
            o[16] = (int32_t)blockIdx.x; o[17] = (int32_t)rt0;
            o[18] = (int32_t)__builtin_amdgcn_s_memrealtime();
            o[0] = (int32_t)r; o[1] = (int32_t)(pt3 - pt0); o[2] = (int32_t)(pt1 - pt0);
            o[3] = (int32_t)(pt2 - pt1); o[4] = (int32_t)(pt3 - pt2); o[5] = nm_total; o[6] = p_nreg; o[9] = p_ext_dp;
            o[7] = p_ext_rows; o[8] = p_cig_rows; o[10] = p_ext_calls;
            o[11] = L.misc[3]; o[12] = L.misc[4]; o[13] = L.misc[5]; o[14] = L.misc[6]; o[15] = L.misc[7];
        }
#endif
        wave_sync();
    }
}

template <bool TAILS>
__global__ void k_pairs(int64_t n_pairs, const int32_t *__restrict__ hits, const ReadRec *__restrict__ recs,
                        af_aln_out out, int32_t *__restrict__ ctrl, const uint8_t *__restrict__ reads, int32_t stride,
                        const int32_t *__restrict__ lens, AfTails tails) {
    const int64_t pp = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (blockIdx.x == 0 && threadIdx.x < 8)  // K2 ran: reset its dequeue heads
        ctrl[AF_CTRL_HEADS2 + AF_HEAD_STRIDE * threadIdx.x] = 0;
    if (pp >= n_pairs) return;
    ReadRec R[2];
#pragma unroll
    for (int m = 0; m < 2; ++m) {
        const int64_t r = 2 * pp + m;
        if (hits[r] > 0) R[m] = recs[r];
        else { R[m].flag = 0x4; R[m].pos = 0; R[m].score = 0; R[m].n_cigar = 0; }
    }
    int o_flag[2], o_pos[2], o_score[2], o_nc[2];
#pragma unroll
    for (int m = 0; m < 2; ++m) {
        const ReadRec &x = R[m], &y = R[m ^ 1];
        const int xf = x.flag, yf = y.flag;
        int f = 0x1 | (m ? 0x80 : 0x40) | (xf & ~0x4 & 0x30000);
        int pos = x.pos;
        if (!(xf & 0x4)) f |= xf & 0x10;
        else f |= 0x4;
        if (yf & 0x4) f |= 0x8;
        else f |= (yf & 0x10) ? 0x20 : 0;
        if ((xf & 0x4) && !(yf & 0x4)) { pos = y.pos; f |= (yf & 0x10); }
        if ((xf & 0x4) && (yf & 0x4)) pos = -1;
        o_flag[m] = f;
        o_pos[m] = pos;
        o_score[m] = x.score;
        o_nc[m] = (xf & 0x4) ? 0 : x.n_cigar;
    }
    // both mates in one 8-byte nontemporal store per field: the 16 B/pair of records go out to
    // HBM during this kernel instead of staying dirty in L2/MALL for the next launch to flush
    typedef int i32x2 __attribute__((ext_vector_type(2)));
    __builtin_nontemporal_store(i32x2{o_flag[0], o_flag[1]}, reinterpret_cast<i32x2 *>(out.flag) + pp);
    __builtin_nontemporal_store(i32x2{o_pos[0], o_pos[1]}, reinterpret_cast<i32x2 *>(out.pos) + pp);
    __builtin_nontemporal_store(i32x2{o_score[0], o_score[1]}, reinterpret_cast<i32x2 *>(out.score) + pp);
    __builtin_nontemporal_store(i32x2{o_nc[0], o_nc[1]}, reinterpret_cast<i32x2 *>(out.n_cigar) + pp);
    if (TAILS) {  // split-read tails for the partner search (af_emit_tail, af_internal.h)
#pragma unroll
        for (int m = 0; m < 2; ++m)
            if (!(o_flag[m] & 0x4) && o_nc[m] == 2)
                af_emit_tail(tails, reads, stride, lens, 2 * pp + m, o_flag[m], out.cigar + (2 * pp + m) * AF_MAX_CIGAR);
    }
}

}  // namespace

#ifdef AF_K2_PROF
extern "C" int af_debug_k2_prof_enable(int64_t max_items) {
    int32_t *d = nullptr;
    if (hipMalloc(&d, sizeof(int32_t) * PROF_W * max_items) != hipSuccess) return -1;
    (void)hipMemset(d, 0, sizeof(int32_t) * PROF_W * max_items);
    return hipMemcpyToSymbol(HIP_SYMBOL(g_k2prof), &d, sizeof d) == hipSuccess ? PROF_W : -1;
}
extern "C" int af_debug_k2_prof_read(int32_t *host, int64_t n_items) {
    int32_t *d = nullptr;
    if (hipMemcpyFromSymbol(&d, HIP_SYMBOL(g_k2prof), sizeof d) != hipSuccess || !d) return -1;
    return hipMemcpy(host, d, sizeof(int32_t) * PROF_W * n_items, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

hipError_t af_launch_align(const DevIndex &ix, const uint8_t *reads, int64_t n_reads, int32_t stride,
                           const int32_t *lens, const af_params &p, const int32_t *cand, const int32_t *n_cand,
                           int32_t *heads, ReadRec *recs, uint32_t *cigar, uint8_t *zscratch, int32_t n_slots,
                           hipStream_t s) {
    (void)n_reads;
    const size_t zstride = (size_t)(AF_MAX_READ + 1) * 1024;
    const int cpl = (stride + 1 + 63) / 64;
    dim3 g(n_slots), b(64);
#define AF_GO(C) hipLaunchKernelGGL((k_align<C, false>), g, b, 0, s, ix, reads, stride, lens, p, cand, n_cand, heads, \
                                    recs, cigar, zscratch, zstride, nullptr, nullptr, 0)
    if (cpl <= 2) AF_GO(2);
    else if (cpl <= 3) AF_GO(3);
    else if (cpl <= 4) AF_GO(4);
    else AF_GO(AF_CPL);
#undef AF_GO
    return hipGetLastError();
}

hipError_t af_launch_place(const DevIndex &ix, const uint8_t *reads, const int32_t *n_queries, int32_t stride,
                           const int32_t *lens, const af_params &p, int32_t *heads, uint8_t *zscratch,
                           int32_t n_slots, af_hit *hits, int32_t *n_hits, int32_t max_hits, hipStream_t s) {
    const size_t zstride = (size_t)(AF_MAX_READ + 1) * 1024;
    const int cpl = (stride + 1 + 63) / 64;
    dim3 g(n_slots), b(64);
#define AF_GO(C) hipLaunchKernelGGL((k_align<C, true>), g, b, 0, s, ix, reads, stride, lens, p, nullptr, n_queries, \
                                    heads, nullptr, nullptr, zscratch, zstride, hits, n_hits, max_hits)
    if (cpl <= 2) AF_GO(2);
    else if (cpl <= 3) AF_GO(3);
    else if (cpl <= 4) AF_GO(4);
    else AF_GO(AF_CPL);
#undef AF_GO
    return hipGetLastError();
}

hipError_t af_launch_pairs(int64_t n_pairs, const int32_t *hits, const ReadRec *recs, af_aln_out out,
                           int32_t *ctrl, hipStream_t s, const uint8_t *reads, int32_t stride, const int32_t *lens,
                           const AfTails *tails) {
    const int bs = 256;
    const int64_t nb = n_pairs > 0 ? (n_pairs + bs - 1) / bs : 1;
    if (tails)
        hipLaunchKernelGGL(k_pairs<true>, dim3((unsigned)nb), dim3(bs), 0, s, n_pairs, hits, recs, out, ctrl, reads,
                           stride, lens, *tails);
    else
        hipLaunchKernelGGL(k_pairs<false>, dim3((unsigned)nb), dim3(bs), 0, s, n_pairs, hits, recs, out, ctrl,
                           nullptr, 0, nullptr, AfTails{});
    return hipGetLastError();
}
