// align_lane.hip -- K2, lane-per-read form (`bwa mem -M` at
// Anchored_Fusion.py:182).
//
// Each lane aligns one candidate read end to end: MEM search, seed sort, seed extension
// (ksw_extend2), band inference and global DP with traceback (ksw_global2, bwa_gen_cigar2).
// The per-read program is the one restated by oracle/af_oracle.c (align_read, find_mems,
// extend_seed, ext_dp, gen_cigar, global_dp); lanes of a wave run 64 reads side by side.
//
// Why lanes, not waves: the row-parallel form (align.hip) spends a serial chain of scalar
// band bookkeeping per DP row for ONE read; here every instruction serves 64 reads and the
// bookkeeping is vector work.
//
// Memory per wave:
//  * LDS (dynamic): query codes q[j][lane] (bytes) and the DP row eh[j][lane] (h, e as two
//    int16 halves of a dword), lane-interleaved so a wave's same-j accesses hit 64 banks;
//  * global scratch per lane: sorted MEM keys (64 x u64), regions (16 x 8 int), traceback
//    bytes (AF_LANE_Z) and a 64-entry CIGAR ring.
// int16 DP cells are exact for the parameter ranges check_params admits (see
// af_lane_params_ok); reads whose traceback matrix exceeds AF_LANE_Z bytes are handed to
// the wave kernel (align.hip) through the deferred list.
#include "af_internal.h"

namespace {

#ifdef AF_K2_PROF
__device__ int32_t *g_lane_prof = nullptr;  // per candidate: [0] r [1] load [2] mem [3] ext [4] cigar [5] trace
#define LPROF(...) __VA_ARGS__
#else
#define LPROF(...)
#endif

constexpr int NEG16 = -16384;  // -inf of the global DP in int16 cells (drift bounded by af_lane_params_ok)

struct Sc { int a, b, o_del, e_del, o_ins, e_ins; };

struct LaneCtx {
    uint8_t *q;        // LDS: q[j * 64 + lane]
    uint32_t *eh;      // LDS: eh[j * 64 + lane]
    int lane;
    __device__ __forceinline__ int qc(int j) const { return q[j * 64 + lane]; }
    __device__ __forceinline__ uint32_t ehg(int j) const { return eh[j * 64 + lane]; }
    __device__ __forceinline__ void ehs(int j, int h, int e) const {
        eh[j * 64 + lane] = (uint32_t)(h & 0xffff) | ((uint32_t)e << 16);
    }
};
__device__ __forceinline__ int eh_h(uint32_t v) { return (int)(int16_t)(v & 0xffff); }
__device__ __forceinline__ int eh_e(uint32_t v) { return (int)(int16_t)(v >> 16); }

__device__ __forceinline__ int sc_of(const Sc &p, int x, int y) {
    return (x > 3 || y > 3) ? -1 : (x == y ? p.a : -p.b);
}

__device__ __forceinline__ int cal_max_gap_l(const Sc &p, int w, int qlen) {
    int l_del = (int)((double)(qlen * p.a - p.o_del) / p.e_del + 1.);
    int l_ins = (int)((double)(qlen * p.a - p.o_ins) / p.e_ins + 1.);
    int l = l_del > l_ins ? l_del : l_ins;
    l = l > 1 ? l : 1;
    return l < w << 1 ? l : w << 1;
}

__device__ __forceinline__ int infer_bw_l(int l1, int l2, int score, int a, int q, int r) {
    if (l1 == l2 && l1 * a - score < (q + r - a) << 1) return 0;
    int w = (int)((double)((l1 < l2 ? l1 : l2) * a - score - q) / r + 2.);
    int d = l1 - l2 < 0 ? l2 - l1 : l1 - l2;
    return w < d ? d : w;
}

struct ExtOut { int max, qle, tle, gtle, gscore, max_off; };

// ksw_extend2 (oracle ext_dp) for one lane.  Query column j is q[qb0 + qdir * j]; target row i
// is D[t0 + tdir * i].  Adds the exact early exit of DESIGN.md §3 (checked every 8 rows).
__device__ ExtOut lane_ext(const LaneCtx &L, const uint8_t *__restrict__ D, int qlen, int qb0, int qdir, int tlen,
                           int64_t t0, int tdir, const Sc &p, int w, int end_bonus, int zdrop, int h0) {
    const int oe_del = p.o_del + p.e_del, oe_ins = p.o_ins + p.e_ins;
    {
        const int v1 = h0 > oe_ins ? h0 - oe_ins : 0;
        L.ehs(0, h0, 0);
        for (int j = 1; j <= qlen; ++j) {
            const int vj = v1 - (j - 1) * p.e_ins;
            L.ehs(j, j == 1 ? v1 : (vj > 0 ? vj : 0), 0);
        }
    }
    {
        int max_ins = (int)((double)(qlen * p.a + end_bonus - p.o_ins) / p.e_ins + 1.);
        max_ins = max_ins > 1 ? max_ins : 1;
        w = w < max_ins ? w : max_ins;
        int max_del = (int)((double)(qlen * p.a + end_bonus - p.o_del) / p.e_del + 1.);
        max_del = max_del > 1 ? max_del : 1;
        w = w < max_del ? w : max_del;
    }
    int mx = h0, max_i = -1, max_j = -1, max_ie = -1, gscore = -1, max_off = 0;
    int beg = 0, end = qlen;
    int ti_next = tlen > 0 ? D[t0] : 4;
    for (int i = 0; i < tlen; ++i) {
        const int ti = ti_next;
        if (i + 1 < tlen) ti_next = D[t0 + (int64_t)tdir * (i + 1)];
        if (beg < i - w) beg = i - w;
        if (end > i + w + 1) end = i + w + 1;
        if (end > qlen) end = qlen;
        int h1 = 0;
        if (beg == 0) {
            h1 = h0 - (p.o_del + p.e_del * (i + 1));
            if (h1 < 0) h1 = 0;
        }
        int f = 0, m = 0, mj = -1;
        int j = beg;
        if (beg < end) {
            uint32_t v = L.ehg(beg);
            int qv = L.qc(qb0 + qdir * beg);
            for (; j < end; ++j) {
                uint32_t vn = 0;
                int qn = 4;
                if (j + 1 < end) { vn = L.ehg(j + 1); qn = L.qc(qb0 + qdir * (j + 1)); }
                int M = eh_h(v), e = eh_e(v);
                M = M ? M + sc_of(p, ti, qv) : 0;
                int h = M > e ? M : e;
                h = h > f ? h : f;
                mj = m > h ? mj : j;
                m = m > h ? m : h;
                int t = M - oe_del;
                t = t > 0 ? t : 0;
                e -= p.e_del;
                e = e > t ? e : t;
                L.ehs(j, h1, e);
                h1 = h;
                t = M - oe_ins;
                t = t > 0 ? t : 0;
                f -= p.e_ins;
                f = f > t ? f : t;
                v = vn; qv = qn;
            }
        }
        L.ehs(end, h1, 0);
        if (j == qlen) {
            max_ie = gscore > h1 ? max_ie : i;
            gscore = gscore > h1 ? gscore : h1;
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
        for (j = beg; j < end && L.ehg(j) == 0u; ++j) {}
        beg = j;
        for (j = end; j >= beg && L.ehg(j) == 0u; --j) {}
        end = j + 2 < qlen ? j + 2 : qlen;
        if ((i & 7) == 7 && gscore > 0) {  // exact early exit
            int U = 0;
            for (int x = beg; x <= qlen; ++x) {
                const uint32_t vv = L.ehg(x);
                const int hv = eh_h(vv), ev = eh_e(vv);
                const int u = (hv > ev ? hv : ev) + (qlen - x) * p.a;
                U = U > u ? U : u;
            }
            if (U <= mx && U < gscore) break;
        }
    }
    ExtOut r;
    r.max = mx; r.qle = max_j + 1; r.tle = max_i + 1; r.gtle = max_ie + 1; r.gscore = gscore; r.max_off = max_off;
    return r;
}

// ksw_global2 + traceback (oracle global_dp) for one lane.  Query j = q[qb0 + qdir*j], target
// i = D[t0 + tdir*i].  z: this lane's traceback bytes (row-major, n_col per row).  The CIGAR is
// left in `ring` in reverse order; returns the op count through *n_ops.
__device__ int lane_global(const LaneCtx &L, const uint8_t *__restrict__ D, int qlen, int qb0, int qdir, int tlen,
                           int64_t t0, int tdir, const Sc &p, int w, uint8_t *__restrict__ z,
                           uint32_t *__restrict__ ring, int *n_ops LPROF(, int *prof_tb)) {
    const int oe_del = p.o_del + p.e_del, oe_ins = p.o_ins + p.e_ins;
    const int n_col = qlen < 2 * w + 1 ? qlen : 2 * w + 1;
    L.ehs(0, 0, NEG16);
    for (int j = 1; j <= qlen; ++j) L.ehs(j, j <= w ? -(p.o_ins + p.e_ins * j) : NEG16, NEG16);
    int ti_next = tlen > 0 ? D[t0] : 4;
    for (int i = 0; i < tlen; ++i) {
        const int ti = ti_next;
        if (i + 1 < tlen) ti_next = D[t0 + (int64_t)tdir * (i + 1)];
        const int beg = i > w ? i - w : 0;
        const int end = i + w + 1 < qlen ? i + w + 1 : qlen;
        int h1 = beg == 0 ? -(p.o_del + p.e_del * (i + 1)) : NEG16;
        int f = NEG16;
        uint8_t *zi = z + (size_t)i * n_col;
        uint32_t v = beg < end ? L.ehg(beg) : 0u;
        int qv = beg < end ? L.qc(qb0 + qdir * beg) : 4;
        uint32_t zw = 0;
        int zn = 0;
        for (int j = beg; j < end; ++j) {
            uint32_t vn = 0;
            int qn = 4;
            if (j + 1 < end) { vn = L.ehg(j + 1); qn = L.qc(qb0 + qdir * (j + 1)); }
            int m = eh_h(v), e = eh_e(v);
            m += sc_of(p, ti, qv);
            int d = m >= e ? 0 : 1;
            int h = m >= e ? m : e;
            d = h >= f ? d : 2;
            h = h >= f ? h : f;
            int t = m - oe_del;
            e -= p.e_del;
            d |= e > t ? 1 << 2 : 0;
            e = e > t ? e : t;
            L.ehs(j, h1, e);
            h1 = h;
            t = m - oe_ins;
            f -= p.e_ins;
            d |= f > t ? 2 << 4 : 0;
            f = f > t ? f : t;
            // pack 4 cells per dword store when the row slice is dword-aligned
            zw |= (uint32_t)d << (8 * zn);
            if (++zn == 4 || j + 1 == end) {
                uint8_t *dst = zi + (j + 1 - zn - beg);
                if (zn == 4 && (((uintptr_t)dst) & 3) == 0) *reinterpret_cast<uint32_t *>(dst) = zw;
                else for (int u = 0; u < zn; ++u) dst[u] = (uint8_t)(zw >> (8 * u));
                zw = 0; zn = 0;
            }
            v = vn; qv = qn;
        }
        L.ehs(end, h1, NEG16);
    }
    const int score = eh_h(L.ehg(qlen));
    LPROF(const int64_t tb0 = clock64();)
    // traceback from the last cell (serial per lane; one byte per step)
    int nc = 0, which = 0, cur_op = -1, cur_len = 0;
    auto push = [&](int op, int len) {
        if (op == cur_op) { cur_len += len; return; }
        if (cur_op >= 0) { ring[nc & 63] = (uint32_t)cur_len << 4 | (uint32_t)cur_op; ++nc; }
        cur_op = op; cur_len = len;
    };
    int i = tlen - 1;
    int k = (i + w + 1 < qlen ? i + w + 1 : qlen) - 1;
    while (i >= 0 && k >= 0) {
        which = z[(size_t)i * n_col + (k - (i > w ? i - w : 0))] >> (which << 1) & 3;
        if (which == 0) { push(0, 1); --i; --k; }
        else if (which == 1) { push(2, 1); --i; }
        else { push(1, 1); --k; }
    }
    if (i >= 0) push(2, i + 1);
    if (k >= 0) push(1, k + 1);
    push(-2, 1);  // flush
    *n_ops = nc;
    LPROF(if (g_lane_prof) *prof_tb += (int)(clock64() - tb0);)
    return score;
}

struct LaneScratch {
    uint64_t *mem;     // [64] sorted MEM keys ((1023-len)<<50 | qb<<40 | rb)
    int32_t *reg;      // [16][8] score, truesc, qb, qe, rb, re, seedlen0, w
    uint8_t *z;        // [AF_LANE_Z]
    uint32_t *ring;    // [64]
};

// 16 bases of the packed doubled reference starting at pos, plus its N mask (bit per base)
__device__ __forceinline__ void getD16l(const DevIndex &ix, int64_t pos, uint32_t &bits, uint32_t &nmask) {
    const int64_t wi = pos >> 4;
    const int sh = (int)(pos & 15) * 2;
    const uint32_t lo = ix.D2[wi], hi = ix.D2[wi + 1];
    bits = sh ? (lo >> sh) | (hi << (32 - sh)) : lo;
    const int64_t ni = pos >> 5;
    const int nsh = (int)(pos & 31);
    const uint32_t nlo = ix.Dn[ni], nhi = ix.Dn[ni + 1];
    nmask = (nsh ? (nlo >> nsh) | (nhi << (32 - nsh)) : nlo) & 0xFFFFu;
}

// One read, one lane (oracle align_read).  Returns false when the read must be deferred to
// the wave kernel (traceback matrix above AF_LANE_Z).
__device__ bool lane_align_read(const DevIndex &ix, const LaneCtx &L, const LaneScratch &S, int l, const af_params &P,
                                const Sc &p, ReadRec &rec, uint32_t *__restrict__ cig_out LPROF(, int *pr)) {
    const int64_t n = ix.n, n2 = 2 * ix.n;
    LPROF(int64_t pt = clock64();)
    rec.flag = 0x4; rec.pos = 0; rec.score = 0; rec.n_cigar = 0;
    // ---- MEMs (find_mems): every left-maximal exact match >= min_seed_len ----------------
    const uint32_t hm = (1u << ix.hbits) - 1u;
    const int max_mems = P.max_mems < 64 ? P.max_mems : 64;
    int nm = 0;
    bool overflow = false;
    uint32_t k = 0;
    int valid = 0;
    for (int x = 0; x < l && !overflow; ++x) {
        const int c = L.qc(x);
        valid = c < 4 ? valid + 1 : 0;
        k = (k >> 2) | ((uint32_t)(c & 3) << 30);
        if (x < AF_K - 1 || valid < AF_K) continue;
        const int qb = x - (AF_K - 1);
        uint32_t s = af_fmix(k) & hm;
        int cnt = 0, st = 0;
        for (;;) {
            const int4 e = ix.hslot[s];
            if (e.z == 0) break;
            if ((uint32_t)e.x == k) { cnt = e.z; st = e.y; break; }
            s = (s + 1) & hm;
        }
        if (cnt == 0 || cnt > P.max_occ) continue;
        const int qprev = qb > 0 ? L.qc(qb - 1) : 4;
        for (int o = 0; o < cnt; ++o) {
            const int64_t rb = ix.kpos[st + o];
            if (qb > 0 && rb != 0 && rb != n && qprev < 4 && qprev == ix.D[rb - 1]) continue;
            const int64_t lim = rb < n ? n : n2;
            int len = AF_K;
            for (;;) {
                const int qp = qb + len;
                const int64_t rp = rb + len;
                const int64_t room64 = min((int64_t)(l - qp), lim - rp);
                if (room64 <= 0) break;
                const int room = (int)min(room64, (int64_t)16);
                uint32_t qk = 0;
                int qn = 16;
                for (int u = 0; u < room; ++u) {
                    const int cq = L.qc(qp + u);
                    if (cq > 3 && qn == 16) qn = u;
                    qk |= (uint32_t)(cq & 3) << (2 * u);
                }
                uint32_t dk, dn;
                getD16l(ix, rp, dk, dn);
                const uint32_t xr = qk ^ dk;
                const int eq = xr ? (__builtin_ctz(xr) >> 1) : 16;
                const int dnf = dn ? __builtin_ctz(dn) : 16;
                const int step = min(min(eq, room), min(qn, dnf));
                len += step;
                if (step < 16) break;
            }
            if (len < P.min_seed_len) continue;
            if (nm >= max_mems) { overflow = true; break; }
            // insertion into the sorted key list (len desc, qb, rb)
            const uint64_t key = ((uint64_t)(1023 - len) << 50) | ((uint64_t)qb << 40) | (uint64_t)rb;
            int y = nm;
            while (y > 0 && S.mem[y - 1] > key) { S.mem[y] = S.mem[y - 1]; --y; }
            S.mem[y] = key;
            ++nm;
        }
    }
    LPROF(pr[2] = (int)(clock64() - pt); pt = clock64();)
    if (overflow) { rec.flag = 0x4 | AF_FLAG_MEM_OVERFLOW; return true; }
    // ---- seeds in order -> regions (mem_chain2aln for single-seed chains) ------------------
    const int max_ext = P.max_ext < 16 ? P.max_ext : 16;
    int n_reg = 0;
    for (int si = 0; si < nm; ++si) {
        const uint64_t key = S.mem[si];
        const int slen = 1023 - (int)(key >> 50);
        const int sqb = (int)((key >> 40) & 1023);
        const int64_t srb = (int64_t)(key & 0xFFFFFFFFFFull);
        bool skip = false;
        for (int rr = 0; rr < n_reg && !skip; ++rr) {
            const int *a = S.reg + rr * 8;
            const int aqb = a[2], aqe = a[3], arb = a[4], are = a[5], asl = a[6], aw = a[7];
            if (srb < arb || srb + slen > are || sqb < aqb || sqb + slen > aqe) continue;
            if (10 * (slen - asl) > l) continue;
            int qd = sqb - aqb, rd = (int)(srb - arb);
            int mg = cal_max_gap_l(p, P.w, qd < rd ? qd : rd);
            int ww = mg < aw ? mg : aw;
            if (qd - rd < ww && rd - qd < ww) { skip = true; break; }
            qd = aqe - (sqb + slen); rd = (int)(are - (srb + slen));
            mg = cal_max_gap_l(p, P.w, qd < rd ? qd : rd);
            ww = mg < aw ? mg : aw;
            if (qd - rd < ww && rd - qd < ww) skip = true;
        }
        if (skip) continue;
        if (n_reg >= max_ext) break;
        const int64_t bq = srb - (sqb + cal_max_gap_l(p, P.w, sqb));
        const int rem = l - sqb - slen;
        const int64_t eq = srb + slen + (rem + cal_max_gap_l(p, P.w, rem));
        int64_t rmax0 = bq > 0 ? bq : 0, rmax1 = eq < n2 ? eq : n2;
        if (rmax0 < n && n < rmax1) {
            if (srb < n) rmax1 = n; else rmax0 = n;
        }
        int a_score = 0, a_truesc = 0, a_qb = 0, a_qe = 0;
        int64_t a_rb = 0, a_re = 0;
        int aw0 = P.w, aw1 = P.w;
        if (sqb) {
            const int tmp = (int)(srb - rmax0);
            ExtOut er;
            for (int it = 0; it < 2; ++it) {
                const int prev = a_score;
                aw0 = P.w << it;
                // reversed query (q[sqb-1-j]) against the reversed target (D[srb-1-i])
                er = lane_ext(L, ix.D, sqb, sqb - 1, -1, tmp, srb - 1, -1, p, aw0, P.pen_clip5, P.zdrop, slen * p.a);
                a_score = er.max;
                if (a_score == prev || er.max_off < (aw0 >> 1) + (aw0 >> 2)) break;
            }
            if (er.gscore <= 0 || er.gscore <= a_score - P.pen_clip5) {
                a_qb = sqb - er.qle; a_rb = srb - er.tle; a_truesc = a_score;
            } else {
                a_qb = 0; a_rb = srb - er.gtle; a_truesc = er.gscore;
            }
        } else {
            a_score = a_truesc = slen * p.a; a_qb = 0; a_rb = srb;
        }
        if (sqb + slen != l) {
            const int qe = sqb + slen;
            const int re = (int)(srb + slen - rmax0);
            const int sc0 = a_score;
            const int tl = (int)(rmax1 - rmax0 - re);
            ExtOut er;
            for (int it = 0; it < 2; ++it) {
                const int prev = a_score;
                aw1 = P.w << it;
                er = lane_ext(L, ix.D, l - qe, qe, 1, tl, rmax0 + re, 1, p, aw1, P.pen_clip3, P.zdrop, sc0);
                a_score = er.max;
                if (a_score == prev || er.max_off < (aw1 >> 1) + (aw1 >> 2)) break;
            }
            if (er.gscore <= 0 || er.gscore <= a_score - P.pen_clip3) {
                a_qe = qe + er.qle; a_re = rmax0 + re + er.tle; a_truesc += a_score - sc0;
            } else {
                a_qe = l; a_re = rmax0 + re + er.gtle; a_truesc += er.gscore - sc0;
            }
        } else {
            a_qe = l; a_re = srb + slen;
        }
        int *a = S.reg + n_reg * 8;
        a[0] = a_score; a[1] = a_truesc; a[2] = a_qb; a[3] = a_qe;
        a[4] = (int)a_rb; a[5] = (int)a_re; a[6] = slen; a[7] = aw0 > aw1 ? aw0 : aw1;
        ++n_reg;
    }
    LPROF(pr[3] = (int)(clock64() - pt); pt = clock64();)
    int best = -1, best_sc = 0;
    for (int rr = 0; rr < n_reg; ++rr) {
        const int s0 = S.reg[rr * 8];
        if (best < 0 || s0 > best_sc) { best = rr; best_sc = s0; }
    }
    if (best < 0 || best_sc < P.T) return true;
    // ---- CIGAR (bwa_gen_cigar2 with the band retry loop) ------------------------------------
    const int *a = S.reg + best * 8;
    const int a_score = a[0], a_truesc = a[1], aqb = a[2], aqe = a[3], awb = a[7];
    const int64_t arb = a[4], are = a[5];
    const bool is_rev = arb >= n;
    const int lq = aqe - aqb, rlen = (int)(are - arb);
    const int tmpw = infer_bw_l(lq, rlen, a_truesc, p.a, p.o_del, p.e_del);
    int w2 = infer_bw_l(lq, rlen, a_truesc, p.a, p.o_ins, p.e_ins);
    w2 = w2 > tmpw ? w2 : tmpw;
    if (w2 > P.w) w2 = w2 < awb ? w2 : awb;
    // forward-reference orientation: reverse hits walk both sequences backwards
    const int qb0 = is_rev ? aqe - 1 : aqb, qdir = is_rev ? -1 : 1;
    const int64_t t0 = is_rev ? are - 1 : arb;
    const int tdir = is_rev ? -1 : 1;
    int score = 0, last_sc = -(1 << 30), it = 0, nc = 0;
    do {
        w2 = w2 < P.w << 2 ? w2 : P.w << 2;
        if (lq == rlen && w2 == 0) {
            score = 0;
            for (int x = 0; x < lq; ++x) score += sc_of(p, ix.D[t0 + (int64_t)tdir * x], L.qc(qb0 + qdir * x));
            S.ring[0] = (uint32_t)lq << 4;
            nc = 1;
        } else {
            int max_ins = (int)((double)(((lq + 1) >> 1) * p.a - p.o_ins) / p.e_ins + 1.);
            int max_del = (int)((double)(((lq + 1) >> 1) * p.a - p.o_del) / p.e_del + 1.);
            int max_gap = max_ins > max_del ? max_ins : max_del;
            max_gap = max_gap > 1 ? max_gap : 1;
            const int d = rlen - lq < 0 ? lq - rlen : rlen - lq;
            int w = (max_gap + d + 1) >> 1;
            w = w < w2 ? w : w2;
            const int min_w = d + 3;
            w = w > min_w ? w : min_w;
            const int n_col = lq < 2 * w + 1 ? lq : 2 * w + 1;
            if ((int64_t)n_col * rlen > AF_LANE_Z) return false;  // defer to the wave kernel
            score = lane_global(L, ix.D, lq, qb0, qdir, rlen, t0, tdir, p, w, S.z, S.ring, &nc LPROF(, &pr[5]));
        }
        if (score == last_sc || w2 == P.w << 2) break;
        last_sc = score;
        w2 <<= 1;
    } while (++it < 3 && score < a_truesc - p.a);
    LPROF(pr[4] = (int)(clock64() - pt);)
    // ---- assemble (ring holds the ops in reverse order) -----------------------------------
    const int ncap = nc < AF_MAX_CIGAR ? nc : AF_MAX_CIGAR;
    bool of = nc > AF_MAX_CIGAR;
    int64_t pos = is_rev ? n2 - are : arb;
    int xs = 0, xe = ncap;
    if (ncap > 0) {
        const uint32_t first = S.ring[(nc - 1) & 63];
        const uint32_t last = S.ring[(nc - ncap) & 63];
        if ((first & 0xf) == 2) { pos += first >> 4; xs = 1; }
        else if ((last & 0xf) == 2) xe = ncap - 1;
    }
    const int clip5 = is_rev ? l - aqe : aqb;
    const int clip3 = is_rev ? aqb : l - aqe;
    int nf = 0;
    if (clip5) cig_out[nf++] = (uint32_t)clip5 << 4 | 4;
    for (int x = xs; x < xe; ++x) {
        if (nf < AF_MAX_CIGAR) cig_out[nf] = S.ring[(nc - 1 - x) & 63];
        ++nf;
    }
    if (clip3) {
        if (nf < AF_MAX_CIGAR) cig_out[nf] = (uint32_t)clip3 << 4 | 4;
        ++nf;
    }
    if (nf > AF_MAX_CIGAR) { of = true; nf = AF_MAX_CIGAR; }
    rec.flag = (is_rev ? 0x10 : 0) | (of ? AF_FLAG_CIGAR_OVERFLOW : 0);
    rec.pos = (int)pos;
    rec.score = a_score;
    rec.n_cigar = nf;
    return true;
}

__global__ __launch_bounds__(64) void k_align_lane(DevIndex ix, const uint8_t *__restrict__ reads, int32_t stride,
                                                  const int32_t *__restrict__ lens, af_params P,
                                                  const int32_t *__restrict__ cand,
                                                  const int32_t *__restrict__ n_cand, int32_t *__restrict__ heads,
                                                  ReadRec *__restrict__ recs, uint32_t *__restrict__ cigar,
                                                  uint8_t *__restrict__ scratch, int32_t *__restrict__ defer,
                                                  int32_t *__restrict__ n_defer) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int lane = threadIdx.x;
    LaneCtx L{lds, reinterpret_cast<uint32_t *>(lds + (size_t)stride * 64), lane};
    const int64_t gl = (int64_t)blockIdx.x * 64 + lane;
    uint8_t *sb = scratch + gl * AF_LANE_SCRATCH;
    LaneScratch S{reinterpret_cast<uint64_t *>(sb), reinterpret_cast<int32_t *>(sb + 512), sb + 1024,
                  reinterpret_cast<uint32_t *>(sb + 1024 + AF_LANE_Z)};
    const Sc p{P.a, P.b, P.o_del, P.e_del, P.o_ins, P.e_ins};
    const int ncand = *n_cand;
    const int nchunks = (ncand + 63) / 64;
    int head = (int)(blockIdx.x & 7), heads_left = 8;
    for (;;) {
        // one dequeue per wave: chunk c of head x covers candidates [(8c + x) * 64, +64)
        int chunk = -1;
        while (heads_left > 0) {
            int v = 0;
            if (lane == 0) v = atomicAdd(&heads[AF_HEAD_STRIDE * head], 1);
            v = __builtin_amdgcn_readfirstlane(v);
            const int64_t c = 8 * (int64_t)v + head;
            if (c < nchunks) { chunk = (int)c; break; }
            head = (head + 1) & 7;
            --heads_left;
        }
        if (chunk < 0) break;
        const int item = chunk * 64 + lane;
        if (item < ncand) {
            const int64_t r = cand[item];
            int l = lens ? lens[r] : stride;
            if (l > stride) l = stride;
            const uint8_t *rd = reads + r * (int64_t)stride;
            LPROF(int pr[8] = {0, 0, 0, 0, 0, 0, 0, 0}; const int64_t pl0 = clock64();)
            for (int x = 0; x < l; ++x) {
                const uint8_t c = rd[x];
                uint8_t v = 4;
                switch (c) {
                case 'A': case 'a': v = 0; break;
                case 'C': case 'c': v = 1; break;
                case 'G': case 'g': v = 2; break;
                case 'T': case 't': v = 3; break;
                default: v = 4;
                }
                lds[x * 64 + lane] = v;
            }
            LPROF(pr[1] = (int)(clock64() - pl0); pr[0] = (int)r;)
            ReadRec rec;
            const bool done = lane_align_read(ix, L, S, l, P, p, rec, cigar + r * AF_MAX_CIGAR LPROF(, pr));
            LPROF(if (g_lane_prof) { for (int u = 0; u < 8; ++u) g_lane_prof[(int64_t)item * 8 + u] = pr[u]; })
            if (done) {
                recs[r] = rec;
            } else {
                const int slot = atomicAdd(n_defer, 1);
                defer[slot] = (int32_t)r;
            }
        }
    }
}

}  // namespace

#ifdef AF_K2_PROF
extern "C" int af_debug_lane_prof_enable(int64_t max_items) {
    int32_t *d = nullptr;
    if (hipMalloc(&d, sizeof(int32_t) * 8 * max_items) != hipSuccess) return -1;
    (void)hipMemset(d, 0, sizeof(int32_t) * 8 * max_items);
    return hipMemcpyToSymbol(HIP_SYMBOL(g_lane_prof), &d, sizeof d) == hipSuccess ? 8 : -1;
}
extern "C" int af_debug_lane_prof_read(int32_t *host, int64_t n_items) {
    int32_t *d = nullptr;
    if (hipMemcpyFromSymbol(&d, HIP_SYMBOL(g_lane_prof), sizeof d) != hipSuccess || !d) return -1;
    return hipMemcpy(host, d, sizeof(int32_t) * 8 * n_items, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

size_t af_align_lane_lds(int32_t stride) { return (size_t)stride * 64 + (size_t)(stride + 1) * 64 * 4; }

bool af_lane_params_ok(const af_params &p, int32_t stride) {
    // int16 DP cells must reproduce the int32 recurrences exactly:
    //  * extension scores stay below h0 + qlen*a <= 2*stride*a;
    //  * global DP: a -inf-derived cell falls by at most b per row along a diagonal and by
    //    e per column, over R <= stride + 4w rows (cal_max_gap <= 2w per side) and C <= stride
    //    columns; it rises by at most a + e per step and must stay below every real value
    //    (>= -(o + e*(R + C))).  NEG16 = -16384 leaves room for both.
    const int64_t R = (int64_t)stride + 4 * (int64_t)p.w, C = stride;
    const int64_t e = p.e_del > p.e_ins ? p.e_del : p.e_ins;
    const int64_t fall = R * p.b + C * e + p.b + p.o_del + p.e_del + p.o_ins + p.e_ins;
    const int64_t rise = (R + C) * (p.a + e) + p.o_del + p.o_ins;
    return (int64_t)2 * stride * p.a < 15000 && fall < 15000 && rise < 15000;
}

hipError_t af_launch_align_lane(const DevIndex &ix, const uint8_t *reads, int32_t stride, const int32_t *lens,
                                const af_params &p, const int32_t *cand, const int32_t *n_cand, int32_t *heads,
                                ReadRec *recs, uint32_t *cigar, uint8_t *scratch, int32_t n_waves, int32_t *defer,
                                int32_t *n_defer, hipStream_t s) {
    const size_t lds = af_align_lane_lds(stride);
    static bool attr_done = false;
    if (!attr_done) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&k_align_lane),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return e;
        attr_done = true;
    }
    hipLaunchKernelGGL(k_align_lane, dim3((unsigned)n_waves), dim3(64), lds, s, ix, reads, stride, lens, p, cand,
                       n_cand, heads, recs, cigar, scratch, defer, n_defer);
    return hipGetLastError();
}
