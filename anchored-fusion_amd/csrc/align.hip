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
#include "ksw_dp.h"

namespace {

#ifndef AF_K2_STATIC_PCT
#define AF_K2_STATIC_PCT 0  // share of candidates assigned round-robin (rest: per-XCD dequeue)
#endif
constexpr int MEMCAP = 64;   // == max allowed af_params.max_mems

// placement kernel state beside the DP slot (g_dp): MEM lists and regions
struct __attribute__((aligned(16))) AlnLds {
    uint64_t mem[MEMCAP];
    uint64_t smem[MEMCAP];
    int32_t regs[16][8];   // score, truesc, qb, qe, -, -, seedlen0, w
    int64_t rpos[16][2];   // rb, re of the regions (genome-scale references exceed 2^31)
};
__shared__ AlnLds g_aln;


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
    DpLds &L = g_dp;
    AlnLds &A = g_aln;
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
                    A.mem[slot] = ((uint64_t)(1023 - len) << 50) | ((uint64_t)qb << 40) | (uint64_t)rb;
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
                const uint64_t ka = A.mem[lane];
                int rank = 0;
                for (int b = 0; b < nm; ++b) rank += A.mem[b] < ka;
                A.smem[rank] = ka;
            }
            wave_sync();
            // ---- 3. seed extension ---------------------------------------------------
            int n_reg = 0;
            for (int si = 0; si < nm; ++si) {
                const uint64_t key = A.smem[si];
                const int slen = 1023 - (int)(key >> 50);
                const int sqb = (int)((key >> 40) & 1023);
                const int64_t srb = (int64_t)(key & 0xFFFFFFFFFFull);
                bool skip = false;
                for (int rr = 0; rr < n_reg; ++rr) {
                    const int *a = A.regs[rr];
                    const int aqb = a[2], aqe = a[3], asl = a[6], aw = a[7];
                    const int64_t arb = A.rpos[rr][0], are = A.rpos[rr][1];
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
                    int *a = A.regs[n_reg];
                    a[0] = a_score; a[1] = a_truesc; a[2] = a_qb; a[3] = a_qe;
                    a[4] = 0; a[5] = 0; a[6] = slen; a[7] = aw0 > aw1 ? aw0 : aw1;
                    A.rpos[n_reg][0] = a_rb; A.rpos[n_reg][1] = a_re;
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
                const int *a = A.regs[ri];
                const int a_score = a[0], a_truesc = a[1], aqb = a[2], aqe = a[3], awb = a[7];
                const int64_t arb = A.rpos[ri][0], are = A.rpos[ri][1];
                const bool is_rev = arb >= n;
                const int lq = aqe - aqb;
                const int tmpw = infer_bw(lq, (int)(are - arb), a_truesc, p.a, p.o_del, p.e_del);
                int w2 = infer_bw(lq, (int)(are - arb), a_truesc, p.a, p.o_ins, p.e_ins);
                w2 = w2 > tmpw ? w2 : tmpw;
                if (w2 > p.w) w2 = w2 < awb ? w2 : awb;
                int score = 0, last_sc = -(1 << 30), it = 0;
                do {
                    w2 = w2 < p.w << 2 ? w2 : p.w << 2;
                    score = gen_cigar_wave<CPL>(ix.D, ix.n, p, w2, lq, aqb, arb, are, L, zg, lane);
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
                    if (best < 0 || A.regs[rr][0] > A.regs[best][0]) best = rr;
                if (best >= 0 && A.regs[best][0] >= p.T) {
                    int mt_unused = 0, span_unused = 0;
                    int64_t pos64 = 0;
                    emit(best, cigar + r * AF_MAX_CIGAR, flag, pos64, out_score, out_nc, false, mt_unused,
                         span_unused);
                    out_pos = (int)pos64;  // hash (anchor) indexes only: < 2^31 (af_align_* check)
                }
            } else {
                // every region scoring >= T, best first (ties: region order), at most max_hits
                int32_t *order = reinterpret_cast<int32_t *>(A.mem);
                if (lane < n_reg) {
                    const int me = A.regs[lane][0];
                    int rank = 0;
                    for (int u = 0; u < n_reg; ++u) {
                        const int su = A.regs[u][0];
                        rank += su > me || (su == me && u < lane);
                    }
                    order[rank] = lane;
                }
                wave_sync();
                int nh = 0;
                for (int k = 0; k < n_reg && nh < max_hits; ++k) {
                    const int *a = A.regs[order[k]];
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
