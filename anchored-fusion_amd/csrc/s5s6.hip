// s5s6.hip -- the genome check of the split reads and the S6 queries, on the device.
//
// `del_too_many_reads` (functions.py:705-768) reads the SAM of `bwa mem -M genome split.fa`
// (fn:716) query by query -- records grouped by consecutive QNAME, the QNAME being
// `read$gene$POS$CIGAR` of the anchored record (fn:710-715) -- and drops a query when a genome
// record aligns it as one operation (fn:749-751) or a genome M straddles the end of an anchored M
// by more than 20 % of that M on both sides (fn:752-756).  The survivors are written as
// pseudo-SAM lines (fn:735, 760) that `Find_fine_block` (fn:506-528) turns into the S6 FASTA:
// deal_cigar's processed SEQ of each, ids = ordinals.  Both CIGARs go through `deal_cigar`
// (fn:656-702) first, the genome one with its first H read as S and, for a reverse record, its
// operations reversed with the running ends recomputed.
//
// k_s5_check: one thread per S5 query (the af_grec records of af_genome_align_se_device, the S2
// record of the read): keep[q] = the query starts a QNAME group and no record of the group is
// bad.  An order-preserving select (hipCUB) lists the survivors; k_s6_rows writes each one's
// processed SEQ (deal_cigar's D -> N insertions and I removals on the anchored CIGAR) as an S6
// query row, with its S5 query index.  Integer and byte work; the 20 % bounds are computed in
// double as Python computes them.
#include <hipcub/hipcub.hpp>

#include "af_internal.h"

namespace {

constexpr int NOPS = AF_MAX_CIGAR + 2;
struct NOp {
    int32_t end, len, op;  // deal_cigar's [end, length, op]; op in BAM codes (M0 I1 D2 N3 S4 H5 P6 =7 X8)
};

// parse (running ends) of BAM ops; the first H (in CIGAR string order) read as S when h_as_s
__host__ __device__ int parse_ops(const uint32_t *cig, int nc, bool h_as_s, NOp *o) {
    int e = 0;
    bool first_h = h_as_s;
    const int n = nc < AF_MAX_CIGAR ? nc : AF_MAX_CIGAR;
    for (int k = 0; k < n; ++k) {
        const int len = (int)(cig[k] >> 4);
        int op = (int)(cig[k] & 0xf);
        if (op == 5 && first_h) { op = 4; first_h = false; }
        e += len;
        o[k] = NOp{e, len, op};
    }
    return n;
}

__host__ __device__ __forceinline__ void del_at(NOp *o, int &n, int k) {
    for (int j = k; j < n - 1; ++j) o[j] = o[j + 1];
    --n;
}

// deal_cigar's operation list (functions.py:656-702; cigar.py `normalize`), ops only
__host__ __device__ int deal_ops(NOp *o, int n) {
    int k = 0;
    while (k < n) {
        const int op = o[k].op;
        if (op == 3 || op == 5 || op == 1) {
            for (int j = k + 1; j < n; ++j) o[j].end -= o[k].len;
            del_at(o, n, k);
        } else if (op == 2) {
            if (k + 1 < n) o[k + 1].len += o[k].len;
            del_at(o, n, k);
        } else {
            ++k;
        }
    }
    int m = 0;
    for (int k2 = 0; k2 < n; ++k2) {
        if (m > 0 && o[m - 1].op == 0 && o[k2].op == 0) {
            o[m - 1].end = o[k2].end;
            o[m - 1].len += o[k2].len;
        } else {
            o[m++] = o[k2];
        }
    }
    return m;
}

// fn:752-756 for one genome record against the anchored ops `bf` (nb)
__host__ __device__ bool record_bad(const af_grec &g, const NOp *bf, int nb) {
    NOp now[NOPS];
    const int flag = g.flag & 0xFFFF;
    const bool rev = flag > 15 && ((flag >> 4) & 1);
    int n = deal_ops(now, parse_ops(g.cigar, g.n_cigar, true, now));
    if (rev) {
        for (int a = 0, b = n - 1; a < b; ++a, --b) { const NOp t = now[a]; now[a] = now[b]; now[b] = t; }
        int run = 0;
        for (int k = 0; k < n; ++k) { run += now[k].len; now[k].end = run; }
    }
    if (n == 1) return true;
    if (n < 2) return false;
    for (int i = 0; i < nb; ++i) {
        if (bf[i].op != 0) continue;
        const double lo = (double)bf[i].end - (double)bf[i].len * 0.2;
        const double hi = (double)bf[i].end + (double)bf[i].len * 0.2;
        for (int k = 0; k < n; ++k)
            if (now[k].op == 0 && (double)(now[k].end - now[k].len) < lo && (double)now[k].end > hi) return true;
    }
    return false;
}

struct S5In {
    const af_grec *recs;
    const int32_t *n_rec;
    const int32_t *q_rows;  // the read row of each S5 query (S2 record index)
    const int32_t *flag, *pos, *n_cigar;
    const uint32_t *cigar;
    const uint8_t *cont;    // optional: cont[q] != 0 when query q continues the QNAME group of q - 1
};

// QNAME of query q: read name (the pair: row >> 1), gene, POS, CIGAR of the anchored record
__host__ __device__ bool same_qname(const S5In &in, int64_t a, int64_t b) {
    const int ra = in.q_rows[a], rb = in.q_rows[b];
    if ((ra >> 1) != (rb >> 1) || in.pos[ra] != in.pos[rb] || in.n_cigar[ra] != in.n_cigar[rb]) return false;
    const int nc = in.n_cigar[ra] < AF_MAX_CIGAR ? in.n_cigar[ra] : AF_MAX_CIGAR;
    for (int k = 0; k < nc; ++k)
        if (in.cigar[(int64_t)ra * AF_MAX_CIGAR + k] != in.cigar[(int64_t)rb * AF_MAX_CIGAR + k]) return false;
    return true;
}

// query u continues the group of u - 1: the caller's flags (a shard of a wider query list,
// whose neighbours in the global order are known to the caller), else the QNAMEs compared
__host__ __device__ bool continues(const S5In &in, int64_t u) {
    return in.cont ? in.cont[u] != 0 : same_qname(in, u - 1, u);
}

__host__ __device__ bool query_bad(const S5In &in, int64_t q, const NOp *bf, int nb) {
    const int nr = in.n_rec[q] < AF_G_MAX_REC ? in.n_rec[q] : AF_G_MAX_REC;
    for (int k = 0; k < nr; ++k)
        if (record_bad(in.recs[q * AF_G_MAX_REC + k], bf, nb)) return true;
    return false;
}

// keep flag of query q of n: it starts a QNAME group and no record of the group is bad
__host__ __device__ uint8_t s5_keep(const S5In &in, int64_t q, int64_t n) {
    if (q > 0 && continues(in, q)) return 0;
    const int r = in.q_rows[q];
    NOp bf[NOPS];
    const int nb = deal_ops(bf, parse_ops(in.cigar + (int64_t)r * AF_MAX_CIGAR, in.n_cigar[r], false, bf));
    bool bad = query_bad(in, q, bf, nb);
    for (int64_t u = q + 1; !bad && u < n && continues(in, u); ++u) bad = query_bad(in, u, bf, nb);
    return bad ? 0 : 1;
}

__global__ void k_s5_check(S5In in, int64_t n, uint8_t *__restrict__ keep) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n) return;
    keep[q] = s5_keep(in, q, n);
}

// Python slice index (negative counts from the end, clamped to [0, len])
__host__ __device__ __forceinline__ int py_idx(int i, int len) {
    if (i < 0) i += len;
    return i < 0 ? 0 : (i > len ? len : i);
}

// deal_cigar's processed SEQ of S5 query qi into `row` (out_stride bytes): the edits run in place
// on the row; bytes past out_stride are dropped (the BLAT kernel takes at most AF_MAX_READ
// bases).  Returns the row length; *over = a byte was dropped.
__host__ __device__ int s6_row(const S5In &in, int32_t qi, const uint8_t *q, int32_t q_stride, const int32_t *q_lens,
                               uint8_t *row, int32_t out_stride, bool *over_out) {
    const int r = in.q_rows[qi];
    int len = q_lens[qi] < q_stride ? q_lens[qi] : q_stride;
    if (len > out_stride) { len = out_stride; *over_out = true; }
    for (int j = 0; j < len; ++j) row[j] = q[(int64_t)qi * q_stride + j];
    NOp o[NOPS];
    int n_op = parse_ops(in.cigar + (int64_t)r * AF_MAX_CIGAR, in.n_cigar[r], false, o);
    bool over = false;
    int kk = 0;
    while (kk < n_op) {
        const int op = o[kk].op;
        if (op == 3 || op == 5 || op == 1) {
            // later ends move back first (so ops[-1] below is the shifted last op, as in Python)
            for (int j = kk + 1; j < n_op; ++j) o[j].end -= o[kk].len;
            if (op == 1) {  // seq = seq[:ops[k-1].end] + seq[end:]
                const int cut = py_idx(o[kk == 0 ? n_op - 1 : kk - 1].end, len);
                const int from = py_idx(o[kk].end, len);
                int nl = cut + (len - from);
                if (from >= cut) {
                    for (int j = 0; j < len - from; ++j) row[cut + j] = row[from + j];
                } else {  // overlapping slices repeat bases: seq[:cut] + seq[from:]
                    for (int j = len - from - 1; j >= 0; --j)
                        if (cut + j < out_stride) row[cut + j] = row[from + j];
                }
                if (nl > out_stride) { nl = out_stride; over = true; }
                len = nl;
            }
            del_at(o, n_op, kk);
        } else if (op == 2) {  // seq = seq[:ops[k-1].end] + 'N' * len + seq[ops[k-1].end:]
            const int ln = o[kk].len;
            const int at = py_idx(o[kk == 0 ? n_op - 1 : kk - 1].end, len);
            int nl = len + ln;
            if (nl > out_stride) { nl = out_stride; over = true; }
            for (int j = nl - 1; j >= at + ln; --j) row[j] = row[j - ln];
            for (int j = at; j < at + ln && j < nl; ++j) row[j] = 'N';
            len = nl;
            if (kk + 1 < n_op) o[kk + 1].len += ln;
            del_at(o, n_op, kk);
        } else {
            ++kk;
        }
    }
    if (over) *over_out = true;
    return len;
}

// S6 row k = survivor k (S5 query sel[k]); rows with dropped bytes are counted in *n_over and / or
// flagged in over_rows[k]
__global__ void k_s6_rows(S5In in, const uint8_t *__restrict__ q, int32_t q_stride, const int32_t *__restrict__ q_lens,
                          const int32_t *__restrict__ sel, const int64_t *__restrict__ n_sel, int64_t cap,
                          uint8_t *__restrict__ out, int32_t out_stride, int32_t *__restrict__ out_lens,
                          int32_t *__restrict__ out_src, int32_t *__restrict__ n_over, uint8_t *__restrict__ over_rows) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t n = *n_sel < cap ? *n_sel : cap;
    if (k >= n) return;
    const int32_t qi = sel[k];
    bool over = false;
    out_lens[k] = s6_row(in, qi, q, q_stride, q_lens, out + k * (int64_t)out_stride, out_stride, &over);
    out_src[k] = qi;
    if (over && n_over) atomicAdd(n_over, 1);
    if (over_rows) over_rows[k] = over ? 1 : 0;
}

// the QNAME-group leaders (fn:718-768 keeps at most a group's first query; no record is read)
__global__ void k_s5_lead(S5In in, int64_t n, uint8_t *__restrict__ keep) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n) return;
    keep[q] = (q == 0 || !continues(in, q)) ? 1 : 0;
}

// ---- the compaction of the leaders' S6 rows and BLAT results to the survivors ----------------------
// live[p] = pre row p's S5 query survived the check (0 past the row count)
__global__ void k_s6_live(const int32_t *__restrict__ src, const int32_t *__restrict__ n_pre, int64_t cap,
                          const uint8_t *__restrict__ keep, uint8_t *__restrict__ live) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= cap) return;
    const int64_t n = *n_pre < cap ? *n_pre : cap;
    live[p] = p < n ? keep[src[p]] : 0;
}
// the scan input of the live flags (0 past the row count)
__global__ void k_s6_pre_flags(const uint8_t *__restrict__ live, const int32_t *__restrict__ n_pre, int64_t cap,
                               int32_t *__restrict__ flag) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= cap) return;
    const int64_t n = *n_pre < cap ? *n_pre : cap;
    flag[p] = p < n ? (int32_t)live[p] : 0;
}

__device__ __forceinline__ void copy_words(int32_t *__restrict__ d, const int32_t *__restrict__ s, int n, int lane, int w) {
    for (int x = lane; x < n; x += w) d[x] = s[x];
}

constexpr int PSL_WORDS = (int)(sizeof(af_psl) / 4);
static_assert(sizeof(af_psl) % 4 == 0 && offsetof(af_psl, query) == 0, "af_psl words");

// one wave per pre row p (grid-stride): survivor k = idx[p] takes p's query row, length, S5 query,
// PSL rows (query field = k) and row count; its clipped flag and cap events are counted, and its
// rows the pre spill pool dropped (a full pool: its ROWS events) added to the out pool's count
__global__ void k_s6_compact(af_s6_set pre, af_s6_set out, const int32_t *__restrict__ flag,
                             const int32_t *__restrict__ idx, int32_t max_rows, int32_t *__restrict__ caps) {
    const int lane = threadIdx.x & 63;
    const int64_t waves = (int64_t)gridDim.x * (blockDim.x >> 6);
    const int64_t n = *pre.n < pre.cap ? *pre.n : pre.cap;
    const int qw = pre.stride / 4;
    for (int64_t p = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); p < n; p += waves) {
        if (!flag[p]) continue;
        const int64_t k = idx[p];
        if (k >= out.cap) continue;
        copy_words(reinterpret_cast<int32_t *>(out.q + k * out.stride), reinterpret_cast<const int32_t *>(pre.q + p * pre.stride),
                   qw, lane, 64);
        const int nr = pre.n_rows[p] < max_rows ? pre.n_rows[p] : max_rows;
        int32_t *dr = reinterpret_cast<int32_t *>(out.rows + k * max_rows);
        const int32_t *sr = reinterpret_cast<const int32_t *>(pre.rows + p * max_rows);
        for (int x = lane; x < nr * PSL_WORDS; x += 64) dr[x] = x % PSL_WORDS == 0 ? (int32_t)k : sr[x];  // af_psl.query = k
        if (lane == 0) {
            out.lens[k] = pre.lens[p];
            out.src[k] = pre.src[p];
            out.n_rows[k] = pre.n_rows[p];
            if (out.n_over && pre.over && pre.over[p]) atomicAdd(out.n_over, 1);
        }
        if (caps && pre.caps && lane < AF_BLAT_CAP_N) {
            const int32_t v = pre.caps[(int64_t)lane * pre.cap + p];
            if (v) atomicAdd(&caps[lane], v);
            if (v && lane == AF_BLAT_CAP_ROWS && out.spill_n && pre.spill_cap > 0) atomicAdd(out.spill_n, v);
        }
    }
}

// sflag[x] = spilled row x belongs to a survivor (0 past the pool's fill)
__global__ void k_s6_spill_flags(af_s6_set pre, const int32_t *__restrict__ flag, int32_t *__restrict__ sflag) {
    const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= pre.spill_cap) return;
    const int64_t n = *pre.spill_n < pre.spill_cap ? *pre.spill_n : pre.spill_cap;
    sflag[x] = x < n ? flag[pre.spill_query[x]] : 0;
}

// the survivors' spilled rows in pool order, their query renumbered; the counts
__global__ void k_s6_spill_copy(af_s6_set pre, af_s6_set out, const int32_t *__restrict__ flag,
                                const int32_t *__restrict__ idx, const int32_t *__restrict__ sflag,
                                const int32_t *__restrict__ sidx, int32_t *__restrict__ caps) {
    const int lane = threadIdx.x & 63;
    const int64_t waves = (int64_t)gridDim.x * (blockDim.x >> 6);
    const int64_t n = *pre.spill_n < pre.spill_cap ? *pre.spill_n : pre.spill_cap;
    for (int64_t x = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); x < n; x += waves) {
        if (!sflag[x]) continue;
        const int64_t j = sidx[x];
        const int32_t k = idx[pre.spill_query[x]];
        if (j >= out.spill_cap) {
            if (lane == 0 && caps) atomicAdd(&caps[AF_BLAT_CAP_ROWS], 1);
            continue;
        }
        int32_t *d = reinterpret_cast<int32_t *>(out.spill_rows + j);
        const int32_t *sr = reinterpret_cast<const int32_t *>(pre.spill_rows + x);
        for (int w = lane; w < PSL_WORDS; w += 64) d[w] = w == 0 ? k : sr[w];
        if (lane == 0) out.spill_query[j] = k;
    }
}

// *out.n = min(survivors, out.cap); *out.spill_n = the survivors' spilled rows in the pre pool (k_s6_compact
// adds those it dropped)
__global__ void k_s6_compact_counts(af_s6_set pre, af_s6_set out, const int32_t *__restrict__ flag,
                                    const int32_t *__restrict__ idx, const int32_t *__restrict__ sflag,
                                    const int32_t *__restrict__ sidx) {
    if (threadIdx.x != 0) return;
    const int64_t t = pre.cap > 0 ? (int64_t)idx[pre.cap - 1] + flag[pre.cap - 1] : 0;
    *out.n = (int32_t)(t < out.cap ? t : out.cap);
    if (out.spill_n) *out.spill_n = pre.spill_cap > 0 ? sidx[pre.spill_cap - 1] + sflag[pre.spill_cap - 1] : 0;
}

__global__ void k_s6_count(const int64_t *__restrict__ n_sel, int64_t cap, int32_t *__restrict__ n_out) {
    if (threadIdx.x == 0) {
        const int64_t v = *n_sel;
        *n_out = (int32_t)(v > cap ? cap : v);
    }
}

}  // namespace

// The per-query rules above compiled for the host, over host arrays (unit tests of the rules
// against the consumer-stage restatements on machines without a GPU; the product path is
// af_s5_filter_device).  keep[q] as k_s5_check writes it; rows[q] / out_lens[q] / over[q] =
// k_s6_rows' output for EVERY query q (survivor or not).
extern "C" int af_s5_rules_host(const af_grec *recs, const int32_t *n_rec, int64_t n, const int32_t *q_rows,
                                const int32_t *pos, const int32_t *n_cigar, const uint32_t *cigar, const uint8_t *cont,
                                const uint8_t *q, int32_t q_stride, const int32_t *q_lens, uint8_t *keep, uint8_t *rows,
                                int32_t out_stride, int32_t *out_lens, uint8_t *over) {
    if (n < 0 || (n > 0 && (!recs || !n_rec || !q_rows || !pos || !n_cigar || !cigar || !q || !q_lens || !keep ||
                            !rows || !out_lens || !over)) || q_stride <= 0 || out_stride <= 0)
        return AF_E_INVALID;
    const S5In in{recs, n_rec, q_rows, nullptr, pos, n_cigar, cigar, cont};
    for (int64_t k = 0; k < n; ++k) {
        keep[k] = s5_keep(in, k, n);
        bool o = false;
        out_lens[k] = s6_row(in, (int32_t)k, q, q_stride, q_lens, rows + k * (int64_t)out_stride, out_stride, &o);
        over[k] = o ? 1 : 0;
    }
    return AF_OK;
}

size_t af_s5_temp_bytes(int64_t n) {
    size_t b = 0;
    (void)hipcub::DeviceSelect::Flagged(nullptr, b, hipcub::CountingInputIterator<int32_t>(0), (const uint8_t *)nullptr,
                                        (int32_t *)nullptr, (int64_t *)nullptr, n);
    return b;
}

hipError_t af_launch_s5_filter(const af_grec *recs, const int32_t *n_rec, int64_t n, const uint8_t *q, int32_t q_stride,
                               const int32_t *q_lens, const int32_t *q_rows, const af_aln_out &s2, const uint8_t *cont,
                               int64_t cap,
                               uint8_t *out, int32_t out_stride, int32_t *out_lens, int32_t *out_src, int32_t *n_out,
                               int32_t *n_over, uint8_t *keep, int32_t *sel, int64_t *n_sel, void *temp,
                               size_t temp_bytes, hipStream_t s) {
    hipError_t e;
    if (n_over && (e = hipMemsetAsync(n_over, 0, sizeof(int32_t), s)) != hipSuccess) return e;
    const S5In in{recs, n_rec, q_rows, s2.flag, s2.pos, s2.n_cigar, s2.cigar, cont};
    if (n <= 0) {
        if ((e = hipMemsetAsync(n_sel, 0, sizeof(int64_t), s)) != hipSuccess) return e;
    } else {
        const int bs = 256;
        hipLaunchKernelGGL(k_s5_check, dim3((unsigned)((n + bs - 1) / bs)), dim3(bs), 0, s, in, n, keep);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        size_t tb = temp_bytes;
        if ((e = hipcub::DeviceSelect::Flagged(temp, tb, hipcub::CountingInputIterator<int32_t>(0), keep, sel, n_sel, n,
                                               s)) != hipSuccess)
            return e;
        hipLaunchKernelGGL(k_s6_rows, dim3((unsigned)((n + bs - 1) / bs)), dim3(bs), 0, s, in, q, q_stride, q_lens, sel,
                           n_sel, cap, out, out_stride, out_lens, out_src, n_over, (uint8_t *)nullptr);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_s6_count, dim3(1), dim3(64), 0, s, n_sel, cap, n_out);
    return hipGetLastError();
}

hipError_t af_launch_s6_queries(int64_t n, const uint8_t *q, int32_t q_stride, const int32_t *q_lens,
                                const int32_t *q_rows, const af_aln_out &s2, const uint8_t *cont, const af_s6_set &pre,
                                uint8_t *keep, int32_t *sel, int64_t *n_sel, void *temp, size_t temp_bytes,
                                hipStream_t s) {
    hipError_t e;
    const S5In in{nullptr, nullptr, q_rows, s2.flag, s2.pos, s2.n_cigar, s2.cigar, cont};
    if (n <= 0) {
        if ((e = hipMemsetAsync(n_sel, 0, sizeof(int64_t), s)) != hipSuccess) return e;
    } else {
        const int bs = 256;
        hipLaunchKernelGGL(k_s5_lead, dim3((unsigned)((n + bs - 1) / bs)), dim3(bs), 0, s, in, n, keep);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        size_t tb = temp_bytes;
        if ((e = hipcub::DeviceSelect::Flagged(temp, tb, hipcub::CountingInputIterator<int32_t>(0), keep, sel, n_sel, n,
                                               s)) != hipSuccess)
            return e;
        hipLaunchKernelGGL(k_s6_rows, dim3((unsigned)((n + bs - 1) / bs)), dim3(bs), 0, s, in, q, q_stride, q_lens, sel,
                           n_sel, pre.cap, pre.q, pre.stride, pre.lens, pre.src, (int32_t *)nullptr, pre.over);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_s6_count, dim3(1), dim3(64), 0, s, n_sel, pre.cap, pre.n);
    return hipGetLastError();
}

size_t af_s6_compact_temp_bytes(int64_t n) {
    size_t b = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, b, (const int32_t *)nullptr, (int32_t *)nullptr, n);
    return b;
}

hipError_t af_launch_s6_check(const af_grec *recs, const int32_t *n_rec, int64_t n, const int32_t *q_rows,
                              const af_aln_out &s2, const uint8_t *cont, const af_s6_set &pre, uint8_t *keep,
                              uint8_t *live, hipStream_t s) {
    const int bs = 256;
    if (n > 0) {
        const S5In in{recs, n_rec, q_rows, s2.flag, s2.pos, s2.n_cigar, s2.cigar, cont};
        hipLaunchKernelGGL(k_s5_check, dim3((unsigned)((n + bs - 1) / bs)), dim3(bs), 0, s, in, n, keep);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    if (pre.cap > 0)
        hipLaunchKernelGGL(k_s6_live, dim3((unsigned)((pre.cap + bs - 1) / bs)), dim3(bs), 0, s, pre.src, pre.n, pre.cap,
                           keep, live);
    return hipGetLastError();
}

hipError_t af_launch_s6_compact(const af_s6_set &pre, const uint8_t *live, const af_s6_set &out, int32_t max_rows,
                                int32_t *caps, int32_t *flag, int32_t *idx, int32_t *sflag, int32_t *sidx, void *temp,
                                size_t temp_bytes, hipStream_t s) {
    hipError_t e;
    const int bs = 256;
    if (out.n_over && (e = hipMemsetAsync(out.n_over, 0, sizeof(int32_t), s)) != hipSuccess) return e;
    // survivor flags and new indices of the pre rows and of the spilled rows, the counts, then the copies
    if (pre.cap > 0) {
        hipLaunchKernelGGL(k_s6_pre_flags, dim3((unsigned)((pre.cap + bs - 1) / bs)), dim3(bs), 0, s, live, pre.n,
                           pre.cap, flag);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        size_t tb = temp_bytes;
        if ((e = hipcub::DeviceScan::ExclusiveSum(temp, tb, flag, idx, pre.cap, s)) != hipSuccess) return e;
    }
    if (pre.spill_cap > 0) {
        hipLaunchKernelGGL(k_s6_spill_flags, dim3((unsigned)((pre.spill_cap + bs - 1) / bs)), dim3(bs), 0, s, pre, flag,
                           sflag);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        size_t tb = temp_bytes;
        if ((e = hipcub::DeviceScan::ExclusiveSum(temp, tb, sflag, sidx, pre.spill_cap, s)) != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_s6_compact_counts, dim3(1), dim3(64), 0, s, pre, out, flag, idx, sflag, sidx);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (pre.cap > 0) {
        hipLaunchKernelGGL(k_s6_compact, dim3(1024), dim3(bs), 0, s, pre, out, flag, idx, max_rows, caps);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if (pre.spill_cap > 0)
        hipLaunchKernelGGL(k_s6_spill_copy, dim3(256), dim3(bs), 0, s, pre, out, flag, idx, sflag, sidx, caps);
    return hipGetLastError();
}
