// api.hip -- C-ABI of libafgpu.so (include/afgpu.h): contexts, anchor index build and the
// align entry points that replace `bwa index` / `bwa mem -M` (Anchored_Fusion.py:172, 182).
#include "af_internal.h"

#include <cstdlib>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <vector>

struct af_ctx {
    int device = 0;
    int n_cu = 0;
    int n_slots = 0;
    std::string err;
    // scratch (device)
    int32_t *ctrl = nullptr;   // af_internal.h: candidate counts (2 epochs) + K2 dequeue heads
    int64_t epoch = 0;         // seed-filter calls so far; the last call used count slot (epoch - 1) & 1
    int32_t *cand = nullptr;
    uint32_t *d_packed = nullptr;  // af_align_pairs: the candidates' CIGAR rows, gathered for one D2H
    int64_t cap_packed = 0;
    int64_t cap_reads = 0;
    uint8_t *zscratch = nullptr;
    uint8_t *bscratch = nullptr;  // k_blat: AF_BLAT_SLOT_BYTES per resident wave (blat_slots)
    int blat_slots = 0;
    void *blat_ord_work = nullptr;  // k_blat's cost-ordered schedule (af_launch_blat_order)
    int32_t *blat_order = nullptr;
    int64_t blat_ord_cap = 0;
    int32_t *blat_caps = nullptr;   // AF_BLAT_CAP_N counters, cumulative until af_blat_caps resets them
    BlatSpill blat_spill;           // af_blat_spill's pool (caller-owned device buffers)
    int32_t *blat_qcaps = nullptr;  // af_blat_query_caps' per-query counters (caller-owned), their query capacity
    int64_t blat_qcap = 0;
    BlatHeavy blat_hv;              // the deferred strands' table
    int32_t blat_heavy_min = AF_BLAT_HEAVY_CLUMPS;
    BlatLaunch blat_pending;        // af_blat_device_begin's search, finished by af_blat_device_end
    bool blat_open = false;
    af_psl *blat_stage = nullptr;   // per (query, strand) rows before k_blat_merge
    int32_t *blat_stage_n = nullptr;
    int64_t blat_stage_rows = 0, blat_stage_items = 0;
    // S2 (bwa mem paired-end) scratch, s2.hip
    S2Reg *s2_pool = nullptr;
    int64_t s2_pool_cap = 0;
    int2 *s2_rmap = nullptr;
    int32_t *s2_plist = nullptr, *s2_ghist = nullptr;
    int64_t s2_ghist_ints = 0;
    int64_t *s2_scan = nullptr;
    void *s2_plan = nullptr;
    int64_t s2_cap_pairs = 0;
    int32_t *s2_nchunks = nullptr;
    S2Pes *s2_pes = nullptr;
    int64_t *s2_cstart = nullptr;
    int32_t s2_max_chunks = 0;
    // S3 (s3.hip)
    uint64_t *s3_keys = nullptr;
    void *s3_temp = nullptr;
    int64_t s3_cap = 0;
    size_t s3_temp_bytes = 0;
    int64_t *s3_counts = nullptr;
    int32_t *g_sel = nullptr;   // af_gather_reads_device: selected rows, their count, select scratch
    int64_t *g_sel_n = nullptr;
    void *g_temp = nullptr;
    int64_t g_cap = 0;
    size_t g_temp_bytes = 0;
    // host-API staging (device)
    uint8_t *d_reads = nullptr;
    int64_t cap_bytes = 0;
    int32_t *d_lens = nullptr;
    int32_t *d_flag = nullptr, *d_pos = nullptr, *d_score = nullptr, *d_ncig = nullptr, *d_hits = nullptr;
    uint32_t *d_cigar = nullptr;
    int64_t cap_out = 0;
    hipStream_t stream = nullptr;
    // the genome calls S4 / S5 (bwa_genome.hip): per-lane / per-wave scratch, per-call pools
    uint8_t *g1_scr = nullptr, *g2_scr = nullptr;
    int g1_threads = 0, g2_waves = 0;
    // the paired-end records beside the single-end ones (af_genome_align_pe_se_device): their own
    // per-wave scratch, and the event that orders them after the shared seed / region kernels
    uint8_t *g2_scr_pe = nullptr, *zscratch_pe = nullptr;
    hipEvent_t g_ev = nullptr;
    // G2's heavy-read pools (GHeavy) and the kept-chain count from which a read is heavy
    GHeavy g_hv{};
    int32_t g_heavy_min = AF_G_HEAVY_CHAINS;
    GPeSpec g_pe{};
    int32_t g_pe_min = AF_G_PE_SPEC_WINDOWS;
    GPeSpec s2_sp{};
    int32_t s2_sp_min = AF_S2_SPEC_WINDOWS;
    int32_t g1_max_ext = AF_G1_HEAVY_EXT;
    bool g1_ext_env = false;        // AF_G1_HEAVY_EXT given: the hand-off threshold is fixed
    // G2 takes the reads with at least this many seeds first (env AF_G2_FIRST_OCC; 0: read order)
    int32_t g2_first_occ = AF_G2_FIRST_OCC;
    int32_t *g2_list = nullptr;
    uint8_t *g2_flag = nullptr;
    int64_t *g1_hv = nullptr;       // G1's heavy-read list (ensure_genome_pools)
    GIv *g_iv = nullptr;
    GReg *g_reg = nullptr;
    int64_t g_iv_cap = 0, g_reg_cap = 0, g_cap_reads = 0;
    unsigned long long *g_iv_fill = nullptr;
    int32_t *g_reg_fill = nullptr, *g_stats = nullptr, *g_iv_n = nullptr, *g_reg_off = nullptr, *g_reg_n = nullptr;
    int64_t *g_iv_off = nullptr;
    int32_t *g_ghist = nullptr, *g_nchunks = nullptr;
    int64_t g_ghist_ints = 0, *g_cstart = nullptr, *g_scan = nullptr, g_scan_cap = 0;
    S2Pes *g_pes = nullptr;
    int32_t g_max_chunks = 0;
    af_grec *g_recs = nullptr;      // host-buffer API staging
    int32_t *g_nrec = nullptr, *g_hlens = nullptr;
    uint8_t *g_hreads = nullptr;
    int64_t g_cap_recs = 0, g_cap_hbytes = 0;
    // the S5 genome check + S6 queries (s5s6.hip)
    uint8_t *s5_keep = nullptr;
    int32_t *s5_sel = nullptr;
    int64_t *s5_nsel = nullptr;
    void *s5_temp = nullptr;
    size_t s5_temp_bytes = 0;
    int64_t s5_cap = 0;
    // af_s6_compact_device: the pre rows' survivor flags and new indices, the spill pool's, scan scratch
    int32_t *s6_flag = nullptr, *s6_idx = nullptr, *s6_sflag = nullptr, *s6_sidx = nullptr;
    void *s6_temp = nullptr;
    size_t s6_temp_bytes = 0;
    int64_t s6_cap = 0, s6_spill_cap = 0;
};

struct af_genome {
    af_ctx *ctx = nullptr;
    DevGenome dev{};
};

struct af_index {
    af_ctx *ctx = nullptr;
    DevIndex dev{};
    std::vector<uint32_t> bloom_host;
    // S2: the bwa text of the anchor (built with the index), its suffix ranks and 16-mer hash
    // (built on first use by an af_align_* call)
    std::vector<uint8_t> text;
    DevText s2{};
    bool s2_ready = false;
    DevTile tile{};        // BLAT tile index (af_tile_index_build*), else unused
    bool is_tile = false;
    void *allocs[24] = {};
    int n_allocs = 0;
};

namespace {

inline void af_free(void *p) {
    if (p) (void)hipFree(p);
}

int fail(af_ctx *c, int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (c) c->err = buf;
    return code;
}

#define HIPCHK(ctx, expr)                                                                       \
    do {                                                                                        \
        hipError_t _e = (expr);                                                                 \
        if (_e != hipSuccess) return fail(ctx, AF_E_HIP, "%s: %s", #expr, hipGetErrorString(_e)); \
    } while (0)

// CIGAR rows of the reads of the listed pairs (the only rows the pair kernel writes), row i =
// read (i & 1) of pair plist[i >> 1], packed for one device-to-host copy
__global__ void k_gather_cigar(const int32_t *__restrict__ plist, int64_t n, const uint32_t *__restrict__ cigar,
                               uint32_t *__restrict__ packed) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n * (AF_MAX_CIGAR / 4);
         t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = t / (AF_MAX_CIGAR / 4), w = t % (AF_MAX_CIGAR / 4);
        const int64_t r = 2 * (int64_t)plist[i >> 1] + (i & 1);
        reinterpret_cast<uint4 *>(packed)[t] = reinterpret_cast<const uint4 *>(cigar + r * AF_MAX_CIGAR)[w];
    }
}

inline uint8_t nt4(uint8_t c) {
    switch (c) {
    case 'A': case 'a': return 0;
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'T': case 't': return 3;
    default: return 4;
    }
}

// srand48(11) / lrand48() of the POSIX drand48 family (glibc): bns_fasta2bntseq replaces every
// ambiguous base of the reference by lrand48() & 3 after srand48(bns->seed = 11)
struct Rand48 {
    uint64_t x;
    explicit Rand48(long seed) : x(((uint64_t)(uint32_t)seed << 16) | 0x330Eu) {}
    long next() {
        x = (0x5DEECE66DULL * x + 0xBULL) & ((1ULL << 48) - 1);
        return (long)(x >> 17);
    }
};

// the bwa text of a one-contig reference: forward pac (N substituted) ++ its reverse complement
std::vector<uint8_t> bwa_text(const char *seq, int64_t n) {
    std::vector<uint8_t> T((size_t)(2 * n));
    Rand48 r(11);
    for (int64_t i = 0; i < n; ++i) {
        int c = nt4((uint8_t)seq[i]);
        if (c >= 4) c = (int)(r.next() & 3);
        T[i] = (uint8_t)c;
        T[2 * n - 1 - i] = (uint8_t)(3 - c);
    }
    return T;
}

// suffix ranks of T (a suffix that ends first sorts first: bwa's '$'), prefix doubling
std::vector<int32_t> suffix_ranks(const std::vector<uint8_t> &T) {
    const int64_t N = (int64_t)T.size();
    std::vector<int64_t> rk(N), tmp(N);
    std::vector<int32_t> idx(N);
    for (int64_t i = 0; i < N; ++i) { rk[i] = T[i]; idx[i] = (int32_t)i; }
    for (int64_t h = 1;; h <<= 1) {
        auto key2 = [&](int32_t i) { return i + h < N ? rk[i + h] : (int64_t)-1; };
        std::sort(idx.begin(), idx.end(), [&](int32_t a, int32_t b) {
            if (rk[a] != rk[b]) return rk[a] < rk[b];
            return key2(a) < key2(b);
        });
        int64_t r = 0;
        for (int64_t j = 0; j < N; ++j) {
            if (j > 0 && (rk[idx[j]] != rk[idx[j - 1]] || key2(idx[j]) != key2(idx[j - 1]))) ++r;
            tmp[idx[j]] = r;
        }
        rk.swap(tmp);
        if (r == N - 1 || h >= N) break;
    }
    std::vector<int32_t> out(N);
    for (int64_t i = 0; i < N; ++i) out[i] = (int32_t)rk[i];
    return out;
}

template <class T>
int dev_upload(af_ctx *ctx, af_index *ix, const std::vector<T> &v, const T **out) {
    void *p = nullptr;
    const size_t bytes = std::max<size_t>(v.size() * sizeof(T), 16);
    HIPCHK(ctx, hipMalloc(&p, bytes));
    ix->allocs[ix->n_allocs++] = p;
    if (!v.empty()) HIPCHK(ctx, hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    *out = static_cast<const T *>(p);
    return AF_OK;
}

int ensure_reads_cap(af_ctx *c, int64_t n_reads) {
    if (n_reads <= c->cap_reads) return AF_OK;
    af_free(c->cand);
    c->cand = nullptr; c->cap_reads = 0;
    const int64_t cap = std::max<int64_t>(n_reads, 1 << 16);
    HIPCHK(c, hipMalloc(&c->cand, sizeof(int32_t) * cap));
    c->cap_reads = cap;
    return AF_OK;
}

int ensure_zscratch(af_ctx *c) {
    if (c->zscratch) return AF_OK;
    const size_t zstride = (size_t)(AF_MAX_READ + 1) * 1024;
    HIPCHK(c, hipMalloc(&c->zscratch, zstride * c->n_slots));
    return AF_OK;
}

// the deferred strands' table for a search of cap queries (grow-only; a strand that does not fit
// is searched by k_blat itself)
int ensure_blat_heavy(af_ctx *c, int64_t cap) {
    BlatHeavy &h = c->blat_hv;
    h.min_clumps = c->blat_heavy_min;
    if (h.min_clumps <= 0) return AF_OK;
    const int64_t strands = std::min<int64_t>(1 << 16, std::max<int64_t>(1024, 2 * cap));
    if (h.ctrl && h.strands_cap >= strands) return AF_OK;
    if (h.ctrl) HIPCHK(c, hipDeviceSynchronize());  // an earlier search may still use the table
    af_free(h.strands); af_free(h.ctrl);
    h = BlatHeavy{};
    h.min_clumps = c->blat_heavy_min;
    HIPCHK(c, hipMalloc(&h.strands, sizeof(int4) * strands));
    HIPCHK(c, hipMalloc(&h.ctrl, sizeof(int32_t) * AF_BLAT_HV_CTRL_WORDS));
    h.strands_cap = strands;
    h.jobs_n = h.ctrl + AF_BLAT_HV_JOBS_N;
    h.strands_n = h.ctrl + AF_BLAT_HV_STRANDS_N;
    return AF_OK;
}

int ensure_blat_order(af_ctx *c, int64_t cap) {
    if (cap <= c->blat_ord_cap) return AF_OK;
    af_free(c->blat_ord_work); af_free(c->blat_order);
    c->blat_ord_work = nullptr; c->blat_order = nullptr; c->blat_ord_cap = 0;
    HIPCHK(c, hipMalloc(&c->blat_ord_work, af_blat_order_bytes(cap)));
    HIPCHK(c, hipMalloc(&c->blat_order, sizeof(int32_t) * cap));
    c->blat_ord_cap = cap;
    return AF_OK;
}

int ensure_blat_stage(af_ctx *c, int64_t cap, int32_t max_rows) {
    const int64_t need = 2 * cap * max_rows;
    if (c->blat_stage && need <= c->blat_stage_rows && 2 * cap <= c->blat_stage_items) return AF_OK;
    af_free(c->blat_stage); af_free(c->blat_stage_n);
    c->blat_stage = nullptr; c->blat_stage_n = nullptr; c->blat_stage_rows = c->blat_stage_items = 0;
    HIPCHK(c, hipMalloc(&c->blat_stage, sizeof(af_psl) * need));
    HIPCHK(c, hipMalloc(&c->blat_stage_n, sizeof(int32_t) * 2 * cap));
    c->blat_stage_rows = need;
    c->blat_stage_items = 2 * cap;
    return AF_OK;
}

// k_blat's per-wave scratch for `items` query strands: one slot per strand up to the resident
// waves of the chip (a search of a few queries -- the partner stages' targets, each a context of
// its own -- holds a few slots, not the 2 MB x 6,144 a genome-wide S6 needs)
int ensure_bscratch(af_ctx *c, int64_t items) {
    const int max_slots = af_blat_slots(c->n_cu);
    const int want = (int)std::min<int64_t>(max_slots, std::max<int64_t>(64, (items + 63) / 64 * 64));
    if (!c->blat_caps) {
        HIPCHK(c, hipMalloc(&c->blat_caps, sizeof(int32_t) * AF_BLAT_CAP_N));
        HIPCHK(c, hipMemset(c->blat_caps, 0, sizeof(int32_t) * AF_BLAT_CAP_N));
    }
    if (c->bscratch && c->blat_slots >= want) return AF_OK;
    if (c->bscratch) {
        HIPCHK(c, hipDeviceSynchronize());  // an earlier search may still use the old slots
        af_free(c->bscratch);
        c->bscratch = nullptr;
    }
    c->blat_slots = want;
    HIPCHK(c, hipMalloc(&c->bscratch, (size_t)AF_BLAT_SLOT_BYTES * c->blat_slots));
    return AF_OK;
}

// S2 structures of an anchor index: suffix ranks of the bwa text, its 16-mer hash (every
// position, including the strand boundary), packed text, base counts
int ensure_s2_text(af_ctx *c, af_index *ix) {
    if (ix->s2_ready) return AF_OK;
    const std::vector<uint8_t> &T = ix->text;
    const int64_t N = (int64_t)T.size(), n = N / 2;
    if (N < AF_K) return fail(c, AF_E_INVALID, "anchor shorter than %d", AF_K / 2);
    std::vector<int32_t> rank = suffix_ranks(T);
    std::vector<uint32_t> T2((N + 15) / 16 + 2, 0);
    for (int64_t i = 0; i < N; ++i) T2[i >> 4] |= (uint32_t)T[i] << (2 * (i & 15));
    std::vector<uint64_t> occ;
    occ.reserve(N);
    for (int64_t q = 0; q + AF_K <= N; ++q) {
        uint32_t k = 0;
        for (int u = 0; u < AF_K; ++u) k |= (uint32_t)T[q + u] << (2 * u);
        occ.push_back((uint64_t)k << 32 | (uint64_t)q);
    }
    std::sort(occ.begin(), occ.end());
    std::vector<uint32_t> keys;
    std::vector<int32_t> starts, cnts, kpos(occ.size());
    for (size_t i = 0; i < occ.size(); ++i) {
        const uint32_t k = (uint32_t)(occ[i] >> 32);
        kpos[i] = (int32_t)(occ[i] & 0xffffffffu);
        if (i == 0 || k != keys.back()) { keys.push_back(k); starts.push_back((int32_t)i); cnts.push_back(0); }
        ++cnts.back();
    }
    const int64_t nd = (int64_t)keys.size();
    int hbits = 10;
    while ((1LL << hbits) < 2 * nd) ++hbits;
    const uint32_t hm = (1u << hbits) - 1u;
    std::vector<int4> hslot(1u << hbits, int4{0, 0, 0, 0});
    for (int64_t i = 0; i < nd; ++i) {
        uint32_t sl = af_fmix(keys[i]) & hm;
        while (hslot[sl].z) sl = (sl + 1) & hm;
        hslot[sl] = int4{(int)keys[i], starts[i], cnts[i], kpos[starts[i]]};
    }
    if (ix->n_allocs + 5 > 24) return fail(c, AF_E_INVALID, "index allocation table full");
    int rc;
    DevText X{};
    if ((rc = dev_upload(c, ix, T, &X.T)) || (rc = dev_upload(c, ix, T2, &X.T2)) ||
        (rc = dev_upload(c, ix, rank, &X.rank)) || (rc = dev_upload(c, ix, hslot, &X.hslot)) ||
        (rc = dev_upload(c, ix, kpos, &X.kpos)))
        return rc;
    X.n = n;
    X.hbits = hbits;
    for (int b = 0; b < 4; ++b) X.base_cnt[b] = 0;
    for (int64_t i = 0; i < N; ++i) ++X.base_cnt[T[i]];
    ix->s2 = X;
    ix->s2_ready = true;
    return AF_OK;
}

// per-context S2 scratch for a batch of n_pairs (chunks of >= chunk_bases bases)
int ensure_s2_work(af_ctx *c, int64_t n_pairs, int32_t stride, int64_t chunk_bases, int32_t max_ins) {
    if (n_pairs > c->s2_cap_pairs) {
        af_free(c->s2_pool); af_free(c->s2_rmap); af_free(c->s2_plist); af_free(c->s2_scan); af_free(c->s2_plan);
        c->s2_pool = nullptr; c->s2_rmap = nullptr; c->s2_plist = nullptr; c->s2_scan = nullptr; c->s2_plan = nullptr;
        c->s2_cap_pairs = 0;
        const int64_t cap = std::max<int64_t>(n_pairs, 1 << 16);
        // regions: 4 per read (40 B each) -- enough when every read is a candidate with a
        // couple of regions (targeted input); a read past the pool is flagged and counted
        c->s2_pool_cap = 8 * cap + (1 << 20);
        HIPCHK(c, hipMalloc(&c->s2_pool, sizeof(S2Reg) * c->s2_pool_cap));
        HIPCHK(c, hipMalloc(&c->s2_rmap, sizeof(int2) * 2 * cap));
        HIPCHK(c, hipMalloc(&c->s2_plist, sizeof(int32_t) * cap));
        HIPCHK(c, hipMalloc(&c->s2_scan, sizeof(int64_t) * cap));
        HIPCHK(c, hipMalloc(&c->s2_plan, af_s2_plan_bytes() * cap));
        // K3c's heavy pairs: one in 8 of the batch's pairs, 16 window slots each on average
        GPeSpec &e = c->s2_sp;
        af_free(e.pair); af_free(e.off); af_free(e.nj); af_free(e.job); af_free(e.res);
        e.pair = e.off = e.nj = e.res = nullptr; e.job = nullptr;
        e.cap_pairs = std::max<int64_t>(cap / 8, 1024); e.cap_jobs = 16 * e.cap_pairs;
        HIPCHK(c, hipMalloc(&e.pair, sizeof(int32_t) * e.cap_pairs));
        HIPCHK(c, hipMalloc(&e.off, sizeof(int32_t) * e.cap_pairs));
        HIPCHK(c, hipMalloc(&e.nj, sizeof(int32_t) * e.cap_pairs));
        HIPCHK(c, hipMalloc(&e.job, sizeof(int2) * e.cap_jobs));
        HIPCHK(c, hipMalloc(&e.res, sizeof(int32_t) * 4 * AF_G_PE_RES_W * e.cap_jobs));
        if (!e.cnt) HIPCHK(c, hipMalloc(&e.cnt, 8 * sizeof(unsigned long long)));
        c->s2_cap_pairs = cap;
    }
    const int64_t mc = std::min<int64_t>(n_pairs, 2 * n_pairs * (int64_t)stride / std::max<int64_t>(chunk_bases, 1) + 2) + 1;
    if (mc > c->s2_max_chunks) {
        af_free(c->s2_pes); af_free(c->s2_cstart); af_free(c->s2_nchunks);
        c->s2_pes = nullptr; c->s2_cstart = nullptr; c->s2_nchunks = nullptr;
        c->s2_max_chunks = 0;
        const int64_t m = std::max<int64_t>(mc, 64);
        HIPCHK(c, hipMalloc(&c->s2_pes, sizeof(S2Pes) * 4 * m));
        HIPCHK(c, hipMalloc(&c->s2_cstart, sizeof(int64_t) * (m + 1)));
        HIPCHK(c, hipMalloc(&c->s2_nchunks, sizeof(int32_t)));
        c->s2_max_chunks = (int32_t)m;
    }
    // insert-size histograms [chunk][orientation][max_ins + 1], zero between calls (K3b clears them)
    const int64_t hints = (int64_t)c->s2_max_chunks * 4 * (max_ins + 1);
    if (hints > c->s2_ghist_ints) {
        af_free(c->s2_ghist);
        c->s2_ghist = nullptr;
        c->s2_ghist_ints = 0;
        HIPCHK(c, hipMalloc(&c->s2_ghist, sizeof(int32_t) * hints));
        HIPCHK(c, hipMemset(c->s2_ghist, 0, sizeof(int32_t) * hints));
        c->s2_ghist_ints = hints;
    }
    return AF_OK;
}

int check_pe(af_ctx *c, const af_pe *e) {
    if (e->pen_unpaired < 0 || e->max_ins < 1 || e->max_ins > 16383 || e->max_matesw < 0 || e->split_width < 0 ||
        e->max_mem_intv < 0 || e->max_chain_gap < 1 || e->chunk_bases < 1 || e->pair_base < 0)
        return fail(c, AF_E_INVALID, "invalid af_pe (1 <= max_ins <= 16383, chunk_bases >= 1, pair_base >= 0)");
    return AF_OK;
}

int check_params(af_ctx *c, const af_params *p) {
    if (!p) return fail(c, AF_E_INVALID, "params is NULL");
    if (p->a <= 0 || p->b < 0 || p->o_del < 0 || p->e_del <= 0 || p->o_ins < 0 || p->e_ins <= 0 || p->w < 0 ||
        p->min_seed_len < AF_K || p->max_ext < 1 || p->max_ext > 16 || p->max_mems < 1 || p->max_mems > 64 ||
        p->max_occ < 1)
        return fail(c, AF_E_INVALID, "invalid af_params (min_seed_len>=%d, 1<=max_ext<=16, 1<=max_mems<=64)", AF_K);
    return AF_OK;
}


// ---- genome calls (bwa_genome.hip) ------------------------------------------------------
// per-lane G1 scratch (AF_G1_WPS waves per SIMD) and per-wave G2-G4 scratch (8 waves per CU, <= n_slots of
// the context's traceback scratch)
int ensure_genome_scratch(af_ctx *c) {
    if (c->g1_scr) return AF_OK;
    c->g1_threads = c->n_cu * 4 * AF_G1_WPS * 64;
    c->g2_waves = std::min(c->n_cu * 8, c->n_slots);
    HIPCHK(c, hipMalloc(&c->g1_scr, af_g1_slot_bytes() * (size_t)c->g1_threads));
    HIPCHK(c, hipMalloc(&c->g2_scr, af_g2_slot_bytes() * (size_t)c->g2_waves));
    // iv fill, G1 next, G1 heavy count / next, G2 first-list count / next
    HIPCHK(c, hipMalloc(&c->g_iv_fill, 8 * sizeof(unsigned long long)));
    HIPCHK(c, hipMalloc(&c->g_reg_fill, sizeof(int32_t)));
    HIPCHK(c, hipMalloc(&c->g_stats, sizeof(int32_t) * AF_GSTAT_N));
    HIPCHK(c, hipMemset(c->g_stats, 0, sizeof(int32_t) * AF_GSTAT_N));
    return ensure_zscratch(c);
}

// pools for a call over n_reads reads: intervals (96 per read on average; a read's list is at
// most AF_G_MAX_INTV) and regions (16 per read on average)
int ensure_genome_pools(af_ctx *c, int64_t n_reads) {
    if (n_reads <= c->g_cap_reads) return AF_OK;
    // the region pool's fill and offsets are int32 (at most 16 regions per read on average)
    if (n_reads > INT32_MAX / 16 - AF_G_MAX_REG) return fail(c, AF_E_INVALID, "too many reads for one genome call");
    af_free(c->g_iv); af_free(c->g_reg); af_free(c->g_iv_off); af_free(c->g_iv_n); af_free(c->g_reg_off);
    af_free(c->g_reg_n); af_free(c->g1_hv);
    c->g_iv = nullptr; c->g_reg = nullptr; c->g_iv_off = nullptr; c->g_iv_n = nullptr; c->g_reg_off = nullptr;
    c->g_reg_n = nullptr; c->g1_hv = nullptr; c->g_cap_reads = 0;
    const int64_t cap = std::max<int64_t>(n_reads, 1 << 14);
    c->g_iv_cap = cap * 96 + AF_G_MAX_INTV;
    c->g_reg_cap = cap * 16 + AF_G_MAX_REG;
    HIPCHK(c, hipMalloc(&c->g_iv, sizeof(GIv) * c->g_iv_cap));
    HIPCHK(c, hipMalloc(&c->g_reg, sizeof(GReg) * c->g_reg_cap));
    HIPCHK(c, hipMalloc(&c->g_iv_off, sizeof(int64_t) * cap));
    HIPCHK(c, hipMalloc(&c->g_iv_n, sizeof(int32_t) * cap));
    HIPCHK(c, hipMalloc(&c->g_reg_off, sizeof(int32_t) * cap));
    HIPCHK(c, hipMalloc(&c->g_reg_n, sizeof(int32_t) * cap));
    HIPCHK(c, hipMalloc(&c->g1_hv, sizeof(int64_t) * cap));
    // heavy reads: at most every read; 8 pooled chains and 16 seeds per read of the call (a read
    // that does not fit is extended by its own wave)
    GHeavy &h = c->g_hv;
    af_free(h.read); af_free(h.nch); af_free(h.ch_off); af_free(h.sd_off); af_free(h.ch_read);
    af_free(h.ch); af_free(h.sd); af_free(h.res);
    h.read = nullptr; h.nch = h.ch_off = h.sd_off = h.ch_read = nullptr; h.ch = h.sd = h.res = nullptr;
    h.cap_reads = cap; h.cap_ch = std::max<int64_t>(cap * 8, 1 << 16); h.cap_sd = 2 * h.cap_ch;
    HIPCHK(c, hipMalloc(&h.read, sizeof(int64_t) * h.cap_reads));
    HIPCHK(c, hipMalloc(&h.nch, sizeof(int32_t) * h.cap_reads));
    HIPCHK(c, hipMalloc(&h.ch_off, sizeof(int32_t) * h.cap_reads));
    HIPCHK(c, hipMalloc(&h.sd_off, sizeof(int32_t) * h.cap_reads));
    HIPCHK(c, hipMalloc(&h.ch_read, sizeof(int32_t) * h.cap_ch));
    HIPCHK(c, hipMalloc(&h.ch, af_g_chain_bytes() * h.cap_ch));
    HIPCHK(c, hipMalloc(&h.sd, af_g_seed_bytes() * h.cap_sd));
    HIPCHK(c, hipMalloc(&h.res, sizeof(GReg) * h.cap_sd));
    if (!h.cnt) HIPCHK(c, hipMalloc(&h.cnt, 8 * sizeof(unsigned long long)));
    // S4's heavy pairs: up to half the call's pairs (cap counts reads), 8 window slots each on
    // average (a pair that does not fit runs its rescues on its own wave; counted by
    // AF_GSTAT_PE_JOBS: 1,628 of the configs[2] step's 26 k pairs hit the round's first cap of 1/32)
    GPeSpec &e = c->g_pe;
    af_free(e.pair); af_free(e.off); af_free(e.nj); af_free(e.job); af_free(e.res);
    e.pair = e.off = e.nj = e.res = nullptr; e.job = nullptr;
    e.cap_pairs = std::max<int64_t>(cap / 4, 1024); e.cap_jobs = 8 * e.cap_pairs;
    HIPCHK(c, hipMalloc(&e.pair, sizeof(int32_t) * e.cap_pairs));
    HIPCHK(c, hipMalloc(&e.off, sizeof(int32_t) * e.cap_pairs));
    HIPCHK(c, hipMalloc(&e.nj, sizeof(int32_t) * e.cap_pairs));
    HIPCHK(c, hipMalloc(&e.job, sizeof(int2) * e.cap_jobs));
    HIPCHK(c, hipMalloc(&e.res, sizeof(int32_t) * 4 * AF_G_PE_RES_W * e.cap_jobs));
    if (!e.cnt) HIPCHK(c, hipMalloc(&e.cnt, 8 * sizeof(unsigned long long)));
    af_free(c->g2_list); af_free(c->g2_flag);
    c->g2_list = nullptr; c->g2_flag = nullptr;
    HIPCHK(c, hipMalloc(&c->g2_list, sizeof(int32_t) * cap));
    HIPCHK(c, hipMalloc(&c->g2_flag, cap));
    c->g_cap_reads = cap;
    return AF_OK;
}

// n_reads: the call's reads.  G1's hand-off threshold follows the load: a lane-path read's time is
// its chain of extensions, each a trip of the whole wave, while the wave path's reads share the
// CUs -- with few reads per CU (a rank's share at N = 8: ~70 S5 reads per CU) the CUs are idle
// and every read finishes sooner on a wave of its own (threshold 1, each read handed off after its
// first extension: the rank-share step 37.1 -> 35.3 ms with the wave path at 6 waves per SIMD),
// with hundreds per CU (one GPU's 50 M pairs: ~580) the waves' work would queue (1,024: 238 vs
// 203 ms)
GWork genome_work(af_ctx *c, int64_t n_reads) {
    GWork w;
    w.iv = c->g_iv; w.iv_cap = c->g_iv_cap; w.iv_fill = c->g_iv_fill; w.iv_off = c->g_iv_off; w.iv_n = c->g_iv_n;
    w.reg = c->g_reg; w.reg_cap = c->g_reg_cap; w.reg_fill = c->g_reg_fill; w.reg_off = c->g_reg_off;
    w.reg_n = c->g_reg_n;
    w.heads = c->ctrl + AF_CTRL_G_HEADS;
    w.g1_next = c->g_iv_fill + 1;
    w.g1_hv = c->g1_hv; w.g1_hv_n = c->g_iv_fill + 2; w.g1_hv_next = c->g_iv_fill + 3;
    int32_t mx = c->g1_max_ext;
    if (!c->g1_ext_env && n_reads > 0) {
        const int64_t per_cu = n_reads / std::max(1, c->n_cu);
        mx = per_cu >= 160 ? mx : per_cu >= 96 ? std::min(mx, 1024) : 1;
    }
    w.g1_max_ext = c->g1_hv ? mx : 0;
    w.hv = c->g_hv;
    w.hv.min_chains = c->g_hv.cnt ? c->g_heavy_min : 0;
    w.pe = c->g_pe;
    w.pe.min_windows = c->g_pe.cnt ? c->g_pe_min : 0;
    w.g2_list = c->g2_list; w.g2_flag = c->g2_flag; w.g2_list_n = c->g_iv_fill + 4; w.g2_list_next = c->g_iv_fill + 5;
    w.g2_first_occ = c->g2_flag ? c->g2_first_occ : 0;
    w.stats = c->g_stats;
    return w;
}

int check_genome_call(af_ctx *c, const af_genome *g, const af_params *p, const af_pe *e, int32_t stride) {
    if (!c || !g || !g->dev.sa) return fail(c, AF_E_INVALID, "null context or genome");
    if (!p || p->a <= 0 || p->b < 0 || p->o_del < 0 || p->e_del <= 0 || p->o_ins < 0 || p->e_ins <= 0 || p->w < 0 ||
        p->min_seed_len < 1 || p->max_occ < 1)
        return fail(c, AF_E_INVALID, "invalid af_params");
    if (stride < 1) return fail(c, AF_E_INVALID, "stride must be >= 1");
    return e ? check_pe(c, e) : AF_OK;
}

// S2Work view of the S4 chunk statistics (k_s2_pestat; ragged chunk starts from the lengths)
int ensure_genome_pe(af_ctx *c, int64_t n_pairs, int32_t stride, int64_t chunk_bases, int32_t max_ins) {
    const int64_t mc = std::min<int64_t>(n_pairs, 2 * n_pairs * (int64_t)stride / std::max<int64_t>(chunk_bases, 1) + 2) + 1;
    if (mc > c->g_max_chunks) {
        af_free(c->g_pes); af_free(c->g_cstart); af_free(c->g_nchunks);
        c->g_pes = nullptr; c->g_cstart = nullptr; c->g_nchunks = nullptr; c->g_max_chunks = 0;
        const int64_t m = std::max<int64_t>(mc, 16);
        HIPCHK(c, hipMalloc(&c->g_pes, sizeof(S2Pes) * 4 * m));
        HIPCHK(c, hipMalloc(&c->g_cstart, sizeof(int64_t) * (m + 1)));
        HIPCHK(c, hipMalloc(&c->g_nchunks, sizeof(int32_t)));
        c->g_max_chunks = (int32_t)m;
    }
    if (n_pairs > c->g_scan_cap) {
        af_free(c->g_scan);
        c->g_scan = nullptr; c->g_scan_cap = 0;
        HIPCHK(c, hipMalloc(&c->g_scan, sizeof(int64_t) * std::max<int64_t>(n_pairs, 1)));
        c->g_scan_cap = std::max<int64_t>(n_pairs, 1);
    }
    const int64_t hints = (int64_t)c->g_max_chunks * 4 * (max_ins + 1);
    if (hints > c->g_ghist_ints) {
        af_free(c->g_ghist);
        c->g_ghist = nullptr; c->g_ghist_ints = 0;
        HIPCHK(c, hipMalloc(&c->g_ghist, sizeof(int32_t) * hints));
        HIPCHK(c, hipMemset(c->g_ghist, 0, sizeof(int32_t) * hints));
        c->g_ghist_ints = hints;
    }
    return AF_OK;
}

int genome_build(af_ctx *c, const char *blob, int64_t n_blob, const int64_t *ctg_off, const int64_t *ctg_len,
                 int32_t n_ctg, af_genome **out, bool on_device) {
    if (!c || !blob || !ctg_off || !ctg_len || !out || n_ctg < 1 || n_blob < 1)
        return fail(c, AF_E_INVALID, "null or empty argument");
    *out = nullptr;
    for (int k = 0; k < n_ctg; ++k)
        if (ctg_off[k] < 0 || ctg_len[k] < 1 || ctg_off[k] + ctg_len[k] > n_blob)
            return fail(c, AF_E_INVALID, "contig %d outside the blob", k);
    (void)hipSetDevice(c->device);
    const uint8_t *d_blob = reinterpret_cast<const uint8_t *>(blob);
    uint8_t *tmp = nullptr;
    if (!on_device) {
        HIPCHK(c, hipMalloc(&tmp, n_blob));
        if (hipMemcpy(tmp, blob, n_blob, hipMemcpyHostToDevice) != hipSuccess) {
            af_free(tmp);
            return fail(c, AF_E_HIP, "genome copy to the device failed");
        }
        d_blob = tmp;
    }
    af_genome *g = new (std::nothrow) af_genome;
    if (!g) { af_free(tmp); return fail(c, AF_E_NOMEM, "out of host memory"); }
    g->ctx = c;
    const hipError_t e = af_fm_build(d_blob, ctg_off, ctg_len, n_ctg, &g->dev, c->stream);
    af_free(tmp);
    if (e != hipSuccess) {
        delete g;
        return fail(c, e == hipErrorOutOfMemory ? AF_E_NOMEM : AF_E_HIP, "genome index build: %s", hipGetErrorString(e));
    }
    *out = g;
    return AF_OK;
}

}  // namespace

extern "C" {

void af_params_default(af_params *p) {
    // bwa mem defaults (bwa 0.7.17 usage text): -A1 -B4 -O6 -E1 -L5 -w100 -d100 -k19 -T30
    p->a = 1; p->b = 4; p->o_del = 6; p->e_del = 1; p->o_ins = 6; p->e_ins = 1;
    p->pen_clip5 = 5; p->pen_clip3 = 5; p->w = 100; p->zdrop = 100;
    p->min_seed_len = 19; p->max_occ = 500; p->T = 30; p->max_ext = 16; p->max_mems = 64;
}

void af_pe_default(af_pe *e) {
    // bwa 0.7.17 mem_opt_init paired-end options; chunk = 10,000,000 bases x threads (the
    // reference runs `bwa mem -t <--thread>`, default 1: Anchored_Fusion.py:29)
    e->pen_unpaired = 17; e->max_ins = 10000; e->max_matesw = 50; e->split_width = 10;
    e->max_mem_intv = 20; e->max_chain_gap = 10000;
    e->chunk_bases = 10000000; e->pair_base = 0;
}

int af_ctx_create(int device, af_ctx **out) {
    if (!out) return AF_E_INVALID;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return AF_E_HIP;
    if (device < 0 || device >= ndev) return AF_E_INVALID;
    if (hipSetDevice(device) != hipSuccess) return AF_E_HIP;
    af_ctx *c = new (std::nothrow) af_ctx;
    if (!c) return AF_E_NOMEM;
    c->device = device;
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
    c->n_cu = std::max(1, cus);
    c->n_slots = c->n_cu * 4 * AF_K2_WPS;  // k_align: AF_K2_WPS waves per SIMD (VGPR and LDS budget)
    if (const char *hv = getenv("AF_G_HEAVY_CHAINS")) c->g_heavy_min = std::max(0, atoi(hv));  // tests: 1 = every read
    if (const char *pw = getenv("AF_G_PE_SPEC_WINDOWS")) c->g_pe_min = std::max(0, atoi(pw));  // tests: 1 = every rescuing pair
    if (const char *sw = getenv("AF_S2_SPEC_WINDOWS")) c->s2_sp_min = std::max(0, atoi(sw));
    if (const char *hv = getenv("AF_BLAT_HEAVY_CLUMPS")) c->blat_heavy_min = std::max(0, atoi(hv));  // 0: none deferred
    if (const char *go = getenv("AF_G2_FIRST_OCC")) c->g2_first_occ = std::max(0, atoi(go));
    if (const char *hv = getenv("AF_G1_HEAVY_EXT")) {  // tests: 1 = every read
        c->g1_max_ext = std::max(0, atoi(hv));
        c->g1_ext_env = true;
    }
    if (hipMalloc(&c->ctrl, AF_CTRL_BYTES) != hipSuccess) { delete c; return AF_E_HIP; }
    if (hipMemset(c->ctrl, 0, AF_CTRL_BYTES) != hipSuccess) { af_free(c->ctrl); delete c; return AF_E_HIP; }
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        af_free(c->ctrl);
        delete c;
        return AF_E_HIP;
    }
    *out = c;
    return AF_OK;
}

void af_ctx_destroy(af_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    af_free(c->ctrl); af_free(c->cand); af_free(c->zscratch); af_free(c->bscratch); af_free(c->blat_caps); af_free(c->blat_ord_work); af_free(c->blat_order); af_free(c->blat_stage); af_free(c->blat_stage_n); af_free(c->d_packed);
    af_free(c->d_reads); af_free(c->d_lens);
    af_free(c->d_flag); af_free(c->d_pos); af_free(c->d_score); af_free(c->d_ncig); af_free(c->d_hits);
    af_free(c->d_cigar);
    af_free(c->s2_pool); af_free(c->s2_rmap); af_free(c->s2_plist); af_free(c->s2_ghist); af_free(c->s2_scan);
    af_free(c->s2_plan);
    af_free(c->s2_pes); af_free(c->s2_cstart); af_free(c->s2_nchunks);
    af_free(c->s3_keys); af_free(c->s3_temp); af_free(c->s3_counts);
    af_free(c->g_sel); af_free(c->g_sel_n); af_free(c->g_temp);
    af_free(c->g2_scr_pe); af_free(c->zscratch_pe);
    af_free(c->g_hv.read); af_free(c->g_hv.nch); af_free(c->g_hv.ch_off); af_free(c->g_hv.sd_off); af_free(c->g_hv.ch_read);
    af_free(c->g_hv.ch); af_free(c->g_hv.sd); af_free(c->g_hv.res); af_free(c->g_hv.cnt);
    af_free(c->g_pe.pair); af_free(c->g_pe.off); af_free(c->g_pe.nj); af_free(c->g_pe.job); af_free(c->g_pe.res);
    af_free(c->g_pe.cnt);
    af_free(c->s2_sp.pair); af_free(c->s2_sp.off); af_free(c->s2_sp.nj); af_free(c->s2_sp.job); af_free(c->s2_sp.res);
    af_free(c->s2_sp.cnt);
    af_free(c->g2_list); af_free(c->g2_flag);
    if (c->g_ev) (void)hipEventDestroy(c->g_ev);
    af_free(c->g1_scr); af_free(c->g2_scr); af_free(c->g_iv); af_free(c->g_reg); af_free(c->g_iv_fill);
    af_free(c->g_reg_fill); af_free(c->g_stats); af_free(c->g_iv_n); af_free(c->g_reg_off); af_free(c->g_reg_n); af_free(c->g1_hv);
    af_free(c->g_iv_off); af_free(c->g_ghist); af_free(c->g_nchunks); af_free(c->g_cstart); af_free(c->g_scan);
    af_free(c->g_pes); af_free(c->g_recs); af_free(c->g_nrec); af_free(c->g_hlens); af_free(c->g_hreads);
    af_free(c->s5_keep); af_free(c->s5_sel); af_free(c->s5_nsel); af_free(c->s5_temp);
    af_free(c->s6_flag); af_free(c->s6_idx); af_free(c->s6_sflag); af_free(c->s6_sidx); af_free(c->s6_temp);
    af_free(c->blat_hv.strands);
    af_free(c->blat_hv.ctrl);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

const char *af_last_error(const af_ctx *c) { return c ? c->err.c_str() : "null context"; }

int af_index_build(af_ctx *c, const char *anchor, int64_t len, af_index **out) {
    if (!c || !anchor || !out) return fail(c, AF_E_INVALID, "null argument");
    *out = nullptr;
    if (len <= 0) return fail(c, AF_E_INVALID, "empty anchor");
    if (len > (1LL << 30)) return fail(c, AF_E_UNSUPPORTED, "anchor longer than 2^30");
    (void)hipSetDevice(c->device);
    const int64_t n = len, n2 = 2 * len;
    std::vector<uint8_t> D(n2);
    for (int64_t i = 0; i < n; ++i) {
        const uint8_t v = nt4((uint8_t)anchor[i]);
        D[i] = v;
        D[n2 - 1 - i] = v < 4 ? 3 - v : 4;
    }
    std::vector<uint32_t> D2((n2 + 15) / 16 + 2, 0), Dn((n2 + 31) / 32 + 2, 0);
    for (int64_t i = 0; i < n2; ++i) {
        D2[i >> 4] |= (uint32_t)(D[i] & 3) << (2 * (i & 15));
        if (D[i] > 3) Dn[i >> 5] |= 1u << (i & 31);
    }
    // 16-mer occurrences that do not cross the strand boundary, sorted by (kmer, pos)
    std::vector<uint64_t> occ;
    occ.reserve(n2);
    for (int64_t p = 0; p + AF_K <= n2; ++p) {
        if (p < n && p + AF_K > n) continue;
        uint32_t k = 0;
        bool ok = true;
        for (int u = 0; u < AF_K && ok; ++u) {
            ok = D[p + u] < 4;
            k |= (uint32_t)(D[p + u] & 3) << (2 * u);
        }
        if (ok) occ.push_back((uint64_t)k << 32 | (uint64_t)p);
    }
    std::sort(occ.begin(), occ.end());
    std::vector<uint32_t> keys;
    std::vector<int32_t> starts, cnts, kpos(occ.size());
    for (size_t i = 0; i < occ.size(); ++i) {
        const uint32_t k = (uint32_t)(occ[i] >> 32);
        kpos[i] = (int32_t)(occ[i] & 0xffffffffu);
        if (i == 0 || k != keys.back()) { keys.push_back(k); starts.push_back((int32_t)i); cnts.push_back(0); }
        ++cnts.back();
    }
    const int64_t nd = (int64_t)keys.size();
    int hbits = 10;
    while ((1LL << hbits) < 2 * nd) ++hbits;
    const uint32_t hm = (1u << hbits) - 1u;
    std::vector<int4> hslot(1u << hbits, int4{0, 0, 0, 0});
    for (int64_t i = 0; i < nd; ++i) {
        uint32_t s = af_fmix(keys[i]) & hm;
        while (hslot[s].z) s = (s + 1) & hm;
        hslot[s] = int4{(int)keys[i], starts[i], cnts[i], kpos[starts[i]]};
    }
    // Bloom filter of the distinct 16-mers of the bwa text that do not cross the strand boundary
    // (K1; S2 seeds never cross it): 2^bl_bits 32-bit words, ~2.4 words per key (at most 2^15
    // words = 128 KiB, a 6.8 kb anchor), four bits in each of two words
    std::vector<uint8_t> T = bwa_text(anchor, n);
    std::vector<uint32_t> tkeys;
    tkeys.reserve(n2);
    for (int64_t q = 0; q + AF_K <= n2; ++q) {
        if (q < n && q + AF_K > n) continue;
        uint32_t k = 0;
        for (int u = 0; u < AF_K; ++u) k |= (uint32_t)T[q + u] << (2 * u);
        tkeys.push_back(k);
    }
    std::sort(tkeys.begin(), tkeys.end());
    tkeys.erase(std::unique(tkeys.begin(), tkeys.end()), tkeys.end());
    const int64_t ntd = (int64_t)tkeys.size();
    int bl_bits = 8;
    while ((double)(1LL << bl_bits) < 2.4 * (double)ntd && bl_bits < AF_K1_MAX_BITS) ++bl_bits;
    std::vector<uint32_t> bloom((size_t)1 << bl_bits, 0);
    for (int64_t i = 0; i < ntd; ++i) {
        const uint64_t h = af_k1_hash(af_k1_key(tkeys[i]));
        const uint32_t lo = (uint32_t)h, hi = (uint32_t)(h >> 32);
        bloom[(hi >> 2) & ((1u << bl_bits) - 1u)] |= af_k1_mask(lo);
        bloom[lo >> (32 - bl_bits)] |= af_k1_mask(hi);
    }
    af_index *ix = new (std::nothrow) af_index;
    if (!ix) return fail(c, AF_E_NOMEM, "out of host memory");
    ix->ctx = c;
    ix->bloom_host = bloom;
    ix->text.swap(T);
    int rc = AF_OK;
    const uint32_t *bld = nullptr;
    if ((rc = dev_upload(c, ix, D, &ix->dev.D)) || (rc = dev_upload(c, ix, D2, &ix->dev.D2)) ||
        (rc = dev_upload(c, ix, Dn, &ix->dev.Dn)) || (rc = dev_upload(c, ix, hslot, &ix->dev.hslot)) ||
        (rc = dev_upload(c, ix, kpos, &ix->dev.kpos)) || (rc = dev_upload(c, ix, bloom, &bld))) {
        af_index_free(ix);
        return rc;
    }
    ix->dev.bloom = bld;
    ix->dev.n = n;
    ix->dev.hbits = hbits;
    ix->dev.bl_bits = bl_bits;
    *out = ix;
    return AF_OK;
}

void af_index_free(af_index *ix) {
    if (!ix) return;
    if (ix->ctx) (void)hipSetDevice(ix->ctx->device);
    for (int i = 0; i < ix->n_allocs; ++i) af_free(ix->allocs[i]);
    delete ix;
}

int64_t af_index_anchor_len(const af_index *ix) { return ix ? ix->dev.n : -1; }
int32_t af_index_filter_words(const af_index *ix) {
    return ix ? (ix->dev.bl_bits < 0 ? 0 : (1 << ix->dev.bl_bits)) : -1;
}

int af_index_filter_table(const af_index *ix, uint32_t *out, int64_t cap) {
    if (!ix || !out) return AF_E_INVALID;
    if (cap < (int64_t)ix->bloom_host.size()) return AF_E_CAPACITY;
    memcpy(out, ix->bloom_host.data(), ix->bloom_host.size() * sizeof(uint32_t));
    return AF_OK;
}

int af_seed_filter_device(af_ctx *c, const af_index *ix, const uint8_t *d_reads, int64_t n_reads, int32_t stride,
                          const int32_t *d_lens, int32_t *d_hits, void *stream) {
    if (ix && ix->is_tile) return fail(c, AF_E_UNSUPPORTED, "a tile index serves af_blat only");
    if (!c || !ix || (!d_reads && n_reads) || !d_hits) return fail(c, AF_E_INVALID, "null argument");
    if (stride <= 0 || stride > AF_MAX_READ) return fail(c, AF_E_INVALID, "stride %d outside [1, %d]", stride, AF_MAX_READ);
    if (((uintptr_t)d_reads & 15) != 0) return fail(c, AF_E_INVALID, "reads buffer must be 16-byte aligned");
    (void)hipSetDevice(c->device);
    hipStream_t s = (hipStream_t)stream;
    int rc = ensure_reads_cap(c, n_reads);
    if (rc) return rc;
    const int slot = (int)(c->epoch & 1);
    HIPCHK(c, af_launch_seed_filter(ix->dev, d_reads, n_reads, stride, d_lens, d_hits, c->cand,
                                    c->ctrl + AF_HEAD_STRIDE * slot, c->ctrl + AF_HEAD_STRIDE * (slot ^ 1),
                                    c->ctrl + AF_CTRL_S2_POOL + AF_HEAD_STRIDE * slot, c->n_cu, s));
    ++c->epoch;
    return AF_OK;
}

int64_t af_last_candidates(af_ctx *c) {
    if (!c) return -1;
    int32_t v = -1;
    (void)hipSetDevice(c->device);
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (c->epoch == 0) return 0;
    const int slot = (int)((c->epoch - 1) & 1);
    if (hipMemcpy(&v, c->ctrl + AF_HEAD_STRIDE * slot, sizeof v, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    return v;
}

int af_align_pairs_device(af_ctx *c, const af_index *ix, const uint8_t *d_reads, int64_t n_pairs, int32_t stride,
                          const int32_t *d_lens, const af_params *p, const af_pe *pe, af_aln_out *o, void *stream) {
    if (!c || !ix || !o) return fail(c, AF_E_INVALID, "null argument");
    int rc = check_params(c, p);
    if (rc) return rc;
    if (n_pairs < 0) return fail(c, AF_E_INVALID, "n_pairs < 0");
    if (n_pairs == 0) return AF_OK;
    if (!o->flag || !o->pos || !o->score || !o->n_cigar || !o->hits || !o->cigar)
        return fail(c, AF_E_INVALID, "output arrays must all be non-NULL");
    if ((rc = af_seed_filter_device(c, ix, d_reads, 2 * n_pairs, stride, d_lens, o->hits, stream))) return rc;
    return af_align_candidates_device(c, ix, d_reads, n_pairs, stride, d_lens, p, pe, o, stream);
}

static int align_candidates(af_ctx *c, af_index *ix, const uint8_t *d_reads, int64_t n_pairs, int32_t stride,
                            const int32_t *d_lens, const af_params *p, const af_pe *pe, af_aln_out *o, void *stream,
                            const AfTails *tails, bool append);

int af_align_candidates_device(af_ctx *c, const af_index *ix, const uint8_t *d_reads, int64_t n_pairs,
                               int32_t stride, const int32_t *d_lens, const af_params *p, const af_pe *pe,
                               af_aln_out *o, void *stream) {
    return align_candidates(c, const_cast<af_index *>(ix), d_reads, n_pairs, stride, d_lens, p, pe, o, stream, nullptr,
                            false);
}

int af_align_candidates_tails_device(af_ctx *c, const af_index *ix, const uint8_t *d_reads, int64_t n_pairs,
                                     int32_t stride, const int32_t *d_lens, const af_params *p, const af_pe *pe,
                                     af_aln_out *o,
                                     int32_t min_clip, int64_t read_base, int32_t append, int64_t cap,
                                     uint8_t *d_tails, int32_t *d_tail_lens, int32_t *d_tail_read,
                                     int32_t *d_n_tails, void *stream) {
    if (!d_n_tails || (cap > 0 && (!d_tails || !d_tail_lens || !d_tail_read)))
        return fail(c, AF_E_INVALID, "null tails argument");
    if (cap < 0) return fail(c, AF_E_INVALID, "cap < 0");
    if (read_base < 0 || read_base + 2 * n_pairs > (1LL << 31) - 1)
        return fail(c, AF_E_INVALID, "read_base + reads exceeds int32");
    const AfTails t{d_tails, d_tail_lens, d_tail_read, d_n_tails, cap, read_base, min_clip < 1 ? 1 : min_clip};
    return align_candidates(c, const_cast<af_index *>(ix), d_reads, n_pairs, stride, d_lens, p, pe, o, stream, &t,
                            append != 0);
}

static int align_candidates(af_ctx *c, af_index *ix, const uint8_t *d_reads, int64_t n_pairs, int32_t stride,
                            const int32_t *d_lens, const af_params *p, const af_pe *pe_in, af_aln_out *o, void *stream,
                            const AfTails *tails, bool append) {
    if (ix && ix->is_tile) return fail(c, AF_E_UNSUPPORTED, "a tile index serves af_blat only");
    if (!c || !ix || !o) return fail(c, AF_E_INVALID, "null argument");
    int rc = check_params(c, p);
    if (rc) return rc;
    if (p->w > 300) return fail(c, AF_E_INVALID, "af_align_*: band w %d above 300", p->w);
    af_pe pe;
    if (pe_in) pe = *pe_in;
    else af_pe_default(&pe);
    if ((rc = check_pe(c, &pe))) return rc;
    if (n_pairs <= 0) return n_pairs == 0 ? AF_OK : fail(c, AF_E_INVALID, "n_pairs < 0");
    if (n_pairs > (1LL << 30)) return fail(c, AF_E_INVALID, "n_pairs above 2^30");
    if (!o->flag || !o->pos || !o->score || !o->n_cigar || !o->hits || !o->cigar)
        return fail(c, AF_E_INVALID, "output arrays must all be non-NULL");
    if ((((uintptr_t)o->flag | (uintptr_t)o->pos | (uintptr_t)o->score | (uintptr_t)o->n_cigar) & 7) != 0)
        return fail(c, AF_E_INVALID, "flag/pos/score/n_cigar arrays must be 8-byte aligned");
    if (2 * n_pairs > c->cap_reads) return fail(c, AF_E_INVALID, "seed filter was not run for this batch");
    (void)hipSetDevice(c->device);
    if ((rc = ensure_zscratch(c))) return rc;
    if ((rc = ensure_s2_text(c, ix))) return rc;
    if ((rc = ensure_s2_work(c, n_pairs, stride, pe.chunk_bases, pe.max_ins))) return rc;
    hipStream_t s = (hipStream_t)stream;
    if (c->epoch == 0) return fail(c, AF_E_INVALID, "seed filter was not run for this batch");
    const int slot = (int)((c->epoch - 1) & 1);
    int32_t *n_cand = c->ctrl + AF_HEAD_STRIDE * slot;
    S2Work w{};
    w.pool = c->s2_pool; w.pool_cap = c->s2_pool_cap;
    w.pool_n = c->ctrl + AF_CTRL_S2_POOL + AF_HEAD_STRIDE * slot;
    w.rmap = c->s2_rmap;
    w.plist = c->s2_plist;
    w.n_plist = c->ctrl + AF_CTRL_S2_NPAIRS + AF_HEAD_STRIDE * slot;
    w.ghist = c->s2_ghist; w.pes = c->s2_pes;
    w.cstart = c->s2_cstart; w.n_chunks = c->s2_nchunks; w.max_chunks = c->s2_max_chunks;
    if (!d_lens) {  // every read has length stride: pairs per chunk is arithmetic (bseq_read)
        w.ppc = (pe.chunk_bases + 2 * (int64_t)stride - 1) / (2 * (int64_t)stride);
        w.n_chunks_u = (int32_t)((n_pairs + w.ppc - 1) / w.ppc);
    }
    w.heads_k2 = c->ctrl + AF_CTRL_HEADS2; w.heads_k3 = c->ctrl + AF_CTRL_S2_HEADS3;
    w.plan = c->s2_plan;
    w.sp = c->s2_sp;
    w.sp.min_windows = c->s2_sp.cnt ? c->s2_sp_min : 0;
    S2Opt opt{pe.pen_unpaired, pe.max_ins, pe.max_matesw, pe.split_width, pe.max_mem_intv, pe.max_chain_gap, pe.pair_base};
    if (d_lens)
        HIPCHK(c, af_launch_s2_chunks(n_pairs, stride, d_lens, pe.chunk_bases, c->s2_cstart, c->s2_scan,
                                      c->s2_max_chunks, c->s2_nchunks, s));
    if (tails && !append) HIPCHK(c, hipMemsetAsync(tails->n_tails, 0, 4, s));
    HIPCHK(c, af_launch_s2(ix->s2, d_reads, n_pairs, stride, d_lens, *p, opt, o->hits, c->cand, n_cand, w, *o,
                           c->zscratch, c->n_slots, c->n_cu, tails, s));
    return AF_OK;
}

int af_align_pairs(af_ctx *c, const af_index *ix, const uint8_t *reads, int64_t n_pairs, int32_t stride,
                   const int32_t *lens, const af_params *p, const af_pe *pe, af_aln_out *out) {
    if (ix && ix->is_tile) return fail(c, AF_E_UNSUPPORTED, "a tile index serves af_blat only");
    if (!c || !ix || !out || (!reads && n_pairs)) return fail(c, AF_E_INVALID, "null argument");
    if (n_pairs == 0) return AF_OK;
    if (stride <= 0 || stride > AF_MAX_READ) return fail(c, AF_E_INVALID, "stride %d outside [1, %d]", stride, AF_MAX_READ);
    (void)hipSetDevice(c->device);
    const int64_t nr = 2 * n_pairs;
    const int64_t bytes = nr * (int64_t)stride;
    if (bytes > c->cap_bytes) {
        af_free(c->d_reads); af_free(c->d_lens);
        c->d_reads = nullptr; c->d_lens = nullptr; c->cap_bytes = 0;
        HIPCHK(c, hipMalloc(&c->d_reads, bytes + 64));
        HIPCHK(c, hipMalloc(&c->d_lens, sizeof(int32_t) * nr + 64));
        c->cap_bytes = bytes;
    }
    if (nr > c->cap_out) {
        af_free(c->d_flag); af_free(c->d_pos); af_free(c->d_score); af_free(c->d_ncig); af_free(c->d_hits);
        af_free(c->d_cigar);
        c->cap_out = 0;
        HIPCHK(c, hipMalloc(&c->d_flag, 4 * nr)); HIPCHK(c, hipMalloc(&c->d_pos, 4 * nr));
        HIPCHK(c, hipMalloc(&c->d_score, 4 * nr)); HIPCHK(c, hipMalloc(&c->d_ncig, 4 * nr));
        HIPCHK(c, hipMalloc(&c->d_hits, 4 * nr));
        HIPCHK(c, hipMalloc(&c->d_cigar, sizeof(uint32_t) * AF_MAX_CIGAR * nr));
        c->cap_out = nr;
    }
    hipStream_t s = c->stream;
    HIPCHK(c, hipMemcpyAsync(c->d_reads, reads, bytes, hipMemcpyHostToDevice, s));
    if (lens) {
        for (int64_t i = 0; i < nr; ++i)
            if (lens[i] < 0 || lens[i] > stride) return fail(c, AF_E_INVALID, "lens[%lld]=%d outside [0, stride]", (long long)i, lens[i]);
        HIPCHK(c, hipMemcpyAsync(c->d_lens, lens, 4 * nr, hipMemcpyHostToDevice, s));
    }
    af_aln_out d{c->d_flag, c->d_pos, c->d_score, c->d_ncig, c->d_hits, c->d_cigar};
    int rc = af_align_pairs_device(c, ix, c->d_reads, n_pairs, stride, lens ? c->d_lens : nullptr, p, pe, &d, s);
    if (rc) return rc;
    if (out->flag) HIPCHK(c, hipMemcpyAsync(out->flag, c->d_flag, 4 * nr, hipMemcpyDeviceToHost, s));
    if (out->pos) HIPCHK(c, hipMemcpyAsync(out->pos, c->d_pos, 4 * nr, hipMemcpyDeviceToHost, s));
    if (out->score) HIPCHK(c, hipMemcpyAsync(out->score, c->d_score, 4 * nr, hipMemcpyDeviceToHost, s));
    if (out->n_cigar) HIPCHK(c, hipMemcpyAsync(out->n_cigar, c->d_ncig, 4 * nr, hipMemcpyDeviceToHost, s));
    if (out->hits) HIPCHK(c, hipMemcpyAsync(out->hits, c->d_hits, 4 * nr, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    if (out->cigar) {
        // only reads of listed pairs (a K1 candidate in the pair) have CIGARs: gather the rows of
        // both reads of every listed pair on the device and copy those
        const int slot = (int)((c->epoch - 1) & 1);
        int32_t np = 0;
        HIPCHK(c, hipMemcpy(&np, c->ctrl + AF_CTRL_S2_NPAIRS + AF_HEAD_STRIDE * slot, sizeof np, hipMemcpyDeviceToHost));
        if (np > 0) {
            const int64_t nrows = 2 * (int64_t)np;
            if (nrows > c->cap_packed) {
                af_free(c->d_packed); c->d_packed = nullptr; c->cap_packed = 0;
                HIPCHK(c, hipMalloc(&c->d_packed, sizeof(uint32_t) * AF_MAX_CIGAR * (size_t)nrows));
                c->cap_packed = nrows;
            }
            hipLaunchKernelGGL(k_gather_cigar, dim3((unsigned)std::min<int64_t>(4096, (nrows * 8 + 255) / 256)),
                               dim3(256), 0, s, c->s2_plist, nrows, c->d_cigar, c->d_packed);
            HIPCHK(c, hipGetLastError());
            std::vector<int32_t> ids((size_t)np);
            std::vector<uint32_t> rows((size_t)nrows * AF_MAX_CIGAR);
            HIPCHK(c, hipMemcpyAsync(ids.data(), c->s2_plist, sizeof(int32_t) * np, hipMemcpyDeviceToHost, s));
            HIPCHK(c, hipMemcpyAsync(rows.data(), c->d_packed, sizeof(uint32_t) * AF_MAX_CIGAR * nrows,
                                     hipMemcpyDeviceToHost, s));
            HIPCHK(c, hipStreamSynchronize(s));
            for (int64_t i = 0; i < nrows; ++i)
                memcpy(out->cigar + (2 * (int64_t)ids[i >> 1] + (i & 1)) * AF_MAX_CIGAR,
                       rows.data() + (size_t)i * AF_MAX_CIGAR, sizeof(uint32_t) * AF_MAX_CIGAR);
        }
    }
    return AF_OK;
}

int af_partition_device(af_ctx *c, const int32_t *d_flag, const int32_t *d_pos, int64_t n_reads, int64_t ref_len,
                        int32_t *d_tmp1, int32_t *d_tmp2, int32_t *d_anchored, int64_t *d_counts, void *stream) {
    if (!c || !d_counts || (n_reads > 0 && (!d_flag || !d_pos || !d_tmp1 || !d_tmp2 || !d_anchored)))
        return fail(c, AF_E_INVALID, "null argument");
    if (n_reads < 0 || n_reads > (1LL << 31) - 1) return fail(c, AF_E_INVALID, "n_reads out of range");
    if (ref_len <= 0 || ref_len > (1LL << 31) - 1) return fail(c, AF_E_INVALID, "ref_len outside [1, 2^31)");
    (void)hipSetDevice(c->device);
    const hipStream_t s = (hipStream_t)stream;
    if (n_reads == 0) {
        HIPCHK(c, hipMemsetAsync(d_counts, 0, 3 * sizeof(int64_t), s));
        return AF_OK;
    }
    if (n_reads > c->s3_cap) {
        HIPCHK(c, hipStreamSynchronize(s));
        if (c->s3_keys) (void)hipFree(c->s3_keys);
        if (c->s3_temp) (void)hipFree(c->s3_temp);
        c->s3_keys = nullptr; c->s3_temp = nullptr; c->s3_cap = 0;
        const size_t tb = af_s3_temp_bytes(n_reads);
        if (hipMalloc(&c->s3_keys, 2 * sizeof(uint64_t) * (size_t)n_reads) != hipSuccess ||
            hipMalloc(&c->s3_temp, tb) != hipSuccess)
            return fail(c, AF_E_NOMEM, "S3 scratch for %lld reads", (long long)n_reads);
        c->s3_cap = n_reads;
        c->s3_temp_bytes = tb;
    }
    if (!c->s3_counts && hipMalloc(&c->s3_counts, 4 * sizeof(int64_t)) != hipSuccess)
        return fail(c, AF_E_NOMEM, "S3 counts");
    HIPCHK(c, af_launch_s3(d_flag, d_pos, n_reads, ref_len, c->s3_keys, c->s3_keys + c->s3_cap, c->s3_temp,
                           c->s3_temp_bytes, c->s3_counts, d_tmp1, d_tmp2, d_anchored, s));
    HIPCHK(c, hipMemcpyAsync(d_counts, c->s3_counts, 3 * sizeof(int64_t), hipMemcpyDeviceToDevice, s));
    return AF_OK;
}

int af_split_tails_device(af_ctx *c, const uint8_t *d_reads, int64_t n_reads, int32_t stride,
                          const int32_t *d_lens, const af_aln_out *d_out, int32_t min_clip, int64_t read_base,
                          int32_t append, int64_t cap, uint8_t *d_tails, int32_t *d_tail_lens,
                          int32_t *d_tail_read, int32_t *d_n_tails, void *stream) {
    if (!c || !d_out || !d_n_tails || (n_reads > 0 && !d_reads) || (cap > 0 && (!d_tails || !d_tail_lens || !d_tail_read)))
        return fail(c, AF_E_INVALID, "null argument");
    if (n_reads < 0 || n_reads > (1LL << 31) - 1) return fail(c, AF_E_INVALID, "n_reads out of range");
    if (cap < 0) return fail(c, AF_E_INVALID, "cap < 0");
    if (read_base < 0 || read_base + n_reads > (1LL << 31) - 1) return fail(c, AF_E_INVALID, "read_base + n_reads exceeds int32");
    if (stride <= 0 || stride > AF_MAX_READ) return fail(c, AF_E_INVALID, "stride %d outside [1, %d]", stride, AF_MAX_READ);
    if (n_reads > 0 && (!d_out->flag || !d_out->n_cigar || !d_out->cigar))
        return fail(c, AF_E_INVALID, "d_out needs flag, n_cigar and cigar");
    (void)hipSetDevice(c->device);
    const AfTails t{d_tails, d_tail_lens, d_tail_read, d_n_tails, cap, read_base, min_clip < 1 ? 1 : min_clip};
    HIPCHK(c, af_launch_split_tails(d_reads, n_reads, stride, d_lens, *d_out, t, append != 0, (hipStream_t)stream));
    return AF_OK;
}

int af_gather_reads_device(af_ctx *c, const uint8_t *d_reads, int32_t stride, const int32_t *d_lens,
                           const int32_t *d_rows, int64_t n_rows, int32_t mode, const af_aln_out *d_out,
                           int64_t first, int64_t step, int64_t cap, uint8_t *d_q, int32_t *d_q_lens,
                           int32_t *d_q_rows, int32_t *d_n_q, void *stream) {
    if (!c) return AF_E_INVALID;
    if (n_rows < 0 || cap < 0 || first < 0 || step < 1 || stride < 1 || stride > AF_MAX_READ)
        return fail(c, AF_E_INVALID, "af_gather_reads_device: n_rows, cap, first >= 0, step >= 1, 1 <= stride <= %d",
                    AF_MAX_READ);
    if (mode != AF_GATHER_SEQUENCED && mode != AF_GATHER_SPLIT_SAM)
        return fail(c, AF_E_INVALID, "af_gather_reads_device: unknown mode %d", mode);
    if ((n_rows > 0 && (!d_reads || !d_rows || !d_q || !d_q_lens)) ||
        (mode == AF_GATHER_SPLIT_SAM && (!d_out || !d_out->flag || !d_out->n_cigar || !d_out->cigar)))
        return fail(c, AF_E_INVALID, "af_gather_reads_device: null buffer");
    (void)hipSetDevice(c->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (mode == AF_GATHER_SPLIT_SAM && n_rows > c->g_cap) {
        af_free(c->g_sel); af_free(c->g_temp);
        c->g_sel = nullptr; c->g_temp = nullptr; c->g_cap = 0;
        const size_t tb = af_gather_temp_bytes(n_rows);
        HIPCHK(c, hipMalloc(&c->g_sel, sizeof(int32_t) * (size_t)n_rows));
        HIPCHK(c, hipMalloc(&c->g_temp, std::max<size_t>(tb, 16)));
        c->g_cap = n_rows;
        c->g_temp_bytes = tb;
    }
    if (mode == AF_GATHER_SPLIT_SAM && !c->g_sel_n) HIPCHK(c, hipMalloc(&c->g_sel_n, sizeof(int64_t)));
    af_aln_out none{};
    HIPCHK(c, af_launch_gather(d_reads, stride, d_lens, d_rows, n_rows, mode, d_out ? *d_out : none, first, step, cap,
                               d_q, d_q_lens, d_q_rows, d_n_q, c->g_sel, c->g_sel_n, c->g_temp, c->g_temp_bytes, s));
    return AF_OK;
}

void af_blat_params_default(af_blat_params *p) {
    // blat's defaults for DNA (usage text of blat v.35): tileSize 11, stepSize = tileSize,
    // minMatch 2, repMatch 1024, minScore 30, minIdentity 90, maxGap 2, maxIntron 750000
    p->step_size = AF_TILE; p->min_match = 2; p->rep_match = 1024; p->min_score = 30;
    p->min_identity = 90; p->max_gap = 2; p->max_intron = 750000;
}

static int tile_build(af_ctx *c, const char *seq, int64_t len, int32_t step, af_index **out, bool dev) {
    if (!c || !seq || !out) return fail(c, AF_E_INVALID, "null argument");
    *out = nullptr;
    if (len < AF_TILE) return fail(c, AF_E_INVALID, "reference shorter than a tile (%d)", AF_TILE);
    if (len >= (1LL << 32) - 1) return fail(c, AF_E_UNSUPPORTED, "reference of 2^32 bases or more");
    if (step < 1 || step > AF_TILE) return fail(c, AF_E_INVALID, "step_size %d outside [1, %d]", step, AF_TILE);
    (void)hipSetDevice(c->device);
    af_index *ix = new (std::nothrow) af_index;
    if (!ix) return fail(c, AF_E_NOMEM, "out of host memory");
    ix->ctx = c;
    ix->is_tile = true;
    const uint8_t *d = reinterpret_cast<const uint8_t *>(seq);
    void *tmp = nullptr;
    hipError_t e = hipSuccess;
    if (!dev) {
        if ((e = hipMalloc(&tmp, (size_t)len)) != hipSuccess ||
            (e = hipMemcpyAsync(tmp, seq, (size_t)len, hipMemcpyHostToDevice, c->stream)) != hipSuccess) {
            af_free(tmp);
            af_index_free(ix);
            return fail(c, AF_E_HIP, "af_tile_index_build: upload: %s", hipGetErrorString(e));
        }
        d = static_cast<const uint8_t *>(tmp);
    }
    e = af_build_tile_index(d, len, step, &ix->tile, ix->allocs, &ix->n_allocs, c->stream);
    af_free(tmp);
    if (e != hipSuccess) {
        af_index_free(ix);
        return fail(c, AF_E_HIP, "af_tile_index_build: %s", hipGetErrorString(e));
    }
    ix->dev.n = len;
    *out = ix;
    return AF_OK;
}

int af_tile_index_build(af_ctx *c, const char *seq, int64_t len, int32_t step, af_index **out) {
    return tile_build(c, seq, len, step, out, false);
}

int af_tile_index_build_device(af_ctx *c, const char *d_seq, int64_t len, int32_t step, af_index **out) {
    return tile_build(c, d_seq, len, step, out, true);
}

static int check_blat(af_ctx *c, const af_index *ix, const af_blat_params *p, int32_t stride, int32_t max_rows) {
    if (!ix || !ix->is_tile) return fail(c, AF_E_INVALID, "af_blat needs a tile index (af_tile_index_build)");
    if (!p) return fail(c, AF_E_INVALID, "params is NULL");
    if (p->step_size != ix->tile.step)
        return fail(c, AF_E_INVALID, "step_size %d differs from the index's %d", p->step_size, ix->tile.step);
    if (p->min_match < 1 || p->rep_match < 1 || p->min_identity < 0 || p->min_identity > 100 || p->max_gap < 0 ||
        p->max_intron < 0)
        return fail(c, AF_E_INVALID, "invalid af_blat_params");
    if (stride <= 0 || stride > AF_MAX_READ) return fail(c, AF_E_INVALID, "stride %d outside [1, %d]", stride, AF_MAX_READ);
    if (max_rows < 1 || max_rows > AF_BLAT_MAX_ROWS)
        return fail(c, AF_E_INVALID, "max_rows must be in [1, %d]", AF_BLAT_MAX_ROWS);
    return AF_OK;
}

// a search's launch arguments on c's scratch; heavy strands are deferred to c->blat_hv's table
static BlatLaunch blat_launch(af_ctx *c, const af_index *ix, const uint8_t *q, const int32_t *n_q, const int32_t *first,
                              int64_t cap, int32_t stride, const int32_t *lens, const af_blat_params &p, af_psl *rows,
                              int32_t *n_rows, int32_t max_rows, const int32_t *order, bool with_spill) {
    BlatLaunch B;
    B.X = ix->tile;
    B.queries = q; B.n_queries = n_q; B.q_first = first; B.cap = cap; B.stride = stride; B.lens = lens; B.p = p;
    B.heads = c->ctrl + AF_CTRL_PLACE_HEADS; B.bscratch = c->bscratch; B.n_slots = c->blat_slots;
    B.rows = rows; B.n_rows = n_rows; B.max_rows = max_rows; B.order = order;
    B.stage = c->blat_stage; B.stage_n = c->blat_stage_n;
    B.caps = BlatCaps{c->blat_caps, with_spill ? c->blat_qcaps : nullptr, with_spill ? c->blat_qcap : 0};
    if (with_spill) B.spill = c->blat_spill;
    B.hv = c->blat_hv;
    return B;
}

int af_blat(af_ctx *c, const af_index *ix, const uint8_t *queries, int64_t n_queries, int32_t stride,
            const int32_t *lens, const af_blat_params *p, int32_t max_rows, af_psl *rows, int32_t *n_rows) {
    static_assert(sizeof(af_psl) == 328, "af_psl layout is part of the C-ABI");
    if (!c || !rows || !n_rows || (!queries && n_queries)) return fail(c, AF_E_INVALID, "null argument");
    int rc = check_blat(c, ix, p, stride, max_rows);
    if (rc) return rc;
    if (n_queries < 0 || n_queries > (1LL << 30)) return fail(c, AF_E_INVALID, "n_queries out of range");
    if (n_queries == 0) return AF_OK;
    if (lens)
        for (int64_t i = 0; i < n_queries; ++i)
            if (lens[i] < 0 || lens[i] > stride) return fail(c, AF_E_INVALID, "lens[%lld]=%d outside [0, stride]", (long long)i, lens[i]);
    (void)hipSetDevice(c->device);
    if ((rc = ensure_bscratch(c, 2 * n_queries)) || (rc = ensure_blat_order(c, n_queries)) ||
        (rc = ensure_blat_stage(c, n_queries, max_rows)) || (rc = ensure_blat_heavy(c, n_queries)))
        return rc;
    const int64_t bytes = n_queries * (int64_t)stride, nr = n_queries * (int64_t)max_rows;
    uint8_t *d_q = nullptr;
    int32_t *d_lens = nullptr, *d_nrows = nullptr;
    af_psl *d_rows = nullptr;
    auto done = [&](int code) {
        af_free(d_q); af_free(d_lens); af_free(d_nrows); af_free(d_rows);
        return code;
    };
    if (hipMalloc(&d_q, bytes + 64) != hipSuccess || hipMalloc(&d_lens, 4 * n_queries + 64) != hipSuccess ||
        hipMalloc(&d_nrows, 4 * n_queries + 64) != hipSuccess || hipMalloc(&d_rows, sizeof(af_psl) * nr) != hipSuccess)
        return done(fail(c, AF_E_NOMEM, "af_blat: device buffers"));
    hipStream_t s = c->stream;
    const int32_t nq = (int32_t)n_queries;
    hipError_t e;
    if ((e = hipMemcpyAsync(d_q, queries, bytes, hipMemcpyHostToDevice, s)) != hipSuccess ||
        (lens && (e = hipMemcpyAsync(d_lens, lens, 4 * n_queries, hipMemcpyHostToDevice, s)) != hipSuccess) ||
        (e = hipMemsetAsync(c->ctrl + AF_CTRL_PLACE_HEADS, 0, 4 * AF_HEAD_STRIDE * 8, s)) != hipSuccess ||
        (e = hipMemcpyAsync(c->ctrl + AF_CTRL_PLACE_N, &nq, 4, hipMemcpyHostToDevice, s)) != hipSuccess ||
        // rows past a query's n_rows come back zeroed, not as stale device memory
        (e = hipMemsetAsync(d_rows, 0, sizeof(af_psl) * nr, s)) != hipSuccess ||
        (e = af_launch_blat_order(ix->tile, d_q, c->ctrl + AF_CTRL_PLACE_N, n_queries, stride,
                                  lens ? d_lens : nullptr, p->rep_match, c->blat_ord_work, c->blat_order, s)) !=
            hipSuccess ||
        (e = af_launch_blat(blat_launch(c, ix, d_q, c->ctrl + AF_CTRL_PLACE_N, nullptr, n_queries, stride,
                                        lens ? d_lens : nullptr, *p, d_rows, d_nrows, max_rows, c->blat_order, false),
                            s)) != hipSuccess ||
        (e = hipMemcpyAsync(rows, d_rows, sizeof(af_psl) * nr, hipMemcpyDeviceToHost, s)) != hipSuccess ||
        (e = hipMemcpyAsync(n_rows, d_nrows, 4 * n_queries, hipMemcpyDeviceToHost, s)) != hipSuccess ||
        (e = hipStreamSynchronize(s)) != hipSuccess)
        return done(fail(c, AF_E_HIP, "af_blat: %s", hipGetErrorString(e)));
    return done(AF_OK);
}

int af_blat_long(af_ctx *c, const af_index *ix, const uint8_t *query, int32_t len, const af_blat_params *p,
                 int32_t max_rows, af_psl *rows, int32_t *n_rows, af_psl_block *blocks, int64_t block_cap,
                 int64_t *block_off, int64_t *n_blocks) {
    if (!c || !n_rows || !n_blocks || (len > 0 && !query) || (max_rows > 0 && (!rows || !block_off)))
        return fail(c, AF_E_INVALID, "null argument");
    int rc = check_blat(c, ix, p, 1, 1);
    if (rc) return rc;
    if (len < 0 || len > AF_BLAT_LONG_MAX) return fail(c, AF_E_INVALID, "query length %d outside [0, %d]", len, AF_BLAT_LONG_MAX);
    if (max_rows < 0 || block_cap < 0) return fail(c, AF_E_INVALID, "max_rows / block_cap out of range");
    (void)hipSetDevice(c->device);
    if (!c->blat_caps) {
        HIPCHK(c, hipMalloc(&c->blat_caps, sizeof(int32_t) * AF_BLAT_CAP_N));
        HIPCHK(c, hipMemset(c->blat_caps, 0, sizeof(int32_t) * AF_BLAT_CAP_N));
    }
    // the codes of both strands (strand 1: the reverse complement)
    std::vector<uint8_t> q2(2 * (size_t)len + 16, 4);
    for (int i = 0; i < len; ++i) {
        const uint8_t ch = query[i];
        const uint8_t x = (ch == 'A' || ch == 'a') ? 0 : (ch == 'C' || ch == 'c') ? 1 : (ch == 'G' || ch == 'g') ? 2
                        : (ch == 'T' || ch == 't') ? 3 : 4;
        q2[i] = x;
        q2[len + (len - 1 - i)] = x > 3 ? 4 : 3 - x;
    }
    uint8_t *d_q2 = nullptr;
    HIPCHK(c, hipMalloc(&d_q2, q2.size()));
    std::vector<af_psl> r;
    std::vector<int32_t> seq;
    std::vector<int64_t> boff;
    std::vector<af_psl_block> blk;
    hipError_t e = hipMemcpyAsync(d_q2, q2.data(), q2.size(), hipMemcpyHostToDevice, c->stream);
    int overflow = 0;
    if (e == hipSuccess)
        e = af_blat_long_run(ix->tile, d_q2, len, *p, c->blat_caps, r, seq, boff, blk, c->n_cu, c->stream, &overflow);
    (void)hipFree(d_q2);
    if (e == hipErrorOutOfMemory) return fail(c, AF_E_NOMEM, "af_blat_long: device memory");
    if (e != hipSuccess) return fail(c, AF_E_HIP, "af_blat_long: %s", hipGetErrorString(e));
    if (overflow) return fail(c, AF_E_CAPACITY, "af_blat_long: the device row list / block arena overflowed");
    // every row best first: score desc, strand, tStart, qStart, tEnd, qEnd, then emission order
    std::vector<int64_t> ord(r.size());
    for (size_t k = 0; k < ord.size(); ++k) ord[k] = (int64_t)k;
    std::sort(ord.begin(), ord.end(), [&](int64_t a, int64_t b) {
        const af_psl &x = r[a], &y = r[b];
        if (x.score != y.score) return x.score > y.score;
        if (x.strand != y.strand) return x.strand < y.strand;
        if (x.t_start != y.t_start) return x.t_start < y.t_start;
        if (x.q_start != y.q_start) return x.q_start < y.q_start;
        if (x.t_end != y.t_end) return x.t_end < y.t_end;
        if (x.q_end != y.q_end) return x.q_end < y.q_end;
        return seq[a] < seq[b];
    });
    const int64_t m = std::min<int64_t>((int64_t)r.size(), max_rows);
    int64_t nb = 0;
    for (int64_t k = 0; k < m; ++k) nb += r[ord[k]].block_count;
    *n_rows = (int32_t)r.size();
    *n_blocks = nb;
    if (nb > block_cap) return fail(c, AF_E_CAPACITY, "af_blat_long: %lld blocks, room for %lld", (long long)nb,
                                    (long long)block_cap);
    int64_t off = 0;
    for (int64_t k = 0; k < m; ++k) {
        const af_psl &h = r[ord[k]];
        rows[k] = h;
        block_off[k] = off;
        for (int b = 0; b < h.block_count; ++b) blocks[off++] = blk[boff[ord[k]] + b];
    }
    if (max_rows > 0) block_off[m] = off;
    return AF_OK;
}

int af_blat_device(af_ctx *c, const af_index *ix, const uint8_t *d_queries, const int32_t *d_n_queries,
                   int64_t cap_queries, int32_t stride, const int32_t *d_lens, const af_blat_params *p,
                   int32_t max_rows, af_psl *d_rows, int32_t *d_n_rows, void *stream) {
    return af_blat_device_range(c, ix, d_queries, nullptr, d_n_queries, cap_queries, stride, d_lens, p, max_rows,
                                d_rows, d_n_rows, stream);
}

// enqueues the first part of a device search (af_launch_blat_begin) and keeps its arguments on c
static int blat_device_begin(af_ctx *c, const af_index *ix, const uint8_t *d_queries, const int32_t *d_first,
                             const int32_t *d_n_queries, int64_t cap_queries, int32_t stride, const int32_t *d_lens,
                             const af_blat_params *p, int32_t max_rows, af_psl *d_rows, int32_t *d_n_rows,
                             hipStream_t s) {
    if (!c || !d_n_queries || (cap_queries > 0 && (!d_queries || !d_rows || !d_n_rows)))
        return fail(c, AF_E_INVALID, "null argument");
    int rc = check_blat(c, ix, p, stride, max_rows);
    if (rc) return rc;
    if (cap_queries < 0 || cap_queries > (1LL << 30)) return fail(c, AF_E_INVALID, "cap_queries out of range");
    c->blat_open = false;
    if (cap_queries == 0) return AF_OK;
    (void)hipSetDevice(c->device);
    if ((rc = ensure_bscratch(c, 2 * cap_queries)) || (rc = ensure_blat_stage(c, cap_queries, max_rows)) ||
        (rc = ensure_blat_heavy(c, cap_queries)))
        return rc;
    HIPCHK(c, hipMemsetAsync(c->ctrl + AF_CTRL_PLACE_HEADS, 0, 4 * AF_HEAD_STRIDE * 8, s));
    HIPCHK(c, af_launch_clamp_count(d_n_queries, cap_queries, c->ctrl + AF_CTRL_PLACE_N, s));
    const int32_t *order = nullptr;  // a subrange keeps query order; the whole set runs heaviest first
    if (!d_first) {
        if ((rc = ensure_blat_order(c, cap_queries))) return rc;
        HIPCHK(c, af_launch_blat_order(ix->tile, d_queries, c->ctrl + AF_CTRL_PLACE_N, cap_queries, stride, d_lens,
                                       p->rep_match, c->blat_ord_work, c->blat_order, s));
        order = c->blat_order;
    }
    c->blat_pending = blat_launch(c, ix, d_queries, c->ctrl + AF_CTRL_PLACE_N, d_first, cap_queries, stride, d_lens, *p,
                                  d_rows, d_n_rows, max_rows, order, true);
    HIPCHK(c, af_launch_blat_begin(c->blat_pending, s));
    c->blat_open = true;
    return AF_OK;
}

int af_blat_device_range(af_ctx *c, const af_index *ix, const uint8_t *d_queries, const int32_t *d_first,
                         const int32_t *d_n_queries, int64_t cap_queries, int32_t stride, const int32_t *d_lens,
                         const af_blat_params *p, int32_t max_rows, af_psl *d_rows, int32_t *d_n_rows, void *stream) {
    if (int rc = blat_device_begin(c, ix, d_queries, d_first, d_n_queries, cap_queries, stride, d_lens, p, max_rows,
                                   d_rows, d_n_rows, (hipStream_t)stream))
        return rc;
    return af_blat_device_end(c, nullptr, stream);
}

int af_blat_device_begin(af_ctx *c, const af_index *ix, const uint8_t *d_queries, const int32_t *d_n_queries,
                         int64_t cap_queries, int32_t stride, const int32_t *d_lens, const af_blat_params *p,
                         int32_t max_rows, af_psl *d_rows, int32_t *d_n_rows, void *stream) {
    return blat_device_begin(c, ix, d_queries, nullptr, d_n_queries, cap_queries, stride, d_lens, p, max_rows, d_rows,
                             d_n_rows, (hipStream_t)stream);
}

int af_blat_device_end(af_ctx *c, const uint8_t *d_live, void *stream) {
    if (!c) return fail(c, AF_E_INVALID, "null argument");
    if (!c->blat_open) return AF_OK;  // nothing begun (or an empty search)
    c->blat_open = false;
    (void)hipSetDevice(c->device);
    HIPCHK(c, af_launch_blat_end(c->blat_pending, d_live, (hipStream_t)stream));
    return AF_OK;
}

int af_blat_spill(af_ctx *c, af_psl *d_rows, int32_t *d_query, int32_t *d_n, int64_t cap) {
    if (!c) return fail(c, AF_E_INVALID, "null argument");
    if (!d_rows || cap <= 0) { c->blat_spill = BlatSpill{}; return AF_OK; }
    if (!d_query || !d_n) return fail(c, AF_E_INVALID, "af_blat_spill: null query / count buffer");
    c->blat_spill = BlatSpill{d_rows, d_query, d_n, cap};
    return AF_OK;
}

int af_blat_query_caps(af_ctx *c, int32_t *d_counts, int64_t cap) {
    if (!c) return fail(c, AF_E_INVALID, "null argument");
    if (!d_counts || cap <= 0) { c->blat_qcaps = nullptr; c->blat_qcap = 0; return AF_OK; }
    c->blat_qcaps = d_counts;
    c->blat_qcap = cap;
    return AF_OK;
}

int af_blat_heavy_stats(af_ctx *c, int32_t *out) {
    if (!c || !out) return fail(c, AF_E_INVALID, "null argument");
    for (int k = 0; k < 4; ++k) out[k] = 0;
    if (!c->blat_hv.ctrl) return AF_OK;
    (void)hipSetDevice(c->device);
    HIPCHK(c, hipDeviceSynchronize());
    const int32_t at[4] = {AF_BLAT_HV_STRANDS_N, AF_BLAT_HV_JOBS_N, AF_BLAT_HV_JOBS_DONE, AF_BLAT_HV_STRANDS_DONE};
    for (int k = 0; k < 4; ++k) HIPCHK(c, hipMemcpy(out + k, c->blat_hv.ctrl + at[k], 4, hipMemcpyDeviceToHost));
    return AF_OK;
}

int af_blat_caps(af_ctx *c, int32_t *out, int reset) {
    if (!c || !out) return fail(c, AF_E_INVALID, "null argument");
    if (!c->blat_caps) { for (int k = 0; k < AF_BLAT_CAP_N; ++k) out[k] = 0; return AF_OK; }
    (void)hipSetDevice(c->device);
    HIPCHK(c, hipDeviceSynchronize());
    HIPCHK(c, hipMemcpy(out, c->blat_caps, sizeof(int32_t) * AF_BLAT_CAP_N, hipMemcpyDeviceToHost));
    if (reset) HIPCHK(c, hipMemset(c->blat_caps, 0, sizeof(int32_t) * AF_BLAT_CAP_N));
    return AF_OK;
}

// ---- genome calls S4 / S5 ------------------------------------------------------------------
int af_genome_build(af_ctx *c, const char *blob, int64_t n_blob, const int64_t *ctg_off, const int64_t *ctg_len,
                    int32_t n_ctg, af_genome **out) {
    return genome_build(c, blob, n_blob, ctg_off, ctg_len, n_ctg, out, false);
}
int af_genome_build_device(af_ctx *c, const char *d_blob, int64_t n_blob, const int64_t *ctg_off,
                           const int64_t *ctg_len, int32_t n_ctg, af_genome **out) {
    return genome_build(c, d_blob, n_blob, ctg_off, ctg_len, n_ctg, out, true);
}
void af_genome_free(af_genome *g) {
    if (!g) return;
    if (g->ctx) (void)hipSetDevice(g->ctx->device);
    af_fm_free(&g->dev);
    delete g;
}
int64_t af_genome_lpac(const af_genome *g) { return g ? g->dev.l_pac : -1; }
int64_t af_genome_primary(const af_genome *g) { return g ? g->dev.primary : -1; }

int af_genome_read(af_ctx *c, const af_genome *g, int32_t what, int64_t first, int64_t n, void *out) {
    if (!c || !g || !out || first < 0 || n < 0) return fail(c, AF_E_INVALID, "bad argument");
    const int64_t rows = what == 0 ? g->dev.N : what == 1 ? g->dev.N + 1 : 8 * g->dev.n_blk;
    if (what < 0 || what > 2 || first + n > rows)
        return fail(c, AF_E_INVALID, "range outside the text / suffix array / occurrence table");
    (void)hipSetDevice(c->device);
    if (what == 0) HIPCHK(c, hipMemcpy(out, g->dev.T + first, n, hipMemcpyDeviceToHost));
    else if (what == 1) HIPCHK(c, hipMemcpy(out, g->dev.sa + first, sizeof(int64_t) * n, hipMemcpyDeviceToHost));
    else HIPCHK(c, hipMemcpy(out, g->dev.occ + first, sizeof(uint64_t) * n, hipMemcpyDeviceToHost));
    return AF_OK;
}

static GOpt genome_opt(const af_pe *e) {
    af_pe d;
    if (!e) { af_pe_default(&d); e = &d; }
    return GOpt{e->pen_unpaired, e->max_ins, e->max_matesw, e->split_width, e->max_mem_intv, e->max_chain_gap,
                e->pair_base};
}

static int genome_se_device(af_ctx *c, const af_genome *g, const uint8_t *d_reads, int64_t n, int32_t stride,
                            const int32_t *d_lens, const af_params *p, const af_pe *pe, int64_t id_base,
                            const int64_t *d_ids, af_grec *d_recs, int32_t *d_n_rec, void *stream) {
    int rc = check_genome_call(c, g, p, pe, stride);
    if (rc) return rc;
    if (n < 0 || (n > 0 && (!d_reads || !d_recs || !d_n_rec))) return fail(c, AF_E_INVALID, "null argument");
    if (n == 0) return AF_OK;
    (void)hipSetDevice(c->device);
    if ((rc = ensure_genome_scratch(c)) || (rc = ensure_genome_pools(c, n))) return rc;
    hipStream_t s = (hipStream_t)stream;
    const GOpt o = genome_opt(pe);
    const GWork w = genome_work(c, n);
    HIPCHK(c, af_launch_genome_regions(g->dev, d_reads, stride, d_lens, nullptr, n, *p, o, w, c->g1_scr, c->g1_threads,
                                       c->g2_scr, c->g2_waves, c->zscratch, s));
    HIPCHK(c, af_launch_genome_se(g->dev, d_reads, stride, d_lens, nullptr, n, *p, id_base, d_ids, w, c->g2_scr,
                                  c->g2_waves, c->zscratch, d_recs, d_n_rec, s));
    return AF_OK;
}

int af_genome_align_se_device(af_ctx *c, const af_genome *g, const uint8_t *d_reads, int64_t n, int32_t stride,
                              const int32_t *d_lens, const af_params *p, const af_pe *pe, int64_t id_base,
                              af_grec *d_recs, int32_t *d_n_rec, void *stream) {
    return genome_se_device(c, g, d_reads, n, stride, d_lens, p, pe, id_base, nullptr, d_recs, d_n_rec, stream);
}

int af_genome_align_se_ids_device(af_ctx *c, const af_genome *g, const uint8_t *d_reads, int64_t n, int32_t stride,
                                  const int32_t *d_lens, const af_params *p, const af_pe *pe, const int64_t *d_ids,
                                  af_grec *d_recs, int32_t *d_n_rec, void *stream) {
    if (n > 0 && !d_ids) return fail(c, AF_E_INVALID, "null argument");
    return genome_se_device(c, g, d_reads, n, stride, d_lens, p, pe, 0, d_ids, d_recs, d_n_rec, stream);
}

int af_genome_align_pe_device(af_ctx *c, const af_genome *g, const uint8_t *d_reads, int64_t n_pairs,
                              int32_t stride, const int32_t *d_lens, const af_params *p, const af_pe *pe,
                              af_grec *d_recs, int32_t *d_n_rec, void *stream) {
    af_pe e;
    if (pe) e = *pe;
    else af_pe_default(&e);
    int rc = check_genome_call(c, g, p, &e, stride);
    if (rc) return rc;
    if (n_pairs < 0 || (n_pairs > 0 && (!d_reads || !d_lens || !d_recs || !d_n_rec)))
        return fail(c, AF_E_INVALID, "null argument (paired-end calls need the read lengths)");
    if (n_pairs == 0) return AF_OK;
    (void)hipSetDevice(c->device);
    if ((rc = ensure_genome_scratch(c)) || (rc = ensure_genome_pools(c, 2 * n_pairs)) ||
        (rc = ensure_genome_pe(c, n_pairs, stride, e.chunk_bases, e.max_ins)))
        return rc;
    hipStream_t s = (hipStream_t)stream;
    const GOpt o = genome_opt(&e);
    const GWork w = genome_work(c, 2 * n_pairs);
    S2Work sw{};
    sw.ghist = c->g_ghist; sw.pes = c->g_pes; sw.ppc = 0; sw.cstart = c->g_cstart; sw.n_chunks = c->g_nchunks;
    sw.max_chunks = c->g_max_chunks;
    HIPCHK(c, af_launch_s2_chunks(n_pairs, stride, d_lens, e.chunk_bases, c->g_cstart, c->g_scan, c->g_max_chunks,
                                  c->g_nchunks, s));
    HIPCHK(c, af_launch_genome_regions(g->dev, d_reads, stride, d_lens, nullptr, 2 * n_pairs, *p, o, w, c->g1_scr,
                                       c->g1_threads, c->g2_scr, c->g2_waves, c->zscratch, s));
    HIPCHK(c, af_launch_genome_pe(g->dev, d_reads, stride, d_lens, nullptr, n_pairs, *p, o, w, sw, c->g2_scr,
                                  c->g2_waves, c->zscratch, d_recs, d_n_rec, s));
    return AF_OK;
}

int af_genome_align_pe_se_device(af_ctx *c, const af_genome *g, const uint8_t *d_reads, int64_t n_pairs, int64_t n_se,
                                 int32_t stride, const int32_t *d_lens, const af_params *p, const af_pe *pe_s4,
                                 const af_pe *pe_s5, int64_t se_id_base, const int64_t *d_se_ids, af_grec *d_recs,
                                 int32_t *d_n_rec, void *stream, void *stream_pe) {
    af_pe e4, e5;
    if (pe_s4) e4 = *pe_s4;
    else af_pe_default(&e4);
    if (pe_s5) e5 = *pe_s5;
    else af_pe_default(&e5);
    int rc = check_genome_call(c, g, p, &e4, stride);
    if (rc || (rc = check_pe(c, &e5))) return rc;
    if (n_pairs < 0 || n_se < 0 || (n_pairs + n_se > 0 && (!d_reads || !d_lens || !d_recs || !d_n_rec)))
        return fail(c, AF_E_INVALID, "null argument (the reads' lengths are required)");
    // one launch of the seed / region kernels holds both calls: their options must agree
    if (e4.split_width != e5.split_width || e4.max_mem_intv != e5.max_mem_intv || e4.max_chain_gap != e5.max_chain_gap)
        return fail(c, AF_E_INVALID, "S4 and S5 seeding options differ (split_width, max_mem_intv, max_chain_gap)");
    const int64_t n = 2 * n_pairs + n_se;
    if (n == 0) return AF_OK;
    if (n > INT32_MAX / 16) return fail(c, AF_E_INVALID, "too many reads for one genome call");
    (void)hipSetDevice(c->device);
    if ((rc = ensure_genome_scratch(c)) || (rc = ensure_genome_pools(c, n)) ||
        (n_pairs && (rc = ensure_genome_pe(c, n_pairs, stride, e4.chunk_bases, e4.max_ins))))
        return rc;
    hipStream_t s = (hipStream_t)stream, spe = stream_pe ? (hipStream_t)stream_pe : s;
    if (spe != s && !c->g2_scr_pe) {
        HIPCHK(c, hipMalloc(&c->g2_scr_pe, af_g2_slot_bytes() * (size_t)c->g2_waves));
        HIPCHK(c, hipMalloc(&c->zscratch_pe, (size_t)(AF_MAX_READ + 1) * 1024 * (size_t)c->n_slots));
    }
    if (!c->g_ev) HIPCHK(c, hipEventCreateWithFlags(&c->g_ev, hipEventDisableTiming));
    const GOpt o = genome_opt(&e4);
    const GWork w = genome_work(c, n);
    if (n_pairs)
        HIPCHK(c, af_launch_s2_chunks(n_pairs, stride, d_lens, e4.chunk_bases, c->g_cstart, c->g_scan, c->g_max_chunks,
                                      c->g_nchunks, s));
    HIPCHK(c, af_launch_genome_regions(g->dev, d_reads, stride, d_lens, nullptr, n, *p, o, w, c->g1_scr, c->g1_threads,
                                       c->g2_scr, c->g2_waves, c->zscratch, s));
    if (n_pairs) {
        S2Work sw{};
        sw.ghist = c->g_ghist; sw.pes = c->g_pes; sw.ppc = 0; sw.cstart = c->g_cstart; sw.n_chunks = c->g_nchunks;
        sw.max_chunks = c->g_max_chunks;
        if (spe != s) {
            HIPCHK(c, hipEventRecord(c->g_ev, s));
            HIPCHK(c, hipStreamWaitEvent(spe, c->g_ev, 0));
        }
        HIPCHK(c, af_launch_genome_pe(g->dev, d_reads, stride, d_lens, nullptr, n_pairs, *p, o, w, sw,
                                      spe != s ? c->g2_scr_pe : c->g2_scr, c->g2_waves,
                                      spe != s ? c->zscratch_pe : c->zscratch, d_recs, d_n_rec, spe));
    }
    if (n_se) {
        // the single-end reads' view: rows [2 n_pairs, n) of the launch
        const int64_t b = 2 * n_pairs;
        GWork ws = w;
        ws.reg_off += b; ws.reg_n += b; ws.iv_off += b; ws.iv_n += b;
        HIPCHK(c, af_launch_genome_se(g->dev, d_reads + b * stride, stride, d_lens + b, nullptr, n_se, *p, se_id_base,
                                      d_se_ids, ws, c->g2_scr, c->g2_waves, c->zscratch, d_recs + b * AF_G_MAX_REC,
                                      d_n_rec + b, s));
    }
    return AF_OK;
}

// host-buffer forms: reads / lens staged through the context's buffers
static int genome_stage(af_ctx *c, const uint8_t *reads, int64_t n_reads, int32_t stride, const int32_t *lens,
                        bool need_lens, const int32_t **d_lens) {
    const int64_t bytes = n_reads * (int64_t)stride;
    if (bytes > c->g_cap_hbytes) {
        af_free(c->g_hreads); c->g_hreads = nullptr; c->g_cap_hbytes = 0;
        HIPCHK(c, hipMalloc(&c->g_hreads, bytes + 16));
        c->g_cap_hbytes = bytes;
    }
    if (n_reads > c->g_cap_recs) {
        af_free(c->g_recs); af_free(c->g_nrec); af_free(c->g_hlens);
        c->g_recs = nullptr; c->g_nrec = nullptr; c->g_hlens = nullptr; c->g_cap_recs = 0;
        HIPCHK(c, hipMalloc(&c->g_recs, sizeof(af_grec) * AF_G_MAX_REC * n_reads));
        HIPCHK(c, hipMalloc(&c->g_nrec, sizeof(int32_t) * n_reads));
        HIPCHK(c, hipMalloc(&c->g_hlens, sizeof(int32_t) * n_reads));
        c->g_cap_recs = n_reads;
    }
    HIPCHK(c, hipMemcpyAsync(c->g_hreads, reads, bytes, hipMemcpyHostToDevice, c->stream));
    *d_lens = nullptr;
    if (lens || need_lens) {
        if (lens) HIPCHK(c, hipMemcpyAsync(c->g_hlens, lens, sizeof(int32_t) * n_reads, hipMemcpyHostToDevice, c->stream));
        else {
            std::vector<int32_t> u((size_t)n_reads, stride);
            HIPCHK(c, hipMemcpyAsync(c->g_hlens, u.data(), sizeof(int32_t) * n_reads, hipMemcpyHostToDevice, c->stream));
            HIPCHK(c, hipStreamSynchronize(c->stream));
        }
        *d_lens = c->g_hlens;
    }
    return AF_OK;
}

static int genome_unstage(af_ctx *c, int64_t n_reads, af_grec *recs, int32_t *n_rec) {
    HIPCHK(c, hipMemcpyAsync(recs, c->g_recs, sizeof(af_grec) * AF_G_MAX_REC * n_reads, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(n_rec, c->g_nrec, sizeof(int32_t) * n_reads, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return AF_OK;
}

int af_genome_align_se(af_ctx *c, const af_genome *g, const uint8_t *reads, int64_t n, int32_t stride,
                       const int32_t *lens, const af_params *p, const af_pe *pe, int64_t id_base, af_grec *recs,
                       int32_t *n_rec) {
    int rc = check_genome_call(c, g, p, pe, stride);
    if (rc) return rc;
    if (n < 0 || (n > 0 && (!reads || !recs || !n_rec))) return fail(c, AF_E_INVALID, "null argument");
    if (n == 0) return AF_OK;
    (void)hipSetDevice(c->device);
    const int32_t *d_lens = nullptr;
    if ((rc = genome_stage(c, reads, n, stride, lens, false, &d_lens))) return rc;
    if ((rc = af_genome_align_se_device(c, g, c->g_hreads, n, stride, d_lens, p, pe, id_base, c->g_recs, c->g_nrec,
                                        c->stream)))
        return rc;
    return genome_unstage(c, n, recs, n_rec);
}

int af_genome_align_pe(af_ctx *c, const af_genome *g, const uint8_t *reads, int64_t n_pairs, int32_t stride,
                       const int32_t *lens, const af_params *p, const af_pe *pe, af_grec *recs, int32_t *n_rec) {
    int rc = check_genome_call(c, g, p, pe, stride);
    if (rc) return rc;
    if (n_pairs < 0 || (n_pairs > 0 && (!reads || !recs || !n_rec))) return fail(c, AF_E_INVALID, "null argument");
    if (n_pairs == 0) return AF_OK;
    (void)hipSetDevice(c->device);
    const int32_t *d_lens = nullptr;
    if ((rc = genome_stage(c, reads, 2 * n_pairs, stride, lens, true, &d_lens))) return rc;
    if ((rc = af_genome_align_pe_device(c, g, c->g_hreads, n_pairs, stride, d_lens, p, pe, c->g_recs, c->g_nrec,
                                        c->stream)))
        return rc;
    return genome_unstage(c, 2 * n_pairs, recs, n_rec);
}

int af_genome_regions(af_ctx *c, const af_genome *g, const uint8_t *reads, int64_t n, int32_t stride,
                      const int32_t *lens, const af_params *p, const af_pe *pe, int32_t max_reg, int64_t *regs,
                      int32_t *n_reg) {
    int rc = check_genome_call(c, g, p, pe, stride);
    if (rc) return rc;
    if (n < 0 || max_reg < 1 || (n > 0 && (!reads || !regs || !n_reg))) return fail(c, AF_E_INVALID, "bad argument");
    if (n == 0) return AF_OK;
    (void)hipSetDevice(c->device);
    const int32_t *d_lens = nullptr;
    if ((rc = genome_stage(c, reads, n, stride, lens, false, &d_lens))) return rc;
    if ((rc = ensure_genome_scratch(c)) || (rc = ensure_genome_pools(c, n))) return rc;
    const GWork w = genome_work(c, n);
    HIPCHK(c, af_launch_genome_regions(g->dev, c->g_hreads, stride, d_lens, nullptr, n, *p, genome_opt(pe), w, c->g1_scr,
                                       c->g1_threads, c->g2_scr, c->g2_waves, c->zscratch, c->stream));
    std::vector<int32_t> off((size_t)n);
    int32_t fill = 0;
    HIPCHK(c, hipMemcpyAsync(n_reg, c->g_reg_n, sizeof(int32_t) * n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(off.data(), c->g_reg_off, sizeof(int32_t) * n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(&fill, c->g_reg_fill, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    std::vector<GReg> pool((size_t)std::max<int64_t>(std::min<int64_t>(fill, c->g_reg_cap), 1));
    if (fill > 0) HIPCHK(c, hipMemcpy(pool.data(), c->g_reg, sizeof(GReg) * std::min<int64_t>(fill, c->g_reg_cap),
                                      hipMemcpyDeviceToHost));
    for (int64_t r = 0; r < n; ++r) {
        for (int k = 0; k < n_reg[r] && k < max_reg; ++k) {
            const GReg &a = pool[(size_t)off[r] + k];
            int64_t *o = regs + (r * max_reg + k) * 12;
            o[0] = a.rb; o[1] = a.re; o[2] = a.qb; o[3] = a.qe; o[4] = a.rid; o[5] = a.score; o[6] = a.truesc;
            o[7] = a.w; o[8] = a.seedcov; o[9] = a.seedlen0; o[10] = 0; o[11] = 0;
        }
    }
    return AF_OK;
}

int af_genome_intervals(af_ctx *c, const af_genome *g, const uint8_t *reads, int64_t n, int32_t stride,
                        const int32_t *lens, const af_params *p, const af_pe *pe, int32_t max_iv, int64_t *ivs,
                        int32_t *n_iv) {
    int rc = check_genome_call(c, g, p, pe, stride);
    if (rc) return rc;
    if (n < 0 || max_iv < 1 || (n > 0 && (!reads || !ivs || !n_iv))) return fail(c, AF_E_INVALID, "bad argument");
    if (n == 0) return AF_OK;
    (void)hipSetDevice(c->device);
    const int32_t *d_lens = nullptr;
    if ((rc = genome_stage(c, reads, n, stride, lens, false, &d_lens))) return rc;
    if ((rc = ensure_genome_scratch(c)) || (rc = ensure_genome_pools(c, n))) return rc;
    const GWork w = genome_work(c, n);
    HIPCHK(c, af_launch_genome_intervals(g->dev, c->g_hreads, stride, d_lens, n, *p, genome_opt(pe), w, c->g1_scr,
                                         c->g1_threads, c->stream));
    std::vector<int64_t> off((size_t)n);
    unsigned long long fill = 0;
    HIPCHK(c, hipMemcpyAsync(n_iv, c->g_iv_n, sizeof(int32_t) * n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(off.data(), c->g_iv_off, sizeof(int64_t) * n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(&fill, c->g_iv_fill, sizeof fill, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const int64_t nf = std::min<int64_t>((int64_t)fill, c->g_iv_cap);
    std::vector<GIv> pool((size_t)std::max<int64_t>(nf, 1));
    if (nf > 0) HIPCHK(c, hipMemcpy(pool.data(), c->g_iv, sizeof(GIv) * nf, hipMemcpyDeviceToHost));
    for (int64_t r = 0; r < n; ++r)
        for (int k = 0; k < n_iv[r] && k < max_iv; ++k) {
            const GIv &v = pool[(size_t)off[r] + k];
            int64_t *o = ivs + (r * max_iv + k) * 4;
            o[0] = v.sa_k; o[1] = v.s; o[2] = v.qb; o[3] = v.qe;
        }
    return AF_OK;
}

int af_genome_stats(af_ctx *c, int32_t *out) {
    if (!c || !out) return fail(c, AF_E_INVALID, "null argument");
    if (!c->g_stats) { for (int k = 0; k < AF_GSTAT_N; ++k) out[k] = 0; return AF_OK; }
    (void)hipSetDevice(c->device);
    HIPCHK(c, hipDeviceSynchronize());
    HIPCHK(c, hipMemcpy(out, c->g_stats, sizeof(int32_t) * AF_GSTAT_N, hipMemcpyDeviceToHost));
    return AF_OK;
}

// the S5 check's per-query flags, selection and select scratch for n queries
static int ensure_s5(af_ctx *c, int64_t n_queries) {
    if (n_queries > c->s5_cap) {
        af_free(c->s5_keep); af_free(c->s5_sel); af_free(c->s5_temp);
        c->s5_keep = nullptr; c->s5_sel = nullptr; c->s5_temp = nullptr; c->s5_cap = 0;
        const int64_t n = std::max<int64_t>(n_queries, 1 << 16);
        c->s5_temp_bytes = af_s5_temp_bytes(n);
        HIPCHK(c, hipMalloc(&c->s5_keep, n));
        HIPCHK(c, hipMalloc(&c->s5_sel, sizeof(int32_t) * n));
        HIPCHK(c, hipMalloc(&c->s5_temp, std::max<size_t>(c->s5_temp_bytes, 16)));
        c->s5_cap = n;
    }
    if (!c->s5_nsel) HIPCHK(c, hipMalloc(&c->s5_nsel, sizeof(int64_t)));
    return AF_OK;
}

int af_s5_filter_device(af_ctx *c, const af_grec *d_recs, const int32_t *d_n_rec, int64_t n_queries,
                        const uint8_t *d_q, int32_t q_stride, const int32_t *d_q_lens, const int32_t *d_q_rows,
                        const af_aln_out *d_s2, const uint8_t *d_cont, int64_t cap, uint8_t *d_s6, int32_t s6_stride,
                        int32_t *d_s6_lens, int32_t *d_s6_src, int32_t *d_n6, int32_t *d_n_over, void *stream) {
    if (!c || !d_s2 || !d_n6) return fail(c, AF_E_INVALID, "null argument");
    if (n_queries < 0 || n_queries > (1LL << 30)) return fail(c, AF_E_INVALID, "n_queries out of range");
    if (n_queries > 0 && (!d_recs || !d_n_rec || !d_q || !d_q_lens || !d_q_rows || !d_s2->flag || !d_s2->pos ||
                          !d_s2->n_cigar || !d_s2->cigar))
        return fail(c, AF_E_INVALID, "null argument");
    if (cap < 0 || (cap > 0 && (!d_s6 || !d_s6_lens || !d_s6_src))) return fail(c, AF_E_INVALID, "null output buffer");
    if (q_stride <= 0 || q_stride > AF_MAX_READ || s6_stride <= 0 || s6_stride > AF_MAX_READ)
        return fail(c, AF_E_INVALID, "strides must be in [1, %d]", AF_MAX_READ);
    (void)hipSetDevice(c->device);
    if (int rc = ensure_s5(c, n_queries)) return rc;
    HIPCHK(c, af_launch_s5_filter(d_recs, d_n_rec, n_queries, d_q, q_stride, d_q_lens, d_q_rows, *d_s2, d_cont, cap, d_s6,
                                  s6_stride, d_s6_lens, d_s6_src, d_n6, d_n_over, c->s5_keep, c->s5_sel, c->s5_nsel, c->s5_temp,
                                  c->s5_temp_bytes, (hipStream_t)stream));
    return AF_OK;
}

static int check_s6_set(af_ctx *c, const af_s6_set *s, bool results, const char *what) {
    if (!s) return fail(c, AF_E_INVALID, "%s: null set", what);
    if (s->cap < 0 || s->cap > (1LL << 30) || s->spill_cap < 0 || s->spill_cap > (1LL << 30))
        return fail(c, AF_E_INVALID, "%s: capacity out of range", what);
    if (s->stride <= 0 || s->stride > AF_MAX_READ || (s->stride & 3))
        return fail(c, AF_E_INVALID, "%s: stride must be a multiple of 4 in [4, %d]", what, AF_MAX_READ);
    if (!s->n || (s->cap > 0 && (!s->q || !s->lens || !s->src)))
        return fail(c, AF_E_INVALID, "%s: null row buffer", what);
    if (results && s->cap > 0 && (!s->rows || !s->n_rows)) return fail(c, AF_E_INVALID, "%s: null PSL buffer", what);
    if (s->spill_cap > 0 && (!s->spill_rows || !s->spill_query || !s->spill_n))
        return fail(c, AF_E_INVALID, "%s: null spill buffer", what);
    return AF_OK;
}

int af_s6_queries_device(af_ctx *c, int64_t n_queries, const uint8_t *d_q, int32_t q_stride, const int32_t *d_q_lens,
                         const int32_t *d_q_rows, const af_aln_out *d_s2, const uint8_t *d_cont, const af_s6_set *pre,
                         void *stream) {
    if (!c || !d_s2) return fail(c, AF_E_INVALID, "null argument");
    if (int rc = check_s6_set(c, pre, false, "af_s6_queries_device")) return rc;
    if (n_queries < 0 || n_queries > (1LL << 30)) return fail(c, AF_E_INVALID, "n_queries out of range");
    if (n_queries > 0 && (!d_q || !d_q_lens || !d_q_rows || !d_s2->flag || !d_s2->pos || !d_s2->n_cigar || !d_s2->cigar))
        return fail(c, AF_E_INVALID, "null argument");
    if (q_stride <= 0 || q_stride > AF_MAX_READ) return fail(c, AF_E_INVALID, "q_stride must be in [1, %d]", AF_MAX_READ);
    (void)hipSetDevice(c->device);
    if (int rc = ensure_s5(c, n_queries)) return rc;
    HIPCHK(c, af_launch_s6_queries(n_queries, d_q, q_stride, d_q_lens, d_q_rows, *d_s2, d_cont, *pre, c->s5_keep,
                                   c->s5_sel, c->s5_nsel, c->s5_temp, c->s5_temp_bytes, (hipStream_t)stream));
    return AF_OK;
}

int af_s6_check_device(af_ctx *c, const af_grec *d_recs, const int32_t *d_n_rec, int64_t n_queries,
                       const int32_t *d_q_rows, const af_aln_out *d_s2, const uint8_t *d_cont, const af_s6_set *pre,
                       uint8_t *d_live, void *stream) {
    if (!c || !d_s2) return fail(c, AF_E_INVALID, "null argument");
    if (int rc = check_s6_set(c, pre, false, "af_s6_check_device")) return rc;
    if (pre->cap > 0 && !d_live) return fail(c, AF_E_INVALID, "af_s6_check_device: null live flags");
    if (n_queries < 0 || n_queries > (1LL << 30)) return fail(c, AF_E_INVALID, "n_queries out of range");
    if (n_queries > 0 && (!d_recs || !d_n_rec || !d_q_rows || !d_s2->flag || !d_s2->pos || !d_s2->n_cigar ||
                          !d_s2->cigar))
        return fail(c, AF_E_INVALID, "null argument");
    (void)hipSetDevice(c->device);
    if (int rc = ensure_s5(c, n_queries)) return rc;
    HIPCHK(c, af_launch_s6_check(d_recs, d_n_rec, n_queries, d_q_rows, *d_s2, d_cont, *pre, c->s5_keep, d_live,
                                 (hipStream_t)stream));
    return AF_OK;
}

int af_s6_compact_device(af_ctx *c, const af_s6_set *pre, const uint8_t *d_live, const af_s6_set *out,
                         int32_t max_rows, void *stream) {
    if (!c) return fail(c, AF_E_INVALID, "null argument");
    if (int rc = check_s6_set(c, pre, true, "af_s6_compact_device (pre)")) return rc;
    if (int rc = check_s6_set(c, out, true, "af_s6_compact_device (out)")) return rc;
    if (pre->cap > 0 && !d_live) return fail(c, AF_E_INVALID, "af_s6_compact_device: null live flags");
    if (pre->stride != out->stride) return fail(c, AF_E_INVALID, "af_s6_compact_device: pre and out strides differ");
    if (max_rows < 1 || max_rows > AF_BLAT_MAX_ROWS) return fail(c, AF_E_INVALID, "max_rows out of range");
    if (pre->spill_cap > 0 && out->spill_cap <= 0)
        return fail(c, AF_E_INVALID, "af_s6_compact_device: pre has a spill pool, out none");
    (void)hipSetDevice(c->device);
    if (!c->blat_caps) {
        HIPCHK(c, hipMalloc(&c->blat_caps, sizeof(int32_t) * AF_BLAT_CAP_N));
        HIPCHK(c, hipMemset(c->blat_caps, 0, sizeof(int32_t) * AF_BLAT_CAP_N));
    }
    if (pre->cap > c->s6_cap || pre->spill_cap > c->s6_spill_cap) {
        af_free(c->s6_flag); af_free(c->s6_idx); af_free(c->s6_sflag); af_free(c->s6_sidx); af_free(c->s6_temp);
        c->s6_flag = c->s6_idx = c->s6_sflag = c->s6_sidx = nullptr;
        c->s6_temp = nullptr;
        c->s6_cap = c->s6_spill_cap = 0;
        const int64_t n = std::max<int64_t>(pre->cap, 1 << 16), ns = std::max<int64_t>(pre->spill_cap, 1 << 16);
        c->s6_temp_bytes = std::max(af_s6_compact_temp_bytes(n), af_s6_compact_temp_bytes(ns));
        HIPCHK(c, hipMalloc(&c->s6_flag, sizeof(int32_t) * n));
        HIPCHK(c, hipMalloc(&c->s6_idx, sizeof(int32_t) * n));
        HIPCHK(c, hipMalloc(&c->s6_sflag, sizeof(int32_t) * ns));
        HIPCHK(c, hipMalloc(&c->s6_sidx, sizeof(int32_t) * ns));
        HIPCHK(c, hipMalloc(&c->s6_temp, std::max<size_t>(c->s6_temp_bytes, 16)));
        c->s6_cap = n;
        c->s6_spill_cap = ns;
    }
    HIPCHK(c, af_launch_s6_compact(*pre, d_live, *out, max_rows, c->blat_caps, c->s6_flag, c->s6_idx, c->s6_sflag,
                                   c->s6_sidx, c->s6_temp, c->s6_temp_bytes, (hipStream_t)stream));
    return AF_OK;
}

}  // extern "C"

