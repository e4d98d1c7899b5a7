// fmindex.hip -- `bwa index <genome.fa>` on the GPU (the index AF:178 builds and AF:188 /
// functions.py:716 search): the bwa text, its suffix array and the FM occurrence table.
//
//   pac   bns_fasta2bntseq: the contigs joined without separators; every non-ACGT base becomes
//         lrand48() & 3 after srand48(11), the j-th ambiguous base taking the (j + 1)-th draw
//         (a jump-ahead of the 48-bit LCG by j + 1 steps, so every base is computed in parallel)
//   T     pac ++ revcomp(pac), N = 2 l_pac codes (one byte each)
//   SA    rows 0..N of the suffix array of T$ ('$' smallest: row 0 is the empty suffix), int64,
//         by prefix doubling (Manber-Myers ranks = group start rows; Larsson-Sadakane's
//         refinement: only unsorted groups are re-sorted, and ranks refined earlier in a pass may
//         be read later in it):
//           - first the 21-character prefixes (3-bit codes, 0 = past the end) in 100 buckets of
//             the first three characters: counting scatter, then a radix sort per bucket;
//           - then, while groups of equal prefixes remain, the rows of those groups in chunks that
//             hold whole groups: key (group ordinal << 33 | rank[sa + h] + 1), radix sorted,
//             new group starts by a max-scan, ranks scattered, singletons dropped; h doubles
//   occ   per 128 rows one 64-B block: the counts of A/C/G/T in the rows before the block
//         (uint64 x 4) and the rows' BWT characters T[sa - 1] at 2 bits (uint64 x 4); the '$'
//         row (sa = 0, bwt "primary") is stored as A and corrected on lookup
//
// The bit-exact contract is oracle/bwa_pe.c (text_new, suffix_array, build_fm); HBM at
// 3.1 Gbp: T 6.2 GB + SA 49.6 GB + occ 3.1 GB resident; the build also holds the ranks
// (49.6 GB) and the unsorted-row list.
#include <hipcub/hipcub.hpp>
#include <vector>

#include "af_internal.h"

namespace {

constexpr int FM_BLK = 128;  // rows per occ block

// ---- pac / T ------------------------------------------------------------------------------
__device__ __forceinline__ int nt4_dev(uint8_t c) {
    switch (c) {
    case 'A': case 'a': return 0;
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'T': case 't': return 3;
    default: return 4;
    }
}

struct Lcg48Jump { uint64_t a[48], c[48]; };  // f^(2^b) of x -> a x + c (mod 2^48)

// ambiguous flags of pac (contig bytes copied from the blob) -> for the scan
__global__ void k_pac_flags(const uint8_t *__restrict__ blob, const int64_t *__restrict__ src_of,
                            const int64_t *__restrict__ pac_off, int n_ctg, int64_t l_pac, uint8_t *__restrict__ T,
                            int32_t *__restrict__ amb) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < l_pac; i += (int64_t)gridDim.x * blockDim.x) {
        int lo = 0, hi = n_ctg;  // pac_off[lo] <= i < pac_off[lo + 1]
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (pac_off[mid] <= i) lo = mid;
            else hi = mid;
        }
        const int c = nt4_dev(blob[src_of[lo] + (i - pac_off[lo])]);
        T[i] = (uint8_t)c;
        amb[i] = c >= 4;
    }
}

// ambiguous bases -> lrand48() & 3 (the draw after `ord` earlier ones); T[N-1-i] = 3 - T[i]
__global__ void k_pac_fill(uint8_t *__restrict__ T, const int32_t *__restrict__ ord, int64_t l_pac, Lcg48Jump J) {
    const uint64_t M48 = (1ull << 48) - 1;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < l_pac; i += (int64_t)gridDim.x * blockDim.x) {
        int c = T[i];
        if (c >= 4) {
            uint64_t x = (11ull << 16) | 0x330Eull;
            const uint64_t k = (uint64_t)ord[i] + 1;  // exclusive scan: earlier ambiguous bases
            for (int b = 0; b < 48; ++b)
                if ((k >> b) & 1) x = (J.a[b] * x + J.c[b]) & M48;
            c = (int)((x >> 17) & 3);
            T[i] = (uint8_t)c;
        }
        T[2 * l_pac - 1 - i] = (uint8_t)(3 - c);
    }
}

// ---- initial buckets ----------------------------------------------------------------------
__device__ __forceinline__ int code3(const uint8_t *T, int64_t N, int64_t p) { return p < N ? T[p] + 1 : 0; }
__device__ __forceinline__ int bucket_of(const uint8_t *T, int64_t N, int64_t i) {
    return ((code3(T, N, i) - 1) * 5 + code3(T, N, i + 1)) * 5 + code3(T, N, i + 2);
}
constexpr int NB = 100;

__global__ void k_bucket_hist(const uint8_t *__restrict__ T, int64_t N, unsigned long long *__restrict__ hist) {
    __shared__ unsigned int h[NB];
    for (int k = threadIdx.x; k < NB; k += blockDim.x) h[k] = 0;
    __syncthreads();
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += (int64_t)gridDim.x * blockDim.x)
        atomicAdd(&h[bucket_of(T, N, i)], 1u);
    __syncthreads();
    for (int k = threadIdx.x; k < NB; k += blockDim.x)
        if (h[k]) atomicAdd(&hist[k], (unsigned long long)h[k]);
}

// positions into their bucket's rows (order inside a bucket is arbitrary: sorted next).  Each
// block takes `per` consecutive positions, reserves its slots per bucket with one atomic each.
__global__ void k_bucket_scatter(const uint8_t *__restrict__ T, int64_t N, int64_t per,
                                 unsigned long long *__restrict__ cursor, int64_t *__restrict__ sa) {
    __shared__ unsigned int h[NB];
    __shared__ unsigned long long base[NB];
    const int64_t b0 = (int64_t)blockIdx.x * per, b1 = min(b0 + per, N);
    for (int k = threadIdx.x; k < NB; k += blockDim.x) h[k] = 0;
    __syncthreads();
    for (int64_t i = b0 + threadIdx.x; i < b1; i += blockDim.x) atomicAdd(&h[bucket_of(T, N, i)], 1u);
    __syncthreads();
    for (int k = threadIdx.x; k < NB; k += blockDim.x) {
        base[k] = h[k] ? atomicAdd(&cursor[k], (unsigned long long)h[k]) : 0;
        h[k] = 0;
    }
    __syncthreads();
    for (int64_t i = b0 + threadIdx.x; i < b1; i += blockDim.x) {
        const int b = bucket_of(T, N, i);
        const unsigned int o = atomicAdd(&h[b], 1u);
        sa[base[b] + o] = i;
    }
}

// 21-character key of suffix p: 3-bit codes (0 past the end), first character most significant
__device__ __forceinline__ uint64_t key21(const uint8_t *T, int64_t N, int64_t p) {
    uint64_t k = 0;
    for (int j = 0; j < 21; ++j) k = (k << 3) | (uint64_t)code3(T, N, p + j);
    return k;
}

__global__ void k_keys21(const uint8_t *__restrict__ T, int64_t N, const int64_t *__restrict__ pos, int64_t n,
                         uint64_t *__restrict__ keys) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x)
        keys[j] = key21(T, N, pos[j]);
}

// group heads of a sorted key run (rows row0 + j): head value = its row, else 0 (max-scan input)
__global__ void k_heads(const uint64_t *__restrict__ keys, int64_t n, int64_t row0, int64_t *__restrict__ hv) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x)
        hv[j] = (j == 0 || keys[j] != keys[j - 1]) ? row0 + j : 0;
}

// ranks (group start rows) into isa; rows of non-singleton groups flagged for the unsorted list
__global__ void k_rank_scatter(const uint64_t *__restrict__ keys, const int64_t *__restrict__ pos,
                               const int64_t *__restrict__ gstart, int64_t n, int64_t *__restrict__ isa,
                               uint8_t *__restrict__ keep) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
        isa[pos[j]] = gstart[j];
        const bool head = j == 0 || keys[j] != keys[j - 1];
        const bool next_head = j + 1 == n || keys[j + 1] != keys[j];
        keep[j] = !(head && next_head);
    }
}

// ---- doubling ----------------------------------------------------------------------------
// group start (rank) of each listed row before this chunk is refined
__global__ void k_gather_gs(const int64_t *__restrict__ U, int64_t n, const int64_t *__restrict__ sa,
                            const int64_t *__restrict__ isa, int64_t *__restrict__ gs) {
    for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < n; u += (int64_t)gridDim.x * blockDim.x)
        gs[u] = isa[sa[U[u]]];
}
// the last group boundary b in (0, n]: gs[b] != gs[b - 1] (b = n counts when gs[n] != gs[n-1])
__global__ void k_last_boundary(const int64_t *__restrict__ gs, int64_t n, unsigned long long *__restrict__ out) {
    for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x + 1; u <= n; u += (int64_t)gridDim.x * blockDim.x)
        if (gs[u] != gs[u - 1]) atomicMax(out, (unsigned long long)u);
}
// the first group boundary b in [1, n]; n + 1 if none
__global__ void k_first_boundary(const int64_t *__restrict__ gs, int64_t n, unsigned long long *__restrict__ out) {
    for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x + 1; u <= n; u += (int64_t)gridDim.x * blockDim.x)
        if (gs[u] != gs[u - 1]) atomicMin(out, (unsigned long long)u);
}
// composite keys of a chunk: dense group ordinal (from the gs changes, via a scan) << 33 | key
__global__ void k_group_flags(const int64_t *__restrict__ gs, int64_t n, int64_t *__restrict__ f) {
    for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < n; u += (int64_t)gridDim.x * blockDim.x)
        f[u] = (u > 0 && gs[u] != gs[u - 1]) ? 1 : 0;
}
__global__ void k_dbl_keys(const int64_t *__restrict__ U, const int64_t *__restrict__ gord, int64_t n,
                           const int64_t *__restrict__ sa, const int64_t *__restrict__ isa, int64_t N, int64_t h,
                           uint64_t *__restrict__ keys, int64_t *__restrict__ pos) {
    for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < n; u += (int64_t)gridDim.x * blockDim.x) {
        const int64_t p = sa[U[u]];
        const uint64_t k = p + h < N ? (uint64_t)isa[p + h] + 1 : 0;
        keys[u] = ((uint64_t)gord[u] << 33) | k;
        pos[u] = p;
    }
}
__global__ void k_dbl_heads(const uint64_t *__restrict__ keys, const int64_t *__restrict__ U, int64_t n,
                            int64_t *__restrict__ hv) {
    for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < n; u += (int64_t)gridDim.x * blockDim.x)
        hv[u] = (u == 0 || keys[u] != keys[u - 1]) ? U[u] : 0;
}
__global__ void k_dbl_write(const uint64_t *__restrict__ keys, const int64_t *__restrict__ pos,
                            const int64_t *__restrict__ U, const int64_t *__restrict__ gstart, int64_t n,
                            int64_t *__restrict__ sa, int64_t *__restrict__ isa, uint8_t *__restrict__ keep) {
    for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < n; u += (int64_t)gridDim.x * blockDim.x) {
        sa[U[u]] = pos[u];
        isa[pos[u]] = gstart[u];
        const bool head = u == 0 || keys[u] != keys[u - 1];
        const bool next_head = u + 1 == n || keys[u + 1] != keys[u];
        keep[u] = !(head && next_head);
    }
}

// ---- BWT and occ ---------------------------------------------------------------------------
// per 128-row block: the 2-bit BWT words and the block's own counts
__global__ void k_occ_blocks(const uint8_t *__restrict__ T, const int64_t *__restrict__ sa, int64_t N, int64_t nblk,
                             uint64_t *__restrict__ occ, uint64_t *__restrict__ cnt, unsigned long long *__restrict__ primary) {
    for (int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nblk; b += (int64_t)gridDim.x * blockDim.x) {
        uint64_t w[4] = {0, 0, 0, 0};
        uint64_t c4[4] = {0, 0, 0, 0};
        for (int k = 0; k < FM_BLK; ++k) {
            const int64_t r = b * FM_BLK + k;
            if (r > N) break;
            const int64_t p = sa[r];
            int c;
            if (p == 0) { c = 0; *primary = (unsigned long long)r; }  // '$' stored as A, not counted
            else {
                c = T[p - 1];
                ++c4[c];
            }
            w[k >> 5] |= (uint64_t)c << (2 * (k & 31));
        }
        uint64_t *o = occ + b * 8;
        for (int k = 0; k < 4; ++k) { o[4 + k] = w[k]; cnt[k * nblk + b] = c4[k]; }
    }
}
__global__ void k_occ_counts(const uint64_t *__restrict__ pre, int64_t nblk, uint64_t *__restrict__ occ) {
    for (int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nblk; b += (int64_t)gridDim.x * blockDim.x)
        for (int k = 0; k < 4; ++k) occ[b * 8 + k] = pre[k * nblk + b];
}

__global__ void k_cpy_i64(const int64_t *__restrict__ src, int64_t *__restrict__ dst, int64_t n) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x)
        dst[j] = src[j];
}

struct Max64 {
    __device__ __forceinline__ int64_t operator()(int64_t a, int64_t b) const { return a > b ? a : b; }
};

inline dim3 grid_for(int64_t n, int bs = 256) {
    int64_t g = (n + bs - 1) / bs;
    return dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>(g, 1 << 20)));
}

#define FMCHK(expr)                                   \
    do {                                              \
        hipError_t _e = (expr);                       \
        if (_e != hipSuccess) { ok = _e; goto done; } \
    } while (0)

}  // namespace

// Builds the index of `n_ctg` contigs of d_blob (device bytes; contig k at blob offset src_off[k],
// src_len[k] bytes).  Fills *G (device pointers it owns: T, sa, occ, ctg_off, ctg_len) and returns
// hipSuccess or the first error.  Synchronous on stream s.
// the contig bucket table (DevGenome::ctg_bkt): one thread per bucket, bns_pos2rid's binary
// search at the bucket's first and last base
__device__ int ctg_search(const int64_t *off, int n_ctg, int64_t pos) {
    int lo = 0, hi = n_ctg;  // the last contig starting at or before pos
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (off[mid] <= pos) lo = mid;
        else hi = mid;
    }
    return lo;
}
__global__ void k_ctg_bkt(const int64_t *__restrict__ off, int n_ctg, int64_t l_pac, int64_t nb, int32_t *__restrict__ bkt) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    const int64_t p0 = b << AF_CTG_BKT_SHIFT;
    const int64_t p1 = min(p0 + ((int64_t)1 << AF_CTG_BKT_SHIFT), l_pac) - 1;
    const int r0 = ctg_search(off, n_ctg, p0), r1 = ctg_search(off, n_ctg, p1);
    bkt[b] = r0 | (r1 != r0 ? (int32_t)0x80000000 : 0);
}

hipError_t af_fm_build(const uint8_t *d_blob, const int64_t *src_off, const int64_t *src_len, int n_ctg, DevGenome *G,
                       hipStream_t s) {
    hipError_t ok = hipSuccess;
    *G = DevGenome{};
    std::vector<int64_t> pac_off(n_ctg);
    int64_t l_pac = 0;
    for (int k = 0; k < n_ctg; ++k) { pac_off[k] = l_pac; l_pac += src_len[k]; }
    const int64_t N = 2 * l_pac;
    int64_t *d_src = nullptr, *d_pacoff = nullptr, *isa = nullptr, *U = nullptr;
    int32_t *amb = nullptr, *ord = nullptr;  // ambiguous-base flags and their exclusive scan (< 2^31)
    uint8_t *Tm = nullptr;
    uint8_t *keep = nullptr;
    void *tmp = nullptr;
    size_t tmp_bytes = 0;
    unsigned long long *cur = nullptr;
    uint64_t *kA = nullptr, *kB = nullptr, *cnt = nullptr;
    int64_t *vA = nullptr, *vB = nullptr, *hv = nullptr, *gs = nullptr, *sel_n = nullptr;
    int64_t *g2 = nullptr;  // a long group's boundary scan (freed at done: on error paths too)
    int64_t cap = 0;  // chunk arrays' capacity
    int64_t nU = 0;
    std::vector<unsigned long long> hist(NB);
    if (l_pac <= 0 || n_ctg < 1) return hipErrorInvalidValue;
    // suffix ranks + 1 are packed in 33 bits (k_dbl_keys), as are the genome kernels' SA-row
    // intervals (bwa_genome.hip G1): 2 l_pac + 1 rows must stay below 2^33
    if (N + 1 >= (int64_t)1 << 33) return hipErrorInvalidValue;
    G->l_pac = l_pac; G->N = N; G->n_ctg = n_ctg;
    FMCHK(hipMalloc(&G->ctg_off_d, sizeof(int64_t) * n_ctg));
    FMCHK(hipMalloc(&G->ctg_len_d, sizeof(int64_t) * n_ctg));
    FMCHK(hipMemcpyAsync(G->ctg_off_d, pac_off.data(), sizeof(int64_t) * n_ctg, hipMemcpyHostToDevice, s));
    FMCHK(hipMemcpyAsync(G->ctg_len_d, src_len, sizeof(int64_t) * n_ctg, hipMemcpyHostToDevice, s));
    {
        const int64_t nb = ((l_pac - 1) >> AF_CTG_BKT_SHIFT) + 1;
        FMCHK(hipMalloc(&G->ctg_bkt, sizeof(int32_t) * nb));
        hipLaunchKernelGGL(k_ctg_bkt, grid_for(nb), dim3(256), 0, s, G->ctg_off_d, n_ctg, l_pac, nb, G->ctg_bkt);
        FMCHK(hipGetLastError());
    }
    FMCHK(hipMalloc(&d_src, sizeof(int64_t) * n_ctg));
    FMCHK(hipMemcpyAsync(d_src, src_off, sizeof(int64_t) * n_ctg, hipMemcpyHostToDevice, s));
    // ---- pac and T
    FMCHK(hipMalloc(&Tm, N + 16));
    G->T = Tm;
    FMCHK(hipMalloc(&amb, sizeof(int32_t) * l_pac));
    FMCHK(hipMalloc(&ord, sizeof(int32_t) * l_pac));
    hipLaunchKernelGGL(k_pac_flags, grid_for(l_pac), dim3(256), 0, s, d_blob, d_src, G->ctg_off_d, n_ctg, l_pac,
                       Tm, amb);
    FMCHK(hipGetLastError());
    FMCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, amb, ord, l_pac, s));
    FMCHK(hipMalloc(&tmp, tmp_bytes));
    FMCHK(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, amb, ord, l_pac, s));
    {
        Lcg48Jump J;
        const uint64_t M48 = (1ull << 48) - 1;
        J.a[0] = 0x5DEECE66DULL; J.c[0] = 0xB;
        for (int b = 1; b < 48; ++b) {
            J.a[b] = (J.a[b - 1] * J.a[b - 1]) & M48;
            J.c[b] = (J.a[b - 1] * J.c[b - 1] + J.c[b - 1]) & M48;
        }
        hipLaunchKernelGGL(k_pac_fill, grid_for(l_pac), dim3(256), 0, s, Tm, ord, l_pac, J);
        FMCHK(hipGetLastError());
    }
    FMCHK(hipFree(amb)); amb = nullptr;
    FMCHK(hipFree(ord)); ord = nullptr;
    FMCHK(hipFree(tmp)); tmp = nullptr; tmp_bytes = 0;
    // base counts and C
    {
        FMCHK(hipMalloc(&cur, sizeof(unsigned long long) * NB));
        FMCHK(hipMemsetAsync(cur, 0, sizeof(unsigned long long) * NB, s));
        hipLaunchKernelGGL(k_bucket_hist, grid_for(N, 256), dim3(256), 0, s, G->T, N, cur);
        FMCHK(hipGetLastError());
        FMCHK(hipMemcpyAsync(hist.data(), cur, sizeof(unsigned long long) * NB, hipMemcpyDeviceToHost, s));
        FMCHK(hipStreamSynchronize(s));
        for (int b = 0; b < NB; ++b) G->base_cnt[b / 25] += (int64_t)hist[b];
        G->C[0] = 1;
        for (int c = 1; c < 4; ++c) G->C[c] = G->C[c - 1] + G->base_cnt[c - 1];
    }
    // ---- SA rows 1..N by bucket, then each bucket sorted by its 21-character keys
    FMCHK(hipMalloc(&G->sa, sizeof(int64_t) * (N + 1)));
    FMCHK(hipMalloc(&isa, sizeof(int64_t) * (N + 1)));
    {
        std::vector<unsigned long long> start(NB);
        unsigned long long acc = 1;  // row 0 is '$'
        int64_t maxb = 1;
        for (int b = 0; b < NB; ++b) { start[b] = acc; acc += hist[b]; maxb = std::max<int64_t>(maxb, (int64_t)hist[b]); }
        FMCHK(hipMemcpyAsync(cur, start.data(), sizeof(unsigned long long) * NB, hipMemcpyHostToDevice, s));
        const int64_t per = 1 << 16;
        hipLaunchKernelGGL(k_bucket_scatter, dim3((unsigned)((N + per - 1) / per)), dim3(256), 0, s, G->T, N, per, cur,
                           G->sa);
        FMCHK(hipGetLastError());
        const int64_t zero = N;
        FMCHK(hipMemcpyAsync(G->sa, &zero, sizeof(int64_t), hipMemcpyHostToDevice, s));
        // chunk arrays sized for the largest bucket and for the doubling chunks
        cap = std::max<int64_t>(maxb, std::min<int64_t>(N, (int64_t)1 << 27)) + 1;
        FMCHK(hipMalloc(&kA, sizeof(uint64_t) * cap));
        FMCHK(hipMalloc(&kB, sizeof(uint64_t) * cap));
        FMCHK(hipMalloc(&vA, sizeof(int64_t) * cap));
        FMCHK(hipMalloc(&vB, sizeof(int64_t) * cap));
        FMCHK(hipMalloc(&hv, sizeof(int64_t) * cap));
        FMCHK(hipMalloc(&gs, sizeof(int64_t) * (cap + 1)));
        FMCHK(hipMalloc(&keep, cap));
        FMCHK(hipMalloc(&sel_n, sizeof(int64_t) * 2));
        FMCHK(hipMalloc(&U, sizeof(int64_t) * (N + 1)));
        {   // scratch sizes for the largest calls
            size_t b1 = 0, b2 = 0, b3 = 0;
            hipcub::DoubleBuffer<uint64_t> dk(kA, kB);
            hipcub::DoubleBuffer<int64_t> dv(vA, vB);
            FMCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, b1, dk, dv, cap, 0, 64, s));
            FMCHK(hipcub::DeviceScan::InclusiveScan(nullptr, b2, hv, gs, Max64(), cap, s));
            hipcub::CountingInputIterator<int64_t> rows(0);
            FMCHK(hipcub::DeviceSelect::Flagged(nullptr, b3, rows, keep, U, sel_n, cap, s));
            size_t b4 = 0;
            FMCHK(hipcub::DeviceScan::InclusiveSum(nullptr, b4, hv, gs, cap, s));
            tmp_bytes = std::max(std::max(b1, b2), std::max(b3, b4));
            FMCHK(hipMalloc(&tmp, tmp_bytes));
        }
        for (int b = 0; b < NB; ++b) {
            const int64_t n = (int64_t)hist[b];
            if (!n) continue;
            const int64_t r0 = (int64_t)start[b];
            hipLaunchKernelGGL(k_cpy_i64, grid_for(n), dim3(256), 0, s, G->sa + r0, vA, n);
            hipLaunchKernelGGL(k_keys21, grid_for(n), dim3(256), 0, s, G->T, N, vA, n, kA);
            FMCHK(hipGetLastError());
            hipcub::DoubleBuffer<uint64_t> dk(kA, kB);
            hipcub::DoubleBuffer<int64_t> dv(vA, vB);
            size_t tb = tmp_bytes;
            FMCHK(hipcub::DeviceRadixSort::SortPairs(tmp, tb, dk, dv, n, 0, 63, s));
            uint64_t *ks = dk.Current();
            int64_t *ps = dv.Current();
            hipLaunchKernelGGL(k_cpy_i64, grid_for(n), dim3(256), 0, s, ps, G->sa + r0, n);
            hipLaunchKernelGGL(k_heads, grid_for(n), dim3(256), 0, s, ks, n, r0, hv);
            FMCHK(hipGetLastError());
            tb = tmp_bytes;
            FMCHK(hipcub::DeviceScan::InclusiveScan(tmp, tb, hv, gs, Max64(), n, s));
            hipLaunchKernelGGL(k_rank_scatter, grid_for(n), dim3(256), 0, s, ks, ps, gs, n, isa, keep);
            FMCHK(hipGetLastError());
            hipcub::CountingInputIterator<int64_t> rows(r0);
            tb = tmp_bytes;
            FMCHK(hipcub::DeviceSelect::Flagged(tmp, tb, rows, keep, U + nU, sel_n, n, s));
            int64_t got = 0;
            FMCHK(hipMemcpyAsync(&got, sel_n, sizeof(int64_t), hipMemcpyDeviceToHost, s));
            FMCHK(hipStreamSynchronize(s));
            nU += got;
        }
    }
    {   // isa of the '$' row (never read as a key: p + h < N only) -- rank 0
        const int64_t z = 0;
        FMCHK(hipMemcpyAsync(isa + N, &z, sizeof(int64_t), hipMemcpyHostToDevice, s));
    }
    // ---- prefix doubling over the unsorted rows
    for (int64_t h = 21; nU > 0; h <<= 1) {
        int64_t u0 = 0, w = 0;  // read position, compacted write position (w <= u0)
        while (u0 < nU) {
            int64_t n = std::min<int64_t>(cap - 1, nU - u0);
            // group starts of [u0, u0 + n] (one past the window to see a boundary at its end)
            const int64_t ng = std::min<int64_t>(n + 1, nU - u0);
            hipLaunchKernelGGL(k_gather_gs, grid_for(ng), dim3(256), 0, s, U + u0, ng, G->sa, isa, gs);
            FMCHK(hipGetLastError());
            if (u0 + n < nU) {  // cut at the last group boundary inside the window
                unsigned long long b = 0;
                FMCHK(hipMemcpyAsync(cur, &b, sizeof b, hipMemcpyHostToDevice, s));
                hipLaunchKernelGGL(k_last_boundary, grid_for(n), dim3(256), 0, s, gs, n, cur);
                FMCHK(hipGetLastError());
                FMCHK(hipMemcpyAsync(&b, cur, sizeof b, hipMemcpyDeviceToHost, s));
                FMCHK(hipStreamSynchronize(s));
                if (b == 0) {
                    // one group longer than the chunk arrays: grow them to hold the whole group
                    int64_t gl = n;
                    for (;;) {
                        const int64_t m = std::min<int64_t>(2 * gl, nU - u0);
                        FMCHK(hipMalloc(&g2, sizeof(int64_t) * (m + 1)));
                        hipLaunchKernelGGL(k_gather_gs, grid_for(m), dim3(256), 0, s, U + u0, m, G->sa, isa, g2);
                        FMCHK(hipGetLastError());
                        unsigned long long fb = ~0ull;
                        FMCHK(hipMemcpyAsync(cur, &fb, sizeof fb, hipMemcpyHostToDevice, s));
                        hipLaunchKernelGGL(k_first_boundary, grid_for(m), dim3(256), 0, s, g2, m - 1, cur);
                        FMCHK(hipGetLastError());
                        FMCHK(hipMemcpyAsync(&fb, cur, sizeof fb, hipMemcpyDeviceToHost, s));
                        FMCHK(hipStreamSynchronize(s));
                        FMCHK(hipFree(g2));
                        g2 = nullptr;
                        if (fb != ~0ull) { gl = (int64_t)fb; break; }
                        if (m == nU - u0) { gl = m; break; }
                        gl = m;
                    }
                    // regrow every chunk array to gl + 1
                    (void)hipFree(kA); (void)hipFree(kB); (void)hipFree(vA); (void)hipFree(vB); (void)hipFree(hv);
                    (void)hipFree(gs); (void)hipFree(keep); (void)hipFree(tmp);
                    kA = kB = nullptr; vA = vB = hv = gs = nullptr; keep = nullptr; tmp = nullptr;
                    cap = gl + 2;
                    FMCHK(hipMalloc(&kA, sizeof(uint64_t) * cap));
                    FMCHK(hipMalloc(&kB, sizeof(uint64_t) * cap));
                    FMCHK(hipMalloc(&vA, sizeof(int64_t) * cap));
                    FMCHK(hipMalloc(&vB, sizeof(int64_t) * cap));
                    FMCHK(hipMalloc(&hv, sizeof(int64_t) * cap));
                    FMCHK(hipMalloc(&gs, sizeof(int64_t) * (cap + 1)));
                    FMCHK(hipMalloc(&keep, cap));
                    {
                        size_t b1 = 0, b2 = 0, b3 = 0, b4 = 0;
                        hipcub::DoubleBuffer<uint64_t> dk(kA, kB);
                        hipcub::DoubleBuffer<int64_t> dv(vA, vB);
                        FMCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, b1, dk, dv, cap, 0, 64, s));
                        FMCHK(hipcub::DeviceScan::InclusiveScan(nullptr, b2, hv, gs, Max64(), cap, s));
                        hipcub::CountingInputIterator<int64_t> rows(0);
                        FMCHK(hipcub::DeviceSelect::Flagged(nullptr, b3, rows, keep, U, sel_n, cap, s));
                        FMCHK(hipcub::DeviceScan::InclusiveSum(nullptr, b4, hv, gs, cap, s));
                        tmp_bytes = std::max(std::max(b1, b2), std::max(b3, b4));
                        FMCHK(hipMalloc(&tmp, tmp_bytes));
                    }
                    n = gl;
                    hipLaunchKernelGGL(k_gather_gs, grid_for(n), dim3(256), 0, s, U + u0, n, G->sa, isa, gs);
                    FMCHK(hipGetLastError());
                } else {
                    n = (int64_t)b;
                }
            }
            // composite keys: dense group ordinal << 33 | (rank of p + h) + 1
            hipLaunchKernelGGL(k_group_flags, grid_for(n), dim3(256), 0, s, gs, n, hv);
            size_t tb = tmp_bytes;
            FMCHK(hipcub::DeviceScan::InclusiveSum(tmp, tb, hv, vB, n, s));
            hipLaunchKernelGGL(k_dbl_keys, grid_for(n), dim3(256), 0, s, U + u0, vB, n, G->sa, isa, N, h, kA, vA);
            FMCHK(hipGetLastError());
            int bits = 33;
            {   // ordinals < n
                int64_t m = n;
                int ob = 0;
                while (m) { ++ob; m >>= 1; }
                bits += ob;
            }
            hipcub::DoubleBuffer<uint64_t> dk(kA, kB);
            hipcub::DoubleBuffer<int64_t> dv(vA, vB);
            tb = tmp_bytes;
            FMCHK(hipcub::DeviceRadixSort::SortPairs(tmp, tb, dk, dv, n, 0, std::min(bits, 64), s));
            uint64_t *ks = dk.Current();
            int64_t *ps = dv.Current();
            hipLaunchKernelGGL(k_dbl_heads, grid_for(n), dim3(256), 0, s, ks, U + u0, n, hv);
            tb = tmp_bytes;
            FMCHK(hipcub::DeviceScan::InclusiveScan(tmp, tb, hv, gs, Max64(), n, s));
            hipLaunchKernelGGL(k_dbl_write, grid_for(n), dim3(256), 0, s, ks, ps, U + u0, gs, n, G->sa, isa, keep);
            FMCHK(hipGetLastError());
            // keep the rows of groups still unsorted (in place: w <= u0, rows staged through kB)
            int64_t *stage = reinterpret_cast<int64_t *>(dk.Alternate());
            tb = tmp_bytes;
            FMCHK(hipcub::DeviceSelect::Flagged(tmp, tb, U + u0, keep, stage, sel_n, n, s));
            int64_t got = 0;
            FMCHK(hipMemcpyAsync(&got, sel_n, sizeof(int64_t), hipMemcpyDeviceToHost, s));
            FMCHK(hipStreamSynchronize(s));
            if (got) {
                hipLaunchKernelGGL(k_cpy_i64, grid_for(got), dim3(256), 0, s, stage, U + w, got);
                FMCHK(hipGetLastError());
            }
            w += got;
            u0 += n;
        }
        nU = w;
        if (h > N) break;  // (cannot happen: every group splits by then)
    }
    FMCHK(hipStreamSynchronize(s));
    (void)hipFree(isa); isa = nullptr;
    (void)hipFree(U); U = nullptr;
    (void)hipFree(kA); (void)hipFree(kB); (void)hipFree(vA); (void)hipFree(vB); (void)hipFree(hv); (void)hipFree(gs);
    (void)hipFree(keep);
    kA = kB = nullptr; vA = vB = hv = gs = nullptr; keep = nullptr;
    (void)hipFree(tmp); tmp = nullptr;
    // ---- BWT + occ
    {
        // one block past the rows: lookups at i = N + 1 (a whole-text interval end) read its
        // counts, the totals
        const int64_t nblk = (N + 1 + FM_BLK - 1) / FM_BLK + 1;
        G->n_blk = nblk;
        FMCHK(hipMalloc(&G->occ, sizeof(uint64_t) * 8 * (nblk + 1)));
        FMCHK(hipMalloc(&cnt, sizeof(uint64_t) * 8 * nblk));  // counts, then their exclusive scans
        unsigned long long prim = 0;
        FMCHK(hipMemcpyAsync(cur, &prim, sizeof prim, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_occ_blocks, grid_for(nblk), dim3(256), 0, s, G->T, G->sa, N, nblk, G->occ, cnt, cur);
        FMCHK(hipGetLastError());
        size_t tb = 0;
        FMCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, cnt, cnt + 4 * nblk, nblk, s));
        FMCHK(hipMalloc(&tmp, tb));
        for (int k = 0; k < 4; ++k) {
            size_t t2 = tb;
            FMCHK(hipcub::DeviceScan::ExclusiveSum(tmp, t2, cnt + k * nblk, cnt + (4 + k) * nblk, nblk, s));
        }
        hipLaunchKernelGGL(k_occ_counts, grid_for(nblk), dim3(256), 0, s, cnt + 4 * nblk, nblk, G->occ);
        FMCHK(hipGetLastError());
        FMCHK(hipMemcpyAsync(&prim, cur, sizeof prim, hipMemcpyDeviceToHost, s));
        FMCHK(hipStreamSynchronize(s));
        G->primary = (int64_t)prim;
    }
done:
    (void)hipStreamSynchronize(s);
    (void)hipFree(d_src); (void)hipFree(d_pacoff); (void)hipFree(amb); (void)hipFree(ord); (void)hipFree(isa); (void)hipFree(U);
    (void)hipFree(keep); (void)hipFree(tmp); (void)hipFree(cur); (void)hipFree(kA); (void)hipFree(kB); (void)hipFree(vA);
    (void)hipFree(vB); (void)hipFree(hv); (void)hipFree(gs); (void)hipFree(sel_n); (void)hipFree(cnt); (void)hipFree(g2);
    if (ok != hipSuccess) af_fm_free(G);
    return ok;
}

void af_fm_free(DevGenome *G) {
    (void)hipFree(const_cast<uint8_t *>(G->T));
    (void)hipFree(G->sa);
    (void)hipFree(G->occ);
    (void)hipFree(G->ctg_bkt);
    (void)hipFree(G->ctg_off_d);
    (void)hipFree(G->ctg_len_d);
    *G = DevGenome{};
}
