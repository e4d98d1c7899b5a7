// genome_index.hip -- genome-scale reference index built on the GPU (SURVEY.md §8 f rank 2:
// `bwa index <genome>` at Anchored_Fusion.py:173-178, used by the genome placements of S4-S8 and
// the homolog search, Anchored_Fusion.py:188, functions.py:341, 530, 716, 1244).
//
// A hash of both strands' 16-mers (the anchor index, api.hip) does not scale to a 3.1 Gbp genome:
// 6.2 G positions overflow int32 and a host sort of them takes minutes.  This index is built in
// HBM by five passes over the sequence:
//   1. codes: ASCII -> the doubled reference D (forward ++ reverse complement, 1 B/base), its
//      2-bit packing D2 and N bitmap Dn -- what K2 reads for extension and CIGARs;
//   2. count: one thread per forward position, the 16-mer key (from D2, skipping windows with an
//      N) -> atomicAdd on a direct table S of 4^16 + 1 uint32 counters (16 GiB);
//   3. scan: S becomes the inclusive prefix sum (three passes: block sums, one scan of those, an
//      in-block scan with the block's offset);
//   4. scatter: atomicSub on S[key] gives each forward position its slot in kposu; S[k] ends as
//      the start of k's run and S[4^16] holds the total, so the run of k is [S[k], S[k + 1]).
// Only forward positions are stored (< 2^32); K2 adds the reverse-strand occurrences of a 16-mer
// as the images n2 - 16 - q of the forward run of its reverse complement (align.hip, MEM search).
// Positions inside a run are in atomic order, not sorted: the MEM set of a read does not depend
// on it (MEMs are rank-sorted by length, query and reference position before use).
#include "af_internal.h"

namespace {

constexpr uint64_t kKeys = 1ull << 32;  // 4^16

__device__ __forceinline__ uint32_t nt4d(uint32_t c) {
    switch (c) {
    case 'A': case 'a': return 0;
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'T': case 't': return 3;
    default: return 4;
    }
}

// one thread per 32 bases of the doubled reference
__global__ void k_gx_codes(const uint8_t *__restrict__ seq, int64_t n, uint8_t *__restrict__ D,
                           uint32_t *__restrict__ D2, uint32_t *__restrict__ Dn) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t n2 = 2 * n, p0 = 32 * t;
    if (p0 >= n2) return;
    uint32_t w[2] = {0, 0}, nm = 0;
    for (int u = 0; u < 32; ++u) {
        const int64_t p = p0 + u;
        if (p >= n2) break;
        uint32_t c;
        if (p < n) c = nt4d(seq[p]);
        else {
            c = nt4d(seq[n2 - 1 - p]);
            c = c < 4 ? 3 - c : 4;
        }
        D[p] = (uint8_t)c;
        w[u >> 4] |= (c & 3u) << (2 * (u & 15));
        if (c > 3) nm |= 1u << u;
    }
    D2[2 * t] = w[0];
    D2[2 * t + 1] = w[1];
    Dn[t] = nm;
}

// the 16-mer at forward position q, or false if it holds an N
__device__ __forceinline__ bool key_at(const uint32_t *__restrict__ D2, const uint32_t *__restrict__ Dn, int64_t q,
                                       uint32_t &k) {
    const int64_t wi = q >> 4;
    const int sh = (int)(q & 15) * 2;
    const uint32_t lo = D2[wi], hi = D2[wi + 1];
    k = sh ? (lo >> sh) | (hi << (32 - sh)) : lo;
    const int64_t ni = q >> 5;
    const int nsh = (int)(q & 31);
    const uint32_t nlo = Dn[ni], nhi = Dn[ni + 1];
    const uint32_t nmask = (nsh ? (nlo >> nsh) | (nhi << (32 - nsh)) : nlo) & 0xFFFFu;
    return nmask == 0;
}

__global__ void k_gx_count(const uint32_t *__restrict__ D2, const uint32_t *__restrict__ Dn, int64_t n_q,
                           uint32_t *__restrict__ S) {
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n_q; q += (int64_t)gridDim.x * blockDim.x) {
        uint32_t k;
        if (key_at(D2, Dn, q, k)) atomicAdd(&S[k], 1u);
    }
}

__global__ void k_gx_scatter(const uint32_t *__restrict__ D2, const uint32_t *__restrict__ Dn, int64_t n_q,
                             uint32_t *__restrict__ S, uint32_t *__restrict__ kposu) {
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n_q; q += (int64_t)gridDim.x * blockDim.x) {
        uint32_t k;
        if (key_at(D2, Dn, q, k)) kposu[atomicSub(&S[k], 1u) - 1u] = (uint32_t)q;
    }
}

// ---- inclusive scan of 2^32 uint32 counters (totals < 2^32: the genome is < 4 Gbp) ----------
constexpr int SCAN_T = 1024, SCAN_V = 16, SCAN_B = SCAN_T * SCAN_V;  // 16 Ki counters per block

__device__ __forceinline__ uint32_t block_incl_scan(uint32_t v, uint32_t *sh, uint32_t &total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t t = __shfl_up(v, d);
        if (lane >= d) v += t;
    }
    if (lane == 63) sh[w] = v;
    __syncthreads();
    if (w == 0) {
        uint32_t x = lane < SCAN_T / 64 ? sh[lane] : 0u;
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t t = __shfl_up(x, d);
            if (lane >= d) x += t;
        }
        if (lane < SCAN_T / 64) sh[lane] = x;
    }
    __syncthreads();
    const uint32_t off = w ? sh[w - 1] : 0u;
    total = sh[SCAN_T / 64 - 1];
    __syncthreads();
    return v + off;
}

__global__ __launch_bounds__(SCAN_T) void k_scan_sums(const uint32_t *__restrict__ S, uint32_t *__restrict__ sums) {
    __shared__ uint32_t sh[SCAN_T / 64];
    const uint64_t b0 = (uint64_t)blockIdx.x * SCAN_B;
    uint32_t v = 0;
    for (int u = 0; u < SCAN_V; ++u) v += S[b0 + (uint64_t)u * SCAN_T + threadIdx.x];
    uint32_t total;
    (void)block_incl_scan(v, sh, total);
    if (threadIdx.x == 0) sums[blockIdx.x] = total;
}

// one block: exclusive scan of nb block sums in place (sequential chunks of SCAN_T)
__global__ __launch_bounds__(SCAN_T) void k_scan_top(uint32_t *__restrict__ sums, int nb) {
    __shared__ uint32_t sh[SCAN_T / 64];
    uint32_t carry = 0;
    for (int c0 = 0; c0 < nb; c0 += SCAN_T) {
        const int i = c0 + threadIdx.x;
        const uint32_t v = i < nb ? sums[i] : 0u;
        uint32_t total;
        const uint32_t incl = block_incl_scan(v, sh, total);
        if (i < nb) sums[i] = carry + incl - v;
        carry += total;
    }
}

// in-block inclusive scan with the block's offset; thread t owns counters [t*16, t*16+16)
__global__ __launch_bounds__(SCAN_T) void k_scan_apply(uint32_t *__restrict__ S, const uint32_t *__restrict__ sums) {
    __shared__ uint32_t sh[SCAN_T / 64];
    const uint64_t b0 = (uint64_t)blockIdx.x * SCAN_B + (uint64_t)threadIdx.x * SCAN_V;
    uint32_t v[SCAN_V], s = 0;
    const uint4 *src = reinterpret_cast<const uint4 *>(S + b0);
#pragma unroll
    for (int u = 0; u < SCAN_V / 4; ++u) {
        const uint4 x = src[u];
        v[4 * u] = x.x; v[4 * u + 1] = x.y; v[4 * u + 2] = x.z; v[4 * u + 3] = x.w;
    }
#pragma unroll
    for (int u = 0; u < SCAN_V; ++u) s += v[u];
    uint32_t total;
    const uint32_t incl = block_incl_scan(s, sh, total);
    uint32_t run = sums[blockIdx.x] + incl - s;
    uint4 *dst = reinterpret_cast<uint4 *>(S + b0);
#pragma unroll
    for (int u = 0; u < SCAN_V; ++u) {
        run += v[u];
        v[u] = run;
    }
#pragma unroll
    for (int u = 0; u < SCAN_V / 4; ++u) dst[u] = make_uint4(v[4 * u], v[4 * u + 1], v[4 * u + 2], v[4 * u + 3]);
}

__global__ void k_set_total(uint32_t *S) { S[kKeys] = S[kKeys - 1]; }

}  // namespace

size_t af_genome_index_table_bytes() { return (size_t)(kKeys + 1) * sizeof(uint32_t); }

// Fills D/D2/Dn (sizes as af_index_build: 2n, (2n+15)/16+2 and (2n+31)/32+2 words, zeroed by the
// caller), S (kKeys + 1 counters) and kposu (>= n - 15 entries) from seq (device, n bytes).
hipError_t af_build_genome_index(const uint8_t *seq, int64_t n, uint8_t *D, uint32_t *D2, uint32_t *Dn,
                                 uint32_t *S, uint32_t *kposu, uint32_t *scan_sums, int n_cu, hipStream_t s) {
    const int64_t n2 = 2 * n;
    const int64_t nt = (n2 + 31) / 32;
    hipLaunchKernelGGL(k_gx_codes, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, s, seq, n, D, D2, Dn);
    hipError_t e = hipMemsetAsync(S, 0, af_genome_index_table_bytes(), s);
    if (e != hipSuccess) return e;
    const int64_t n_q = n >= AF_K ? n - AF_K + 1 : 0;
    const dim3 grid((unsigned)(n_cu * 8)), block(256);
    hipLaunchKernelGGL(k_gx_count, grid, block, 0, s, D2, Dn, n_q, S);
    const int nb = (int)(kKeys / SCAN_B);
    hipLaunchKernelGGL(k_scan_sums, dim3(nb), dim3(SCAN_T), 0, s, S, scan_sums);
    hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(SCAN_T), 0, s, scan_sums, nb);
    hipLaunchKernelGGL(k_scan_apply, dim3(nb), dim3(SCAN_T), 0, s, S, scan_sums);
    hipLaunchKernelGGL(k_set_total, dim3(1), dim3(1), 0, s, S);
    hipLaunchKernelGGL(k_gx_scatter, grid, block, 0, s, D2, Dn, n_q, S, kposu);
    return hipGetLastError();
}

int af_genome_scan_blocks() { return (int)(kKeys / SCAN_B); }
