// seed_filter.hip -- K1: HBM-streaming anchor seed filter (the seeding
// pass of `bwa mem` at Anchored_Fusion.py:182).
//
// Layout and schedule:
//  * persistent grid, one 1024-thread workgroup per CU, block tiles of AF_SEED_BTILE whole
//    reads taken round-robin; the 16 waves sweep a tile together, 16 KiB contiguous per
//    round (lane l of wave w loads one 16-byte chunk: a coalesced 1-KiB dwordx4 per wave),
//    unrolled x3 with two rounds of loads in flight;
//  * ASCII -> 2-bit codes by SWAR ((c>>1)^(c>>2))&3, 4 bases per byte; each lane forms the
//    four 16-mers starting at its 4-byte-aligned offsets, borrowing the next lane's packed
//    chunk through a shuffle (lane 63 uses the first chunk of the next round);
//  * stage 1: one bit test in an LDS bitmap of anchor 16-mers (no false negatives);
//  * stage 2: the few 16-mers that pass are appended to a wave-local LDS queue and probed in
//    full 64-lane batches against the fingerprint table (LDS; 8 x u16 buckets), so the exact
//    probe never runs divergent;
//  * per-read hit counts live in 8-bit LDS counters; the wave writes one int32 per read and
//    appends reads with hits to the candidate list (one global atomic per 64 reads).
//
// Exactness: any MEM >= 19 nt (bwa -k 19) contains a 16-mer starting at an offset that is a
// multiple of 4, so hits == 0 implies no seed; the filter can over-report, never drop.
#include "af_internal.h"

#include <algorithm>

namespace {

constexpr int QCAP = 128;  // queue entries per wave (drained whenever >= 64)

__device__ __forceinline__ uint32_t codes4(uint32_t x) { return ((x >> 1) ^ (x >> 2)) & 0x03030303u; }

// bytes y0..y3 (2-bit codes) -> y0 | y1<<2 | y2<<4 | y3<<6
__device__ __forceinline__ uint32_t pack4(uint32_t y) {
    const uint32_t t = y | (y >> 6);
    return (t & 0xFu) | ((t >> 12) & 0xF0u);
}

__device__ __forceinline__ uint32_t pack_chunk(const uint4 v) {
    return pack4(codes4(v.x)) | (pack4(codes4(v.y)) << 8) | (pack4(codes4(v.z)) << 16) |
           (pack4(codes4(v.w)) << 24);
}

__device__ __forceinline__ bool has_zero_half(uint32_t x) { return ((x - 0x00010001u) & ~x & 0x80008000u) != 0; }

__device__ bool probe_exact(const uint4 *__restrict__ tab, int nb_bits, uint32_t k) {
    const uint32_t h = af_fmix(k);
    uint32_t b = h >> (32 - nb_bits);
    const uint32_t f = af_ffp(h);
    const uint32_t ff = f | (f << 16);
    const uint32_t nbm = (1u << nb_bits) - 1u;
    for (;;) {
        const uint4 bk = tab[b];
        if ((int)has_zero_half(bk.x ^ ff) | (int)has_zero_half(bk.y ^ ff) | (int)has_zero_half(bk.z ^ ff) |
            (int)has_zero_half(bk.w ^ ff))
            return true;
        if ((bk.w >> 16) != 1u) return false;
        b = (b + 1u) & nbm;
    }
}

// chunk c of the tile when it is only partly inside the tile (bytes past the end read 'N')
__device__ __noinline__ uint4 load_tail(const uint8_t *__restrict__ base, int c, int64_t tile_bytes) {
    uint32_t w[4] = {0x4E4E4E4Eu, 0x4E4E4E4Eu, 0x4E4E4E4Eu, 0x4E4E4E4Eu};
    const int64_t o = 16 * (int64_t)c;
    for (int b = 0; b < 16; ++b)
        if (o + b < tile_bytes) {
            w[b >> 2] &= ~(0xFFu << (8 * (b & 3)));
            w[b >> 2] |= (uint32_t)base[o + b] << (8 * (b & 3));
        }
    return make_uint4(w[0], w[1], w[2], w[3]);
}

struct TileGeo {
    const uint8_t *base;
    int64_t bytes;
    int nfull, nchunks, nround;
};

template <bool HAS_LENS>
__device__ __forceinline__ void drain(const uint4 *tab, int nb_bits, const uint32_t *qk, const uint32_t *qo, int lo,
                                      int hi, int lane, int32_t stride, const int32_t *lens, int64_t r0,
                                      uint32_t *cnt) {
    const int i = lo + lane;
    if (i < hi) {
        const uint32_t k = qk[i], off = qo[i];
        if (probe_exact(tab, nb_bits, k)) {
            const int r = (int)(off / (uint32_t)stride);
            const int rem = (int)off - r * stride;
            const int l = HAS_LENS ? lens[r0 + r] : stride;
            if (rem + AF_K <= l) atomicAdd(&cnt[r >> 2], 1u << (8 * (r & 3)));
        }
    }
}

// copies n uint4 from global to LDS with the whole workgroup, 8 loads in flight per thread
__device__ __forceinline__ void fill_lds(uint4 *dst, const uint4 *__restrict__ src, int n) {
    int i0 = 0;
    for (; i0 + 8 * 1024 <= n; i0 += 8 * 1024) {
        uint4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = src[i0 + u * 1024 + threadIdx.x];
#pragma unroll
        for (int u = 0; u < 8; ++u) dst[i0 + u * 1024 + threadIdx.x] = v[u];
    }
    for (int i = i0 + (int)threadIdx.x; i < n; i += 1024) dst[i] = src[i];
}

// One round of a wave: chunk c (packed P), the chunk right after lane 63's (packed Px).
template <bool HAS_LENS>
__device__ __forceinline__ void scan_round(uint32_t P, uint32_t Px, int c, bool in, int lane, int bsh,
                                           const uint32_t *bm, const uint4 *tab, int nb_bits, uint32_t *qk,
                                           uint32_t *qo, int &qn, int32_t stride, const int32_t *lens, int64_t r0,
                                           uint32_t *cnt) {
    uint32_t Pn = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)P, 0x130, 0xf, 0xf, false);  // wave_shl:1
    if (lane == 63) Pn = Px;
    const uint64_t PP = ((uint64_t)Pn << 32) | P;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t k = (uint32_t)(PP >> (8 * j));
        const uint32_t bi = af_fmix(k) >> bsh;
        const bool pass = in && ((bm[bi >> 5] >> (bi & 31)) & 1u);
        const uint64_t m = __ballot(pass);
        if (m) {
            if (pass) {
                const int pos = qn + (int)__popcll(m & ((1ull << lane) - 1ull));
                qk[pos] = k;
                qo[pos] = (uint32_t)(c * 16 + 4 * j);
            }
            qn += (int)__popcll(m);
            if (qn >= 64) {
                drain<HAS_LENS>(tab, nb_bits, qk, qo, qn - 64, qn, lane, stride, lens, r0, cnt);
                qn -= 64;
            }
        }
    }
}

// Block tile = AF_SEED_BTILE whole reads, swept by the 16 waves together: in round r wave w
// loads chunk block (r * 16 + w), i.e. the workgroup streams 16 KiB of contiguous bytes per
// round (DRAM row locality), while each wave still owns 64 consecutive chunks.
template <bool HAS_LENS>
__global__ __launch_bounds__(64 * AF_SEED_WAVES) void k_seed_filter(
    const uint8_t *__restrict__ reads, int64_t n_reads, int32_t stride, const int32_t *__restrict__ lens,
    const uint4 *__restrict__ ftab, int nb_bits, const uint32_t *__restrict__ bitmap, int bm_bits,
    int32_t *__restrict__ hits, int32_t *__restrict__ cand, int32_t *__restrict__ ctrl) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int nb = 1 << nb_bits;
    const int bmw = 1 << (bm_bits - 5);
    uint4 *tab = reinterpret_cast<uint4 *>(smem);
    uint32_t *bm = reinterpret_cast<uint32_t *>(smem + (size_t)nb * 16);
    uint32_t *cnt = bm + bmw;                       // AF_SEED_BTILE 8-bit counters
    uint32_t *qbase = cnt + AF_SEED_BTILE / 4;
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // provably wave-uniform
    uint32_t *qk = qbase + wv * 2 * QCAP;
    uint32_t *qo = qk + QCAP;
    {   // table + bitmap fill (uint4), loads batched ahead of the LDS stores
        const uint4 *bm4 = reinterpret_cast<const uint4 *>(bitmap);
        uint4 *bml = reinterpret_cast<uint4 *>(bm);
        const int n4 = bmw / 4;
        fill_lds(tab, ftab, nb);
        fill_lds(bml, bm4, n4);
    }
    const int64_t ntiles = (n_reads + AF_SEED_BTILE - 1) / AF_SEED_BTILE;
    const int bsh = 32 - bm_bits;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t r0 = tile * AF_SEED_BTILE;
        const int nr = __builtin_amdgcn_readfirstlane((int)min((int64_t)AF_SEED_BTILE, n_reads - r0));
        for (int i = threadIdx.x; i < AF_SEED_BTILE / 4; i += blockDim.x) cnt[i] = 0;
        __syncthreads();
        TileGeo g;
        g.base = reads + r0 * (int64_t)stride;
        g.bytes = (int64_t)nr * stride;
        g.nfull = __builtin_amdgcn_readfirstlane((int)(g.bytes >> 4));
        g.nchunks = __builtin_amdgcn_readfirstlane((int)((g.bytes + 15) >> 4));
        const int nblk = (g.nchunks + 63) >> 6;                      // 64-chunk blocks in the tile
        const int nround = (nblk + AF_SEED_WAVES - 1) / AF_SEED_WAVES;  // rounds of this wave
        int qn = 0;
        if (g.nfull == g.nchunks) {
            // every chunk is whole: branch-free loads, addresses clamped into the tile (clamped
            // lanes are masked by `in`; a clamped neighbour only feeds 16-mers that cross the
            // tile end, which drain() rejects).  Three named round buffers, unrolled by 3, so
            // each load lands in the registers consumed two rounds later.
            const uint4 *cb = reinterpret_cast<const uint4 *>(g.base);
            const int last = g.nfull - 1;
#define AF_CH(rr) ((((rr) * AF_SEED_WAVES + wv) << 6))
            uint4 vA = cb[min(AF_CH(0) + lane, last)], xA = cb[min(AF_CH(0) + 64, last)];
            uint4 vB = cb[min(AF_CH(1) + lane, last)], xB = cb[min(AF_CH(1) + 64, last)];
            uint4 vC = cb[min(AF_CH(2) + lane, last)], xC = cb[min(AF_CH(2) + 64, last)];
            for (int r = 0; r < nround; r += 3) {
                scan_round<HAS_LENS>(pack_chunk(vA), pack_chunk(xA), AF_CH(r) + lane, AF_CH(r) + lane < g.nchunks,
                                     lane, bsh, bm, tab, nb_bits, qk, qo, qn, stride, lens, r0, cnt);
                vA = cb[min(AF_CH(r + 3) + lane, last)];
                xA = cb[min(AF_CH(r + 3) + 64, last)];
                if (r + 1 < nround)
                    scan_round<HAS_LENS>(pack_chunk(vB), pack_chunk(xB), AF_CH(r + 1) + lane,
                                         AF_CH(r + 1) + lane < g.nchunks, lane, bsh, bm, tab, nb_bits, qk, qo, qn,
                                         stride, lens, r0, cnt);
                vB = cb[min(AF_CH(r + 4) + lane, last)];
                xB = cb[min(AF_CH(r + 4) + 64, last)];
                if (r + 2 < nround)
                    scan_round<HAS_LENS>(pack_chunk(vC), pack_chunk(xC), AF_CH(r + 2) + lane,
                                         AF_CH(r + 2) + lane < g.nchunks, lane, bsh, bm, tab, nb_bits, qk, qo, qn,
                                         stride, lens, r0, cnt);
                vC = cb[min(AF_CH(r + 5) + lane, last)];
                xC = cb[min(AF_CH(r + 5) + 64, last)];
            }
        } else {
            for (int r = 0; r < nround; ++r) {
                const int b = r * AF_SEED_WAVES + wv;
                const int c = (b << 6) + lane;
                const uint4 v = c < g.nfull ? *reinterpret_cast<const uint4 *>(g.base + 16 * (int64_t)c)
                                            : (c < g.nchunks ? load_tail(g.base, c, g.bytes)
                                                             : make_uint4(0x4E4E4E4Eu, 0x4E4E4E4Eu, 0x4E4E4E4Eu,
                                                                          0x4E4E4E4Eu));
                const int cx = (b + 1) << 6;
                const uint4 x = cx < g.nfull ? *reinterpret_cast<const uint4 *>(g.base + 16 * (int64_t)cx)
                                             : (cx < g.nchunks ? load_tail(g.base, cx, g.bytes)
                                                               : make_uint4(0x4E4E4E4Eu, 0x4E4E4E4Eu, 0x4E4E4E4Eu,
                                                                            0x4E4E4E4Eu));
                scan_round<HAS_LENS>(pack_chunk(v), pack_chunk(x), c, c < g.nchunks, lane, bsh, bm, tab, nb_bits,
                                     qk, qo, qn, stride, lens, r0, cnt);
            }
        }
#undef AF_CH
        if (qn > 0) drain<HAS_LENS>(tab, nb_bits, qk, qo, 0, qn, lane, stride, lens, r0, cnt);
        __syncthreads();
        for (int i0 = wv * 64; i0 < nr; i0 += 64 * AF_SEED_WAVES) {
            const int i = i0 + lane;
            uint32_t h = 0;
            if (i < nr) {
                h = (cnt[i >> 2] >> (8 * (i & 3))) & 0xFFu;
                hits[r0 + i] = (int32_t)h;
            }
            const uint64_t bal = __ballot(h != 0);
            if (bal) {
                int basei = 0;
                if (lane == 0) basei = atomicAdd(&ctrl[0], (int)__popcll(bal));
                basei = __shfl(basei, 0);
                if (h) cand[basei + __popcll(bal & ((1ull << lane) - 1ull))] = (int32_t)(r0 + i);
            }
        }
        __syncthreads();
    }
}

}  // namespace

size_t af_seed_filter_lds(int nb_bits, int bm_bits) {
    return ((size_t)1 << nb_bits) * 16 + ((size_t)1 << (bm_bits - 3)) + AF_SEED_BTILE +
           (size_t)AF_SEED_WAVES * QCAP * 8;
}

hipError_t af_launch_seed_filter(const DevIndex &ix, const uint8_t *reads, int64_t n_reads, int32_t stride,
                                 const int32_t *lens, int32_t *hits, int32_t *cand, int32_t *ctrl, int n_cu,
                                 hipStream_t s) {
    if (n_reads <= 0) return hipSuccess;
    const int64_t want = (n_reads + AF_SEED_BTILE - 1) / AF_SEED_BTILE;
    const size_t lds = af_seed_filter_lds(ix.nb_bits, ix.bm_bits);
    const int per_cu = (int)std::max<size_t>(1, (160 * 1024) / lds);
    const int64_t blocks = std::min<int64_t>(want, (int64_t)n_cu * per_cu);
    static bool attr_done = false;
    if (!attr_done) {  // dynamic LDS above 64 KiB needs the opt-in on both instantiations
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_seed_filter<true>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_seed_filter<false>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_done = true;
    }
    dim3 grid((unsigned)blocks), block(64 * AF_SEED_WAVES);
    if (lens)
        hipLaunchKernelGGL(k_seed_filter<true>, grid, block, lds, s, reads, n_reads, stride, lens, ix.ftab,
                           ix.nb_bits, ix.bitmap, ix.bm_bits, hits, cand, ctrl);
    else
        hipLaunchKernelGGL(k_seed_filter<false>, grid, block, lds, s, reads, n_reads, stride, lens, ix.ftab,
                           ix.nb_bits, ix.bitmap, ix.bm_bits, hits, cand, ctrl);
    return hipGetLastError();
}
