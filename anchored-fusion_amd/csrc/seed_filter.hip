// seed_filter.hip -- K1: HBM-streaming anchor seed filter (the seeding
// pass of `bwa mem` at Anchored_Fusion.py:182).
//
// Layout and schedule:
//  * persistent grid, one or two 1024-thread workgroups per CU (LDS-bound); block tiles of AF_SEED_BTILE whole
//    reads taken round-robin; the 16 waves of a workgroup sweep a tile together, so every
//    round moves ~16 KiB of contiguous bytes (lane l of wave w loads one 16-byte chunk: one
//    coalesced 1-KiB global_load_dwordx4 per wave), unrolled x3 with two rounds in flight;
//  * wave blocks overlap by one chunk (63 new chunks per block): lane 63 only feeds lane 62,
//    so the loop carries no scalar loads and no cross-wave data;
//  * ASCII -> 2-bit codes by SWAR ((c>>1)^(c>>2))&3, four bases per byte; each lane forms the
//    four 16-mers starting at its 4-byte-aligned offsets, taking the next lane's packed chunk
//    through a DPP wave shift;
//  * each 16-mer is tested against a blocked Bloom filter of the anchor's 16-mers held in
//    LDS: one ds_read_b64 returns two 32-bit words, three hash-chosen bits must be set in
//    each (~1e-7 false positives per probe for a 6.8 kb anchor), no data-dependent control
//    flow on the hot path;
//  * Bloom-positive 16-mers add to 8-bit per-read counters in LDS; after the tile each wave
//    writes one int32 per read; the tile's reads with hits are appended to the candidate
//    list with ONE global atomic per tile (LDS prefix over the tile's 64-read ballots).
//
// Exactness: any MEM >= 19 nt (bwa -k 19) contains a 16-mer starting at an offset that is a
// multiple of 4 and a Bloom filter has no false negatives, so hits == 0 implies no seed; the
// filter can over-report, never drop.  oracle/af_oracle.c restates the same hits.
#include "af_internal.h"

#include <algorithm>

namespace {

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

// copies n uint2 from global to LDS with the whole workgroup, 8 loads in flight per thread
__device__ __forceinline__ void fill_lds(uint2 *dst, const uint2 *__restrict__ src, int n) {
    int i0 = 0;
    for (; i0 + 8 * 1024 <= n; i0 += 8 * 1024) {
        uint2 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = src[i0 + u * 1024 + threadIdx.x];
#pragma unroll
        for (int u = 0; u < 8; ++u) dst[i0 + u * 1024 + threadIdx.x] = v[u];
    }
    for (int i = i0 + (int)threadIdx.x; i < n; i += 1024) dst[i] = src[i];
}

// One round of a wave: lane l holds chunk c (packed P); lanes >= 63 or past the tile are off.
__device__ __forceinline__ void scan_round(uint32_t P, int c, bool in, const uint2 *bloom, int bshift,
                                           int32_t stride, uint32_t *cnt) {
    const uint32_t Pn = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)P, 0x130, 0xf, 0xf, false);  // wave_shl:1
    const uint64_t PP = ((uint64_t)Pn << 32) | P;
    bool pass[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t k = (uint32_t)(PP >> (8 * j));
        const uint32_t h1 = af_fmix(k), h2 = af_fmix2(h1);
        const uint2 w = bloom[h1 >> bshift];
        const uint32_t m0 = af_bloom_mask(h1), m1 = af_bloom_mask(h2);
        pass[j] = in && ((w.x & m0) == m0) && ((w.y & m1) == m1);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if (pass[j]) {
            const int off = c * 16 + 4 * j;
            const int r = off / stride;
            if (off - r * stride + AF_K <= stride) atomicAdd(&cnt[r >> 2], 1u << (8 * (r & 3)));
        }
    }
}

template <bool HAS_LENS>
__global__ __launch_bounds__(64 * AF_SEED_WAVES) void k_seed_filter(
    const uint8_t *__restrict__ reads, int64_t n_reads, int32_t stride, const int32_t *__restrict__ lens,
    const uint2 *__restrict__ bloom_g, int bl_bits, int32_t *__restrict__ hits, int32_t *__restrict__ cand,
    int32_t *__restrict__ cnt_g, int32_t *__restrict__ cnt_next) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ uint64_t gbal[AF_SEED_GROUPS];  // per 64-read group: ballot of reads with hits
    __shared__ int gbase[AF_SEED_GROUPS];      // per group: first cand slot
    const int nbl = 1 << bl_bits;
    uint2 *bloom = reinterpret_cast<uint2 *>(smem);
    uint32_t *cnt = reinterpret_cast<uint32_t *>(smem + (size_t)nbl * 8);  // AF_SEED_BTILE 8-bit counters
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // provably wave-uniform
    const int bshift = 32 - bl_bits;
    if (blockIdx.x == 0 && threadIdx.x == 0) *cnt_next = 0;  // next epoch's count (see af_internal.h)
    fill_lds(bloom, bloom_g, nbl);

    const int64_t ntiles = (n_reads + AF_SEED_BTILE - 1) / AF_SEED_BTILE;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t r0 = tile * AF_SEED_BTILE;
        const int nr = __builtin_amdgcn_readfirstlane((int)min((int64_t)AF_SEED_BTILE, n_reads - r0));
        for (int i = threadIdx.x; i < AF_SEED_BTILE / 4; i += blockDim.x) cnt[i] = 0;
        __syncthreads();
        const uint8_t *base = reads + r0 * (int64_t)stride;
        const int64_t bytes = (int64_t)nr * stride;
        const int nfull = __builtin_amdgcn_readfirstlane((int)(bytes >> 4));
        const int nchunks = __builtin_amdgcn_readfirstlane((int)((bytes + 15) >> 4));
        const int nblk = (nchunks + 62) / 63;                            // 63-chunk wave blocks
        const int nround = (nblk + AF_SEED_WAVES - 1) / AF_SEED_WAVES;  // rounds of this wave
        const bool l63 = lane < 63;
#define AF_CH(rr) ((((rr) * AF_SEED_WAVES + wv) * 63))
        if (nfull == nchunks) {
            // every chunk is whole: branch-free loads, addresses clamped into the tile (clamped
            // lanes are masked by `in`; a clamped neighbour only feeds 16-mers that cross the
            // tile end, which the per-read bound rejects).  Three named round buffers,
            // unrolled by 3: each load lands in the registers consumed two rounds later.
            const uint4 *cb = reinterpret_cast<const uint4 *>(base);
            const int last = nfull - 1;
            uint4 vA = cb[min(AF_CH(0) + lane, last)];
            uint4 vB = cb[min(AF_CH(1) + lane, last)];
            uint4 vC = cb[min(AF_CH(2) + lane, last)];
            for (int r = 0; r < nround; r += 3) {
                scan_round(pack_chunk(vA), AF_CH(r) + lane, l63 && AF_CH(r) + lane < nchunks, bloom, bshift, stride,
                           cnt);
                vA = cb[min(AF_CH(r + 3) + lane, last)];
                if (r + 1 < nround)
                    scan_round(pack_chunk(vB), AF_CH(r + 1) + lane, l63 && AF_CH(r + 1) + lane < nchunks, bloom,
                               bshift, stride, cnt);
                vB = cb[min(AF_CH(r + 4) + lane, last)];
                if (r + 2 < nround)
                    scan_round(pack_chunk(vC), AF_CH(r + 2) + lane, l63 && AF_CH(r + 2) + lane < nchunks, bloom,
                               bshift, stride, cnt);
                vC = cb[min(AF_CH(r + 5) + lane, last)];
            }
        } else {
            for (int r = 0; r < nround; ++r) {
                const int c = AF_CH(r) + lane;
                const uint4 v = c < nfull ? *reinterpret_cast<const uint4 *>(base + 16 * (int64_t)c)
                                          : (c < nchunks ? load_tail(base, c, bytes)
                                                         : make_uint4(0x4E4E4E4Eu, 0x4E4E4E4Eu, 0x4E4E4E4Eu,
                                                                      0x4E4E4E4Eu));
                scan_round(pack_chunk(v), c, l63 && c < nchunks, bloom, bshift, stride, cnt);
            }
        }
#undef AF_CH
        __syncthreads();
        if (HAS_LENS) {
            // ragged batch: recount reads shorter than stride exactly (rare path; the streamed
            // count above used the stride bound)
            for (int i = threadIdx.x; i < nr; i += blockDim.x) {
                const int l = lens[r0 + i];
                if (l >= stride) continue;
                uint32_t h = 0;
                const int64_t rb = (r0 + i) * (int64_t)stride;
                for (int o = (int)((4 - (rb & 3)) & 3); o + AF_K <= l; o += 4) {
                    uint32_t k = 0;
                    for (int u = 0; u < AF_K; ++u) {
                        const uint32_t ch = reads[rb + o + u];
                        k |= (((ch >> 1) ^ (ch >> 2)) & 3u) << (2 * u);
                    }
                    const uint32_t h1 = af_fmix(k), h2 = af_fmix2(h1);
                    const uint2 w = bloom[h1 >> bshift];
                    const uint32_t m0 = af_bloom_mask(h1), m1 = af_bloom_mask(h2);
                    h += ((w.x & m0) == m0) && ((w.y & m1) == m1);
                }
                const uint32_t sh = 8 * (i & 3);
                const uint32_t old = (cnt[i >> 2] >> sh) & 0xFFu;
                atomicAdd(&cnt[i >> 2], (h - old) << sh);  // per-byte replace, no carry (h, old < 256)
            }
            __syncthreads();
        }
        // candidate append: ONE device atomic per tile.  A device-scope atomic on a single
        // address is serialised across all 8 XCDs; one per 64-read group (~30k per launch)
        // cost more than the whole scan.
        for (int g = wv; g < AF_SEED_GROUPS; g += AF_SEED_WAVES) {
            const int i = g * 64 + lane;
            uint32_t h = 0;
            if (i < nr) {
                h = (cnt[i >> 2] >> (8 * (i & 3))) & 0xFFu;
                hits[r0 + i] = (int32_t)h;
            }
            const uint64_t bal = __ballot(h != 0);
            if (lane == 0) gbal[g] = bal;
        }
        __syncthreads();
        if (wv == 0) {
            const int c = lane < AF_SEED_GROUPS ? (int)__popcll(gbal[lane]) : 0;
            int incl = c;  // inclusive prefix over the tile's groups
            for (int d = 1; d < AF_SEED_GROUPS; d <<= 1) {
                const int t = __shfl_up(incl, d);
                if (lane >= d) incl += t;
            }
            const int total = __shfl(incl, AF_SEED_GROUPS - 1);
            int basei = 0;
            if (lane == 0 && total) basei = atomicAdd(cnt_g, total);
            basei = __shfl(basei, 0);
            if (lane < AF_SEED_GROUPS) gbase[lane] = basei + incl - c;
        }
        __syncthreads();
        for (int g = wv; g < AF_SEED_GROUPS; g += AF_SEED_WAVES) {
            const uint64_t bal = gbal[g];
            if ((bal >> lane) & 1ull)
                cand[gbase[g] + __popcll(bal & ((1ull << lane) - 1ull))] = (int32_t)(r0 + g * 64 + lane);
        }
        __syncthreads();
    }
}

}  // namespace

size_t af_seed_filter_lds(int bl_bits) { return ((size_t)1 << bl_bits) * 8 + AF_SEED_BTILE; }

hipError_t af_launch_seed_filter(const DevIndex &ix, const uint8_t *reads, int64_t n_reads, int32_t stride,
                                 const int32_t *lens, int32_t *hits, int32_t *cand, int32_t *cnt, int32_t *cnt_next,
                                 int n_cu, hipStream_t s) {
    if (n_reads <= 0) {
        hipError_t e = hipMemsetAsync(cnt, 0, sizeof(int32_t), s);
        return e == hipSuccess ? hipMemsetAsync(cnt_next, 0, sizeof(int32_t), s) : e;
    }
    const int64_t want = (n_reads + AF_SEED_BTILE - 1) / AF_SEED_BTILE;
    const size_t lds = af_seed_filter_lds(ix.bl_bits);
    const int per_cu = (int)std::max<size_t>(1, std::min<size_t>(2, (160 * 1024) / (lds + 1024)));
    const int64_t blocks = std::min<int64_t>(want, (int64_t)n_cu * per_cu);
    static bool attr_done = false;
    if (!attr_done) {  // dynamic LDS above 64 KiB needs the opt-in on both instantiations
        // (static + dynamic must stay within the CU's 160 KiB: leave 1 KiB for the static arrays)
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&k_seed_filter<true>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 159 * 1024);
        if (e == hipSuccess)
            e = hipFuncSetAttribute(reinterpret_cast<const void *>(&k_seed_filter<false>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, 159 * 1024);
        if (e != hipSuccess) return e;
        attr_done = true;
    }
    dim3 grid((unsigned)blocks), block(64 * AF_SEED_WAVES);
    if (lens)
        hipLaunchKernelGGL((k_seed_filter<true>), grid, block, lds, s, reads, n_reads, stride, lens, ix.bloom,
                           ix.bl_bits, hits, cand, cnt, cnt_next);
    else
        hipLaunchKernelGGL((k_seed_filter<false>), grid, block, lds, s, reads, n_reads, stride, lens, ix.bloom,
                           ix.bl_bits, hits, cand, cnt, cnt_next);
    return hipGetLastError();
}
