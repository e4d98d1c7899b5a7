// seed_filter.hip -- K1: HBM-streaming anchor seed filter (the seeding
// pass of `bwa mem` at Anchored_Fusion.py:182).
//
// Every read of the batch is streamed once from HBM (1 B/base, 16-B coalesced loads).  A
// wave owns a tile of AF_SEED_TILE whole reads; lane l of the wave loads 16-byte chunk l
// of the tile, converts ASCII to 2-bit codes with SWAR arithmetic, and takes the next
// lane's packed chunk by a shuffle, so each lane forms the four 16-mers that start at its
// 4-byte-aligned offsets.  Each 16-mer is probed in the anchor filter table held in LDS
// (bucket of 8 x u16: seven 15-bit fingerprints + an overflow flag, one ds_read_b128 per
// probe).  Hits are counted per read in 8-bit LDS counters; the wave then writes one int32
// per read and appends reads with hits to the candidate list (one atomic per 64 reads).
//
// Exactness: any MEM >= 19 nt (bwa -k 19) contains a 16-mer starting at an offset that is
// a multiple of 4, so hits == 0 implies the read has no seed; the filter can only
// over-report (fingerprint collisions), never drop a seeded read.
#include "af_internal.h"

namespace {

__device__ __forceinline__ uint32_t codes4(uint32_t x) { return ((x >> 1) ^ (x >> 2)) & 0x03030303u; }

// bytes y0..y3 (2-bit codes) -> y0 | y1<<2 | y2<<4 | y3<<6
__device__ __forceinline__ uint32_t pack4(uint32_t y) {
    uint32_t t = y | (y >> 6);
    return (t & 0xFu) | ((t >> 12) & 0xF0u);
}

// 1 if the 4 bytes of x are all A/C/G/T (either case)
__device__ __forceinline__ uint32_t valid4(uint32_t x, uint32_t y) {
    const uint32_t expect = __builtin_amdgcn_perm(0u, 0x54474341u, y);  // "ACGT"[code] per byte
    return (x & 0xDFDFDFDFu) == expect ? 1u : 0u;
}

__device__ __forceinline__ void pack_chunk(const uint4 v, uint32_t &P, uint32_t &vm) {
    const uint32_t y0 = codes4(v.x), y1 = codes4(v.y), y2 = codes4(v.z), y3 = codes4(v.w);
    P = pack4(y0) | (pack4(y1) << 8) | (pack4(y2) << 16) | (pack4(y3) << 24);
    vm = valid4(v.x, y0) | (valid4(v.y, y1) << 1) | (valid4(v.z, y2) << 2) | (valid4(v.w, y3) << 3);
}

__device__ __forceinline__ bool has_zero_half(uint32_t x) { return ((x - 0x00010001u) & ~x & 0x80008000u) != 0; }

__device__ __forceinline__ bool probe(const uint4 *__restrict__ tab, int nb_bits, uint32_t k) {
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

// 16 bytes of the tile at chunk c; bytes past the tile read as 'N'
__device__ __forceinline__ uint4 load_chunk(const uint8_t *__restrict__ base, int c, int nfull, int64_t tile_bytes) {
    if (c < nfull) return *reinterpret_cast<const uint4 *>(base + 16 * (int64_t)c);
    uint32_t w[4] = {0x4E4E4E4Eu, 0x4E4E4E4Eu, 0x4E4E4E4Eu, 0x4E4E4E4Eu};
    const int64_t o = 16 * (int64_t)c;
    if (o < tile_bytes) {
        for (int b = 0; b < 16; ++b)
            if (o + b < tile_bytes) {
                w[b >> 2] &= ~(0xFFu << (8 * (b & 3)));
                w[b >> 2] |= (uint32_t)base[o + b] << (8 * (b & 3));
            }
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
}

template <bool HAS_LENS>
__global__ __launch_bounds__(64 * AF_SEED_WAVES) void k_seed_filter(
    const uint8_t *__restrict__ reads, int64_t n_reads, int32_t stride, const int32_t *__restrict__ lens,
    const uint4 *__restrict__ ftab, int nb_bits, int32_t *__restrict__ hits, int32_t *__restrict__ cand,
    int32_t *__restrict__ n_cand) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint4 *tab = reinterpret_cast<uint4 *>(smem);
    const int nb = 1 << nb_bits;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t *cnt = reinterpret_cast<uint32_t *>(smem + (size_t)nb * 16) + wv * (AF_SEED_TILE / 4);
    for (int i = threadIdx.x; i < nb; i += blockDim.x) tab[i] = ftab[i];
    for (int i = lane; i < AF_SEED_TILE / 4; i += 64) cnt[i] = 0;
    __syncthreads();

    const int64_t r0 = ((int64_t)blockIdx.x * AF_SEED_WAVES + wv) * AF_SEED_TILE;
    if (r0 >= n_reads) return;
    const int nr = (int)min((int64_t)AF_SEED_TILE, n_reads - r0);
    const uint8_t *base = reads + r0 * (int64_t)stride;
    const int64_t tile_bytes = (int64_t)nr * stride;
    const int nchunks = (int)((tile_bytes + 15) >> 4);
    const int nfull = (int)(tile_bytes >> 4);

    for (int c0 = 0; c0 < nchunks; c0 += 128) {
        // two chunks per lane in flight
        const int ca = c0 + lane, cb = c0 + 64 + lane;
        const uint4 va = load_chunk(base, ca, nfull, tile_bytes);
        const uint4 vb = load_chunk(base, cb, nfull, tile_bytes);
        uint4 vx = make_uint4(0x4E4E4E4Eu, 0x4E4E4E4Eu, 0x4E4E4E4Eu, 0x4E4E4E4Eu);
        if (lane == 63) vx = load_chunk(base, cb + 1, nfull, tile_bytes);
        uint32_t Pa, ma, Pb, mb, Px, mx;
        pack_chunk(va, Pa, ma);
        pack_chunk(vb, Pb, mb);
        pack_chunk(vx, Px, mx);
        uint32_t Pan = __shfl_down(Pa, 1), man = __shfl_down(ma, 1);
        uint32_t Pbn = __shfl_down(Pb, 1), mbn = __shfl_down(mb, 1);
        const uint32_t Pb0 = __shfl(Pb, 0), mb0 = __shfl(mb, 0);
        if (lane == 63) { Pan = Pb0; man = mb0; Pbn = Px; mbn = mx; }
#pragma unroll
        for (int half = 0; half < 2; ++half) {
            const int c = half ? cb : ca;
            if (c >= nchunks) continue;
            const uint32_t P = half ? Pb : Pa, Pn = half ? Pbn : Pan;
            const uint32_t vv = (half ? mb : ma) | ((half ? mbn : man) << 4);
            const uint64_t PP = ((uint64_t)Pn << 32) | P;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (((vv >> j) & 0xFu) != 0xFu) continue;
                const uint32_t k = (uint32_t)(PP >> (8 * j));
                if (probe(tab, nb_bits, k)) {
                    const int off = c * 16 + 4 * j;
                    const int r = off / stride;
                    const int rem = off - r * stride;
                    const int l = HAS_LENS ? lens[r0 + r] : stride;
                    if (rem + AF_K <= l) atomicAdd(&cnt[r >> 2], 1u << (8 * (r & 3)));
                }
            }
        }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    for (int i0 = 0; i0 < nr; i0 += 64) {
        const int i = i0 + lane;
        uint32_t h = 0;
        if (i < nr) {
            h = (cnt[i >> 2] >> (8 * (i & 3))) & 0xFFu;
            hits[r0 + i] = (int32_t)h;
        }
        const uint64_t bal = __ballot(h != 0);
        if (bal) {
            int basei = 0;
            if (lane == 0) basei = atomicAdd(n_cand, (int)__popcll(bal));
            basei = __shfl(basei, 0);
            if (h) cand[basei + __popcll(bal & ((1ull << lane) - 1ull))] = (int32_t)(r0 + i);
        }
    }
}

}  // namespace

hipError_t af_launch_seed_filter(const DevIndex &ix, const uint8_t *reads, int64_t n_reads, int32_t stride,
                                 const int32_t *lens, int32_t *hits, int32_t *cand, int32_t *n_cand,
                                 hipStream_t s) {
    if (n_reads <= 0) return hipSuccess;
    const int64_t tiles = (n_reads + AF_SEED_TILE - 1) / AF_SEED_TILE;
    const int64_t blocks = (tiles + AF_SEED_WAVES - 1) / AF_SEED_WAVES;
    const size_t lds = ((size_t)1 << ix.nb_bits) * 16 + (size_t)AF_SEED_WAVES * AF_SEED_TILE;
    dim3 grid((unsigned)blocks), block(64 * AF_SEED_WAVES);
    static bool attr_done = false;
    if (!attr_done) {  // dynamic LDS above 64 KiB needs the opt-in on both instantiations
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_seed_filter<true>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_seed_filter<false>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_done = true;
    }
    if (lens)
        hipLaunchKernelGGL(k_seed_filter<true>, grid, block, lds, s, reads, n_reads, stride, lens, ix.ftab,
                           ix.nb_bits, hits, cand, n_cand);
    else
        hipLaunchKernelGGL(k_seed_filter<false>, grid, block, lds, s, reads, n_reads, stride, lens, ix.ftab,
                           ix.nb_bits, hits, cand, n_cand);
    return hipGetLastError();
}
