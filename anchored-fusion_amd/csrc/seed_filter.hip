// seed_filter.hip -- K1: HBM-streaming anchor seed filter (the seeding
// pass of `bwa mem` at Anchored_Fusion.py:182).
//
// Layout and schedule:
//  * persistent grid, one 1024-thread workgroup per CU (the 128 KiB Bloom table sets the LDS
//    budget); block B streams ONE contiguous range of reads, an equal share of the batch (ranges
//    start on 16-byte boundaries); the first chunk loads are issued before the table is copied
//    to LDS;
//  * the 16 waves sweep the range together in 63-chunk wave blocks (one coalesced 1-KiB
//    global_load_dwordx4 per wave and round, blocks overlapping by one 16-byte chunk), two
//    loads in flight per wave, no stores, barriers or returning atomics in the loop;
//  * a byte's 2-bit code is a table lookup on its low 3 bits (v_and + v_perm_b32 for four
//    bytes); 16-mer keys are "word-transposed" (base 4w+b at bits 8b+2w) so the chunk's code
//    words and the next lane's (DPP wave_shl:1) form the four keys at its 4-aligned offsets;
//  * probe: one 32x32->64 multiply per key; two ds_read_b32 (absolute LDS offsets) into the
//    2^bits-word table, four one-hot bits per word must be set (af_k1_hash/af_k1_mask);
//  * positives add to 8-bit per-read counters in LDS; the epilogue writes one int32 per read,
//    ballots per 64 reads and an LDS prefix, and ONE device atomic reserves the block's
//    candidate-list slots.
//
// Exactness: any MEM >= 19 nt (bwa -k 19) contains a 16-mer starting at an offset that is a
// multiple of 4 and a Bloom filter has no false negatives, so hits == 0 implies no seed; the
// filter can over-report, never drop.  oracle/af_oracle.c restates the same hits.
#include "af_internal.h"

#include <algorithm>

#ifndef AF_K1_ABL
#define AF_K1_ABL 0    // 1 = stream-only timing build (scripts/k1_ablate.sh); 0 = the product kernel
#endif
#ifndef AF_K1_DEPTH
#define AF_K1_DEPTH 2  // chunk loads in flight per wave in k_seed_stream (2: 40.6 us, 3: 40.9, 4: 41.5, 6: 43.3, 8: 43.6)
#endif
#ifndef AF_K1_TWO_STAGE
#define AF_K1_TWO_STAGE 0  // 1 = word 2 of a probe read only where word 1 passed
#endif
#ifndef AF_K1_NT
#define AF_K1_NT 0     // 1 = nontemporal (nt) stream loads of the reads
#endif
#ifndef AF_K1_PASS
#define AF_K1_PASS 8   // full tiles per streaming pass of k_seed_stream (8-bit counters in LDS)
#endif

namespace {

// four read bytes -> four 2-bit codes, one per byte (af_k1_code: v_and + v_perm_b32)
__device__ __forceinline__ uint32_t codes_w(uint32_t x) {
    return __builtin_amdgcn_perm(0x02000003u, 0x01000000u, x & 0x07070707u);
}

__device__ __forceinline__ uint32_t next_lane(uint32_t x) {  // lane l <- lane l+1 (DPP wave_shl:1)
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x130, 0xf, 0xf, true);  // lane 63 reads 0
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

// the last round(s) of a range: the chunk that straddles the range end is re-read byte-wise
// (out of line, so the common rounds carry no per-lane test)
__device__ __noinline__ uint4 tail_fix(uint4 v, int cb, int nfull, int nchunks, const uint8_t *__restrict__ base,
                                       int64_t bytes) {
    const int c = cb + (int)__lane_id();
    return c >= nfull && c < nchunks ? load_tail(base, c, bytes) : v;
}

// One Bloom probe of a key (af_k1_hash): both words are read from LDS, no branches.
__device__ __forceinline__ uint32_t onehot_bytes(uint32_t v) {  // af_k1_mask
    return __builtin_amdgcn_perm(0x80402010u, 0x08040201u, v & 0x07070707u);
}
// The Bloom table starts at LDS address 0 (the kernels have no static LDS; the launcher checks),
// so a probe addresses it with plain byte offsets and no base add.
__device__ __forceinline__ uint32_t lds_word(uint32_t byte_off) {
    return *reinterpret_cast<const __attribute__((address_space(3))) uint32_t *>((size_t)byte_off);
}
__device__ __forceinline__ bool probe(uint32_t key, int bshift, uint32_t wmask4) {
    const uint64_t h = af_k1_hash(key);
    const uint32_t lo = (uint32_t)h, hi = (uint32_t)(h >> 32);
    const uint32_t w1 = lds_word(hi & wmask4);
    const uint32_t w2 = lds_word((lo >> bshift) << 2);
    const uint32_t m1 = onehot_bytes(lo), m2 = onehot_bytes(hi);
    return ((m1 & ~w1) | (m2 & ~w2)) == 0u;
}
// Four probes with the eight LDS reads issued back to back (one wait for the round).  The
// residual of a probe is zero iff all its bits are set (the key may be in the anchor).
__device__ __forceinline__ void probe4(const uint32_t (&key)[4], int bshift, uint32_t wmask4, uint32_t (&res)[4]) {
    uint32_t lo[4], hi[4], w1[4], w2[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint64_t h = af_k1_hash(key[i]);
        lo[i] = (uint32_t)h;
        hi[i] = (uint32_t)(h >> 32);
    }
#if AF_K1_TWO_STAGE
    // Word 1 of every probe first; word 2 only where word 1 passed (P ~ 1e-4 per probe for a
    // key that is not in the anchor), under an exec mask: the LDS array -- the busiest unit of
    // this kernel -- serves half the random reads.  The outcome is the same conjunction.
#pragma unroll
    for (int i = 0; i < 4; ++i) w1[i] = lds_word(hi[i] & wmask4);
#pragma unroll
    for (int i = 0; i < 4; ++i) res[i] = onehot_bytes(lo[i]) & ~w1[i];
    if (min(min(res[0], res[1]), min(res[2], res[3])) == 0u) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (res[i] == 0u) res[i] = onehot_bytes(hi[i]) & ~lds_word((lo[i] >> bshift) << 2);
    }
#else
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#if AF_K1_ABL == 5  // timing only: no LDS reads (address-dependent stand-ins)
        w1[i] = (hi[i] & wmask4) * 0x01010101u;
        w2[i] = ((lo[i] >> bshift) << 2) * 0x01010101u;
#else
        w1[i] = lds_word(hi[i] & wmask4);
        w2[i] = lds_word((lo[i] >> bshift) << 2);
#endif
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) res[i] = (onehot_bytes(lo[i]) & ~w1[i]) | (onehot_bytes(hi[i]) & ~w2[i]);
#endif
}

// One round of a wave: lane l holds chunk c (16 read bytes = 4 code words); lanes >= 63 or
// past the tile are off.  The four 16-mers starting in the chunk take the next lane's first
// three code words through DPP.  Positives (rare) add to 8-bit per-read counters in LDS.
//
// The positives' read index: r = floor((off + 0.5) / stride) in f32 is exact here (off < 2^23
// is a tile-relative byte offset, stride <= AF_MAX_READ, so the quotient sits >= 0.5 / stride
// from an integer, far beyond f32 error); a chunk spans at most two reads, so at most two adds.
__device__ __forceinline__ void scan_round(const uint4 v, int cb, int c_end, int bshift,
                                           uint32_t wmask4, int32_t stride, float inv_stride, uint32_t *cnt) {
    const uint32_t c0 = codes_w(v.x), c1 = codes_w(v.y), c2 = codes_w(v.z), c3 = codes_w(v.w);
    const uint32_t a0 = c0 | (c1 << 2), a1 = c1 | (c2 << 2), a2 = c2 | (c3 << 2);
    const uint32_t a3 = c3 | (next_lane(c0) << 2);
    const uint32_t a4 = next_lane(a0), a5 = next_lane(a1);
    const uint32_t key[4] = {a0 | (a2 << 4), a1 | (a3 << 4), a2 | (a4 << 4), a3 | (a5 << 4)};
    uint32_t res[4];
    probe4(key, bshift, wmask4, res);
    // one compare for the round: some probe passed iff the least residual is zero
    const uint32_t rmin = min(min(min(res[0], res[1]), res[2]), res[3]);
    // lanes that own no chunk (lane 63, chunks >= c_end) probed clamped data: drop them here,
    // on the rare positive path, not with a compare per round
#if AF_K1_ABL == 4  // timing only: positives are kept live but not counted
    if (rmin == 0u && cb == -12345) {
#else
    if (rmin == 0u) {
#endif
        const int c = cb + (int)__lane_id();
        if ((int)__lane_id() == 63 || c >= c_end) return;
        const bool p0 = res[0] == 0u, p1 = res[1] == 0u, p2 = res[2] == 0u, p3 = res[3] == 0u;
        const uint32_t off = (uint32_t)c * 16u;
        const uint32_t r = (uint32_t)(((float)off + 0.5f) * inv_stride);
        const int o = (int)(off - r * (uint32_t)stride);
        // read r holds the chunk's k-mers j < ja (o + 4j + 16 <= stride); read r + 1 those with
        // jb <= j < jc (o + 4j >= stride, o + 4j - stride + 16 <= stride)
        const uint32_t pm = (uint32_t)p0 | ((uint32_t)p1 << 1) | ((uint32_t)p2 << 2) | ((uint32_t)p3 << 3);
        const int ja = min(max((stride - 12 - o) >> 2, 0), 4);
        const int jb = min((stride - o + 3) >> 2, 4);
        const int jc = min(max((2 * stride - 12 - o) >> 2, 0), 4);
        const uint32_t na = __builtin_popcount(pm & ((1u << ja) - 1u));
        const uint32_t nb = __builtin_popcount((pm >> jb) & ((1u << max(jc - jb, 0)) - 1u));
        if (na) atomicAdd(&cnt[r >> 2], na << (8 * (r & 3)));
        if (nb) atomicAdd(&cnt[(r + 1) >> 2], nb << (8 * ((r + 1) & 3)));
    }
}

// All tiles a block processes share this state (LDS pointers and wave coordinates).
struct K1 {
    int bshift;
    uint32_t wmask4;
    float inv_stride;
    int32_t stride;
    int lane, wv;
};

#define AF_CH(rr) ((((rr) * AF_SEED_WAVES + k.wv) * 63))

// One tile, unpipelined: rounds, optional ragged recount, and an epilogue with its own
// atomic.  Used for ragged batches and for the partial last tile of k_seed_stream.
template <bool HAS_LENS>
__device__ void one_tile(const K1 &k, const uint8_t *__restrict__ reads, int64_t n_reads, int64_t tile,
                         const int32_t *__restrict__ lens, uint32_t *cnt, uint64_t *gbal, int *gbase,
                         int32_t *__restrict__ hits, int32_t *__restrict__ cand, int32_t *__restrict__ cnt_g) {
    const int32_t stride = k.stride;
    const int lane = k.lane, wv = k.wv;
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
    [[maybe_unused]] const bool l63 = lane < 63;
    for (int r = 0; r < nround; ++r) {
        const int c = AF_CH(r) + lane;
        const uint4 v = c < nfull ? *reinterpret_cast<const uint4 *>(base + 16 * (int64_t)c)
                                  : (c < nchunks ? load_tail(base, c, bytes)
                                                 : make_uint4(0x4E4E4E4Eu, 0x4E4E4E4Eu, 0x4E4E4E4Eu, 0x4E4E4E4Eu));
        scan_round(v, c - lane, nchunks, k.bshift, k.wmask4, stride, k.inv_stride, cnt);
    }
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
                uint32_t key = 0;
                for (int u = 0; u < AF_K; ++u)
                    key |= af_k1_code(reads[rb + o + u]) << (8 * (u & 3) + 2 * (u >> 2));
                h += probe(key, k.bshift, k.wmask4);
            }
            const uint32_t sh = 8 * (i & 3);
            const uint32_t old = (cnt[i >> 2] >> sh) & 0xFFu;
            atomicAdd(&cnt[i >> 2], (h - old) << sh);  // per-byte replace, no carry (h, old < 256)
        }
        __syncthreads();
    }
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

// Ragged batches (lens != nullptr): one unpipelined tile at a time.
__global__ __launch_bounds__(64 * AF_SEED_WAVES) void k_seed_ragged(
    const uint8_t *__restrict__ reads, int64_t n_reads, int32_t stride, const int32_t *__restrict__ lens,
    const uint32_t *__restrict__ bloom_g, int bl_bits, int32_t *__restrict__ hits, int32_t *__restrict__ cand,
    int32_t *__restrict__ cnt_g, int32_t *__restrict__ cnt_next, int32_t *__restrict__ s2z) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int nw = 1 << bl_bits;
    uint32_t *cnt = reinterpret_cast<uint32_t *>(smem + (size_t)nw * 4);
    uint64_t *gbal = reinterpret_cast<uint64_t *>(cnt + AF_K1_PASS * (AF_SEED_BTILE / 4));
    int *gbase = reinterpret_cast<int *>(gbal + AF_K1_PASS * AF_SEED_GROUPS);
    const K1 k{32 - bl_bits, (uint32_t)(nw - 1) << 2, 1.0f / (float)stride, stride, (int)(threadIdx.x & 63),
               __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6))};
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // next epoch's count; this epoch's S2 words (af_internal.h)
        *cnt_next = 0;
        s2z[0] = 0;
        s2z[2 * AF_HEAD_STRIDE] = 0;
    }
    fill_lds(reinterpret_cast<uint2 *>(smem), reinterpret_cast<const uint2 *>(bloom_g), nw / 2);
    const int64_t ntiles = (n_reads + AF_SEED_BTILE - 1) / AF_SEED_BTILE;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x)
        one_tile<true>(k, reads, n_reads, tile, lens, cnt, gbal, gbase, hits, cand, cnt_g);
}

// Uniform-length batches.  Block B streams ONE contiguous range of reads, an equal share of
// the batch (ranges differ by at most one alignment unit of u = 16 / gcd(stride, 16) reads,
// so every range starts on a 16-byte boundary).  Inside the range the waves sweep 63-chunk
// blocks round-robin with AF_K1_DEPTH chunk loads in flight per wave; the loop body has no
// global stores, no returning atomics and no barriers, so every wait is a counted
// `vmcnt(DEPTH-1)`.  Per-read 8-bit counters for the whole range live in LDS (ranges longer
// than AF_K1_PASS * AF_SEED_BTILE reads are streamed in sub-ranges); one epilogue writes the
// hits, and one device atomic reserves the candidate slots.  The first loads are issued
// before the Bloom table is copied to LDS, so HBM streaming starts with the launch.
__global__ __launch_bounds__(64 * AF_SEED_WAVES) void k_seed_stream(
    const uint8_t *__restrict__ reads, int64_t n_reads, int32_t stride, const uint32_t *__restrict__ bloom_g,
    int bl_bits, int32_t *__restrict__ hits, int32_t *__restrict__ cand, int32_t *__restrict__ cnt_g,
    int32_t *__restrict__ cnt_next, int32_t *__restrict__ s2z) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int CAP = AF_K1_PASS * AF_SEED_BTILE;  // reads per sub-range (LDS counters)
    const int nw = 1 << bl_bits;
    uint32_t *cnt = reinterpret_cast<uint32_t *>(smem + (size_t)nw * 4);  // [CAP / 4]
    uint64_t *gbal = reinterpret_cast<uint64_t *>(cnt + CAP / 4);
    int *gbase = reinterpret_cast<int *>(gbal + CAP / 64);
    const K1 k{32 - bl_bits, (uint32_t)(nw - 1) << 2, 1.0f / (float)stride, stride, (int)(threadIdx.x & 63),
               __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6))};
    const int lane = k.lane, wv = k.wv;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        *cnt_next = 0;
        s2z[0] = 0;
        s2z[2 * AF_HEAD_STRIDE] = 0;
    }
    // this block's range [ra, rb) in units of u reads
    const int lowbit = stride & -stride;  // gcd(stride, 16) = min(lowbit, 16)
    const int u = 16 / (lowbit < 16 ? lowbit : 16);
    const int64_t nunits = (n_reads + u - 1) / u;
    const int64_t G = gridDim.x, B = blockIdx.x;
    const int64_t ra = min(n_reads, (B * nunits / G) * u), rb = min(n_reads, ((B + 1) * nunits / G) * u);
    [[maybe_unused]] const bool l63 = lane < 63;
    // sub-range state: [sa, sa + nr) of the block's range, its bytes and 16-byte chunks
    int64_t sa = ra;
    int nr = 0, nfull = 0, nchunks = 0, total = 0, clast = 0, lr = 0, sr = 0;
    int64_t bytes = 0;
    const uint8_t *base = reads;
    auto setup = [&]() {
        nr = (int)min((int64_t)CAP, rb - sa);
        base = reads + sa * (int64_t)stride;
        bytes = (int64_t)nr * stride;
        nfull = (int)(bytes >> 4);
        nchunks = (int)((bytes + 15) >> 4);
        const int nblk = (nchunks + 62) / 63;
        total = (nblk + AF_SEED_WAVES - 1) / AF_SEED_WAVES;  // rounds of every wave
        clast = nfull > 0 ? nfull - 1 : 0;
        lr = 0;
        sr = 0;
    };
    // round r of wave wv covers chunks AF_CH(r) + lane; chunks past the last full one are
    // loaded (clamped) and then re-read byte-wise by load_tail in the scan
    // (32-bit byte offsets from the sub-range base: one add and one min per load)
    // (scalar chunk base clamped to the last full chunk, then one v_min per load)
    const uint32_t lane_off = 16u * (uint32_t)lane;
    auto next_load = [&]() -> uint4 {
        const int cb = min(AF_CH(min(lr, total - 1)), clast);
        const uint8_t *rbase = base + 16 * (int64_t)cb;
        const uint32_t off = min(lane_off, 16u * (uint32_t)(clast - cb));
        ++lr;
#if AF_K1_NT
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(rbase + off));
        return make_uint4(v.x, v.y, v.z, v.w);
#else
        return *reinterpret_cast<const uint4 *>(rbase + off);
#endif
    };
#define AF_PIN asm volatile("" ::: "memory")
    uint4 b[AF_K1_DEPTH];
    if (sa < rb) {
        setup();
#pragma unroll
        for (int q = 0; q < AF_K1_DEPTH; ++q) {
            b[q] = next_load();
            AF_PIN;
        }
    }
    // the Bloom table, while the first chunk loads are in flight
    fill_lds(reinterpret_cast<uint2 *>(smem), reinterpret_cast<const uint2 *>(bloom_g), nw / 2);
    while (sa < rb) {
        for (int i = threadIdx.x; i < (nr + 3) / 4; i += blockDim.x) cnt[i] = 0;
        __syncthreads();
#if AF_K1_ABL
        uint32_t abl = 0;
#endif
        auto scan = [&](uint4 v) {
            const int cb = AF_CH(sr);
            if (cb + 63 >= nfull) v = tail_fix(v, cb, nfull, nchunks, base, bytes);  // wave-uniform test
#if AF_K1_ABL == 1
            abl ^= v.x ^ v.y ^ v.z ^ v.w;
#else
            scan_round(v, cb, nchunks, k.bshift, k.wmask4, stride, k.inv_stride, cnt);
#endif
            ++sr;
        };
        int g = 0;
        for (; g + AF_K1_DEPTH <= total; g += AF_K1_DEPTH) {
#pragma unroll
            for (int q = 0; q < AF_K1_DEPTH; ++q) {
                scan(b[q]);
                b[q] = next_load();
                AF_PIN;
            }
        }
#pragma unroll
        for (int q = 0; q < AF_K1_DEPTH - 1; ++q)
            if (g + q < total) scan(b[q]);
#if AF_K1_ABL
        if (abl == 0x12345679u) cnt[0] = abl;  // keep the ablated work live
#endif
        // the next sub-range's first loads go out before this one's epilogue (no stream bubble)
        const int64_t sa_c = sa;
        const int nr_c = nr;
        sa += CAP;
        if (sa < rb) {
            setup();
#pragma unroll
            for (int q = 0; q < AF_K1_DEPTH; ++q) {
                b[q] = next_load();
                AF_PIN;
            }
        }
        __syncthreads();  // the sub-range is counted
        // epilogue: hits and 64-read ballots, one atomic for the sub-range
        const int ng = (nr_c + 63) / 64;
        for (int q = wv; q < ng; q += AF_SEED_WAVES) {
            const int i = q * 64 + lane;
            uint32_t h = 0;
            if (i < nr_c) {
                h = (cnt[i >> 2] >> (8 * (i & 3))) & 0xFFu;
                hits[sa_c + i] = (int32_t)h;
            }
            const uint64_t bal = __ballot(h != 0);
            if (lane == 0) gbal[q] = bal;
        }
        __syncthreads();
        if (wv == 0) {
            int carry = 0;  // exclusive prefix over the groups, 64 per step
            for (int q0 = 0; q0 < ng; q0 += 64) {
                const int q = q0 + lane;
                const int c = q < ng ? (int)__popcll(gbal[q]) : 0;
                int incl = c;
                for (int d = 1; d < 64; d <<= 1) {
                    const int t = __shfl_up(incl, d);
                    if (lane >= d) incl += t;
                }
                if (q < ng) gbase[q] = carry + incl - c;
                carry += __shfl(incl, 63);
            }
            int bse = 0;
#if AF_K1_ABL == 6  // timing only: no returning device atomic (candidate slots overlap)
            if (lane == 0 && carry) bse = (int)(blockIdx.x & 7);
#else
            if (lane == 0 && carry) bse = atomicAdd(cnt_g, carry);
#endif
            bse = __shfl(bse, 0);
            for (int q = lane; q < ng; q += 64) gbase[q] += bse;
        }
        __syncthreads();
        for (int q = wv; q < ng; q += AF_SEED_WAVES) {
            const uint64_t bal = gbal[q];
            if ((bal >> lane) & 1ull)
                cand[gbase[q] + __popcll(bal & ((1ull << lane) - 1ull))] = (int32_t)(sa_c + q * 64 + lane);
        }
        __syncthreads();
    }
#undef AF_PIN
}
#undef AF_CH

}  // namespace

// dynamic LDS: Bloom words, then 8-bit read counters (AF_K1_PASS * AF_SEED_BTILE reads),
// then 64-read ballots and candidate bases
size_t af_seed_filter_lds(int bl_bits) {
    return ((size_t)1 << bl_bits) * 4 + AF_K1_PASS * AF_SEED_BTILE + AF_K1_PASS * AF_SEED_GROUPS * 12;
}

hipError_t af_launch_seed_filter(const DevIndex &ix, const uint8_t *reads, int64_t n_reads, int32_t stride,
                                 const int32_t *lens, int32_t *hits, int32_t *cand, int32_t *cnt, int32_t *cnt_next,
                                 int32_t *s2z, int n_cu, hipStream_t s) {
    if (n_reads <= 0) {
        hipError_t e = hipMemsetAsync(cnt, 0, sizeof(int32_t), s);
        if (e == hipSuccess) e = hipMemsetAsync(cnt_next, 0, sizeof(int32_t), s);
        if (e == hipSuccess) e = hipMemsetAsync(s2z, 0, sizeof(int32_t), s);
        return e == hipSuccess ? hipMemsetAsync(s2z + 2 * AF_HEAD_STRIDE, 0, sizeof(int32_t), s) : e;
    }
    const int64_t want = (n_reads + AF_SEED_BTILE - 1) / AF_SEED_BTILE;
    const size_t lds = af_seed_filter_lds(ix.bl_bits);
    const int per_cu = (int)std::max<size_t>(1, std::min<size_t>(2, (160 * 1024) / (lds + 1024)));
    const int64_t blocks = std::min<int64_t>(want, (int64_t)n_cu * per_cu);
    static bool attr_done = false;
    if (!attr_done) {  // dynamic LDS above 64 KiB needs the opt-in; static + dynamic stays within 160 KiB
        const void *fns[2] = {reinterpret_cast<const void *>(&k_seed_ragged),
                              reinterpret_cast<const void *>(&k_seed_stream)};
        for (const void *fn : fns) {
            hipFuncAttributes fa;
            hipError_t e = hipFuncGetAttributes(&fa, fn);
            if (e == hipSuccess && fa.sharedSizeBytes != 0) e = hipErrorInvalidKernelFile;  // lds_word: table at 0
            if (e == hipSuccess)
                e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                        (int)(160 * 1024 - fa.sharedSizeBytes));
            if (e != hipSuccess) return e;
        }
        attr_done = true;
    }
    dim3 grid((unsigned)blocks), block(64 * AF_SEED_WAVES);
    if (lens)
        hipLaunchKernelGGL(k_seed_ragged, grid, block, lds, s, reads, n_reads, stride, lens, ix.bloom, ix.bl_bits,
                           hits, cand, cnt, cnt_next, s2z);
    else
        hipLaunchKernelGGL(k_seed_stream, grid, block, lds, s, reads, n_reads, stride, ix.bloom, ix.bl_bits, hits,
                           cand, cnt, cnt_next, s2z);
    return hipGetLastError();
}
