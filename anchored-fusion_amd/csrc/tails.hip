// tails.hip -- split-read tails for partner placement, on the device.
//
// k_split_tails turns the S2 records (af_align_*_device output) into the placement queries of
// the reference's split-read stages: a split read is a mapped primary whose CIGAR has exactly
// two operations, one M and one soft clip S (deal_cigar's two-op case, functions.py:713, and
// the SM / MS types of fn:917-931).  Its tail is the clipped part of SEQ in SAM orientation
// (reverse-complemented read for 0x10), the part `Find_Anchored_split` searches for the
// partner (fn:1001-1005).  One thread per read: the flag / n_cigar loads are coalesced, the
// CIGAR row and the read bytes are touched only for split reads (a few per thousand).  Output
// slots come from one device counter, so the tails' order varies between runs; tail_read maps
// each tail back to its read.
//
// k_clamp_count copies min(count, cap) to the placement kernel's query count, so af_place_device
// never reads past the tails buffer whatever the count says.
#include "af_internal.h"

namespace {

__device__ __forceinline__ uint8_t comp_base(uint8_t c) {
    switch (c | 0x20) {
        case 'a': return 'T';
        case 'c': return 'G';
        case 'g': return 'C';
        case 't': return 'A';
        default: return 'N';
    }
}

__global__ void k_split_tails(const uint8_t *__restrict__ reads, int64_t n_reads, int32_t stride,
                              const int32_t *__restrict__ lens, const int32_t *__restrict__ flag,
                              const int32_t *__restrict__ n_cigar, const uint32_t *__restrict__ cigar,
                              int32_t min_clip, int64_t cap, uint8_t *__restrict__ tails,
                              int32_t *__restrict__ tail_lens, int32_t *__restrict__ tail_read,
                              int32_t *__restrict__ n_tails) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_reads) return;
    const int f = flag[r];
    if ((f & 0x4) || n_cigar[r] != 2) return;
    const uint32_t c0 = cigar[r * AF_MAX_CIGAR], c1 = cigar[r * AF_MAX_CIGAR + 1];
    const int op0 = c0 & 0xf, op1 = c1 & 0xf;  // 0 = M, 4 = S
    int clip, head;
    if (op0 == 4 && op1 == 0) { clip = (int)(c0 >> 4); head = 1; }
    else if (op0 == 0 && op1 == 4) { clip = (int)(c1 >> 4); head = 0; }
    else return;
    const int len = lens ? lens[r] : stride;
    if (clip < min_clip || clip > len) return;
    const int slot = atomicAdd(n_tails, 1);
    if (slot >= cap) return;
    const uint8_t *q = reads + r * (int64_t)stride;
    uint8_t *o = tails + (int64_t)slot * stride;
    const bool rev = (f & 0x10) != 0;
    // SEQ[i] = rev ? comp(read[len - 1 - i]) : read[i]; the tail is SEQ[0, clip) or SEQ[len - clip, len)
    const int s0 = head ? 0 : len - clip;
    for (int i = 0; i < clip; ++i) {
        const int k = s0 + i;
        o[i] = rev ? comp_base(q[len - 1 - k]) : q[k];
    }
    tail_lens[slot] = clip;
    tail_read[slot] = (int32_t)r;
}

__global__ void k_clamp_count(const int32_t *__restrict__ count, int64_t cap, int32_t *__restrict__ dst) {
    if (threadIdx.x == 0) {
        const int64_t v = *count;
        *dst = (int32_t)(v < 0 ? 0 : (v > cap ? cap : v));
    }
}

}  // namespace

hipError_t af_launch_split_tails(const uint8_t *reads, int64_t n_reads, int32_t stride, const int32_t *lens,
                                 const af_aln_out &out, int32_t min_clip, int64_t cap, uint8_t *tails,
                                 int32_t *tail_lens, int32_t *tail_read, int32_t *n_tails, hipStream_t s) {
    hipError_t e = hipMemsetAsync(n_tails, 0, 4, s);
    if (e != hipSuccess || n_reads == 0) return e;
    const int bs = 256;
    hipLaunchKernelGGL(k_split_tails, dim3((unsigned)((n_reads + bs - 1) / bs)), dim3(bs), 0, s, reads, n_reads,
                       stride, lens, out.flag, out.n_cigar, out.cigar, min_clip, cap, tails, tail_lens, tail_read,
                       n_tails);
    return hipGetLastError();
}

hipError_t af_launch_clamp_count(const int32_t *count, int64_t cap, int32_t *dst, hipStream_t s) {
    hipLaunchKernelGGL(k_clamp_count, dim3(1), dim3(64), 0, s, count, cap, dst);
    return hipGetLastError();
}
