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
// each tail back to its read (read_base + row).  With `append` the counter is not reset, so the
// batches of a group (one stream each) can fill one tails buffer for a single placement launch.
//
// The per-read rule is af_emit_tail (af_internal.h), which K3 (k_pairs) also runs when
// af_align_candidates_tails_device asks for the tails with the records.
//
// k_clamp_count copies min(count, cap) to the placement kernel's query count, so af_place_device
// never reads past the tails buffer whatever the count says.
#include "af_internal.h"

namespace {

__global__ void k_split_tails(const uint8_t *__restrict__ reads, int64_t n_reads, int32_t stride,
                              const int32_t *__restrict__ lens, const int32_t *__restrict__ flag,
                              const int32_t *__restrict__ n_cigar, const uint32_t *__restrict__ cigar,
                              AfTails t) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_reads) return;
    const int f = flag[r];
    if ((f & 0x4) || n_cigar[r] != 2) return;
    af_emit_tail(t, reads, stride, lens, r, f, cigar + r * AF_MAX_CIGAR);
}

__global__ void k_clamp_count(const int32_t *__restrict__ count, int64_t cap, int32_t *__restrict__ dst) {
    if (threadIdx.x == 0) {
        const int64_t v = *count;
        *dst = (int32_t)(v < 0 ? 0 : (v > cap ? cap : v));
    }
}

}  // namespace

hipError_t af_launch_split_tails(const uint8_t *reads, int64_t n_reads, int32_t stride, const int32_t *lens,
                                 const af_aln_out &out, const AfTails &t, bool append, hipStream_t s) {
    hipError_t e = append ? hipSuccess : hipMemsetAsync(t.n_tails, 0, 4, s);
    if (e != hipSuccess || n_reads == 0) return e;
    const int bs = 256;
    hipLaunchKernelGGL(k_split_tails, dim3((unsigned)((n_reads + bs - 1) / bs)), dim3(bs), 0, s, reads, n_reads,
                       stride, lens, out.flag, out.n_cigar, out.cigar, t);
    return hipGetLastError();
}

hipError_t af_launch_clamp_count(const int32_t *count, int64_t cap, int32_t *dst, hipStream_t s) {
    hipLaunchKernelGGL(k_clamp_count, dim3(1), dim3(64), 0, s, count, cap, dst);
    return hipGetLastError();
}
