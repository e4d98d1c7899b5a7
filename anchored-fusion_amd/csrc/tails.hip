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
// k_gather_reads turns row lists of S3 (af_partition_device) into the genome searches' queries:
// S4's `samtools fastq` of tmp1 / tmp2 (Anchored_Fusion.py:186-188: the reads as sequenced, the
// two lists interleaved as bwa's two input files pair them) and S5's split-read FASTA
// (functions.py:705-716: rows whose CIGAR deal_cigar reduces to two operations, SEQ as SAM prints
// it).  The S5 selection is an order-preserving select (hipCUB), so queries keep realign.bam order.
//
// k_clamp_count copies min(count, cap) to the placement kernel's query count, so af_place_device
// never reads past the tails buffer whatever the count says.
#include <hipcub/hipcub.hpp>

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

// deal_cigar (functions.py:656-702) leaves exactly two operations for an S2 primary CIGAR (M, I,
// D, S only) when it has one soft clip and an aligned part: I and D vanish, M runs merge
__device__ __forceinline__ bool deal_cigar_split(int nc, const uint32_t *cig) {
    int ns = 0, nm = 0;
    for (int k = 0; k < nc && k < AF_MAX_CIGAR; ++k) {
        const int op = cig[k] & 0xf;
        ns += op == 4;
        nm += op == 0;
    }
    return ns == 1 && nm > 0;
}

struct IsSplit {
    const int32_t *flag, *n_cigar;
    const uint32_t *cigar;
    __device__ bool operator()(int32_t r) const {
        return !(flag[r] & 0x4) && deal_cigar_split(n_cigar[r], cigar + (int64_t)r * AF_MAX_CIGAR);
    }
};

// one wave per query row: lanes copy the bases (reverse complement for SAM-oriented 0x10 reads)
__global__ void k_gather_reads(const uint8_t *__restrict__ reads, int32_t stride, const int32_t *__restrict__ lens,
                               const int32_t *__restrict__ rows, const int64_t *__restrict__ n_rows_dev,
                               int64_t n_rows, const int32_t *__restrict__ flag, int32_t sam_orient,
                               int64_t first, int64_t step, int64_t cap, uint8_t *__restrict__ q,
                               int32_t *__restrict__ q_lens, int32_t *__restrict__ q_rows) {
    const int lane = threadIdx.x & 63;
    const int64_t k = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t n = n_rows_dev ? min(*n_rows_dev, n_rows) : n_rows;
    if (k >= n) return;
    const int64_t slot = first + k * step;
    if (slot >= cap) return;
    const int32_t r = rows[k];
    const int l = lens ? min(lens[r], stride) : stride;
    const bool rc = sam_orient && (flag[r] & 0x10);
    const uint8_t *src = reads + (int64_t)r * stride;
    uint8_t *dst = q + slot * stride;
    for (int j = lane; j < stride; j += 64) {
        uint8_t b = 'N';
        if (j < l) {
            b = src[rc ? l - 1 - j : j];
            if (rc) b = b == 'A' ? 'T' : b == 'C' ? 'G' : b == 'G' ? 'C' : b == 'T' ? 'A' : b == 'a' ? 't' : b == 'c' ? 'g' : b == 'g' ? 'c' : b == 't' ? 'a' : 'N';
        }
        dst[j] = b;
    }
    if (lane == 0) {
        q_lens[slot] = l;
        if (q_rows) q_rows[slot] = r;
    }
}

__global__ void k_store_count(const int64_t *__restrict__ n_dev, int64_t n_host, int64_t first, int64_t step,
                              int64_t cap, int32_t *__restrict__ dst) {
    if (threadIdx.x == 0) {
        const int64_t n = n_dev ? min(*n_dev, n_host) : n_host;
        const int64_t end = n > 0 ? first + (n - 1) * step + 1 : first;
        *dst = (int32_t)(end > cap ? cap : end);
    }
}

}  // namespace

size_t af_gather_temp_bytes(int64_t n_rows) {
    size_t b = 0;
    (void)hipcub::DeviceSelect::If(nullptr, b, (const int32_t *)nullptr, (int32_t *)nullptr, (int64_t *)nullptr,
                                   n_rows, IsSplit{nullptr, nullptr, nullptr});
    return b;
}

hipError_t af_launch_gather(const uint8_t *reads, int32_t stride, const int32_t *lens, const int32_t *rows,
                            int64_t n_rows, int32_t mode, const af_aln_out &out, int64_t first, int64_t step,
                            int64_t cap, uint8_t *q, int32_t *q_lens, int32_t *q_rows, int32_t *n_q, int32_t *sel,
                            int64_t *sel_n, void *temp, size_t temp_bytes, hipStream_t s) {
    hipError_t e;
    const int64_t *n_dev = nullptr;
    if (mode == AF_GATHER_SPLIT_SAM) {
        size_t tb = temp_bytes;
        if (n_rows > 0 && (e = hipcub::DeviceSelect::If(temp, tb, rows, sel, sel_n, n_rows,
                                                        IsSplit{out.flag, out.n_cigar, out.cigar}, s)) != hipSuccess)
            return e;
        if (n_rows == 0 && (e = hipMemsetAsync(sel_n, 0, sizeof(int64_t), s)) != hipSuccess) return e;
        rows = sel;
        n_dev = sel_n;
    }
    if (n_rows > 0) {
        const int64_t waves = n_rows;
        hipLaunchKernelGGL(k_gather_reads, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, s, reads, stride, lens,
                           rows, n_dev, n_rows, out.flag, mode == AF_GATHER_SPLIT_SAM ? 1 : 0, first, step, cap, q,
                           q_lens, q_rows);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if (n_q) {
        hipLaunchKernelGGL(k_store_count, dim3(1), dim3(64), 0, s, n_dev, n_rows, first, step, cap, n_q);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    return hipSuccess;
}

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
