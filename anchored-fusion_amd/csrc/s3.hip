// s3.hip -- S3 on the device: the coordinate sort of `bwa mem ... | samtools sort` and the three
// flag filters that follow it (Anchored_Fusion.py:182, 186-194).
//
// samtools' coordinate order on the anchor: placed records by (pos, strand), ties in input order
// (pair, mate), then the unplaced ones.  Every record the filters keep is placed (a mapped read,
// or an unmapped read carrying its mapped mate's position), so only the placed records that pass
// at least one filter are sorted:
//   1. select + key   every such row r becomes key (2 pos + is_rev) << 32 | r (unique keys, so
//                     any sort gives the stable order); order-preserving select (hipCUB)
//   2. radix sort     of the M selected keys over the bits the positions need (hipCUB onesweep)
//   3. split          three order-preserving selects of the sorted rows by filter:
//                       tmp1      -f 8 -F 260   mapped primary, mate unmapped       (AF:186)
//                       tmp2      -f 4 -F 264   unmapped, mate mapped               (AF:187)
//                       anchored  -F 772        mapped primary                       (AF:194)
// The key/row arrays are 8 + 4 bytes per selected record; the pass reads 8 bytes per record.
#include <hipcub/hipcub.hpp>

#include "af_internal.h"

namespace {

constexpr uint64_t kNone = ~0ull;

__device__ __forceinline__ bool s3_keep(int32_t f) {
    return (f & 772) == 0 || ((f & 0x8) && !(f & 260)) || ((f & 0x4) && !(f & 264));
}

struct SelKey {
    const int32_t *flag, *pos;
    __device__ uint64_t operator()(int64_t r) const {
        const int32_t p = pos[r], f = flag[r];
        if (p < 0 || !s3_keep(f)) return kNone;
        return (uint64_t)(2u * (uint32_t)p + ((f & 0x10) ? 1u : 0u)) << 32 | (uint32_t)r;
    }
};
struct IsSome {
    __device__ bool operator()(uint64_t k) const { return k != kNone; }
};
struct KeyRow {
    __device__ int32_t operator()(uint64_t k) const { return (int32_t)(uint32_t)k; }
};
struct Filter {
    const int32_t *flag;
    int which;  // 0 tmp1, 1 tmp2, 2 anchored
    __device__ bool operator()(int32_t r) const {
        const int32_t f = flag[r];
        return which == 0 ? ((f & 0x8) && !(f & 260)) : which == 1 ? ((f & 0x4) && !(f & 264)) : (f & 772) == 0;
    }
};

using CountIt = hipcub::CountingInputIterator<int64_t>;
using KeyIt = hipcub::TransformInputIterator<uint64_t, SelKey, CountIt>;
using RowIt = hipcub::TransformInputIterator<int32_t, KeyRow, const uint64_t *>;

}  // namespace

size_t af_s3_temp_bytes(int64_t n_reads) {
    size_t a = 0, b = 0, c = 0;
    KeyIt in(CountIt(0), SelKey{nullptr, nullptr});
    (void)hipcub::DeviceSelect::If(nullptr, a, in, (uint64_t *)nullptr, (int64_t *)nullptr, n_reads, IsSome());
    (void)hipcub::DeviceRadixSort::SortKeys(nullptr, b, (const uint64_t *)nullptr, (uint64_t *)nullptr, n_reads, 0, 64);
    RowIt rows((const uint64_t *)nullptr, KeyRow());
    (void)hipcub::DeviceSelect::If(nullptr, c, rows, (int32_t *)nullptr, (int64_t *)nullptr, n_reads,
                                   Filter{nullptr, 0});
    return std::max(a, std::max(b, c));
}

hipError_t af_launch_s3(const int32_t *flag, const int32_t *pos, int64_t n_reads, int64_t ref_len, uint64_t *keys,
                        uint64_t *keys_alt, void *temp, size_t temp_bytes, int64_t *counts, int32_t *tmp1,
                        int32_t *tmp2, int32_t *anchored, hipStream_t s) {
    hipError_t e;
    KeyIt in(CountIt(0), SelKey{flag, pos});
    size_t tb = temp_bytes;
    if ((e = hipcub::DeviceSelect::If(temp, tb, in, keys, counts + 3, n_reads, IsSome(), s)) != hipSuccess) return e;
    int64_t m = 0;
    if ((e = hipMemcpyAsync(&m, counts + 3, sizeof(m), hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;  // M sizes the sort
    int end_bit = 32;
    while (end_bit < 64 && (1ull << (end_bit - 32)) < (uint64_t)(2 * ref_len + 2)) ++end_bit;
    const uint64_t *sorted = keys;
    if (m > 1) {
        tb = temp_bytes;
        if ((e = hipcub::DeviceRadixSort::SortKeys(temp, tb, keys, keys_alt, m, 0, end_bit, s)) != hipSuccess) return e;
        sorted = keys_alt;
    }
    RowIt rows(sorted, KeyRow());
    int32_t *outs[3] = {tmp1, tmp2, anchored};
    for (int w = 0; w < 3; ++w) {
        tb = temp_bytes;
        if ((e = hipcub::DeviceSelect::If(temp, tb, rows, outs[w], counts + w, m, Filter{flag, w}, s)) != hipSuccess)
            return e;
    }
    return hipSuccess;
}
