// af_internal.h -- shared definitions for the libafgpu HIP kernels and host code.
// gfx950 (CDNA4) only; wave64 is assumed everywhere.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <vector>
#include "../../include/afgpu.h"

#define AF_NEG_INF (-0x40000000)
#define AF_SEED_BTILE 2048      // reads per workgroup tile in the seed filter
#define AF_SEED_WAVES 16        // waves per seed-filter workgroup (1024 threads)
#define AF_SEED_GROUPS (AF_SEED_BTILE / 64)  // 64-read ballot groups per tile
#ifndef AF_G1_WPS
#define AF_G1_WPS 4             // genome G1 (k_g_seeds) waves per SIMD: one read per lane, refilled as lanes finish (126 VGPRs)
#endif
#ifndef AF_G2_FIRST_OCC
#define AF_G2_FIRST_OCC 128     // G2 takes the reads with at least this many seeds first (env AF_G2_FIRST_OCC; 0: read order)
#endif
#ifndef AF_G1W_WPS
#define AF_G1W_WPS 6            // G1's wave path (k_g_seeds_wave): waves per SIMD, one read per wave (80 VGPRs)
#endif
#ifndef AF_G1_HEAVY_EXT
#define AF_G1_HEAVY_EXT 2048    // G1: a read past this many FM extensions moves to the wave-per-read kernel (env AF_G1_HEAVY_EXT)
#endif
#ifndef AF_S2_SPEC_WINDOWS
#define AF_S2_SPEC_WINDOWS 4    // S2 K3c: pairs with this many rescue windows run their SWs as grid jobs (env AF_S2_SPEC_WINDOWS)
#endif
#ifndef AF_G_PE_SPEC_WINDOWS
#define AF_G_PE_SPEC_WINDOWS 4  // S4: pairs with this many rescue windows run their SWs as grid jobs (env AF_G_PE_SPEC_WINDOWS)
#endif
#ifndef AF_G_HEAVY_CHAINS
#define AF_G_HEAVY_CHAINS 16    // G2: reads with this many kept chains extend them one job per chain (env AF_G_HEAVY_CHAINS)
#endif
#ifndef AF_K2_WPS
#define AF_K2_WPS 6             // S2 K2 waves per SIMD (launch bound; persistent slots = 4 x this per CU)
#endif
#define AF_CPL 6                // DP columns per lane: 6*64 = 384 >= AF_MAX_READ+1

// Device view of an anchor index (all pointers are device memory).
struct DevIndex {
    const uint8_t *D;       // doubled reference codes (anchor ++ revcomp), N = 4, length 2n
    const uint32_t *D2;     // 2-bit packed D, 16 bases per word (base i at bits 2i), padded
    const uint32_t *Dn;     // N bitmap of D, 32 bases per word, padded
    // 16-mer position hash, one 16-byte slot per entry (one load per probe): {key, first index
    // into kpos, occurrences (0 = empty slot), kpos[first] (a unique 16-mer needs no kpos load)}
    const int4 *hslot;
    const int32_t *kpos;    // positions grouped by 16-mer, ascending
    const uint32_t *bloom;  // Bloom filter of the anchor 16-mers (2^bl_bits words, see af_k1_hash)
    int64_t n;              // anchor length
    int32_t hbits;          // log2 position-hash slots
    int32_t bl_bits;        // log2 Bloom words
};

// BLAT tile index (blat.hip): target codes, every step-th 11-mer's positions grouped by key
// (start[key] .. start[key + 1]) ascending; the target's N bases as one bit per base (nmask, 64
// bases per word) and N counts before each 64-base block (ncum): any N count in O(1)
struct DevTile {
    const uint8_t *T;
    const uint32_t *start, *pos, *ncum;
    const uint64_t *nmask;
    const uint32_t *nnext;  // per 64-base block: the first N at or after its start (0xFFFFFFFF: none)
    int64_t n;
    int32_t step;
};

__host__ __device__ static inline uint32_t af_fmix(uint32_t k) { return (k ^ (k >> 16)) * 0x45D9F3Bu; }
// reverse complement of a 2-bit packed 16-mer (base i at bits 2i; A0 C1 G2 T3, complement = 3 - c)
__host__ __device__ static inline uint32_t af_rc16(uint32_t k) {
    uint32_t x = ~k;
    x = ((x >> 2) & 0x33333333u) | ((x & 0x33333333u) << 2);  // swap 2-bit fields in nibbles
    x = ((x >> 4) & 0x0F0F0F0Fu) | ((x & 0x0F0F0F0Fu) << 4);  // nibbles in bytes
    x = ((x >> 8) & 0x00FF00FFu) | ((x & 0x00FF00FFu) << 8);  // bytes in halves
    return (x >> 16) | (x << 16);
}

// ---- K1 seed-filter keys and Bloom filter --------------------------------
// Base code of a read byte: a 2-bit table indexed by the byte's low 3 bits (A/a 1 -> 0,
// C/c 3 -> 1, G/g 7 -> 2, T/t 4 -> 3; N 6 and the unused slots -> 0).  On the device this is
// one v_and + one v_perm_b32 per four bytes.
#define AF_K1_CODE_TBL 0x8340u
__host__ __device__ static inline uint32_t af_k1_code(uint32_t ch) { return (AF_K1_CODE_TBL >> (2 * (ch & 7))) & 3u; }
// A sampled 16-mer's key is its codes in "word-transposed" order: base 4w+b of the 16-mer at
// bits 8b+2w, so four byte-wise code words of consecutive 4-base groups combine with three
// shift-ors.  The map from the 2-bit packing (base i at bits 2i) is a bijection.
__host__ __device__ static inline uint32_t af_k1_key(uint32_t packed) {
    uint32_t t = 0;
    for (int i = 0; i < 16; ++i) t |= ((packed >> (2 * i)) & 3u) << (8 * (i & 3) + 2 * (i >> 2));
    return t;
}
// One 32x32->64 multiply per key (h = key * AF_K1_MUL = hi:lo).  The filter is 2^bits 32-bit
// words (bits <= 15); a key sets four bits, one per byte, in each of two words:
//   word 1 = hi[bits+1:2],   bit (byte i) = lo byte i & 7;
//   word 2 = lo[31:32-bits], bit (byte i) = hi byte i & 7,
// so neither word's bits come from the half of h that indexes it.  On the device a mask is
// one v_and + one v_perm_b32 over the one-hot bytes 01 02 .. 80.
#define AF_K1_MUL 0x9E3779B1u
#ifndef AF_K1_MAX_BITS
#define AF_K1_MAX_BITS 15
#endif
__host__ __device__ static inline uint64_t af_k1_hash(uint32_t key) { return (uint64_t)key * AF_K1_MUL; }
__host__ __device__ static inline uint32_t af_k1_mask(uint32_t v) {
    uint32_t m = 0;
    for (int b = 0; b < 4; ++b) m |= 1u << (8 * b + ((v >> (8 * b)) & 7));
    return m;
}

// ---- S2: bwa mem paired-end (s2.hip; the contract is oracle/bwa_pe.c) ---------------------
// Per-read caps, identical to the oracle's AFO_PE_MAX_* (a read past one is reported unmapped
// with AF_FLAG_MEM_OVERFLOW on both sides).
#define AF_S2_MAX_PMEM 128
#define AF_S2_MAX_SEED 64
#define AF_S2_MAX_OCC 128
#define AF_S2_MAX_CHAIN 32
#define AF_S2_MAX_REG 32
#define AF_S2_MAX_TSPAN 1024  // longest reference span mem_patch_reg merges (the DP target window)

// The bwa text of the anchor (bns_fasta2bntseq: forward pac with N -> lrand48() & 3, then its
// reverse complement), its suffix ranks (bwt_sa order) and a position hash of ALL its 16-mers
// (including those across the strand boundary: SMEM counts see them, as bwa's BWT does).
struct DevText {
    const uint8_t *T;        // codes 0..3, length 2n
    const uint32_t *T2;      // 2-bit packed T, 16 bases per word, padded
    const int32_t *rank;     // suffix rank of T[i..]
    const int4 *hslot;       // {key, first index into kpos, count, kpos[first]}
    const int32_t *kpos;
    int64_t n;
    int32_t hbits;
    int32_t base_cnt[4];     // occurrences of each base in T
};

// one alignment region (mem_alnreg_t fields the paired-end stage reads)
struct S2Reg {
    int64_t rb, re;
    int32_t qb, qe, score, truesc, w, seedlen0;
};
// insert-size statistics of one chunk and orientation (mem_pestat_t)
struct S2Pes {
    int32_t low, high, failed, pad;
    double avg, std;
};
// Heavy pairs of S2 / S4 (at least min_windows mate-rescue windows, mem_matesw calls): their
// rescue SWs (ksw_align2 per window and direction) run as grid-wide jobs (k_s2_pe_jobs /
// k_g_pe_jobs) before a wave per pair finishes it with their results (k_s2_pairs / k_g_pe, mode 2)
constexpr int AF_G_PE_RES_W = 8;  // ints per (window, direction) result: sc te qe tb qb ran
struct GPeSpec {
    int32_t *pair;                    // [cap_pairs] the pair (S2: its pair-list item; -1: reservation failed)
    int32_t *off;                     // [cap_pairs] its first window slot
    int32_t *nj;                      // [cap_pairs] its windows per end: n0 | n1 << 16
    int2 *job;                        // [cap_jobs] window slot -> {heavy pair, i << 16 | j} (y -1: none)
    int32_t *res;                     // [cap_jobs * 4 * AF_G_PE_RES_W] results per slot and direction
    unsigned long long *cnt;          // [0] heavy pairs, [1] slots, [2] job / [3] finish dequeue, [4] slots written below
    int64_t cap_pairs = 0, cap_jobs = 0;
    int32_t min_windows = 0;          // 0: every pair rescued by its own wave
};
// bwa options of the paired-end path that af_params does not carry (af_pe)
struct S2Opt {
    int32_t pen_unpaired, max_ins, max_matesw, split_width, max_mem_intv, max_chain_gap;
    int64_t pair_base;
};
// per-context device scratch of the S2 kernels
struct S2Work {
    S2Reg *pool;        // region pool (K2 allocates with one atomic per read)
    int64_t pool_cap;
    int32_t *pool_n;    // pool fill (ctrl word of the current epoch)
    int2 *rmap;         // per read: {pool offset, n regions (-1 overflow)}; candidate reads only
    int32_t *plist;     // candidate pairs (K3a), consumed by K3c
    int32_t *n_plist;
    int32_t *ghist;     // [chunk][orientation][max_ins + 1] insert-size counts (zeroed by K3b after use)
    S2Pes *pes;         // [n_chunks][4]
    int64_t ppc;        // pairs per chunk when every read has length stride (0: ragged, use cstart)
    const int64_t *cstart;  // ragged: chunk start pairs, *n_chunks + 1 entries
    const int32_t *n_chunks;  // ragged: device word
    int32_t n_chunks_u; // uniform: the chunk count
    int32_t max_chunks;
    int32_t *heads_k2, *heads_k3;  // per-XCD dequeue heads (8 lines each)
    void *plan;         // per listed pair: the record choice of K3c for K3d (s2.hip S2Plan)
    GPeSpec sp{};       // K3c's heavy pairs (rescue SWs as jobs)
};

// split-read tails output (af_split_tails_device / af_align_candidates_tails_device)
struct AfTails {
    uint8_t *tails;       // cap rows of `stride` bytes
    int32_t *tail_lens, *tail_read, *n_tails;
    int64_t cap, read_base;
    int32_t min_clip;
};

// One read's tail (tails.hip): mapped read with n_cigar == 2 (checked by the caller), CIGAR
// exactly S+M or M+S with clip >= min_clip -> SEQ's clipped part (SAM orientation) appended.
__device__ __forceinline__ void af_emit_tail(const AfTails &t, const uint8_t *reads, int32_t stride,
                                             const int32_t *lens, int64_t r, int f, const uint32_t *cig) {
    const uint32_t c0 = cig[0], c1 = cig[1];
    const int op0 = c0 & 0xf, op1 = c1 & 0xf;  // 0 = M, 4 = S
    int clip, head;
    if (op0 == 4 && op1 == 0) { clip = (int)(c0 >> 4); head = 1; }
    else if (op0 == 0 && op1 == 4) { clip = (int)(c1 >> 4); head = 0; }
    else return;
    const int len = lens ? lens[r] : stride;
    if (clip < t.min_clip || clip > len) return;
    const int slot = atomicAdd(t.n_tails, 1);
    if (slot >= t.cap) return;
    const uint8_t *q = reads + r * (int64_t)stride;
    uint8_t *o = t.tails + (int64_t)slot * stride;
    const bool rev = (f & 0x10) != 0;
    // SEQ[i] = rev ? comp(read[len - 1 - i]) : read[i]; the tail is SEQ[0, clip) or SEQ[len - clip, len)
    const int s0 = head ? 0 : len - clip;
    for (int i = 0; i < clip; ++i) {
        const int k = s0 + i;
        uint8_t c = q[rev ? len - 1 - k : k];
        if (rev) {
            const uint8_t lc = c | 0x20;
            c = lc == 'a' ? 'T' : lc == 'c' ? 'G' : lc == 'g' ? 'C' : lc == 't' ? 'A' : 'N';
        }
        o[i] = c;
    }
    t.tail_lens[slot] = clip;
    t.tail_read[slot] = (int32_t)(t.read_base + r);
}

// ---- the genome index of S4 / S5 (fmindex.hip; `bwa index <genome.fa>`) -----------------
// The bwa text T of l_pac contig bases (N = 2 l_pac), its suffix array (rows 0..N, '$' smallest)
// and the FM occurrence table: per 128 rows, counts of A/C/G/T before the block then the rows'
// BWT characters at 2 bits (row k of the block at bits 2 (k & 31) of word k >> 5); the '$' row
// (`primary`) is stored as A and corrected on lookup.
constexpr int AF_CTG_BKT_SHIFT = 16;
struct DevGenome {
    const uint8_t *T = nullptr;    // codes 0..3
    int64_t *sa = nullptr;
    uint64_t *occ = nullptr;
    int64_t *ctg_off_d = nullptr, *ctg_len_d = nullptr;  // contigs in pac (bns anns)
    // contig of each 2^AF_CTG_BKT_SHIFT-base bucket of pac: the rid at its start, bit 31 set when a
    // contig boundary falls inside (bns_pos2rid then steps from that rid)
    int32_t *ctg_bkt = nullptr;
    int64_t l_pac = 0, N = 0, primary = -1, n_blk = 0;
    int64_t C[4] = {0, 0, 0, 0};   // first row of the suffixes starting with c
    int64_t base_cnt[4] = {0, 0, 0, 0};
    int32_t n_ctg = 0;
};
hipError_t af_fm_build(const uint8_t *d_blob, const int64_t *src_off, const int64_t *src_len, int n_ctg, DevGenome *G,
                       hipStream_t s);
void af_fm_free(DevGenome *G);

// ---- S4 / S5 on the genome (bwa_genome.hip) -------------------------------------------------
using GOpt = S2Opt;
struct GIv { int64_t sa_k, s; int32_t qb, qe; };     // a seed interval: SA rows [sa_k, sa_k + s), query [qb, qe)
struct GReg {                                        // mem_alnreg_t
    int64_t rb, re;
    int32_t qb, qe, rid, score, truesc, w, seedcov, seedlen0, secondary, sub;
    uint64_t hash;
};
// G2's heavy reads (at least min_chains kept chains): the extensions of their chains run as
// one job per chain (k_g_ext_jobs) before a wave per read finishes it (k_g_heavy)
struct GHeavy {
    int64_t *read;                    // [cap_reads] the read (-1: reservation failed)
    int32_t *nch, *ch_off, *sd_off;   // [cap_reads] its kept chains and seeds in the pools
    int32_t *ch_read;                 // [cap_ch] each pooled chain's heavy read (-1: unused)
    void *ch, *sd, *res;              // GChain [cap_ch], GSeed [cap_sd], GReg [cap_sd] (each seed's region)
    unsigned long long *cnt;          // [0] heavy reads, [1] chains, [2] seeds, [3] job / [4] finish dequeue
    int64_t cap_reads, cap_ch, cap_sd;
    int32_t min_chains;               // 0: every read extended by its own wave
};
// per-call pools and counters of the genome kernels (per context)
struct GWork {
    GIv *iv;                    // intervals of every read (G1)
    int64_t iv_cap;
    unsigned long long *iv_fill;
    int64_t *iv_off;
    int32_t *iv_n;              // per read; -1 overflow
    GReg *reg;                  // regions of every read (G2)
    int64_t reg_cap;
    int32_t *reg_fill;
    int32_t *reg_off, *reg_n;   // per read; reg_n -1 overflow
    int32_t *heads;             // G2 dequeue heads (8 lines)
    int32_t *stats;             // AF_GSTAT_*
    unsigned long long *g1_next;  // G1: the next read to hand to an idle lane
    // G1's heavy reads: a lane whose read needs more than g1_max_ext FM extensions hands it to
    // k_g_seeds_wave (one wave per read) through g1_hv[0, *g1_hv_n); 0 = never
    int64_t *g1_hv = nullptr;
    unsigned long long *g1_hv_n = nullptr, *g1_hv_next = nullptr;
    int32_t g1_max_ext = 0;
    GHeavy hv;
    GPeSpec pe{};
    // G2's dequeue order: G1 lists the reads with at least g2_first_occ seeds (bwa's occurrences
    // per interval, at most max_occ, summed) in g2_list[0, *g2_list_n) and flags them; G2 takes
    // that list first, then the other reads in order (0 = read order)
    int32_t *g2_list = nullptr;
    uint8_t *g2_flag = nullptr;
    unsigned long long *g2_list_n = nullptr, *g2_list_next = nullptr;
    int32_t g2_first_occ = 0;
};
size_t af_g1_slot_bytes();
size_t af_g2_slot_bytes();
size_t af_g_chain_bytes();
size_t af_g_seed_bytes();
hipError_t af_launch_genome_regions(const DevGenome &G, const uint8_t *reads, int32_t stride, const int32_t *lens,
                                    const int32_t *d_n, int64_t cap, const af_params &p, const GOpt &o, const GWork &w,
                                    uint8_t *g1_scratch, int n_g1_threads, uint8_t *g2_scratch, int n_g2_waves,
                                    uint8_t *zscratch, hipStream_t s);
hipError_t af_launch_genome_intervals(const DevGenome &G, const uint8_t *reads, int32_t stride, const int32_t *lens,
                                      int64_t cap, const af_params &p, const GOpt &o, const GWork &w,
                                      uint8_t *g1_scratch, int n_g1_threads, hipStream_t s);
hipError_t af_launch_genome_se(const DevGenome &G, const uint8_t *reads, int32_t stride, const int32_t *lens,
                               const int32_t *d_n, int64_t cap, const af_params &p, int64_t id_base, const int64_t *ids,
                               const GWork &w, uint8_t *g2_scratch, int n_waves, uint8_t *zscratch, af_grec *recs,
                               int32_t *n_rec, hipStream_t s);
hipError_t af_launch_genome_pe(const DevGenome &G, const uint8_t *reads, int32_t stride, const int32_t *lens,
                               const int32_t *d_npairs, int64_t cap_pairs, const af_params &p, const GOpt &o,
                               const GWork &w, const S2Work &sw, uint8_t *g2_scratch, int n_waves, uint8_t *zscratch,
                               af_grec *recs, int32_t *n_rec, hipStream_t s);
hipError_t af_launch_s2_pestat(const S2Work &w, int32_t max_ins, hipStream_t s);

// launch helpers (defined in the .hip files)
// ctrl (AF_CTRL_BYTES, one 128-B line per word, no memsets on the hot path):
//  [AF_HEAD_STRIDE * e], e = 0, 1: candidate count of K1 epoch e (K1 of epoch e zeroes the
//                                  other epoch's count for the next call);
//  [AF_HEAD_STRIDE * (10 + x)], x = 0..7: dequeue heads of K2 (k_pairs zeroes them after K2);
//  (word 18 is unused).
#define AF_HEAD_STRIDE 32
#define AF_CTRL_BYTES (4 * AF_HEAD_STRIDE * 41)
#define AF_CTRL_HEADS2 (10 * AF_HEAD_STRIDE)
//  [AF_HEAD_STRIDE * (19 + x)]: dequeue heads of af_place; [AF_HEAD_STRIDE * 27]: its query count.
//  [AF_HEAD_STRIDE * (29 + x)]: dequeue heads of the S2 pair kernel (K3c);
//  [AF_HEAD_STRIDE * (37 + e)], e = 0, 1: S2 region-pool fill of epoch e;
//  [AF_HEAD_STRIDE * (39 + e)]: S2 candidate-pair count of epoch e (K1 of epoch e zeroes both
//  words of its epoch).
#define AF_CTRL_PLACE_HEADS (19 * AF_HEAD_STRIDE)
//  [AF_HEAD_STRIDE * (2 + x)], x = 0..7: dequeue heads of the genome region kernel (bwa_genome.hip)
#define AF_CTRL_G_HEADS (2 * AF_HEAD_STRIDE)
#define AF_CTRL_PLACE_N (27 * AF_HEAD_STRIDE)
#define AF_CTRL_S2_HEADS3 (29 * AF_HEAD_STRIDE)
#define AF_CTRL_S2_POOL (37 * AF_HEAD_STRIDE)
#define AF_CTRL_S2_NPAIRS (39 * AF_HEAD_STRIDE)
size_t af_seed_filter_lds(int bl_bits);
hipError_t af_launch_seed_filter(const DevIndex &ix, const uint8_t *reads, int64_t n_reads, int32_t stride,
                                 const int32_t *lens, int32_t *hits, int32_t *cand, int32_t *cnt, int32_t *cnt_next,
                                 int32_t *s2z, int n_cu, hipStream_t s);
hipError_t af_launch_s2(const DevText &X, const uint8_t *reads, int64_t n_pairs, int32_t stride, const int32_t *lens,
                        const af_params &p, const S2Opt &o, const int32_t *hits, const int32_t *cand,
                        const int32_t *n_cand, const S2Work &w, af_aln_out out, uint8_t *zscratch, int32_t n_slots,
                        int32_t n_cu, const AfTails *tails, hipStream_t s);
size_t af_s2_plan_bytes();
hipError_t af_launch_s2_chunks(int64_t n_pairs, int32_t stride, const int32_t *lens, int64_t chunk_bases,
                               int64_t *cstart, int64_t *scan_tmp, int32_t max_chunks, int32_t *n_chunks_dev,
                               hipStream_t s);
hipError_t af_launch_split_tails(const uint8_t *reads, int64_t n_reads, int32_t stride, const int32_t *lens,
                                 const af_aln_out &out, const AfTails &t, bool append, hipStream_t s);
size_t af_gather_temp_bytes(int64_t n_rows);
// s5s6.hip: the genome check of the split reads (fn:718-768) and the S6 query rows (fn:512-528)
size_t af_s5_temp_bytes(int64_t n);
hipError_t af_launch_s5_filter(const af_grec *recs, const int32_t *n_rec, int64_t n, const uint8_t *q, int32_t q_stride,
                               const int32_t *q_lens, const int32_t *q_rows, const af_aln_out &s2, const uint8_t *cont,
                               int64_t cap,
                               uint8_t *out, int32_t out_stride, int32_t *out_lens, int32_t *out_src, int32_t *n_out,
                               int32_t *n_over, uint8_t *keep, int32_t *sel, int64_t *n_sel, void *temp,
                               size_t temp_bytes, hipStream_t s);
hipError_t af_launch_gather(const uint8_t *reads, int32_t stride, const int32_t *lens, const int32_t *rows,
                            int64_t n_rows, int32_t mode, const af_aln_out &out, int64_t first, int64_t step,
                            int64_t cap, uint8_t *q, int32_t *q_lens, int32_t *q_rows, int32_t *n_q, int32_t *sel,
                            int64_t *sel_n, void *temp, size_t temp_bytes, hipStream_t s);
// k_blat's per-wave global scratch (blat.hip layout) and its resident waves on n_cu CUs
constexpr size_t AF_BLAT_SLOT_BYTES = 872 << 10;  // blat.hip SC_END
int af_blat_slots(int n_cu);
// the rows past max_rows (af_blat_spill): appended at rows[atomicAdd(n, 1)] with their query
struct BlatSpill {
    af_psl *rows = nullptr;
    int32_t *query = nullptr, *n = nullptr;
    int64_t cap = 0;
};
// where a search's cap events (AF_BLAT_CAP_*) are counted: per query in q[k * qcap + query] when
// registered (af_blat_query_caps; queries past qcap and no registration: the context's counters)
struct BlatCaps {
    int32_t *ctx = nullptr;
    int32_t *q = nullptr;
    int64_t qcap = 0;
    __device__ void hit(int64_t query, int k) const {
        if (q && query >= 0 && query < qcap) atomicAdd(&q[k * qcap + query], 1);
        else if (ctx) atomicAdd(&ctx[k], 1);
    }
};
// A heavy strand (more than min_clumps clumps) is deferred by k_blat: its entry {2 query + strand, 0,
// clumps, 0} goes to the strand table and k_blat_heavy searches it, for the live queries only, once
// the caller's live flags exist (S6: after S5's check).  ctrl: AF_BLAT_HV_CTRL_WORDS words, one 128-B
// line apart: the table's fill, the deferred strands' clumps, k_blat_heavy's dequeue heads and
// counters.
#define AF_BLAT_HV_JOBS_N 0                            // clumps of the deferred strands
#define AF_BLAT_HV_STRANDS_N (2 * AF_HEAD_STRIDE)
#define AF_BLAT_HV_STRAND_HEADS (11 * AF_HEAD_STRIDE)
#define AF_BLAT_HV_JOBS_DONE (19 * AF_HEAD_STRIDE)     // clumps of the strands k_blat_heavy searched
#define AF_BLAT_HV_STRANDS_DONE (20 * AF_HEAD_STRIDE)  // deferred strands searched (k_blat_heavy)
#define AF_BLAT_HV_CTRL_WORDS (21 * AF_HEAD_STRIDE)
#ifndef AF_BLAT_HEAVY_CLUMPS
#define AF_BLAT_HEAVY_CLUMPS 512  // default: strands with more clumps are deferred (env AF_BLAT_HEAVY_CLUMPS)
#endif
struct BlatHeavy {
    int32_t min_clumps = 0;   // 0: no strand is deferred
    int4 *strands = nullptr;  // {item, 0, clumps, 0}
    int64_t strands_cap = 0;
    int32_t *ctrl = nullptr, *jobs_n = nullptr, *strands_n = nullptr;
};
// one BLAT search's launch arguments
struct BlatLaunch {
    DevTile X;
    const uint8_t *queries = nullptr;
    const int32_t *n_queries = nullptr, *q_first = nullptr;
    int64_t cap = 0;
    int32_t stride = 0;
    const int32_t *lens = nullptr;
    af_blat_params p{};
    int32_t *heads = nullptr;
    uint8_t *bscratch = nullptr;
    int32_t n_slots = 0;
    af_psl *rows = nullptr;
    int32_t *n_rows = nullptr;
    int32_t max_rows = 0;
    const int32_t *order = nullptr;
    af_psl *stage = nullptr;
    int32_t *stage_n = nullptr;
    BlatCaps caps;
    BlatSpill spill;
    BlatHeavy hv;
};
// af_launch_blat = _begin (k_blat: every strand with at most hv.min_clumps clumps searched) + _end
// (the deferred strands' jobs and chains, then the rows of every query: live[q] == 0 -> no rows)
hipError_t af_launch_blat_begin(const BlatLaunch &B, hipStream_t s);
hipError_t af_launch_blat_end(const BlatLaunch &B, const uint8_t *live, hipStream_t s);
hipError_t af_launch_blat(const BlatLaunch &B, hipStream_t s);
// blat_long.hip: one long query (codes of both strands at d_q2, strand s at d_q2 + s L) -> every
// row (unsorted), its strand's emission order, its first block in `blocks`; cap events to caps;
// *overflow = 1 (and no rows) when the device row list or block arena overflowed
hipError_t af_blat_long_run(const DevTile &X, const uint8_t *d_q2, int L, const af_blat_params &bp, int32_t *caps,
                            std::vector<af_psl> &rows, std::vector<int32_t> &seq, std::vector<int64_t> &boff,
                            std::vector<af_psl_block> &blocks, int n_cu, hipStream_t s, int *overflow);
// s5s6.hip: S6 rows of the QNAME-group leaders before the check, and their compaction after it
hipError_t af_launch_s6_queries(int64_t n, const uint8_t *q, int32_t q_stride, const int32_t *q_lens,
                                const int32_t *q_rows, const af_aln_out &s2, const uint8_t *cont, const af_s6_set &pre,
                                uint8_t *keep, int32_t *sel, int64_t *n_sel, void *temp, size_t temp_bytes,
                                hipStream_t s);
size_t af_s6_compact_temp_bytes(int64_t n);
hipError_t af_launch_s6_check(const af_grec *recs, const int32_t *n_rec, int64_t n, const int32_t *q_rows,
                              const af_aln_out &s2, const uint8_t *cont, const af_s6_set &pre, uint8_t *keep,
                              uint8_t *live, hipStream_t s);
hipError_t af_launch_s6_compact(const af_s6_set &pre, const uint8_t *live, const af_s6_set &out, int32_t max_rows,
                                int32_t *caps, int32_t *flag, int32_t *idx, int32_t *sflag, int32_t *sidx, void *temp,
                                size_t temp_bytes, hipStream_t s);
// k_blat's schedule: the queries by estimated cost, heaviest first (work: af_blat_order_bytes(cap))
size_t af_blat_order_bytes(int64_t cap);
hipError_t af_launch_blat_order(const DevTile &X, const uint8_t *queries, const int32_t *n_queries, int64_t cap,
                                int32_t stride, const int32_t *lens, int32_t rep_match, void *work,
                                int32_t *order, hipStream_t s);
hipError_t af_build_tile_index(const uint8_t *d_seq, int64_t n, int32_t step, DevTile *X, void **allocs, int *na,
                               hipStream_t s);
hipError_t af_launch_clamp_count(const int32_t *count, int64_t cap, int32_t *dst, hipStream_t s);
// s3.hip: S3 (samtools sort + flag filters) on the device
size_t af_s3_temp_bytes(int64_t n_reads);
hipError_t af_launch_s3(const int32_t *flag, const int32_t *pos, int64_t n_reads, int64_t ref_len, uint64_t *keys,
                        uint64_t *keys_alt, void *temp, size_t temp_bytes, int64_t *counts, int32_t *tmp1,
                        int32_t *tmp2, int32_t *anchored, hipStream_t s);

