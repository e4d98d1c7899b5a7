// sim.hip -- libafsim.so: seeded synthetic inputs for BASELINE.json configs[2]-[4], made on the
// device (bench and test infrastructure; the product library libafgpu.so never loads it).
//
// The reference benchmarks on reads simulated with `wgsim -d 200 -1 L -2 L` from fusion
// transcripts (utils/simulate_reads.py:4-20) and aligns against hg38.  Neither hg38 nor wgsim is
// available offline, so this restates both generators:
//
//   k_sim_genome  an hg38-scale genome (contigs joined by N runs), every base a pure function of
//                 (seed, contig, position), so it is deterministic at any launch shape:
//                   - telomere N runs and one centromere N gap per contig, flanked by tandem arrays
//                     of a 171-bp satellite monomer (hundreds of thousands of copies genome-wide:
//                     the highest 16-mer multiplicities, as alpha satellite gives in hg38);
//                   - interspersed repeat families (Alu-, L1-, MIR-, L2-, LTR-, DNA-transposon-like,
//                     several subfamilies each, per-copy divergence, strand, truncation and one
//                     small indel) placed in 1024-base slots, plus simple tandem repeats;
//                   - segmental duplications: 16 kb blocks copied from elsewhere at 1-4 %;
//                   - background at 41 % GC.
//                 The consensus library is host-generated (numpy, seeded) and passed in.
//   k_sim_pairs   wgsim's read model, one thread per pair: fragment ~ N(frag_mean, frag_sd) from a
//                 fusion transcript (probability fusion_frac, transcripts weighted by length) or
//                 from the genome (uniform; re-drawn when it crosses an N), mate 1 = the first L
//                 bases, mate 2 = the reverse complement of the last L, the pair flipped with
//                 probability 1/2; substitutions at `err`, a 1-3 nt indel on `indel_frac` of the
//                 reads, N at `n_rate`.  Every pair is distinct (counter-based randomness).
#include <hip/hip_runtime.h>
#include <stdint.h>

#define SIM_MAX_CTG 64
#define SIM_MAX_FAM 16

struct SimFamily {
    int32_t cons_off;   // first consensus base (codes 0-3) in the library
    int32_t cons_len;   // bases per subfamily consensus
    int32_t n_sub;      // subfamilies (consecutive in the library)
    int32_t min_len, max_len;  // copy length range (truncated copies)
    int32_t kind;       // 0 interspersed, 1 simple tandem repeat (unit 1-6 from the slot hash)
    float div_lo, div_hi;      // per-copy divergence range (subfamily k adds k * div_step)
    float div_step;
    float prob;         // probability that a slot holds a copy of this family
};

struct SimGenomeSpec {
    int32_t n_ctg, n_fam;
    int64_t off[SIM_MAX_CTG], len[SIM_MAX_CTG];  // contig offsets in the joined sequence, lengths
    SimFamily fam[SIM_MAX_FAM];
    int32_t sat_off, sat_len;   // satellite monomer in the library
    int32_t telomere;           // N bases at each contig end
    int32_t cen_gap, sat_flank; // centromere N gap and the satellite array on each side of it
    float cen_at;               // centromere position as a fraction of the contig
    float segdup_prob;          // per 16 kb block
    float gc;
    uint64_t seed;
};

namespace {

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t h2(uint64_t seed, uint64_t a, uint64_t b) {
    return mix64(seed ^ mix64(a * 0x9e3779b97f4a7c15ull + b + 0x632be59bd9b4e019ull));
}
__device__ __forceinline__ float u01(uint64_t h) { return (float)(uint32_t)(h >> 40) * (1.0f / 16777216.0f); }

__device__ __forceinline__ int bg_base(uint64_t h, float gc) {
    const float u = u01(h), at = (1.0f - gc) * 0.5f;
    return u < at ? 0 : u < at + gc * 0.5f ? 1 : u < at + gc ? 2 : 3;
}
__device__ __forceinline__ int mutate(int b, uint64_t h, float d) {
    return u01(h) < d ? ((b + 1 + (int)((h >> 8) % 3)) & 3) : b;
}

// base of the genome before segmental duplication: code 0-3, or 4 for N
__device__ int pass1(const SimGenomeSpec &S, const uint8_t *lib, int c, int64_t lp) {
    const int64_t Lc = S.len[c];
    if (lp < S.telomere || lp >= Lc - S.telomere) return 4;
    const int64_t cen = (int64_t)(S.cen_at * (float)Lc);
    if (lp >= cen && lp < cen + S.cen_gap) return 4;
    const uint64_t pkey = ((uint64_t)c << 40) | (uint64_t)lp;
    if ((lp >= cen - S.sat_flank && lp < cen) || (lp >= cen + S.cen_gap && lp < cen + S.cen_gap + S.sat_flank)) {
        const int64_t o = lp - (lp < cen ? cen - S.sat_flank : cen + S.cen_gap);
        const int64_t mono = o / S.sat_len;
        // monomers diverge 2-10 % from the consensus; each array is one higher-order unit repeated
        const float d = 0.02f + 0.08f * u01(h2(S.seed ^ 0x5a7, (uint64_t)c, (uint64_t)(mono % 12)));
        const int b = lib[S.sat_off + (int)(o % S.sat_len)];
        return mutate(b, h2(S.seed ^ 0x5a8, (uint64_t)c * 64 + (uint64_t)(mono % 12), (uint64_t)(o % S.sat_len)), d);
    }
    const int64_t slot = lp >> 10;
    const int so = (int)(lp & 1023);
    const uint64_t hs = h2(S.seed, ((uint64_t)c << 32) | (uint64_t)slot, 1);
    float u = u01(hs);
    for (int f = 0; f < S.n_fam; ++f) {
        const SimFamily &F = S.fam[f];
        if (u >= F.prob) { u -= F.prob; continue; }
        const uint64_t a = mix64(hs + 1), b = mix64(hs + 2);
        const int len = F.min_len + (int)(a % (uint64_t)(F.max_len - F.min_len + 1));
        const int off = (int)((a >> 20) % (uint64_t)(1024 - len + 1));
        if (so < off || so >= off + len) break;
        const int j = so - off;
        if (F.kind == 1) {  // simple repeat: a 1-6 base unit, 3 % divergence
            const int unit = 1 + (int)(b % 6);
            const int base = (int)((b >> (8 + 2 * (j % unit))) & 3);
            return mutate(base, h2(S.seed ^ 0x51, pkey, 0), 0.03f);
        }
        const int sub = (int)((b >> 4) % (uint64_t)F.n_sub);
        const bool rev = (b >> 12) & 1;
        const int cs = (int)((b >> 16) % (uint64_t)(F.cons_len - len + 1));  // truncation start
        const int ip = 1 + (int)((b >> 32) % (uint64_t)len);
        const int sh = (int)((b >> 48) % 7) - 3;  // -3..3: one small indel inside the copy
        const int jj = rev ? len - 1 - j : j;
        int ci = cs + jj + (jj >= ip ? sh : 0);
        ci = ci < 0 ? 0 : ci >= F.cons_len ? F.cons_len - 1 : ci;
        int base = lib[F.cons_off + sub * F.cons_len + ci];
        if (rev) base = 3 - base;
        const float d = F.div_lo + (F.div_hi - F.div_lo) * u01(mix64(hs + 3)) + F.div_step * (float)sub;
        return mutate(base, h2(S.seed ^ 0x52, pkey, 0), d);
    }
    return bg_base(h2(S.seed ^ 0xb9, pkey, 0), S.gc);
}

__device__ int genome_base(const SimGenomeSpec &S, const uint8_t *lib, int c, int64_t lp) {
    const int64_t blk = lp >> 14;
    const uint64_t hb = h2(S.seed ^ 0xd0, ((uint64_t)c << 32) | (uint64_t)blk, 7);
    if (u01(hb) < S.segdup_prob && lp >= S.telomere && lp < S.len[c] - S.telomere) {
        // a copy of another 16 kb block (any contig), 1-4 % diverged
        const int sc = (int)(mix64(hb + 1) % (uint64_t)S.n_ctg);
        const int64_t nb = S.len[sc] >> 14;
        if (nb > 2) {
            const int64_t sb = 1 + (int64_t)(mix64(hb + 2) % (uint64_t)(nb - 2));
            const int b = pass1(S, lib, sc, (sb << 14) | (lp & 16383));
            if (b == 4) return 4;
            const float d = 0.01f + 0.03f * u01(mix64(hb + 3));
            return mutate(b, h2(S.seed ^ 0xd1, ((uint64_t)c << 40) | (uint64_t)lp, 0), d);
        }
    }
    return pass1(S, lib, c, lp);
}

// 16 bases per thread, one 16-byte store
__global__ void k_sim_genome(uint8_t *__restrict__ out, int64_t n, SimGenomeSpec S, const uint8_t *__restrict__ lib) {
    const int64_t g = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 16;
    if (g >= n) return;
    int c = 0;
    while (c + 1 < S.n_ctg && S.off[c + 1] <= g) ++c;
    uint8_t v[16];
    for (int k = 0; k < 16; ++k) {
        const int64_t p = g + k;
        if (c + 1 < S.n_ctg && p >= S.off[c + 1]) ++c;
        int b = 4;
        if (p < n && p >= S.off[c] && p < S.off[c] + S.len[c]) b = genome_base(S, lib, c, p - S.off[c]);
        v[k] = (uint8_t)"ACGTN"[b];
    }
    if (g + 16 <= n) {
        *reinterpret_cast<uint4 *>(out + g) = *reinterpret_cast<const uint4 *>(v);
    } else {
        for (int k = 0; g + k < n; ++k) out[g + k] = v[k];
    }
}

struct SimReads {
    const uint8_t *genome;  // joined ASCII sequence
    int64_t n_genome;
    int32_t n_ctg;
    int64_t off[SIM_MAX_CTG], len[SIM_MAX_CTG];
    int64_t cum[SIM_MAX_CTG + 1];  // cumulative sampleable contig lengths
    const uint8_t *tx;       // fusion transcripts, joined ASCII
    const int64_t *tx_off;   // n_tx + 1 offsets
    const double *tx_cum;    // n_tx cumulative weights (length-proportional), last = 1
    int32_t n_tx;
    int32_t L;
    float fusion_frac, frag_mean, frag_sd, err, indel_frac, n_rate;
    uint64_t seed;
    int64_t pair_base;       // global index of the first pair (seeds the pair's randomness)
};

__device__ __forceinline__ uint8_t comp(uint8_t b) {
    return b == 'A' ? 'T' : b == 'C' ? 'G' : b == 'G' ? 'C' : b == 'T' ? 'A' : 'N';
}

// one mate: bases src[0..L) (rev: reverse complement of src[-(L-1)..0]) with errors
__device__ void write_mate(uint8_t *dst, const uint8_t *src, int64_t avail, bool rev, int L, const SimReads &R,
                           uint64_t h) {
    const bool indel = u01(mix64(h + 11)) < R.indel_frac;
    const int ipos = 10 + (int)(mix64(h + 12) % (uint64_t)(L - 20 > 0 ? L - 20 : 1));
    const int ik = 1 + (int)(mix64(h + 13) % 3);
    const bool ins = (mix64(h + 14) & 1) != 0;
    int s = 0;  // source index
    for (int k = 0; k < L; ++k) {
        uint8_t b;
        const uint64_t hk = h2(R.seed ^ 0x77, h, (uint64_t)k);
        if (indel && ins && k >= ipos && k < ipos + ik) {
            b = (uint8_t)"ACGT"[hk & 3];  // inserted base
        } else {
            if (indel && !ins && k == ipos) s += ik;  // deleted bases
            if (s < avail) {
                b = rev ? comp(src[-(int64_t)s]) : src[s];
            } else {
                b = (uint8_t)"ACGT"[hk & 3];
            }
            ++s;
        }
        if (b != 'N' && u01(mix64(hk + 9)) < R.err) {
            const int code = b == 'A' ? 0 : b == 'C' ? 1 : b == 'G' ? 2 : 3;
            b = (uint8_t)"ACGT"[(code + 1 + (int)((hk >> 32) % 3)) & 3];
        }
        if (u01(mix64(hk + 5)) < R.n_rate) b = 'N';
        dst[k] = b;
    }
}

__device__ float normal01(uint64_t h) {
    const float u1 = fmaxf(u01(h), 1e-7f), u2 = u01(mix64(h + 1));
    return sqrtf(-2.0f * logf(u1)) * cospif(2.0f * u2);
}

__global__ void k_sim_pairs(uint8_t *__restrict__ reads, int64_t n_pairs, SimReads R, int32_t *__restrict__ src) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_pairs) return;
    const int L = R.L;
    const uint64_t h = h2(R.seed, (uint64_t)(R.pair_base + i), 0x1234);
    int64_t frag = (int64_t)rintf(R.frag_mean + R.frag_sd * normal01(mix64(h + 1)));
    const uint8_t *base = nullptr;
    int32_t where = -1;
    if (R.n_tx > 0 && u01(mix64(h + 2)) < R.fusion_frac) {
        const double u = (double)(mix64(h + 3) >> 11) * (1.0 / 9007199254740992.0);
        int t = 0;
        while (t + 1 < R.n_tx && R.tx_cum[t] <= u) ++t;
        const int64_t tl = R.tx_off[t + 1] - R.tx_off[t];
        frag = frag < L ? L : frag > tl ? tl : frag;
        const int64_t st = (int64_t)(mix64(h + 4) % (uint64_t)(tl - frag + 1));
        base = R.tx + R.tx_off[t] + st;
        where = t;
    } else {
        frag = frag < L ? L : frag;
        for (int tr = 0; tr < 16 && !base; ++tr) {
            const int64_t u = (int64_t)(mix64(h + 20 + tr) % (uint64_t)R.cum[R.n_ctg]);
            int c = 0;
            while (c + 1 < R.n_ctg && R.cum[c + 1] <= u) ++c;
            const int64_t lp = u - R.cum[c];
            if (lp + frag > R.len[c]) continue;
            const uint8_t *p = R.genome + R.off[c] + lp;
            bool has_n = false;
            for (int64_t k = 0; k < frag && !has_n; k += 8) has_n = p[k] == 'N';
            if (has_n || p[frag - 1] == 'N') continue;
            base = p;
            where = R.n_tx + c;
        }
        if (!base) {  // give up: an all-N pair (never seeds)
            for (int k = 0; k < L; ++k) { reads[2 * i * L + k] = 'N'; reads[(2 * i + 1) * L + k] = 'N'; }
            if (src) src[i] = -1;
            return;
        }
    }
    const bool flip = (mix64(h + 5) & 1) != 0;
    uint8_t *m1 = reads + (2 * i + (flip ? 1 : 0)) * (int64_t)L;
    uint8_t *m2 = reads + (2 * i + (flip ? 0 : 1)) * (int64_t)L;
    write_mate(m1, base, frag, false, L, R, mix64(h + 6));
    write_mate(m2, base + frag - 1, frag, true, L, R, mix64(h + 7));
    if (src) src[i] = where;
}

}  // namespace

extern "C" {

// The joined genome (n bytes, ASCII) into d_out; spec->off/len describe the contigs (bytes between
// them are N).  lib: device consensus library (codes 0-3).  Returns a hipError_t.
int afs_genome(uint8_t *d_out, int64_t n, const SimGenomeSpec *spec, const uint8_t *d_lib, void *stream) {
    if (!d_out || !spec || n <= 0 || spec->n_ctg < 1 || spec->n_ctg > SIM_MAX_CTG || spec->n_fam > SIM_MAX_FAM)
        return (int)hipErrorInvalidValue;
    const int64_t threads = (n + 15) / 16;
    const int bs = 256;
    hipLaunchKernelGGL(k_sim_genome, dim3((unsigned)((threads + bs - 1) / bs)), dim3(bs), 0,
                       static_cast<hipStream_t>(stream), d_out, n, *spec, d_lib);
    return (int)hipGetLastError();
}

// n_pairs pairs, pair-major rows of L bytes (row 2i = mate 1); d_src[i] (optional) = the source:
// fusion transcript t (< n_tx), n_tx + contig, or -1.
int afs_pairs(uint8_t *d_reads, int64_t n_pairs, const SimReads *spec, int32_t *d_src, void *stream) {
    if (!d_reads || !spec || n_pairs < 0 || spec->L < 24 || spec->n_ctg < 1 || spec->n_ctg > SIM_MAX_CTG)
        return (int)hipErrorInvalidValue;
    if (n_pairs == 0) return 0;
    const int bs = 256;
    hipLaunchKernelGGL(k_sim_pairs, dim3((unsigned)((n_pairs + bs - 1) / bs)), dim3(bs), 0,
                       static_cast<hipStream_t>(stream), d_reads, n_pairs, *spec, d_src);
    return (int)hipGetLastError();
}

int afs_spec_sizes(int32_t *genome_spec, int32_t *reads_spec) {
    if (genome_spec) *genome_spec = (int32_t)sizeof(SimGenomeSpec);
    if (reads_spec) *reads_spec = (int32_t)sizeof(SimReads);
    return 0;
}

}  // extern "C"
