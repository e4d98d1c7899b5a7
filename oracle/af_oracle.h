/*
 * af_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the anchored split-read alignment path used
 * as the parity oracle for the HIP product path in anchored-fusion_amd/csrc.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 *
 * What it restates: the reference drives `bwa mem -M` (bwa >= 0.7.17, README.md:18;
 * third-party, NOT vendored under /root/reference) at Anchored_Fusion.py:182.  bwa is
 * absent from this image, so this file restates bwa-mem's published algorithm
 * (Li 2013, arXiv:1303.3997; ksw extension/global DP as published in bwa 0.7.17):
 * S2 (bwa_pe.c) restates bwa 0.7.17's paired-end path: SMEM seeding with re-seeding and the
 * third pass, chaining and the chain filter, seed extension, dedup/patch, insert-size
 * estimation per chunk, mate rescue (ksw_align2), -M primary marking with bwa's hash
 * tie-break, pair selection, and the record/flag rules of mem_aln2sam.
 * The same restatement runs the genome calls S4 / S5 (bwa_pe.c, afo_genome_*: bwa index of a
 * multi-contig genome with an FM index, bwt_smem1 / bwt_seed_strategy1 / bwt_sa).
 * Parity with the bwa binary itself is UNPINNED; the oracle is
 * pinned by the wgsim truth in the bundled test FASTQ names and the junction known-answers.
 */
#ifndef AF_ORACLE_H
#define AF_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define AFO_K 16
#define AFO_MAX_CIGAR 32
#define AFO_MAX_READ 512

typedef struct {
    int32_t a, b;                       /* match score / mismatch penalty (bwa -A -B)      */
    int32_t o_del, e_del, o_ins, e_ins; /* affine gaps (bwa -O -E)                          */
    int32_t pen_clip5, pen_clip3;       /* clipping penalty (bwa -L)                        */
    int32_t w;                          /* band width (bwa -w)                              */
    int32_t zdrop;                      /* z-drop (bwa -d)                                  */
    int32_t min_seed_len;               /* bwa -k                                           */
    int32_t max_occ;                    /* k-mer occurrence cap                             */
    int32_t T;                          /* min output score (bwa -T)                        */
    int32_t max_ext;                    /* max seeds extended per read                      */
    int32_t max_mems;                   /* MEM cap per read (overflow -> unmapped + flag)   */
} afo_params;

typedef struct {
    int32_t *flag, *pos, *score, *n_cigar, *hits;
    uint32_t *cigar; /* [n_reads * AFO_MAX_CIGAR], BAM op encoding len<<4|op */
} afo_out;

typedef struct afo_index afo_index;

/* bwa mem paired-end options (bwa 0.7.17 mem_opt_init defaults, afo_pe_default) and the
 * batch's place in bwa's input stream */
typedef struct {
    int32_t pen_unpaired;   /* -U 17                                                         */
    int32_t max_ins;        /* 10000: insert sizes above are ignored by mem_pestat             */
    int32_t max_matesw;     /* 50: mate-SW rounds per end                                      */
    int32_t split_width;    /* 10: re-seed an SMEM occurring at most this often (-r 1.5 split) */
    int32_t max_mem_intv;   /* 20: third seeding pass (-y)                                      */
    int32_t max_chain_gap;  /* 10000                                                           */
    int64_t chunk_bases;    /* bases per bwa batch: 10,000,000 x threads (-K)                   */
    int64_t pair_base;      /* global index of the first pair (bwa's n_processed / 2)           */
} afo_pe;

/* per-read caps of the S2 restatement (AF_S2_MAX_* on the GPU); overflow -> unmapped + flag */
#define AFO_PE_MAX_PMEM 128
#define AFO_PE_MAX_SEED 64
#define AFO_PE_MAX_OCC 128
#define AFO_PE_MAX_CHAIN 32
#define AFO_PE_MAX_REG 32
#define AFO_PE_MAX_TSPAN 1024  /* longest reference span mem_patch_reg merges */

/* ---- the genome calls S4 / S5 (bwa_pe.c, FM mode): `bwa mem -M` against a multi-contig genome.
 * Per-read caps of the restatement (the GPU's AF_G_MAX_*); past one the read is reported
 * unmapped with AF_FLAG_MEM_OVERFLOW (bwa has none). */
#define AFO_G_MAX_PMEM 65536   /* MEM-set cross-check mode only */
#define AFO_G_MAX_INTV 512     /* seed intervals (mem_collect_intv) */
#define AFO_G_MAX_OCC 8192     /* chain seeds (max_occ-sampled occurrences) */
#define AFO_G_MAX_CHAIN 8192
#define AFO_G_MAX_REG 1024
#define AFO_G_MAX_REC 8        /* SAM records per read (primary + -M parts) */
typedef struct afo_text afo_genome;
/* one printed SAM record (mem_aln2sam): FLAG as printed (0x100 for -M parts), contig / 0-based
 * position (-1: '*'), the mate's, AS, CIGAR in BAM op codes (H = 5 on parts after the first),
 * SEQ = the read in the record's orientation, sliced [seq_b, seq_e) */
typedef struct {
    int32_t read, flag, rid, mrid;
    int64_t pos, mpos;
    int32_t score, n_cigar, seq_b, seq_e;
    uint32_t cigar[AFO_MAX_CIGAR];
} afo_grec;
/* one region of mem_align1_core (mem_alnreg_t) */
typedef struct {
    int64_t rb, re;
    int32_t qb, qe, rid, score, truesc, w, seedcov, seedlen0;
} afo_reg;
/* blob: the contigs at ctg_off[k], ctg_len[k] (bytes between them ignored); memset_too: also
 * the MEM-set seeding structures (suffix ranks, 16-mer positions) for the cross-check */
afo_genome *afo_genome_build(const char *blob, const int64_t *ctg_off, const int64_t *ctg_len, int n_ctg,
                             int memset_too);
void afo_genome_free(afo_genome *G);
int64_t afo_genome_lpac(const afo_genome *G);
/* test hook: the SA-IS suffix array equals the prefix-doubling one on T (0), else first differing row + 1 */
int64_t afo_suffix_array_check(const uint8_t *T, int64_t N);
const uint8_t *afo_genome_text(const afo_genome *G);   /* the bwa text T, 2 l_pac codes */
const int64_t *afo_genome_sa(const afo_genome *G);     /* suffix array rows 0..2 l_pac */
int64_t afo_genome_primary(const afo_genome *G);
int afo_genome_seeds(const afo_genome *G, const uint8_t *read, int32_t l, const afo_params *p, const afo_pe *pe,
                     int memset_mode, int64_t *rbeg, int32_t *qbeg, int32_t *len, int32_t cap);
int afo_genome_intervals(const afo_genome *G, const uint8_t *reads, int64_t n, int32_t stride, const int32_t *lens,
                         const afo_params *p, const afo_pe *pe, int n_threads, int32_t max_iv, int64_t *out,
                         int32_t *n_iv);
int afo_genome_regions(const afo_genome *G, const uint8_t *reads, int64_t n, int32_t stride, const int32_t *lens,
                       const afo_params *p, const afo_pe *pe, int n_threads, int32_t max_reg, afo_reg *regs,
                       int32_t *n_reg);
int afo_genome_align_se(const afo_genome *G, const uint8_t *reads, int64_t n, int32_t stride, const int32_t *lens,
                        const afo_params *p, const afo_pe *pe, int64_t id_base, int n_threads, int32_t max_rec,
                        afo_grec *recs, int32_t *n_rec);
int afo_genome_align_se_ids(const afo_genome *G, const uint8_t *reads, int64_t n, int32_t stride, const int32_t *lens,
                            const afo_params *p, const afo_pe *pe, const int64_t *ids, int n_threads, int32_t max_rec,
                            afo_grec *recs, int32_t *n_rec);
int afo_genome_align_pe(const afo_genome *G, const uint8_t *reads, int64_t n_pairs, int32_t stride, const int32_t *lens,
                        const afo_params *p, const afo_pe *pe, int n_threads, int32_t max_rec, afo_grec *recs,
                        int32_t *n_rec);

void afo_params_default(afo_params *p);
afo_index *afo_index_build(const char *anchor, int64_t n);
void afo_index_free(afo_index *idx);
int64_t afo_index_len(const afo_index *idx);
int32_t afo_filter_words(const afo_index *idx);
const uint32_t *afo_filter_table(const afo_index *idx);
/* K1 restatement: per read, number of sampled 16-mers passing the anchor filter */
void afo_seed_filter(const afo_index *idx, const uint8_t *reads, int64_t n_reads, int32_t stride,
                     const int32_t *lens, int32_t *hits);
/* S2 restatement (bwa_pe.c): bwa mem paired-end alignment of every pair (reads pair-major:
 * 2p, 2p+1), one primary record per read.  The batch starts at a bwa chunk boundary; chunks of
 * >= pe->chunk_bases bases share insert-size statistics.  pe may be NULL (defaults). */
void afo_pe_default(afo_pe *pe);
int afo_align_pairs(const afo_index *idx, const uint8_t *reads, int64_t n_pairs, int32_t stride,
                    const int32_t *lens, const afo_params *p, const afo_pe *pe, int n_threads, afo_out *out);

/* BLAT restatement (blat.c): tile index, options, PSL rows (layout of af_psl, afgpu.h) */
#define AFO_PSL_MAX_BLOCKS 16
#define AFO_BLAT_MAX_ROWS 16
typedef struct afo_tiles afo_tiles;
typedef struct {
    int32_t step_size, min_match, rep_match, min_score, min_identity, max_gap, max_intron;
} afo_blat_params;
typedef struct {
    int32_t query, strand, score, matches, mismatches, n_count;
    int32_t q_num_insert, q_base_insert, t_num_insert, t_base_insert;
    int32_t q_start, q_end, q_size, block_count;
    int64_t t_start, t_end;
    int32_t block_sizes[AFO_PSL_MAX_BLOCKS], q_starts[AFO_PSL_MAX_BLOCKS];
    int64_t t_starts[AFO_PSL_MAX_BLOCKS];
} afo_psl;
afo_tiles *afo_tiles_build(const char *seq, int64_t n, int32_t step);
void afo_tiles_free(afo_tiles *X);
void afo_blat_params_default(afo_blat_params *p);
int afo_blat(const afo_tiles *X, const uint8_t *queries, int64_t n_queries, int32_t stride, const int32_t *lens,
             const afo_blat_params *bp, int32_t max_rows, afo_psl *rows, int32_t *n_rows, int threads);
/* afo_blat that also counts how often its caps bound (caps[4] added to, the order of
 * af_blat_caps: hits past MAXH per strand, MAXCL clumps reached, MAXR parts reached with clumps
 * left, per query rows past max_rows) */
void afo_blat_set_literal(int on);  /* test switch: the chain DP recomputes every part each round */
/* comparison switch: 1 = the round-5 gapped parts (ksw_extend2 per clump), 0 = gapless HSPs (default) */
void afo_blat_set_gapped(int on);
/* Long queries (afo_blat_long, af_blat_long): one query of up to AFO_BLAT_LONG_MAX bases searched
 * whole with the same algorithm -- caps: AFO_BLAT_LONG_HITS tile hits and AFO_BLAT_LONG_CLUMPS
 * clumps per strand, AFO_BLAT_LONG_PART_BLOCKS blocks per part; rows of any block count.  Every
 * row of both strands best first; the first max_rows to rows (block_count = all the row's blocks,
 * the first 16 also in the row), their blocks to blocks[block_off[k], block_off[k + 1]).  *n_rows
 * = all rows; *n_blocks = the returned rows' blocks (-3 when more than block_cap, nothing
 * written); caps[0..2] added to as afo_blat_caps counts them per strand. */
#define AFO_BLAT_LONG_MAX 131072
#define AFO_BLAT_LONG_HITS (1 << 22)
#define AFO_BLAT_LONG_CLUMPS (1 << 17)
#define AFO_BLAT_LONG_PART_BLOCKS 256
typedef struct { int32_t size, q_start; int64_t t_start; } afo_psl_block;
int afo_blat_long(const afo_tiles *X, const uint8_t *query, int32_t len, const afo_blat_params *bp, int32_t max_rows,
                  afo_psl *rows, int32_t *n_rows, afo_psl_block *blocks, int64_t block_cap, int64_t *block_off,
                  int64_t *n_blocks, int32_t *caps);
int afo_blat_caps(const afo_tiles *X, const uint8_t *queries, int64_t n_queries, int32_t stride, const int32_t *lens,
                  const afo_blat_params *bp, int32_t max_rows, afo_psl *rows, int32_t *n_rows, int threads,
                  int32_t *caps);

#ifdef __cplusplus
}
#endif
#endif
