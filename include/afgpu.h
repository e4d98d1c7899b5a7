/*
 * afgpu.h -- C-ABI of libafgpu.so, the MI355X-native anchored split-read aligner.
 *
 * Drop-in boundary (SURVEY.md §8 b).  The reference has no plugin API: the hot path is a
 * shell string plus files.  Each entry point below replaces one of those tool calls:
 *
 *   af_index_build        <- `bwa index <G>_fusion_anchored_gene_sequence.fa`
 *                            (Anchored_Fusion.py:167-172; FASTA written at AF:154-163)
 *   af_align_pairs        <- `bwa mem -M -t T anchor fq1 fq2 | samtools view -bSu -`
 *                            (Anchored_Fusion.py:182); per-read primary records carrying the
 *                            SAM fields the callers read (FLAG/POS/CIGAR, functions.py:380-385,
 *                            515-516, 712-714, 917-918; AF:186-194 flag filters)
 *   af_align_pairs_device <- same, device-resident buffers, enqueued on a HIP stream
 *   af_seed_filter_device <- the seeding pass of the same call (the HBM-bound kernel)
 *   af_align_candidates_device <- the extension/CIGAR/pairing pass of the same call
 *   af_split_tails_device <- the split-read selection + query FASTA of the partner search
 *                            (functions.py:705-716, 1001-1005), from device-resident records
 *   af_align_candidates_tails_device <- af_align_candidates_device + the same tails, fused
 *   af_partition_device   <- `| samtools sort` of the same call and the three
 *                            `samtools view -f/-F` filters of Anchored_Fusion.py:186-194
 *   af_gather_reads_device <- `samtools fastq` of the S3 partitions (AF:186-188) and the split-read
 *                            FASTA of functions.py:705-716: the genome searches' queries
 *   af_genome_build(_device) <- `bwa index <genome.fa>` (AF:173-178): the bwa text, suffix array
 *                            and FM index of a multi-contig genome, built on the GPU
 *   af_genome_align_pe(_device) <- `bwa mem -M -t T <genome> tmp1.fq tmp2.fq` (AF:188, S4): every
 *                            SAM record of every pair, as bwa prints them (Find_blocks input)
 *   af_genome_align_se(_device) <- `bwa mem -M -t T <genome> split_reads.fa` (functions.py:716, S5)
 *   af_tile_index_build / af_blat(_device) <- `blat [opts] target.fa query.fa out.psl`
 *                            (functions.py:341, 530, 966, 1007, 1071, 1122, 1244)
 *   af_fastq_*            <- the fq1/fq2 inputs of the AF:182 call (host-side reader)
 *
 * Conventions: plain pointers and sizes only; every function returns AF_OK (0) or a
 * negative AF_E_* code and sets a message readable with af_last_error().  No C++
 * exception crosses this boundary.  One context per GPU; calls on a context are not
 * re-entrant (one host thread per GPU is the supported model).
 *
 * Reads are pair-major, one byte per base (ASCII): row 2p = mate 1, row 2p+1 = mate 2,
 * `stride` bytes per row; `lens` may be NULL when every read has length `stride`.
 * Output arrays are caller-owned (flag/pos/score/n_cigar 8-byte aligned), 2*n_pairs entries each (cigar: 2*n_pairs*AF_MAX_CIGAR,
 * of which only the first n_cigar entries of a row are written,
 * BAM op encoding len<<4|op, M=0 I=1 D=2 S=4).  pos is the 0-based leftmost position of
 * the primary alignment (or of the mate, for an unmapped read with a mapped mate, as bwa
 * prints it); flag carries the SAM bits 0x1 0x4 0x8 0x10 0x20 0x40 0x80 plus
 * AF_FLAG_MEM_OVERFLOW / AF_FLAG_CIGAR_OVERFLOW.
 */
#ifndef AFGPU_H
#define AFGPU_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define AF_OK 0
#define AF_E_INVALID (-1)
#define AF_E_HIP (-2)
#define AF_E_CAPACITY (-3)
#define AF_E_NOMEM (-4)
#define AF_E_UNSUPPORTED (-5)

#define AF_K 16
#define AF_MAX_CIGAR 32
#define AF_MAX_READ 320
#define AF_FLAG_MEM_OVERFLOW 0x10000
#define AF_FLAG_CIGAR_OVERFLOW 0x20000

typedef struct af_ctx af_ctx;
typedef struct af_index af_index;

/* bwa mem scoring/seeding parameters (defaults = bwa mem defaults, see af_params_default) */
typedef struct {
    int32_t a, b;                       /* -A -B */
    int32_t o_del, e_del, o_ins, e_ins; /* -O -E */
    int32_t pen_clip5, pen_clip3;       /* -L    */
    int32_t w;                          /* -w    */
    int32_t zdrop;                      /* -d    */
    int32_t min_seed_len;               /* -k    */
    int32_t max_occ;                    /* k-mer occurrence cap */
    int32_t T;                          /* -T    */
    int32_t max_ext;                    /* seeds extended per read (<= 16) */
    int32_t max_mems;                   /* MEM cap per read (<= 64; more -> unmapped + AF_FLAG_MEM_OVERFLOW) */
} af_params;

typedef struct {
    int32_t *flag, *pos, *score, *n_cigar, *hits;
    uint32_t *cigar;
} af_aln_out;

/* bwa mem paired-end options (bwa 0.7.17 defaults, af_pe_default) and the batch's place in
 * bwa's input stream.  bwa estimates insert sizes per chunk of >= chunk_bases bases
 * (10,000,000 x the -t thread count); a batch must start at a chunk boundary, pair_base being
 * the global index of its first pair (bwa's read-id hash tie-breaks depend on it). */
typedef struct {
    int32_t pen_unpaired;   /* -U, 17 */
    int32_t max_ins;        /* 10000 (<= 16383 here) */
    int32_t max_matesw;     /* 50 */
    int32_t split_width;    /* 10: re-seed SMEMs occurring at most this often */
    int32_t max_mem_intv;   /* 20: third seeding pass (-y) */
    int32_t max_chain_gap;  /* 10000 */
    int64_t chunk_bases;    /* 10,000,000 x threads (-K) */
    int64_t pair_base;
} af_pe;

int af_ctx_create(int device, af_ctx **out);
void af_ctx_destroy(af_ctx *ctx);
const char *af_last_error(const af_ctx *ctx);
void af_params_default(af_params *p);
void af_pe_default(af_pe *pe);

/* anchor index (doubled reference anchor ++ revcomp, 16-mer position map, Bloom seed filter) */
int af_index_build(af_ctx *ctx, const char *anchor, int64_t len, af_index **out);
void af_index_free(af_index *idx);
int64_t af_index_anchor_len(const af_index *idx);
int32_t af_index_filter_words(const af_index *idx);
/* copies the seed-filter Bloom words (af_index_filter_words uint32) to host memory */
int af_index_filter_table(const af_index *idx, uint32_t *out, int64_t cap);

/* host buffers in, host buffers out; synchronous */
int af_align_pairs(af_ctx *ctx, const af_index *idx, const uint8_t *reads, int64_t n_pairs, int32_t stride,
                   const int32_t *lens, const af_params *p, const af_pe *pe, af_aln_out *out);
/* device buffers in/out, asynchronous on `stream` (hipStream_t; NULL = default stream) */
int af_align_pairs_device(af_ctx *ctx, const af_index *idx, const uint8_t *d_reads, int64_t n_pairs,
                          int32_t stride, const int32_t *d_lens, const af_params *p, const af_pe *pe,
                          af_aln_out *d_out, void *stream);
int af_seed_filter_device(af_ctx *ctx, const af_index *idx, const uint8_t *d_reads, int64_t n_reads,
                          int32_t stride, const int32_t *d_lens, int32_t *d_hits, void *stream);
/* the rest of af_align_pairs_device after af_seed_filter_device ran on the same context and
 * stream with d_hits = d_out->hits for these reads: candidate alignment + pair flags */
int af_align_candidates_device(af_ctx *ctx, const af_index *idx, const uint8_t *d_reads, int64_t n_pairs,
                               int32_t stride, const int32_t *d_lens, const af_params *p, const af_pe *pe,
                               af_aln_out *d_out, void *stream);
/* af_align_candidates_device that also writes the split-read tails of af_split_tails_device
 * (same arguments and semantics, see below) from the pair-flag pass, without a pass of its own. */
int af_align_candidates_tails_device(af_ctx *ctx, const af_index *idx, const uint8_t *d_reads, int64_t n_pairs,
                                     int32_t stride, const int32_t *d_lens, const af_params *p, const af_pe *pe,
                                     af_aln_out *d_out,
                                     int32_t min_clip, int64_t read_base, int32_t append, int64_t cap,
                                     uint8_t *d_tails, int32_t *d_tail_lens, int32_t *d_tail_read,
                                     int32_t *d_n_tails, void *stream);
/* number of candidate reads found by the last seed-filter pass on this context (synchronises) */
int64_t af_last_candidates(af_ctx *ctx);

/* Split-read tails on the device, from the records of af_align_pairs_device /
 * af_align_candidates_device (d_out; device buffers, asynchronous on `stream`).  A split read is
 * a mapped read whose CIGAR is exactly M + S or S + M (deal_cigar's two-operation case,
 * functions.py:713) with a clip of at least min_clip bases; its tail is the clipped part of
 * SEQ in SAM orientation (the read reverse-complemented for 0x10), the query of the partner
 * search (functions.py:1001-1005).  Writes up to cap tails: row t of d_tails (`stride` bytes,
 * bytes past d_tail_lens[t] undefined), d_tail_lens[t], d_tail_read[t] = read_base + the read's
 * row; the number of split reads (which may exceed cap) goes to *d_n_tails, which is zeroed
 * first unless `append` is non-zero (then the tails add to those already there: several
 * batches, even on different streams, can fill one buffer for one af_blat_device launch).
 * Tail order varies between runs; d_tail_read identifies them.  Replaces the split-read
 * selection and FASTA writing of functions.py:705-716 and fn:1001-1005. */
int af_split_tails_device(af_ctx *ctx, const uint8_t *d_reads, int64_t n_reads, int32_t stride,
                          const int32_t *d_lens, const af_aln_out *d_out, int32_t min_clip, int64_t read_base,
                          int32_t append, int64_t cap, uint8_t *d_tails, int32_t *d_tail_lens,
                          int32_t *d_tail_read, int32_t *d_n_tails, void *stream);

/* ---------------------------------------------------------------------------------------------
 * BLAT searches (functions.py:341, 530, 966, 1007, 1071, 1122, 1244).  BLAT (Kent 2002) is a
 * third-party binary, absent here; its published search is restated:
 *   index   non-overlapping 11-mer tiles of the target every step_size bases (-stepSize, default
 *           the tile size), tiles with N skipped, tiles occurring > rep_match times ignored;
 *   hits    every 11-mer of the query and of its reverse complement looked up;
 *   clumps  hits sorted by diagonal, split where successive diagonals drift by > max_gap + 2;
 *           a clump needs >= min_match hits (-minMatch);
 *   HSPs    within a clump, hits of one diagonal whose tiles touch form a range; a range not
 *           inside an HSP made before is extended without gaps both ways (+1 match, -1 mismatch
 *           or N, each end stopping XDOWN = 10 positions past its last new best, at its first best);
 *   stitch  HSPs of one strand and target that advance on both sequences, up to max_intron apart,
 *           joined into one multi-block hit (overlaps trimmed from the later HSP; each joint one
 *           q / t insert: the only gaps), best chain first;
 *   filter  PSL score = matches + repMatches/2 - misMatches - qNumInsert - tNumInsert >= min_score
 *           and identity 100 - milliBad / 10 >= min_identity (pslCalcMilliBad, mRNA mode).
 * One row per hit, the PSL columns (qStarts on the reverse-complemented query for '-'). */
typedef struct {
    int32_t step_size;     /* -stepSize (the index's; checked against it)                    */
    int32_t min_match;     /* -minMatch (2)                                                   */
    int32_t rep_match;     /* -repMatch (1024 x 11 / stepSize when not given)                 */
    int32_t min_score;     /* -minScore (30)                                                  */
    int32_t min_identity;  /* -minIdentity, percent (90)                                      */
    int32_t max_gap;       /* -maxGap (2)                                                     */
    int32_t max_intron;    /* -maxIntron (750000)                                             */
} af_blat_params;

#define AF_TILE 11
#define AF_PSL_MAX_BLOCKS 16
#define AF_BLAT_MAX_ROWS 16
typedef struct {
    int32_t query, strand;            /* strand 0 '+', 1 '-'                                       */
    int32_t score;                    /* PSL score                                                 */
    int32_t matches, mismatches, n_count;
    int32_t q_num_insert, q_base_insert, t_num_insert, t_base_insert;
    int32_t q_start, q_end, q_size, block_count;
    int64_t t_start, t_end;           /* forward coordinates of the indexed sequence               */
    int32_t block_sizes[AF_PSL_MAX_BLOCKS], q_starts[AF_PSL_MAX_BLOCKS];
    int64_t t_starts[AF_PSL_MAX_BLOCKS];
} af_psl;

void af_blat_params_default(af_blat_params *p);
/* tile index of `seq` (host or device bytes) for af_blat; step_size 1..11 */
int af_tile_index_build(af_ctx *ctx, const char *seq, int64_t len, int32_t step_size, af_index **out);
int af_tile_index_build_device(af_ctx *ctx, const char *d_seq, int64_t len, int32_t step_size, af_index **out);
/* BLAT search of queries (host buffers, synchronous): rows[q * max_rows + k] for k < n_rows[q],
 * best score first; max_rows 1..AF_BLAT_MAX_ROWS */
int af_blat(af_ctx *ctx, const af_index *idx, const uint8_t *queries, int64_t n_queries, int32_t stride,
            const int32_t *lens, const af_blat_params *p, int32_t max_rows, af_psl *rows, int32_t *n_rows);
/* the same on device buffers, the query count read on the device (clamped to cap_queries) */
int af_blat_device(af_ctx *ctx, const af_index *idx, const uint8_t *d_queries, const int32_t *d_n_queries,
                   int64_t cap_queries, int32_t stride, const int32_t *d_lens, const af_blat_params *p,
                   int32_t max_rows, af_psl *d_rows, int32_t *d_n_rows, void *stream);
/* af_blat_device over the queries [*d_first, min(*d_n_queries, cap_queries)) only (both device
 * words, read when the launch runs): a batch of queries still being appended to a buffer (the
 * split-read tails of the S2 batches done so far) is searched while later batches append.
 * Rows of query k still go to d_rows[k * max_rows ..]. */
int af_blat_device_range(af_ctx *ctx, const af_index *idx, const uint8_t *d_queries, const int32_t *d_first,
                         const int32_t *d_n_queries, int64_t cap_queries, int32_t stride, const int32_t *d_lens,
                         const af_blat_params *p, int32_t max_rows, af_psl *d_rows, int32_t *d_n_rows, void *stream);
/* One long query searched whole (functions.py:341 `Find_homo_genes` and fn:966 hand BLAT the anchor
 * transcript, kilobases long, as one query): the same search as af_blat with caps sized for it --
 * AF_BLAT_LONG_HITS tile hits and AF_BLAT_LONG_CLUMPS clumps per strand, AF_BLAT_LONG_PART_BLOCKS
 * blocks per part -- and rows of any block count.  Host buffers, synchronous.  Every row of both
 * strands best first (the af_blat order, then emission order); *n_rows = all of them, the first
 * max_rows written to rows (block_count = all the row's blocks; its first 16 also in the row) with
 * their blocks at blocks[block_off[k], block_off[k + 1]) (block_off: max_rows + 1 entries);
 * *n_blocks = the blocks of the rows written -- more than block_cap: AF_E_CAPACITY, no row written.
 * Cap events are counted on the context (af_blat_caps). */
#define AF_BLAT_LONG_MAX 131072
#define AF_BLAT_LONG_HITS (1 << 22)
#define AF_BLAT_LONG_CLUMPS (1 << 17)
#define AF_BLAT_LONG_PART_BLOCKS 256
typedef struct {
    int32_t size, q_start;  /* q_start on the reverse-complemented query for '-', as af_psl */
    int64_t t_start;
} af_psl_block;
int af_blat_long(af_ctx *ctx, const af_index *idx, const uint8_t *query, int32_t len, const af_blat_params *p,
                 int32_t max_rows, af_psl *rows, int32_t *n_rows, af_psl_block *blocks, int64_t block_cap,
                 int64_t *block_off, int64_t *n_blocks);
/* af_blat_device in two parts, so that a caller can drop queries while the search runs (S6 searched
 * beside S5's genome check, discover.py): _begin enqueues the per-strand pass -- every query strand
 * with at most 32 clumps (env AF_BLAT_HEAVY_CLUMPS) searched to its rows; the heavier strands' clumps
 * left as jobs -- and _end the rest: the jobs' alignments spread over the chip, those strands' chains,
 * then every query's rows, for the queries with d_live[q] != 0 (NULL: all; a query not live gets 0
 * rows).  Between the two the context holds the search: no other search may run on it.
 * af_blat_device = _begin + _end(NULL); the rows of the live queries are the same either way. */
int af_blat_device_begin(af_ctx *ctx, const af_index *idx, const uint8_t *d_queries, const int32_t *d_n_queries,
                         int64_t cap_queries, int32_t stride, const int32_t *d_lens, const af_blat_params *p,
                         int32_t max_rows, af_psl *d_rows, int32_t *d_n_rows, void *stream);
int af_blat_device_end(af_ctx *ctx, const uint8_t *d_live, void *stream);
/* A device pool for the rows past max_rows (BLAT prints every row; the fixed per-query row slots
 * keep the first max_rows): once registered on ctx, every later af_blat_device(_range) call on ctx
 * appends each query's rows past its first max_rows to d_rows[k] with d_query[k] = the query's
 * index, k from the device counter *d_n (the caller zeroes it; k >= cap: the row is dropped and
 * counted in AF_BLAT_CAP_ROWS).  Spilled rows come in no particular order; in the search's order
 * (best score first, the af_blat order) every one of them follows the query's max_rows kept rows.
 * d_rows == NULL or cap == 0 unregisters.
 * (BLAT prints all of a query's alignments, which functions.py:630-649 reads one by one.) */
int af_blat_spill(af_ctx *ctx, af_psl *d_rows, int32_t *d_query, int32_t *d_n, int64_t cap);
/* How often the search's fixed caps bound (BLAT itself has none), counted per query strand on the
 * context since the last reset: [HITS] tile hits past 32768 (the first 32768 in query order are
 * clumped), [CLUMPS] 4096 clumps reached (the first in diagonal order kept), [PARTS] the stitching
 * work budget reached (the chain DP's rescans after emitted chains; no further chain emitted --
 * every clump is aligned, parts have no cap of their own); [ROWS] without a spill pool: queries
 * with rows past max_rows dropped, with one: rows dropped because the pool was full.
 * Synchronises; reset != 0 zeroes the counters after reading. */
#define AF_BLAT_CAP_HITS 0
#define AF_BLAT_CAP_CLUMPS 1
#define AF_BLAT_CAP_PARTS 2
#define AF_BLAT_CAP_ROWS 3
#define AF_BLAT_CAP_N 4
int af_blat_caps(af_ctx *ctx, int32_t *out, int reset);
/* The last device search's deferred strands (af_blat_device_begin): out[0] strands deferred, [1] their
 * clump jobs, [2] jobs aligned, [3] strands chained (synchronises) */
int af_blat_heavy_stats(af_ctx *ctx, int32_t *out);
/* Per-query cap counters: once registered on ctx, the searches on ctx count each cap event of query q
 * (q < cap) in d_counts[k * cap + q] (k = AF_BLAT_CAP_*; the caller zeroes them) instead of the
 * context's counters, so a caller that later drops queries counts its survivors' events only
 * (af_s6_compact_device).  d_counts == NULL or cap == 0 unregisters. */
int af_blat_query_caps(af_ctx *ctx, int32_t *d_counts, int64_t cap);

/* S3 on the device (Anchored_Fusion.py:182 `| samtools sort`, then AF:186-194): the records
 * d_flag/d_pos of n_reads reads (pair-major, as written by af_align_pairs*) in samtools'
 * coordinate order -- placed records by (pos, strand), ties in input order -- filtered into
 *   d_tmp1      `samtools view -f 8 -F 260`   (AF:186, mapped primary, mate unmapped)
 *   d_tmp2      `samtools view -f 4 -F 264`   (AF:187, unmapped, mate mapped)
 *   d_anchored  `samtools view -F 772`        (AF:194, mapped primary)
 * as read rows in that order; d_counts[0..2] = their lengths (int64, device).  Each output
 * needs room for n_reads rows in the worst case.  ref_len bounds pos (the anchor length).
 * Enqueued on `stream`; synchronizes it once (the selected count sizes the sort). */
int af_partition_device(af_ctx *ctx, const int32_t *d_flag, const int32_t *d_pos, int64_t n_reads, int64_t ref_len,
                        int32_t *d_tmp1, int32_t *d_tmp2, int32_t *d_anchored, int64_t *d_counts, void *stream);

/* The genome searches' queries from S3's row lists (af_partition_device), on the device:
 *   AF_GATHER_SEQUENCED  every listed read as sequenced -- `samtools fastq` of tmp1 / tmp2 for the
 *                        paired genome search (Anchored_Fusion.py:186-188); call once per list with
 *                        first = 0 / 1 and step = 2 to interleave them as bwa pairs its two files;
 *   AF_GATHER_SPLIT_SAM  the listed mapped reads whose CIGAR deal_cigar reduces to two operations
 *                        (one soft clip + the aligned part), SEQ as SAM prints it (reverse complement
 *                        for 0x10): the split-read FASTA of functions.py:705-716; list order kept.
 * Query k goes to slot first + k * step of d_q (`stride` bytes per row, N-padded), d_q_lens and
 * d_q_rows (the read row; may be NULL); slots at or past cap are dropped.  *d_n_q (may be NULL) =
 * min(cap, last slot written + 1, or `first` when no row is written): the query count of the
 * genome calls (af_genome_align_pe_device / _se_device) when the calls fill slots 0.. in order.  d_out supplies FLAG and
 * CIGAR (AF_GATHER_SPLIT_SAM only).  Asynchronous on `stream`. */
#define AF_GATHER_SEQUENCED 0
#define AF_GATHER_SPLIT_SAM 1
int af_gather_reads_device(af_ctx *ctx, const uint8_t *d_reads, int32_t stride, const int32_t *d_lens,
                           const int32_t *d_rows, int64_t n_rows, int32_t mode, const af_aln_out *d_out,
                           int64_t first, int64_t step, int64_t cap, uint8_t *d_q, int32_t *d_q_lens,
                           int32_t *d_q_rows, int32_t *d_n_q, void *stream);

/* ---- the genome `bwa mem` calls S4 / S5 ---------------------------------------------------
 * bwa 0.7.17's algorithm restated on the GPU over bwa's own index construction: contigs joined
 * without separators, ambiguous bases -> lrand48() & 3 after srand48(11) (bns_fasta2bntseq), the
 * suffix array of pac ++ revcomp(pac), SMEM seeding with re-seeding and the third pass
 * (bwt_smem1, bwt_seed_strategy1), max_occ sampling in suffix-array order, chains and the chain
 * filter, ksw extension, dedup/patch, -M primary marking, and for S4 the paired-end statistics per
 * chunk, mate rescue and pairing.  Contract: oracle/bwa_pe.c (FM mode), bit-exact.
 * Per-read caps (bwa has none): a read past one is reported unmapped with AF_FLAG_MEM_OVERFLOW and
 * counted in af_genome_stats. */
#define AF_G_MAX_INTV 512     /* seed intervals (SMEMs, re-seeds, third-pass seeds) */
#define AF_G_MAX_OCC 8192     /* chain seeds (occurrences after max_occ sampling) */
#define AF_G_MAX_CHAIN 8192
#define AF_G_MAX_REG 1024     /* regions (after extension; with mate-rescue hits) */
#define AF_G_MAX_REC 8        /* SAM records per read (primary + -M parts) */
typedef struct af_genome af_genome;
/* One printed SAM record (mem_aln2sam): FLAG as printed (0x100 marks -M parts; AF_FLAG_* bits
 * above 0xFFFF), contig index and 0-based POS (-1: '*'), the mate's (paired-end), AS, CIGAR in BAM
 * op codes (H = 5 on the parts after the first), and SEQ = the read in the record's orientation
 * (reverse complement for 0x10) sliced [seq_b, seq_e). */
typedef struct {
    int32_t read, flag, rid, mrid;
    int64_t pos, mpos;
    int32_t score, n_cigar, seq_b, seq_e;
    uint32_t cigar[AF_MAX_CIGAR];
} af_grec;
/* counters of the last genome call on a context: [0] reads past a per-read cap, [1] reads whose
 * intervals / regions did not fit the call's pools (also flagged), [2] reads with more than
 * AF_G_MAX_REC records, [3] S4 pairs whose mate-rescue SWs ran as grid-wide jobs (informational) */
#define AF_GSTAT_OVERFLOW 0
#define AF_GSTAT_POOL 1
#define AF_GSTAT_RECS 2
#define AF_GSTAT_PE_JOBS 3
#define AF_GSTAT_N 4
/* blob: contig k is blob[ctg_off[k], ctg_off[k] + ctg_len[k]) (host arrays; bytes between contigs
 * are ignored, as a FASTA's headers are).  Synchronous; the index stays in HBM. */
int af_genome_build(af_ctx *ctx, const char *blob, int64_t n_blob, const int64_t *ctg_off, const int64_t *ctg_len,
                    int32_t n_ctg, af_genome **out);
int af_genome_build_device(af_ctx *ctx, const char *d_blob, int64_t n_blob, const int64_t *ctg_off,
                           const int64_t *ctg_len, int32_t n_ctg, af_genome **out);
void af_genome_free(af_genome *g);
int64_t af_genome_lpac(const af_genome *g);
int64_t af_genome_primary(const af_genome *g);
/* copies rows [first, first + n) of the bwa text (what = 0, uint8 codes), of the suffix array
 * (what = 1, int64, rows 0..2 l_pac) or words of the occurrence table (what = 2, uint64: per
 * 128-row block, the A/C/G/T counts before the block then its four 2-bit BWT words; '$' stored as
 * A and not counted) to host memory (tests) */
int af_genome_read(af_ctx *ctx, const af_genome *g, int32_t what, int64_t first, int64_t n, void *out);
/* S5 (single-end): records of reads [0, n) (`stride` bytes per row, d_lens may be NULL) into
 * d_recs[r * AF_G_MAX_REC + k] for k < d_n_rec[r]; read ids id_base + r (bwa's hash tie-breaks),
 * or d_ids[r] with af_genome_align_se_ids_device (a shard of a query list: the reads' ordinals in
 * the whole list).
 * Device buffers, asynchronous on `stream`; calls on one context must be stream-ordered. */
int af_genome_align_se_device(af_ctx *ctx, const af_genome *g, const uint8_t *d_reads, int64_t n, int32_t stride,
                              const int32_t *d_lens, const af_params *p, const af_pe *pe, int64_t id_base,
                              af_grec *d_recs, int32_t *d_n_rec, void *stream);
int af_genome_align_se_ids_device(af_ctx *ctx, const af_genome *g, const uint8_t *d_reads, int64_t n, int32_t stride,
                                  const int32_t *d_lens, const af_params *p, const af_pe *pe, const int64_t *d_ids,
                                  af_grec *d_recs, int32_t *d_n_rec, void *stream);
/* S4 (paired-end): pair-major reads [0, 2 n_pairs) with their lengths (d_lens required); every
 * record of read 2i + m at d_recs[(2i + m) * AF_G_MAX_REC ..]; pe->chunk_bases / pair_base as for
 * af_align_pairs (insert-size statistics per bwa chunk). */
int af_genome_align_pe_device(af_ctx *ctx, const af_genome *g, const uint8_t *d_reads, int64_t n_pairs,
                              int32_t stride, const int32_t *d_lens, const af_params *p, const af_pe *pe,
                              af_grec *d_recs, int32_t *d_n_rec, void *stream);
/* S4 and S5 of one gene step with one launch of the seed and region kernels (bwa's per-read work
 * up to mem_align1_core is the same for both calls; one launch fills the chip once instead of
 * twice): reads [0, 2 n_pairs) are S4's pairs as af_genome_align_pe_device takes them (pe_s4),
 * reads [2 n_pairs, 2 n_pairs + n_se) S5's queries as af_genome_align_se_device (id_base
 * se_id_base) or af_genome_align_se_ids_device (d_se_ids, when not NULL) take them; d_lens covers
 * every read.  Records at d_recs[r * AF_G_MAX_REC ..], d_n_rec[r] for every read r of the call,
 * equal to the two calls made separately.  The seed / region kernels and S5's records run on
 * `stream`; S4's records on `stream_pe` (ordered after the region kernels; NULL: `stream`), so
 * the caller can run S5's consumers on `stream` beside them.  pe_s4 and pe_s5 must agree on the
 * seeding options (split_width, max_mem_intv, max_chain_gap).
 * Replaces Anchored_Fusion.py:188 (`bwa mem -M genome tmp1.fq tmp2.fq`) together with
 * functions.py:716 (`bwa mem -M genome split.fa`) of the same gene. */
int af_genome_align_pe_se_device(af_ctx *ctx, const af_genome *g, const uint8_t *d_reads, int64_t n_pairs,
                                 int64_t n_se, int32_t stride, const int32_t *d_lens, const af_params *p,
                                 const af_pe *pe_s4, const af_pe *pe_s5, int64_t se_id_base, const int64_t *d_se_ids,
                                 af_grec *d_recs, int32_t *d_n_rec, void *stream, void *stream_pe);
/* host-buffer forms (synchronous) */
int af_genome_align_se(af_ctx *ctx, const af_genome *g, const uint8_t *reads, int64_t n, int32_t stride,
                       const int32_t *lens, const af_params *p, const af_pe *pe, int64_t id_base, af_grec *recs,
                       int32_t *n_rec);
int af_genome_align_pe(af_ctx *ctx, const af_genome *g, const uint8_t *reads, int64_t n_pairs, int32_t stride,
                       const int32_t *lens, const af_params *p, const af_pe *pe, af_grec *recs, int32_t *n_rec);
/* regions after mem_align1_core (rb, re on bwa's doubled text; parity tests): regs[r * max_reg +
 * k] as 12 int64 words {rb, re, qb, qe, rid, score, truesc, w, seedcov, seedlen0, 0, 0}, n_reg[r]
 * (-1: overflow); host buffers */
/* mem_collect_intv's seed intervals per read (parity tests): ivs[(r * max_iv + k) * 4] as int64
 * words {SA row k, occurrences s, qb, qe} in mem_chain's order, n_iv[r] (-1: overflow); host
 * buffers */
int af_genome_intervals(af_ctx *ctx, const af_genome *g, const uint8_t *reads, int64_t n, int32_t stride,
                        const int32_t *lens, const af_params *p, const af_pe *pe, int32_t max_iv, int64_t *ivs,
                        int32_t *n_iv);
int af_genome_regions(af_ctx *ctx, const af_genome *g, const uint8_t *reads, int64_t n, int32_t stride,
                      const int32_t *lens, const af_params *p, const af_pe *pe, int32_t max_reg, int64_t *regs,
                      int32_t *n_reg);
/* the counters of the last genome call on ctx (AF_GSTAT_N int32; synchronises) */
int af_genome_stats(af_ctx *ctx, int32_t *out);

/* The genome check of the split reads and the S6 queries, on the device (`del_too_many_reads`,
 * functions.py:718-768, and the FASTA of `Find_fine_block`, fn:506-528).  Input: the n_queries
 * S5 queries (d_q rows of q_stride bytes as af_gather_reads_device's AF_GATHER_SPLIT_SAM wrote
 * them, d_q_lens, d_q_rows = the read rows), their af_genome_align_se_device records (d_recs,
 * d_n_rec) and the S2 records d_s2 of af_align_*_device (FLAG / POS / CIGAR of the anchored
 * read).  A query is dropped when a genome record aligns it as one deal_cigar operation or a
 * genome M straddles the end of an anchored M by more than 20 % of it on both sides; records are
 * grouped by consecutive QNAME (pair, POS, CIGAR), as the reference's file walk groups them, or,
 * when d_cont is given (one process's share of a query list sharded over GPUs), by the caller's
 * flags: d_cont[q] != 0 when query q continues the group of query q - 1.
 * Each survivor, in query order, becomes S6 query row k of d_s6 (s6_stride bytes): deal_cigar's
 * processed SEQ (N for each deleted base, inserted bases removed), d_s6_lens[k] (clipped to
 * s6_stride; the clipped rows are counted in *d_n_over, which may be NULL), d_s6_src[k] = its S5
 * query index; *d_n6 = min(survivors, cap): the query count af_blat_device reads.  Asynchronous
 * on `stream`. */
int af_s5_filter_device(af_ctx *ctx, const af_grec *d_recs, const int32_t *d_n_rec, int64_t n_queries,
                        const uint8_t *d_q, int32_t q_stride, const int32_t *d_q_lens, const int32_t *d_q_rows,
                        const af_aln_out *d_s2, const uint8_t *d_cont, int64_t cap, uint8_t *d_s6, int32_t s6_stride,
                        int32_t *d_s6_lens, int32_t *d_s6_src, int32_t *d_n6, int32_t *d_n_over, void *stream);
/* The same two steps split so that S6's BLAT runs beside S5's genome call (the S6 queries depend
 * only on the S2 records; the check only decides which of them are kept):
 *   af_s6_queries_device   the S6 row of every QNAME-group leader (a query that does not continue
 *                          the group of the one before it -- the only queries the check can keep),
 *                          rows as af_s5_filter_device writes them, in query order, into `pre`
 *                          (q / lens / src / n; over[k] = 1 when row k was clipped);
 *   af_blat_device_begin   on pre's rows (with af_blat_spill / af_blat_query_caps registered on pre's
 *                          spill pool and per-query cap counters), beside the S5 genome call;
 *   af_s6_check_device     the genome check of the n_queries S5 queries (as af_s5_filter_device):
 *                          d_live[k] = 1 when pre row k's query survives (pre->cap bytes);
 *   af_blat_device_end     with d_live: the deferred heavy strands of the survivors only;
 *   af_s6_compact_device   pre's rows of the survivors, renumbered 0.. in query order, to `out` with
 *                          their PSL rows (query field renumbered), row counts and spilled rows (pool
 *                          order kept); the survivors' clipped rows are counted in *out->n_over and
 *                          their cap events added to ctx's af_blat_caps counters.
 * The result equals af_s5_filter_device followed by af_blat_device on its rows, byte for byte. */
typedef struct {
    uint8_t *q;           /* query rows, `stride` bytes each                                  */
    int32_t stride, pad0;
    int32_t *lens, *src;  /* row lengths; the S5 query index of each row                     */
    int32_t *n;           /* row count (device word)                                         */
    uint8_t *over;        /* pre: per row, 1 when the processed SEQ was clipped to the stride */
    int32_t *n_over;      /* out: clipped rows (may be NULL)                                 */
    af_psl *rows;         /* max_rows PSL row slots per query                                */
    int32_t *n_rows;      /* PSL rows per query                                              */
    int32_t *caps;        /* pre: the search's per-query cap counters (af_blat_query_caps)   */
    af_psl *spill_rows;   /* rows past max_rows (af_blat_spill pool), their query, the count */
    int32_t *spill_query, *spill_n;
    int64_t spill_cap;
    int64_t cap;          /* row capacity                                                     */
} af_s6_set;
int af_s6_queries_device(af_ctx *ctx, int64_t n_queries, const uint8_t *d_q, int32_t q_stride, const int32_t *d_q_lens,
                         const int32_t *d_q_rows, const af_aln_out *d_s2, const uint8_t *d_cont, const af_s6_set *pre,
                         void *stream);
int af_s6_check_device(af_ctx *ctx, const af_grec *d_recs, const int32_t *d_n_rec, int64_t n_queries,
                       const int32_t *d_q_rows, const af_aln_out *d_s2, const uint8_t *d_cont, const af_s6_set *pre,
                       uint8_t *d_live, void *stream);
int af_s6_compact_device(af_ctx *ctx, const af_s6_set *pre, const uint8_t *d_live, const af_s6_set *out,
                         int32_t max_rows, void *stream);
/* Test hook: the same per-query rules (one source, compiled for the host too) over host arrays --
 * the S2 fields indexed by the read rows q_rows (pos, n_cigar, cigar[row * AF_MAX_CIGAR ..]).
 * keep[q] = 1 when af_s5_filter_device keeps query q; rows[q] (out_stride bytes), out_lens[q] and
 * over[q] (bytes dropped) = the S6 row it writes for q, for every query.  Not a product path. */
int af_s5_rules_host(const af_grec *recs, const int32_t *n_rec, int64_t n, const int32_t *q_rows, const int32_t *pos,
                     const int32_t *n_cigar, const uint32_t *cigar, const uint8_t *cont, const uint8_t *q,
                     int32_t q_stride, const int32_t *q_lens, uint8_t *keep, uint8_t *rows, int32_t out_stride,
                     int32_t *out_lens, uint8_t *over);

/* Paired FASTQ(.gz) ingest into the read layout above (host only, no GPU).  Replaces the
 * fq1/fq2 inputs of `bwa mem -M -t T anchor fq1 fq2` (Anchored_Fusion.py:182): records as
 * bwa's reader takes them (name = header up to the first blank, "/<digit>" trimmed; multi-line
 * records; FASTA records allowed), the two files paired record by record with equal names.
 * Usage: af_fastq_open; then repeatedly af_fastq_next (parses the next <= max_pairs pairs:
 * *n_pairs = 0 at the end of input; the longest read and the NUL-terminated name bytes of the
 * batch are reported) and af_fastq_export (rows of `stride` >= the longest read, 'N'-padded;
 * lens[2 * n]; names arena + name_off[n]; any output pointer may be NULL); af_fastq_close.
 * Errors return AF_E_* with the message in af_fastq_error (also after a failed open, whose
 * handle must still be closed). */
typedef struct af_fastq af_fastq;
int af_fastq_open(const char *fq1, const char *fq2, int threads, af_fastq **out);
int af_fastq_next(af_fastq *f, int64_t max_pairs, int64_t *n_pairs, int32_t *max_len, int64_t *names_bytes);
int af_fastq_export(af_fastq *f, int32_t stride, uint8_t *reads, int32_t *lens, char *names, int64_t names_cap,
                    int64_t *name_off);
const char *af_fastq_error(const af_fastq *f);
void af_fastq_close(af_fastq *f);
/* Sharded ingest (one process per GPU, cli --gpus N): part `part` of `parts` of ONE BGZF FASTQ
 * file -- the records whose header starts in the BGZF blocks at compressed offsets
 * [part S / parts, (part + 1) S / parts) of the file (S its size); a record that continues into
 * the next blocks is completed from them, and a part after the first starts at the first line
 * that opens a 4-line FASTQ record.  The parts of a file hold every record once, in order.
 * Returns AF_E_UNSUPPORTED (handle set, message in af_fastq_part_error) for input that is not
 * BGZF; then every rank reads the whole file (af_fastq_*).  Export: rows of `stride` bytes
 * ('N'-padded), lens[n], the names (trim_readno applied) in one arena with an offset per record. */
typedef struct af_fastq_part af_fastq_part;
int af_fastq_part_read(const char *path, int part, int parts, int threads, af_fastq_part **out, int64_t *n_records,
                       int32_t *max_len, int64_t *names_bytes);
int af_fastq_part_export(af_fastq_part *p, int32_t stride, uint8_t *seqs, int32_t *lens, char *names, int64_t names_cap,
                         int64_t *name_off);
const char *af_fastq_part_error(const af_fastq_part *p);
void af_fastq_part_free(af_fastq_part *p);

#ifdef __cplusplus
}
#endif
#endif
