"""The genome `bwa mem` calls of the partner stages on the GPU.

The reference runs bwa 0.7.17 against the whole genome twice per anchor gene:

- S4, paired: ``bwa mem -M -t T genome tmp1.fq tmp2.fq`` (Anchored_Fusion.py:188), whose every
  record `Find_blocks` reads (functions.py:376-496);
- S5, single-end: ``bwa mem -M -t T genome split_reads.fa`` (functions.py:716), whose every
  record `del_too_many_reads` reads (fn:705-768).

`GenomeIndex` is ``bwa index genome.fa`` (AF:173-178) built on the GPU (csrc/fmindex.hip: the
bwa text with bns_fasta2bntseq's lrand48 substitution of ambiguous bases, its suffix array and
FM index) and the two calls (csrc/bwa_genome.hip: SMEM seeding with max_occ sampling in
suffix-array order, chains and the chain filter, extension, dedup/patch, -M primary marking,
paired-end statistics, mate rescue and pairing, mem_reg2sam's records).  The records come back
as `af_grec` rows (REC_DTYPE) and are printed as bwa prints them by `sam_lines`.  Bit-exact
contract: oracle/bwa_pe.c in FM mode (tests/test_gpu_genome.py); parity with the bwa binary is
unpinned (absent here), the seeding restatement is cross-checked against the MEM-set form the
anchor path uses (tests/test_oracle_fm.py).
"""
import ctypes

import numpy as np

from . import _lib

MAX_REC = _lib.AF_G_MAX_REC
REC_DTYPE = np.dtype([("read", "<i4"), ("flag", "<i4"), ("rid", "<i4"), ("mrid", "<i4"), ("pos", "<i8"),
                      ("mpos", "<i8"), ("score", "<i4"), ("n_cigar", "<i4"), ("seq_b", "<i4"), ("seq_e", "<i4"),
                      ("cigar", "<u4", (_lib.AF_MAX_CIGAR,))])
assert REC_DTYPE.itemsize == 176
_OPS = "MIDNSHP=X"
_COMP = str.maketrans("ACGTNacgtn", "TGCANtgcan")
STAT_NAMES = ("cap_overflow", "pool_overflow", "record_overflow", "pe_rescue_job_pairs")


def _need(t, nbytes, what, dtype=None):
    """A kernel operand: a contiguous device tensor of at least nbytes (checked on the host before
    the launch, so a short buffer is an error, not an out-of-bounds access)."""
    if t is None or not t.is_cuda or not t.is_contiguous():
        raise ValueError(f"{what}: a contiguous device tensor is required")
    if dtype is not None and t.dtype != dtype:
        raise ValueError(f"{what}: dtype {t.dtype}, expected {dtype}")
    if t.numel() * t.element_size() < nbytes:
        raise ValueError(f"{what}: {t.numel() * t.element_size()} bytes, the call reads or writes {nbytes}")


def _check_se(reads_t, n, stride, recs_t, nrec_t, lens_t):
    n, stride = int(n), int(stride)
    if n < 0 or stride <= 0:
        raise ValueError("n must be >= 0 and stride > 0")
    _need(reads_t, n * stride, "reads_t")
    _need(recs_t, n * MAX_REC * REC_DTYPE.itemsize, "recs_t")
    _need(nrec_t, 4 * n, "nrec_t")
    if lens_t is not None:
        _need(lens_t, 4 * n, "lens_t")


def _stream_handle(stream):
    if stream is None:
        return None
    return stream if isinstance(stream, int) else stream.cuda_stream


class GenomeIndex:
    """`bwa index` of contigs [(name, seq)] (host strings/bytes) on GPU `device`."""

    def __init__(self, contigs, device=0, ctx=None):
        self.names = [n for n, _ in contigs]
        self.lens = [len(s) for _, s in contigs]
        blob = b"".join(s.encode() if isinstance(s, str) else bytes(s) for _, s in contigs)
        off = np.concatenate([[0], np.cumsum(self.lens)[:-1]]).astype(np.int64)
        self._open(ctx, device)
        ln = np.asarray(self.lens, dtype=np.int64)
        self.g = ctypes.c_void_p()
        _lib.check(self.ctx, _lib.lib().af_genome_build(self.ctx, blob, len(blob), off.ctypes.data, ln.ctypes.data,
                                                        len(contigs), ctypes.byref(self.g)), "af_genome_build")
        self.l_pac = int(_lib.lib().af_genome_lpac(self.g))

    @classmethod
    def from_device(cls, blob_t, names, offsets, lens, device=0, ctx=None):
        """Contigs already in HBM: blob_t a uint8 device tensor holding contig k at offsets[k]
        (lens[k] bytes; bytes between contigs are ignored)."""
        self = cls.__new__(cls)
        self.names, self.lens = list(names), [int(v) for v in lens]
        off = np.asarray(offsets, dtype=np.int64)
        ln = np.asarray(self.lens, dtype=np.int64)
        self._open(ctx, device)
        self.g = ctypes.c_void_p()
        _lib.check(self.ctx, _lib.lib().af_genome_build_device(
            self.ctx, blob_t.data_ptr(), int(blob_t.numel()), off.ctypes.data, ln.ctypes.data, len(self.names),
            ctypes.byref(self.g)), "af_genome_build_device")
        self.l_pac = int(_lib.lib().af_genome_lpac(self.g))
        return self

    def _open(self, ctx, device):
        self._own_ctx = ctx is None
        if ctx is None:
            ctx = ctypes.c_void_p()
            _lib.check(None, _lib.lib().af_ctx_create(int(device), ctypes.byref(ctx)), "af_ctx_create")
        self.ctx = ctx

    def close(self):
        L = _lib._L
        if L is None:
            return
        if getattr(self, "g", None):
            L.af_genome_free(self.g)
            self.g = None
        if getattr(self, "_own_ctx", False) and getattr(self, "ctx", None):
            L.af_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass

    # ---- index access (tests) -------------------------------------------------------------
    def text(self, first=0, n=None):
        n = 2 * self.l_pac - first if n is None else n
        out = np.zeros(n, np.uint8)
        _lib.check(self.ctx, _lib.lib().af_genome_read(self.ctx, self.g, 0, first, n, out.ctypes.data), "af_genome_read")
        return out

    def sa(self, first=0, n=None):
        n = 2 * self.l_pac + 1 - first if n is None else n
        out = np.zeros(n, np.int64)
        _lib.check(self.ctx, _lib.lib().af_genome_read(self.ctx, self.g, 1, first, n, out.ctypes.data), "af_genome_read")
        return out

    def occ(self, first_blk=0, n_blk=None):
        """Occurrence-table blocks [first_blk, first_blk + n_blk) as uint64 [n, 8]: counts of
        A/C/G/T before the block, then the block's 128 BWT codes at 2 bits (row k of the block at
        bits 2 (k & 31) of word 4 + (k >> 5)); the '$' row is stored as A and not counted."""
        total = (2 * self.l_pac + 1 + 127) // 128 + 1  # fmindex.hip: one block past the last row
        n_blk = total - first_blk if n_blk is None else n_blk
        out = np.zeros((n_blk, 8), np.uint64)
        _lib.check(self.ctx, _lib.lib().af_genome_read(self.ctx, self.g, 2, 8 * first_blk, 8 * n_blk, out.ctypes.data),
                   "af_genome_read")
        return out

    def primary(self):
        return int(_lib.lib().af_genome_primary(self.g))

    def stats(self, ctx=None):
        c = self.ctx if ctx is None else ctx
        out = np.zeros(_lib.AF_GSTAT_N, np.int32)
        _lib.check(c, _lib.lib().af_genome_stats(c, out.ctypes.data), "af_genome_stats")
        return dict(zip(STAT_NAMES, (int(v) for v in out)))

    # ---- the calls (host buffers) ----------------------------------------------------------
    def align_se(self, reads, lens=None, params=None, pe=None, id_base=0):
        """S5 on reads uint8 [n, stride]: (records [n, MAX_REC] REC_DTYPE, counts [n])."""
        reads = np.ascontiguousarray(reads, dtype=np.uint8)
        n = reads.shape[0]
        recs = np.zeros((n, MAX_REC), REC_DTYPE)
        nrec = np.zeros(n, np.int32)
        if n == 0:
            return recs, nrec
        lp = None if lens is None else np.ascontiguousarray(lens, dtype=np.int32)
        _lib.check(self.ctx, _lib.lib().af_genome_align_se(
            self.ctx, self.g, reads.ctypes.data, n, reads.shape[1], None if lp is None else lp.ctypes.data,
            ctypes.byref(params or _lib.default_params()), ctypes.byref(pe or _lib.default_pe()), int(id_base),
            recs.ctypes.data, nrec.ctypes.data), "af_genome_align_se")
        return recs, nrec

    def align_pe(self, reads, lens=None, params=None, pe=None):
        """S4 on pair-major reads uint8 [2N, stride]: (records [2N, MAX_REC], counts [2N])."""
        reads = np.ascontiguousarray(reads, dtype=np.uint8)
        nr = reads.shape[0]
        if nr % 2:
            raise ValueError("pair-major reads: an even number of rows")
        recs = np.zeros((nr, MAX_REC), REC_DTYPE)
        nrec = np.zeros(nr, np.int32)
        if nr == 0:
            return recs, nrec
        lp = None if lens is None else np.ascontiguousarray(lens, dtype=np.int32)
        _lib.check(self.ctx, _lib.lib().af_genome_align_pe(
            self.ctx, self.g, reads.ctypes.data, nr // 2, reads.shape[1], None if lp is None else lp.ctypes.data,
            ctypes.byref(params or _lib.default_params()), ctypes.byref(pe or _lib.default_pe()), recs.ctypes.data,
            nrec.ctypes.data), "af_genome_align_pe")
        return recs, nrec

    def intervals(self, reads, lens=None, params=None, pe=None, max_iv=512):
        """mem_collect_intv's seed intervals per read (tests): int64 [n, max_iv, 4] {sa_k, s, qb, qe},
        counts [n] (-1: overflow)."""
        reads = np.ascontiguousarray(reads, dtype=np.uint8)
        n = reads.shape[0]
        ivs = np.zeros((n, max_iv, 4), np.int64)
        niv = np.zeros(n, np.int32)
        lp = None if lens is None else np.ascontiguousarray(lens, dtype=np.int32)
        _lib.check(self.ctx, _lib.lib().af_genome_intervals(
            self.ctx, self.g, reads.ctypes.data, n, reads.shape[1], None if lp is None else lp.ctypes.data,
            ctypes.byref(params or _lib.default_params()), ctypes.byref(pe or _lib.default_pe()), max_iv,
            ivs.ctypes.data, niv.ctypes.data), "af_genome_intervals")
        return ivs, niv

    def regions(self, reads, lens=None, params=None, pe=None, max_reg=64):
        """mem_align1_core's regions per read (tests): int64 [n, max_reg, 12], counts [n]."""
        reads = np.ascontiguousarray(reads, dtype=np.uint8)
        n = reads.shape[0]
        regs = np.zeros((n, max_reg, 12), np.int64)
        nreg = np.zeros(n, np.int32)
        lp = None if lens is None else np.ascontiguousarray(lens, dtype=np.int32)
        _lib.check(self.ctx, _lib.lib().af_genome_regions(
            self.ctx, self.g, reads.ctypes.data, n, reads.shape[1], None if lp is None else lp.ctypes.data,
            ctypes.byref(params or _lib.default_params()), ctypes.byref(pe or _lib.default_pe()), max_reg,
            regs.ctypes.data, nreg.ctypes.data), "af_genome_regions")
        return regs, nreg

    # ---- the calls (device buffers, asynchronous) -----------------------------------------
    def align_se_device(self, reads_t, n, stride, recs_t, nrec_t, lens_t=None, params=None, pe=None, id_base=0,
                        stream=None, ctx=None):
        c = self.ctx if ctx is None else ctx
        _check_se(reads_t, n, stride, recs_t, nrec_t, lens_t)
        _lib.check(c, _lib.lib().af_genome_align_se_device(
            c, self.g, reads_t.data_ptr(), int(n), int(stride), None if lens_t is None else lens_t.data_ptr(),
            ctypes.byref(params or _lib.default_params()), ctypes.byref(pe or _lib.default_pe()), int(id_base),
            recs_t.data_ptr(), nrec_t.data_ptr(), _stream_handle(stream)), "af_genome_align_se_device")

    def align_se_ids_device(self, reads_t, n, stride, ids_t, recs_t, nrec_t, lens_t=None, params=None, pe=None,
                            stream=None, ctx=None):
        """S5 on a shard of a query list: read r's bwa id is ids_t[r] (int64, its ordinal in the
        whole list), which decides mem_mark_primary_se's hash tie-breaks."""
        import torch
        c = self.ctx if ctx is None else ctx
        _check_se(reads_t, n, stride, recs_t, nrec_t, lens_t)
        _need(ids_t, 8 * int(n), "ids_t", torch.int64)
        _lib.check(c, _lib.lib().af_genome_align_se_ids_device(
            c, self.g, reads_t.data_ptr(), int(n), int(stride), None if lens_t is None else lens_t.data_ptr(),
            ctypes.byref(params or _lib.default_params()), ctypes.byref(pe or _lib.default_pe()), ids_t.data_ptr(),
            recs_t.data_ptr(), nrec_t.data_ptr(), _stream_handle(stream)), "af_genome_align_se_ids_device")

    def align_pe_device(self, reads_t, n_pairs, stride, lens_t, recs_t, nrec_t, params=None, pe=None, stream=None,
                        ctx=None):
        c = self.ctx if ctx is None else ctx
        _check_se(reads_t, 2 * int(n_pairs), stride, recs_t, nrec_t, lens_t)
        _lib.check(c, _lib.lib().af_genome_align_pe_device(
            c, self.g, reads_t.data_ptr(), int(n_pairs), int(stride), lens_t.data_ptr(),
            ctypes.byref(params or _lib.default_params()), ctypes.byref(pe or _lib.default_pe()), recs_t.data_ptr(),
            nrec_t.data_ptr(), _stream_handle(stream)), "af_genome_align_pe_device")

    def align_pe_se_device(self, reads_t, n_pairs, n_se, stride, lens_t, recs_t, nrec_t, params=None, pe_s4=None,
                           pe_s5=None, se_id_base=0, se_ids_t=None, stream=None, stream_pe=None, ctx=None):
        """S4 (reads [0, 2 n_pairs), pair-major) and S5 (reads [2 n_pairs, 2 n_pairs + n_se)) of one
        gene step with one launch of the seed / region kernels (af_genome_align_pe_se_device):
        records of every read equal to align_pe_device + align_se_device (or align_se_ids_device
        with se_ids_t).  S5's records are ordered on `stream`, S4's on `stream_pe`."""
        import torch
        c = self.ctx if ctx is None else ctx
        n = 2 * int(n_pairs) + int(n_se)
        _check_se(reads_t, n, stride, recs_t, nrec_t, lens_t)
        if lens_t is None:
            raise ValueError("lens_t: the reads' lengths are required")
        if se_ids_t is not None:
            _need(se_ids_t, 8 * int(n_se), "se_ids_t", torch.int64)
        _lib.check(c, _lib.lib().af_genome_align_pe_se_device(
            c, self.g, reads_t.data_ptr(), int(n_pairs), int(n_se), int(stride), lens_t.data_ptr(),
            ctypes.byref(params or _lib.default_params()), ctypes.byref(pe_s4 or _lib.default_pe()),
            ctypes.byref(pe_s5 or _lib.default_pe()), int(se_id_base),
            None if se_ids_t is None else se_ids_t.data_ptr(), recs_t.data_ptr(), nrec_t.data_ptr(),
            _stream_handle(stream), _stream_handle(stream_pe)), "af_genome_align_pe_se_device")

    # ---- SAM text --------------------------------------------------------------------------
    def sam_lines(self, name, seq, recs, n):
        """The SAM lines bwa prints for one read (its af_grec rows recs[:n]): QNAME FLAG RNAME POS
        MAPQ CIGAR RNEXT PNEXT TLEN SEQ QUAL.  MAPQ (60 / 0 unmapped) and TLEN (0) are not
        bwa's: no consumer reads them (SURVEY.md §8 b)."""
        return sam_lines(self.names, name, seq, recs, n)


def s5_filter_device(ctx, recs_t, nrec_t, n, q_t, q_stride, q_lens_t, q_rows_t, s2_out, cap, s6_t, s6_lens_t,
                     s6_src_t, n6_t, n_over_t=None, stream=None, cont_t=None):
    """af_s5_filter_device: the genome check of the n S5 queries (`del_too_many_reads`,
    functions.py:718-768) and the S6 query rows of the survivors (fn:506-528) on the device.
    s2_out: the S2 record tensors (flag / pos / score / n_cigar / hits / cigar) the queries' rows
    index; s6_t uint8 [cap, stride], s6_lens_t / s6_src_t int32 [cap], n6_t int32 [1]; n_over_t
    (int32 [1], optional) counts rows whose processed sequence was clipped to the stride; cont_t
    (uint8 [n], optional): the QNAME groups given by the caller (cont_t[q] != 0: query q continues
    the group of q - 1), for a shard of a wider query list."""
    import torch
    n, cap = int(n), int(cap)
    if int(s6_t.shape[0]) < cap or s6_lens_t.numel() < cap or s6_src_t.numel() < cap:
        raise ValueError("S6 buffers hold fewer than cap rows")
    _need(recs_t, n * MAX_REC * REC_DTYPE.itemsize, "recs_t")
    _need(nrec_t, 4 * n, "nrec_t")
    _need(q_t, n * int(q_stride), "q_t")
    _need(q_lens_t, 4 * n, "q_lens_t")
    _need(q_rows_t, 4 * n, "q_rows_t", torch.int32)
    _need(s6_t, cap * int(s6_t.shape[1]), "s6_t", torch.uint8)
    _need(n6_t, 4, "n6_t")
    if cont_t is not None:
        _need(cont_t, n, "cont_t", torch.uint8)
    for k in ("flag", "pos", "n_cigar"):
        _need(s2_out[k], 4, f"s2_out[{k}]", torch.int32)
    if s2_out["cigar"].numel() != s2_out["flag"].numel() * _lib.AF_MAX_CIGAR:
        raise ValueError("s2_out['cigar'] must hold AF_MAX_CIGAR words per record")
    o = _lib.AlnOut(*(s2_out[k].data_ptr() for k in ("flag", "pos", "score", "n_cigar", "hits", "cigar")))
    _lib.check(ctx, _lib.lib().af_s5_filter_device(
        ctx, recs_t.data_ptr(), nrec_t.data_ptr(), int(n), q_t.data_ptr(), int(q_stride), q_lens_t.data_ptr(),
        q_rows_t.data_ptr(), ctypes.byref(o), None if cont_t is None else cont_t.data_ptr(), int(cap), s6_t.data_ptr(),
        int(s6_t.shape[1]), s6_lens_t.data_ptr(),
        s6_src_t.data_ptr(), n6_t.data_ptr(), None if n_over_t is None else n_over_t.data_ptr(),
        _stream_handle(stream)), "af_s5_filter_device")


def _s2_aln(s2_out):
    import torch
    for k in ("flag", "pos", "n_cigar"):
        _need(s2_out[k], 4, f"s2_out[{k}]", torch.int32)
    if s2_out["cigar"].numel() != s2_out["flag"].numel() * _lib.AF_MAX_CIGAR:
        raise ValueError("s2_out['cigar'] must hold AF_MAX_CIGAR words per record")
    return _lib.AlnOut(*(s2_out[k].data_ptr() for k in ("flag", "pos", "score", "n_cigar", "hits", "cigar")))


_MAX_PSL_ROWS = 16  # blat.MAX_ROWS (af_s6_compact_device's max_rows)


def s6_set(d):
    """af_s6_set of a dict of device tensors (discover.CandidateDiscovery._alloc_s6's layout; absent
    keys are NULL)."""
    def ptr(k):
        t = d.get(k)
        return None if t is None else t.data_ptr()
    cap = int(d["q"].shape[0])
    spill_cap = 0
    if d.get("spill_rows") is not None:
        spill_cap = min(d["spill_rows"].numel() // 328, int(d["spill_q"].numel()))
    if d.get("rows") is not None and d["rows"].numel() < cap * _MAX_PSL_ROWS * 328:
        raise ValueError("rows hold fewer than cap * max_rows PSL rows")
    for k in ("lens", "src", "n_rows"):
        if d.get(k) is not None and d[k].numel() < cap:
            raise ValueError(f"{k} holds fewer than cap entries")
    if d.get("caps") is not None and d["caps"].numel() < 4 * cap:
        raise ValueError("caps holds fewer than 4 * cap counters")
    return _lib.S6Set(ptr("q"), int(d["q"].shape[1]), 0, ptr("lens"), ptr("src"), ptr("n"), ptr("over"), ptr("n_over"),
                      ptr("rows"), ptr("n_rows"), ptr("caps"), ptr("spill_rows"), ptr("spill_q"), ptr("spill_n"),
                      spill_cap, cap)


def s6_queries_device(ctx, n, q_t, q_stride, q_lens_t, q_rows_t, s2_out, pre, stream=None, cont_t=None):
    """af_s6_queries_device: the S6 row of every QNAME-group leader among the n S5 queries (the
    queries fn:718-768 can keep), before the genome check, into the dict `pre`."""
    import torch
    n = int(n)
    _need(q_t, n * int(q_stride), "q_t")
    _need(q_lens_t, 4 * n, "q_lens_t")
    _need(q_rows_t, 4 * n, "q_rows_t", torch.int32)
    if cont_t is not None:
        _need(cont_t, n, "cont_t", torch.uint8)
    o, st = _s2_aln(s2_out), s6_set(pre)
    _lib.check(ctx, _lib.lib().af_s6_queries_device(
        ctx, n, q_t.data_ptr(), int(q_stride), q_lens_t.data_ptr(), q_rows_t.data_ptr(), ctypes.byref(o),
        None if cont_t is None else cont_t.data_ptr(), ctypes.byref(st), _stream_handle(stream)), "af_s6_queries_device")


def s6_check_device(ctx, recs_t, nrec_t, n, q_rows_t, s2_out, pre, live_t, stream=None, cont_t=None):
    """af_s6_check_device: the genome check of the n S5 queries (fn:718-768); live_t[k] (uint8
    [pre cap]) = 1 when pre row k's query survives."""
    import torch
    n = int(n)
    _need(recs_t, n * MAX_REC * REC_DTYPE.itemsize, "recs_t")
    _need(nrec_t, 4 * n, "nrec_t")
    _need(q_rows_t, 4 * n, "q_rows_t", torch.int32)
    _need(live_t, int(pre["q"].shape[0]), "live_t", torch.uint8)
    if cont_t is not None:
        _need(cont_t, n, "cont_t", torch.uint8)
    o, sp = _s2_aln(s2_out), s6_set(pre)
    _lib.check(ctx, _lib.lib().af_s6_check_device(
        ctx, recs_t.data_ptr(), nrec_t.data_ptr(), n, q_rows_t.data_ptr(), ctypes.byref(o),
        None if cont_t is None else cont_t.data_ptr(), ctypes.byref(sp), live_t.data_ptr(), _stream_handle(stream)),
        "af_s6_check_device")


def s6_compact_device(ctx, pre, live_t, out, stream=None):
    """af_s6_compact_device: pre's S6 rows and BLAT results of the live rows into `out`,
    renumbered in order; their cap events go to ctx's af_blat_caps counters."""
    import torch
    _need(live_t, int(pre["q"].shape[0]), "live_t", torch.uint8)
    sp, so = s6_set(pre), s6_set(out)
    _lib.check(ctx, _lib.lib().af_s6_compact_device(ctx, ctypes.byref(sp), live_t.data_ptr(), ctypes.byref(so),
                                                    _MAX_PSL_ROWS, _stream_handle(stream)), "af_s6_compact_device")


def sam_lines(names, name, seq, recs, n):
    out = []
    rc = None
    for k in range(min(int(n), MAX_REC)):
        e = recs[k]
        flag = int(e["flag"])
        rid = int(e["rid"])
        if flag & 0x10:
            if rc is None:
                rc = seq.translate(_COMP)[::-1]
            s = rc
        else:
            s = seq
        s = s[int(e["seq_b"]):int(e["seq_e"])]
        nc = int(e["n_cigar"])
        cig = "".join(f"{int(c) >> 4}{_OPS[int(c) & 15]}" for c in e["cigar"][:nc]) if nc else "*"
        mrid = int(e["mrid"])
        if mrid < 0:
            rnext, pnext = "*", 0
        else:
            rnext, pnext = ("=" if mrid == rid else names[mrid]), int(e["mpos"]) + 1
        rname = names[rid] if rid >= 0 else "*"
        pos1 = int(e["pos"]) + 1 if rid >= 0 else 0
        mapq = 0 if flag & 4 else 60
        out.append(f"{name}\t{flag & 0xFFFF}\t{rname}\t{pos1}\t{mapq}\t{cig}\t{rnext}\t{pnext}\t0\t{s}\t*\n")
    return out
