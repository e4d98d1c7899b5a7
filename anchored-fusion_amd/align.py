"""Anchor alignment of read pairs on the GPU: the drop-in for ``bwa index`` + ``bwa mem -M``
against the anchored transcript (Anchored_Fusion.py:167-172, 181-182).

``AnchorAligner(anchor).align_pairs(reads, lens)`` returns per-read primary records (the SAM
fields Anchored-Fusion consumes: FLAG, POS, CIGAR) computed by the HIP kernels in csrc/.
``partition`` then applies the samtools flag filters and coordinate sort of
Anchored_Fusion.py:183-194 (S3) to those records.
"""
import ctypes

import numpy as np

from . import _lib

CIGAR_OPS = "MIDNSHP=X"


class AlignResult:
    """Per-read arrays (pair-major rows: 2p = mate 1, 2p+1 = mate 2)."""

    def __init__(self, flag, pos, score, n_cigar, cigar, hits):
        self.flag, self.pos, self.score = flag, pos, score
        self.n_cigar, self.cigar, self.hits = n_cigar, cigar, hits

    def __len__(self):
        return len(self.flag)

    def as_dict(self):
        return dict(flag=self.flag, pos=self.pos, score=self.score, n_cigar=self.n_cigar,
                    cigar=self.cigar, hits=self.hits)

    def cigar_ops(self, r):
        return [(int(c >> 4), CIGAR_OPS[c & 0xF]) for c in self.cigar[r][: self.n_cigar[r]]]

    def cigar_str(self, r):
        if self.flag[r] & 0x4:
            return "*"
        return "".join(f"{n}{op}" for n, op in self.cigar_ops(r))

    def mapped(self):
        return (self.flag & 0x4) == 0

    # the record API consume_gene reads (shared with shard.SparseCandidates)
    @property
    def n_reads(self):
        return len(self.flag)

    def flag_at(self, r):
        return int(self.flag[r])

    def pos_at(self, r):
        return int(self.pos[r])

    def n_mapped(self):
        return int(((self.flag & 4) == 0).sum())

    def n_overflow(self):
        """Reads reported unmapped because a per-read cap of the S2 restatement bound
        (AF_FLAG_MEM_OVERFLOW: MEMs / seeds / chains / regions or the region pool;
        AF_FLAG_CIGAR_OVERFLOW: a CIGAR past AF_MAX_CIGAR ops).  bwa has no such caps."""
        return int(((self.flag & (_lib.AF_FLAG_MEM_OVERFLOW | _lib.AF_FLAG_CIGAR_OVERFLOW)) != 0).sum())

    def partition(self):
        return partition(self)


class AnchorAligner:
    """One GPU context + one anchor index.  Not thread-safe (one host thread per GPU)."""

    def __init__(self, anchor: bytes, device: int = 0, params=None, pe=None):
        L = _lib.lib()
        self._ctx = ctypes.c_void_p()
        rc = L.af_ctx_create(int(device), ctypes.byref(self._ctx))
        if rc != _lib.AF_OK:
            raise _lib.AFError(f"af_ctx_create(device={device}) failed (rc={rc}): no usable GPU?")
        self._idx = ctypes.c_void_p()
        self.anchor = bytes(anchor)
        _lib.check(self._ctx, L.af_index_build(self._ctx, self.anchor, len(self.anchor), ctypes.byref(self._idx)),
                   "af_index_build")
        self.params = params or _lib.default_params()
        self.pe = pe or _lib.default_pe()
        self.device = device

    def _pe(self, pair_base):
        """af_pe for a batch starting at global pair index pair_base (bwa's read ids)."""
        e = _lib.Pe.from_buffer_copy(self.pe)
        e.pair_base = int(pair_base)
        return e

    def close(self):
        L = _lib._L
        if L is None:
            return
        if getattr(self, "_idx", None):
            L.af_index_free(self._idx)
            self._idx = None
        if getattr(self, "_ctx", None):
            L.af_ctx_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def filter_table(self):
        L = _lib.lib()
        nw = L.af_index_filter_words(self._idx)
        out = np.zeros(nw, dtype=np.uint32)
        _lib.check(self._ctx, L.af_index_filter_table(self._idx, out.ctypes.data, out.size), "af_index_filter_table")
        return out

    def align_pairs(self, reads, lens=None, pair_base=0) -> AlignResult:
        """reads: uint8 [2N, stride] pair-major ASCII; lens: optional int32 [2N].  The batch is
        bwa's input from pair ``pair_base`` on, starting at one of its chunk boundaries."""
        reads = np.ascontiguousarray(reads, dtype=np.uint8)
        nr, stride = reads.shape
        if nr % 2:
            raise ValueError("reads must hold an even number of rows (pair-major mates)")
        out = {k: np.zeros(nr, dtype=np.int32) for k in ("flag", "pos", "score", "n_cigar", "hits")}
        out["cigar"] = np.zeros((nr, _lib.AF_MAX_CIGAR), dtype=np.uint32)
        o = _lib.AlnOut(*(out[k].ctypes.data for k in ("flag", "pos", "score", "n_cigar", "hits", "cigar")))
        lp = None if lens is None else np.ascontiguousarray(lens, dtype=np.int32)
        _lib.check(self._ctx, _lib.lib().af_align_pairs(self._ctx, self._idx, reads.ctypes.data, nr // 2, stride,
                                                        None if lp is None else lp.ctypes.data,
                                                        ctypes.byref(self.params), ctypes.byref(self._pe(pair_base)),
                                                        ctypes.byref(o)),
                   "af_align_pairs")
        return AlignResult(**out)

    def align_segments(self, reads, lens, seg_pairs) -> AlignResult:
        """One batch holding several independent inputs (e.g. single-cell cells), each aligned
        as its own ``bwa mem`` run: read ids from 0 and insert-size chunks from the segment's
        first pair.  ``seg_pairs``: pairs per segment, in row order.  One H2D copy of the
        batch, one device call per segment on one stream, one D2H copy of the records."""
        import torch
        reads = np.ascontiguousarray(reads, dtype=np.uint8)
        nr, stride = reads.shape
        if nr % 2 or 2 * int(sum(seg_pairs)) != nr:
            raise ValueError("seg_pairs must cover the batch's pairs exactly")
        dev = torch.device("cuda", self.device)
        # segments start on 16-byte boundaries of one device buffer (the seed filter's loads)
        starts, off = [], 0
        for n in seg_pairs:
            starts.append(off)
            off = (off + 2 * int(n) * stride + 15) // 16 * 16
        host = np.zeros(max(off, 16), np.uint8)
        r0 = 0
        for n, b in zip(seg_pairs, starts):
            r1 = r0 + 2 * int(n)
            host[b:b + (r1 - r0) * stride] = reads[r0:r1].reshape(-1)
            r0 = r1
        flat = torch.from_numpy(host).to(dev)
        lt = None if lens is None else torch.from_numpy(np.ascontiguousarray(lens, dtype=np.int32)).to(dev)
        out = {k: torch.zeros(nr, dtype=torch.int32, device=dev) for k in ("flag", "pos", "score", "n_cigar", "hits")}
        out["cigar"] = torch.zeros((nr, _lib.AF_MAX_CIGAR), dtype=torch.int32, device=dev)
        s = torch.cuda.current_stream(dev)
        r0 = 0
        for n, b in zip(seg_pairs, starts):
            n = int(n)
            if n:
                r1 = r0 + 2 * n
                rt = flat[b:b + 2 * n * stride].view(2 * n, stride)
                self.align_pairs_device(rt, n, stride, {k: v[r0:r1] for k, v in out.items()},
                                        None if lt is None else lt[r0:r1], stream=s, pair_base=0)
                r0 = r1
        torch.cuda.synchronize(dev)
        got = {k: v.cpu().numpy() for k, v in out.items()}
        got["cigar"] = got["cigar"].view(np.uint32)
        return AlignResult(**got)

    def align_fastq(self, fq1, fq2, batch_pairs=1 << 20, threads=0):
        """FASTQ(.gz) pair -> records, streamed: the native reader (io.iter_pairs) parses batch
        k + 1 on host threads while batch k is aligned (both ctypes calls release the GIL).
        Alignment calls end on bwa chunk boundaries (``chunk_ends``), so insert-size statistics
        and read ids are those of one ``bwa mem`` run over the whole input.
        Returns ``(names, reads, lens, AlignResult)`` over all pairs, as io.read_pairs + align_pairs
        would (lens None when every read has the common length)."""
        import threading

        from . import io as afio
        it = afio.iter_pairs(fq1, fq2, batch_pairs=batch_pairs, threads=threads)
        box = {}

        def fetch():
            try:
                box["next"] = next(it, None)
            except BaseException as e:  # re-raised on the caller's thread
                box["err"] = e

        parts, pend = [], []
        done = 0
        th = threading.Thread(target=fetch)
        th.start()
        while True:
            th.join()
            if "err" in box:
                raise box.pop("err")
            cur = box.pop("next")
            if cur is not None:
                th = threading.Thread(target=fetch)
                th.start()
                pend.append(cur)
            if not pend:
                break
            names, reads, lens = _concat_batches(pend)
            pb = lens.reshape(-1, 2).sum(axis=1)
            cut = len(pb) if cur is None else complete_chunks(pb, int(self.pe.chunk_bases))
            pend = [] if cut == len(pb) else [(names.slice(cut, len(pb)), reads[2 * cut:], lens[2 * cut:])]
            if cut:
                sub_reads, sub_lens = reads[:2 * cut], lens[:2 * cut]
                uniform = bool((sub_lens == sub_reads.shape[1]).all())
                parts.append((names.slice(0, cut), sub_reads, sub_lens,
                              self.align_pairs(sub_reads, None if uniform else sub_lens, pair_base=done)))
                done += cut
            if cur is None:
                break
        if not parts:
            empty = np.zeros(0, np.int32)
            return (afio.Names(b"", np.zeros(0, np.int64)), np.full((0, 1), ord("N"), np.uint8), None,
                    AlignResult(empty, empty, empty, empty, np.zeros((0, _lib.AF_MAX_CIGAR), np.uint32), empty))
        stride = max(r.shape[1] for _, r, _, _ in parts)
        reads = np.full((sum(r.shape[0] for _, r, _, _ in parts), stride), ord("N"), np.uint8)
        row = 0
        for _, r, _, _ in parts:
            reads[row:row + r.shape[0], :r.shape[1]] = r
            row += r.shape[0]
        lens = np.concatenate([x for _, _, x, _ in parts])
        res = AlignResult(**{k: np.concatenate([getattr(a, k) for _, _, _, a in parts])
                             for k in ("flag", "pos", "score", "n_cigar", "cigar", "hits")})
        names = afio.Names.concat([nm for nm, _, _, _ in parts])
        return names, reads, (None if (lens == stride).all() else lens), res

    # ---- device-resident entry points (torch tensors as HBM buffers) ----------------------
    def align_pairs_device(self, reads_t, n_pairs, stride, out_t, lens_t=None, stream=None, pair_base=0):
        """Enqueues S2 on ``stream`` (torch.cuda.Stream or raw handle); all tensors on-device.
        out_t: dict flag/pos/score/n_cigar/hits (int32 [2N]) and cigar (int32/uint32 [2N, 32])."""
        o = _lib.AlnOut(*(out_t[k].data_ptr() for k in ("flag", "pos", "score", "n_cigar", "hits", "cigar")))
        sh = _stream_handle(stream)
        _lib.check(self._ctx, _lib.lib().af_align_pairs_device(
            self._ctx, self._idx, reads_t.data_ptr(), int(n_pairs), int(stride),
            None if lens_t is None else lens_t.data_ptr(), ctypes.byref(self.params), ctypes.byref(self._pe(pair_base)),
            ctypes.byref(o), sh), "af_align_pairs_device")

    def align_candidates_device(self, reads_t, n_pairs, stride, out_t, lens_t=None, stream=None, pair_base=0):
        """Second half of align_pairs_device; seed_filter_device(hits_t=out_t['hits']) must have
        run on the same stream for this batch."""
        o = _lib.AlnOut(*(out_t[k].data_ptr() for k in ("flag", "pos", "score", "n_cigar", "hits", "cigar")))
        _lib.check(self._ctx, _lib.lib().af_align_candidates_device(
            self._ctx, self._idx, reads_t.data_ptr(), int(n_pairs), int(stride),
            None if lens_t is None else lens_t.data_ptr(), ctypes.byref(self.params), ctypes.byref(self._pe(pair_base)),
            ctypes.byref(o), _stream_handle(stream)), "af_align_candidates_device")

    def align_candidates_tails_device(self, reads_t, n_pairs, stride, out_t, tails, lens_t=None, stream=None,
                                      pair_base=0):
        """align_candidates_device that also cuts the split-read tails in the pair-flag pass.
        tails: dict(tails=uint8 [cap, stride], lens=int32 [cap], read=int32 [cap], n=int32 [1],
        min_clip=20, read_base=0, append=False), as split_tails_device."""
        o = _lib.AlnOut(*(out_t[k].data_ptr() for k in ("flag", "pos", "score", "n_cigar", "hits", "cigar")))
        tt = tails["tails"]
        cap = int(tt.shape[0])
        if tt.shape[1] != stride or tails["lens"].numel() < cap or tails["read"].numel() < cap:
            raise ValueError("tails buffers: [cap, stride] bytes and cap lens / read entries")
        _lib.check(self._ctx, _lib.lib().af_align_candidates_tails_device(
            self._ctx, self._idx, reads_t.data_ptr(), int(n_pairs), int(stride),
            None if lens_t is None else lens_t.data_ptr(), ctypes.byref(self.params), ctypes.byref(self._pe(pair_base)),
            ctypes.byref(o), int(tails.get("min_clip", 20)), int(tails.get("read_base", 0)), int(bool(tails.get("append", False))), cap,
            tt.data_ptr(), tails["lens"].data_ptr(), tails["read"].data_ptr(), tails["n"].data_ptr(),
            _stream_handle(stream)), "af_align_candidates_tails_device")

    def seed_filter_device(self, reads_t, n_reads, stride, hits_t, lens_t=None, stream=None):
        sh = _stream_handle(stream)
        _lib.check(self._ctx, _lib.lib().af_seed_filter_device(
            self._ctx, self._idx, reads_t.data_ptr(), int(n_reads), int(stride),
            None if lens_t is None else lens_t.data_ptr(), hits_t.data_ptr(), sh), "af_seed_filter_device")

    def split_tails_device(self, reads_t, stride, out_t, tails_t, tail_lens_t, tail_read_t, n_tails_t,
                           min_clip=20, lens_t=None, stream=None, read_base=0, append=False):
        """af_split_tails_device over the records in out_t (rows of reads_t): the soft-clipped
        tails of split reads (CIGAR exactly M+S / S+M, clip >= min_clip) into tails_t
        (uint8 [cap, stride]), their lengths and read rows (+ read_base); *n_tails_t = number
        of split reads (may exceed cap), added to the current value when append=True.
        Asynchronous on stream; tail order varies between runs."""
        o = _lib.AlnOut(*(out_t[k].data_ptr() for k in ("flag", "pos", "score", "n_cigar", "hits", "cigar")))
        cap = int(tails_t.shape[0])
        if tail_lens_t.numel() < cap or tail_read_t.numel() < cap:
            raise ValueError("tail_lens_t / tail_read_t hold fewer than cap entries")
        if tails_t.shape[1] != stride:
            raise ValueError("tails_t rows must be `stride` bytes")
        _lib.check(self._ctx, _lib.lib().af_split_tails_device(
            self._ctx, reads_t.data_ptr(), int(reads_t.shape[0]), int(stride),
            None if lens_t is None else lens_t.data_ptr(), ctypes.byref(o), int(min_clip), int(read_base),
            int(bool(append)), cap, tails_t.data_ptr(),
            tail_lens_t.data_ptr(), tail_read_t.data_ptr(), n_tails_t.data_ptr(), _stream_handle(stream)),
            "af_split_tails_device")

    def partition_device(self, flag_t, pos_t, outs=None, stream=None):
        """S3 on the device (af_partition_device; AF:182 `samtools sort` + AF:186-194): read rows
        of tmp1 / tmp2 / anchored in samtools' coordinate order, as ``partition`` returns them.
        outs: optional (tmp1, tmp2, anchored, counts) device tensors to reuse (int32 [n_reads] x 3,
        int64 [3]).  Returns (tmp1, tmp2, anchored, counts); the first three are the full-size
        buffers, valid up to counts[k] (read counts with .cpu() when needed)."""
        import torch
        n = int(flag_t.numel())
        if pos_t.numel() != n:
            raise ValueError("flag and pos must have one entry per read")
        if outs is None:
            dev = flag_t.device
            outs = tuple(torch.empty(max(n, 1), dtype=torch.int32, device=dev) for _ in range(3)) + (
                torch.zeros(3, dtype=torch.int64, device=dev),)
        t1, t2, an, cnt = outs
        if min(t1.numel(), t2.numel(), an.numel()) < n or cnt.numel() < 3:
            raise ValueError("partition outputs need n_reads rows each and 3 counts")
        _lib.check(self._ctx, _lib.lib().af_partition_device(
            self._ctx, flag_t.data_ptr(), pos_t.data_ptr(), n, max(1, len(self.anchor)), t1.data_ptr(),
            t2.data_ptr(), an.data_ptr(), cnt.data_ptr(), _stream_handle(stream)), "af_partition_device")
        return t1, t2, an, cnt

    def gather_reads_device(self, reads_t, stride, rows_t, n_rows, mode, q_t, q_lens_t, q_rows_t=None, n_q_t=None,
                            out_t=None, lens_t=None, first=0, step=1, stream=None):
        """af_gather_reads_device: queries of the genome searches from an S3 row list (rows_t, the
        first n_rows entries; n_rows a host count).  mode _lib.AF_GATHER_SEQUENCED (S4's `samtools
        fastq`, AF:186-188) or _lib.AF_GATHER_SPLIT_SAM (S5's split reads, functions.py:705-716;
        out_t gives FLAG / CIGAR).  Query k goes to row first + k * step of q_t (uint8 [cap, stride]);
        n_q_t (int32 [1], optional) receives the slot count (the query count the genome calls and BLAT read on the device)."""
        cap = int(q_t.shape[0])
        if q_t.dim() != 2 or int(q_t.shape[1]) != int(stride) or q_lens_t.numel() < cap:
            raise ValueError("q_t must be [cap, stride] and q_lens_t hold cap entries")
        if q_rows_t is not None and q_rows_t.numel() < cap:
            raise ValueError("q_rows_t holds fewer than cap entries")
        if int(n_rows) > rows_t.numel():
            raise ValueError("n_rows exceeds the row list")
        o = None
        if out_t is not None:
            o = _lib.AlnOut(*(out_t[k].data_ptr() for k in ("flag", "pos", "score", "n_cigar", "hits", "cigar")))
        elif mode == _lib.AF_GATHER_SPLIT_SAM:
            raise ValueError("AF_GATHER_SPLIT_SAM needs out_t")
        _lib.check(self._ctx, _lib.lib().af_gather_reads_device(
            self._ctx, reads_t.data_ptr(), int(stride), None if lens_t is None else lens_t.data_ptr(),
            rows_t.data_ptr(), int(n_rows), int(mode), None if o is None else ctypes.byref(o), int(first), int(step),
            cap, q_t.data_ptr(), q_lens_t.data_ptr(), None if q_rows_t is None else q_rows_t.data_ptr(),
            None if n_q_t is None else n_q_t.data_ptr(), _stream_handle(stream)), "af_gather_reads_device")

    @property
    def ctx(self):
        """The raw af_ctx handle (e.g. for a search on this slot's stream)."""
        return self._ctx

    def last_candidates(self):
        return int(_lib.lib().af_last_candidates(self._ctx))


class AlignerGroup:
    """Several device-resident batches in flight on one GPU: one AnchorAligner context and one
    stream per batch slot.  ``run_device`` enqueues a group of batches so that their seed-filter
    launches (K1) run back to back and their alignment launches (K2 + K3) then run on all the
    slots' streams at once (see run_device): K2 is a persistent kernel whose waves leave one by one as the
    candidate queue drains, and the next batch's K2 waves take the CUs they free, so one K2's
    tail overlaps the next K2's body instead of idling the chip.  K1 (a whole CU's LDS per
    workgroup) cannot share a CU with K2 waves, so the next group's K1s wait for this group's
    K2s.  Records are those of ``AnchorAligner.align_pairs_device`` per batch."""

    def __init__(self, anchor: bytes, device: int = 0, inflight: int = 4, params=None):
        import torch
        if inflight < 1:
            raise ValueError("inflight must be >= 1")
        self.aligners = [AnchorAligner(anchor, device=device, params=params) for _ in range(inflight)]
        self.streams = [torch.cuda.Stream(torch.device("cuda", device)) for _ in range(inflight)]
        self.inflight = inflight

    def close(self):
        for a in self.aligners:
            a.close()

    def run_device(self, batches, events=None, wait=None, post=None, finish=None, tails=None, before=None):
        """batches: up to ``inflight`` tuples (reads_t, n_pairs, stride, out_t[, lens_t[, pair_base]])
        with every tensor on the device (pair_base: the batch's first pair in bwa's input stream).  Enqueues them and returns without synchronising.

        All K1s go to slot 0's stream, back to back (no cross-queue wait between them); batch
        j's K2 + K3 go to slot j's stream after one wait for the last K1.  wait (optional):
        events slot 0's stream waits for first (pass the previous group's return value when
        buffers or slots are reused).  events (optional): two timing events, recorded on slot
        0's stream before the first K1 and after the last.  post (optional): post(j, aligner,
        stream) enqueues more work for batch j after its K2 + K3; before (optional), the same
        signature, enqueues work ahead of batch j's K2 (after the group's K1s).  tails (optional): tails(j)
        gives batch j's split-read tails spec (align_candidates_tails_device), cut in its K3.
        finish (optional): finish(stream) enqueues work for the whole group on slot 0's
        stream once every batch is done (e.g. one placement launch over all the group's tails).
        Returns the events marking the group's completion."""
        import torch
        if len(batches) > self.inflight:
            raise ValueError(f"{len(batches)} batches for {self.inflight} slots")
        s0 = self.streams[0]
        for e in wait or ():
            s0.wait_event(e)
        if events is not None:
            events[0].record(s0)
        for j, b in enumerate(batches):
            reads_t, n_pairs, stride, out_t = b[:4]
            lens_t = b[4] if len(b) > 4 else None
            self.aligners[j].seed_filter_device(reads_t, 2 * n_pairs, stride, out_t["hits"], lens_t, stream=s0)
        if events is not None:
            events[1].record(s0)
        k1_done = torch.cuda.Event()
        k1_done.record(s0)
        done = []
        for j, b in enumerate(batches):
            s = self.streams[j]
            if j:
                s.wait_event(k1_done)
            reads_t, n_pairs, stride, out_t = b[:4]
            lens_t = b[4] if len(b) > 4 else None
            if before is not None:
                before(j, self.aligners[j], s)
            pb = b[5] if len(b) > 5 else 0
            if tails is not None:
                self.aligners[j].align_candidates_tails_device(reads_t, n_pairs, stride, out_t, tails(j), lens_t,
                                                               stream=s, pair_base=pb)
            else:
                self.aligners[j].align_candidates_device(reads_t, n_pairs, stride, out_t, lens_t, stream=s,
                                                         pair_base=pb)
            if post is not None:
                post(j, self.aligners[j], s)
            e = torch.cuda.Event()
            e.record(s)
            done.append(e)
        if finish is not None:
            for e in done[1:]:
                s0.wait_event(e)
            finish(s0)
            e = torch.cuda.Event()
            e.record(s0)
            done = [e]
        return done

    def join(self, done, stream=None):
        """Makes ``stream`` (default: torch's current stream) wait for a group's events."""
        import torch
        s = stream or torch.cuda.current_stream()
        for e in done:
            s.wait_event(e)


def chunk_ends(pair_bases, chunk_bases):
    """End (exclusive pair index) of each bwa input chunk: bseq_read stops after the pair that
    brings the chunk to >= chunk_bases bases (10,000,000 x threads).  The last entry is the
    input's end when the final chunk is short."""
    cum = np.cumsum(np.asarray(pair_bases, dtype=np.int64))
    ends, start, before = [], 0, 0
    n = len(cum)
    while start < n:
        e = int(np.searchsorted(cum, before + chunk_bases, side="left"))
        end = n if e >= n else e + 1
        ends.append(end)
        before = int(cum[end - 1])
        start = end
    return np.asarray(ends, dtype=np.int64)


def complete_chunks(pair_bases, chunk_bases):
    """Pairs in the complete bwa chunks at the start of ``pair_bases`` (the last chunk of a
    stream that may still grow is left out)."""
    cum = np.cumsum(np.asarray(pair_bases, dtype=np.int64))
    ends = chunk_ends(pair_bases, chunk_bases)
    cut, before = 0, 0
    for e in ends:
        if int(cum[e - 1]) - before < chunk_bases:
            break
        cut, before = int(e), int(cum[e - 1])
    return cut


def _concat_batches(batches):
    """(names, reads, lens) batches of io.iter_pairs joined into one (rows padded with N)."""
    from . import io as afio
    if len(batches) == 1:
        return batches[0]
    stride = max(r.shape[1] for _, r, _ in batches)
    reads = np.full((sum(r.shape[0] for _, r, _ in batches), stride), ord("N"), np.uint8)
    row = 0
    for _, r, _ in batches:
        reads[row:row + r.shape[0], :r.shape[1]] = r
        row += r.shape[0]
    return afio.Names.concat([b[0] for b in batches]), reads, np.concatenate([b[2] for b in batches])


def _stream_handle(stream):
    if stream is None:
        return None
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream


def partition(res: AlignResult):
    """S3 of Anchored_Fusion.py:183-194 on the records of ``res``.

    ``realign.bam`` is coordinate-sorted (``samtools sort``, AF:182): key (ref, pos, strand),
    unmapped-with-unmapped-mate last, ties in input order (pair, mate).  Returns read indices:
      tmp1      ``samtools view -f 8 -F 260``  mapped primary reads whose mate is unmapped (AF:186)
      tmp2      ``samtools view -f 4 -F 264``  unmapped reads whose mate is mapped (AF:187)
      anchored  ``samtools view -F 772``       mapped primary reads (AF:194)
    each in realign.bam order.
    """
    flag = res.flag
    pos = res.pos
    # samtools coordinate order: placed records by (pos, is_rev), ties in input order, then the
    # unplaced ones.  Every record the three filters keep is placed (a mapped read, or an
    # unmapped read carrying its mapped mate's position), so only the placed few % are sorted.
    placed = np.nonzero(pos >= 0)[0]
    key = pos[placed].astype(np.int64) * 2 + ((flag[placed] & 0x10) != 0)
    order = placed[np.argsort(key, kind="stable")]
    f = flag[order]
    tmp1 = order[((f & 0x8) != 0) & ((f & 260) == 0)]
    tmp2 = order[((f & 0x4) != 0) & ((f & 264) == 0)]
    anchored = order[(f & 772) == 0]
    return tmp1, tmp2, anchored
