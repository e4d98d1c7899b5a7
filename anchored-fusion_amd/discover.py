"""Candidate discovery over a read set resident in HBM: S2, S3 and the genome searches of the
partner stages, all on the device with no host round trip for the data.

| reference step | device work here |
|---|---|
| AF:182 `bwa mem -M anchor fq1 fq2` | K1 + K2 + K3 per batch (`AlignerGroup`), batches on bwa's chunk grid |
| AF:182 `\\| samtools sort`, AF:186-194 filters | `af_partition_device` over every record of the set |
| AF:186-188 `samtools fastq` + `bwa mem -M genome tmp1 tmp2` (S4) | `af_gather_reads_device` (SEQUENCED) + `af_genome_align_pe_device` |
| fn:705-716 split reads + `bwa mem -M genome` (S5) | `af_gather_reads_device` (SPLIT_SAM) + `af_genome_align_se_device` |
| fn:506-528 S6 FASTA (of every S5 query that can be kept) | `af_s6_queries_device` right after the gathers |
| fn:530 `blat -minScore=20 genome split.fa` (S6) | `af_blat_device_begin` on slot 1 beside S4 / S5, `_end` after the check |
| fn:718-768 genome check of the split reads | `af_s6_check_device` (live flags), `af_s6_compact_device` (survivors' rows) |

`run()` enqueues one pass; S3 synchronises twice (its select count sizes the sort; the partition
counts size the gathers) and the gathers once (the split-read count sizes S5).  Everything else
stays on the device: the records, the row lists, the queries, the genome calls' SAM records
(af_grec), the S6 queries and their PSL rows (dist_discover exchanges them between ranks over
RCCL, one process per GPU).  S6 runs beside S5: its queries depend only on the S2 records, so every
S5 query that can be kept is searched while S4 / S5 align, and S5's check then keeps the
survivors' rows (the heavy BLAT strands wait for the check: survivors only).
Per-call caps (query buffers, the genome calls' per-read caps) are counted in `summary()`.
"""
import os
import sys

from . import _lib
from . import blat as _blat
from . import genome as _genome
from .align import AlignerGroup, chunk_ends
from .shard import chunk_pairs

MAX_REC = _genome.MAX_REC
# S4 and S5 as two concurrent genome calls on two contexts (1) or one call whose seed / region
# launches cover both (0); bench A/B: AF_S4_SPLIT
_S4_SPLIT = os.environ.get("AF_S4_SPLIT", "1") == "1"
# S6 (BLAT) of every S5 query that can be kept, beside S5's genome call, compacted after the check
# (1), or of the check's survivors after it (0, round 4's order); bench A/B: AF_S6_EARLY
_S6_EARLY = os.environ.get("AF_S6_EARLY", "1") == "1"
# the early S6 search's heavy strands (af_blat_device_end) right behind its first part on slot 1,
# for every pre-check query (1), or after the check for its survivors only (0, the default: on
# configs[2] a query the check drops holds a 3,559-part strand whose serial chain DP costs
# 177 ms of step -- 428.8 vs 252.0 ms per step, profiles/r05/knobs_s6_heavy.txt)
# (experiment knob only: with it, the heavy strands of queries the check drops also spill their
# rows past MAX_ROWS into the shared pre-check pool, so a full pool can drop survivors' rows in
# atomic order -- afgpu.h's byte-for-byte equality holds for the default, end(live), only)
_S6_HEAVY_EARLY = os.environ.get("AF_S6_HEAVY_EARLY", "0") == "1"
_DEBUG = os.environ.get("AF_DEBUG_DISCOVER") == "1"


def _log(msg):
    print(f"[discover] {msg}", file=sys.stderr, flush=True)


class CandidateDiscovery:
    """S2 + S3 + S4/S5/S6 genome searches for `n_pairs` resident pairs, rows of `read_len` bytes.

    reference: genome.GenomeIndex (`bwa index` of the genome, HBM-resident, for the bwa calls); tiles:
    blat.TileReference of the same genome at BLAT's default step (S6).  pair_base: the set's first pair in
    bwa's input stream (a chunk boundary).  batch_chunks: bwa chunks per S2 batch; inflight:
    batches in flight (AlignerGroup).  pair_bases (optional, int [n_pairs]): the pairs' base counts
    when the reads are ragged (run() then takes their lengths); bwa's chunks are cut on them, and
    read_len (the row stride) must be a multiple of 8 so that every batch starts on a 16-byte
    boundary."""

    def __init__(self, anchor: bytes, reference, tiles, n_pairs, read_len, device=0, inflight=8, batch_chunks=30,
                 pair_base=0, chunk_bases=10_000_000, query_frac=0.004, pair_bases=None):
        self.chunk_bases = int(chunk_bases)
        import numpy as np
        import torch
        self.dev = torch.device("cuda", device)
        self.anchor, self.ref, self.tiles_ref = bytes(anchor), reference, tiles
        self.n_pairs, self.L, self.pair_base = int(n_pairs), int(read_len), int(pair_base)
        if pair_bases is None:
            pc = chunk_pairs(self.L, chunk_bases)
            if self.pair_base % pc:
                raise ValueError("pair_base must be on bwa's chunk grid")
            # batches start on 16-byte boundaries of reads_t (the seed filter's vector loads): a
            # whole number of chunks whose bytes are a multiple of 16
            m = 1
            while (m * pc * 2 * self.L) % 16:
                m += 1
            bp = pc * m * max(1, -(-int(batch_chunks) // m))
            self.batches = [(p, min(bp, self.n_pairs - p)) for p in range(0, self.n_pairs, bp)]
        else:
            if self.L % 8:
                raise ValueError("ragged reads: the row stride must be a multiple of 8")
            ends = chunk_ends(np.asarray(pair_bases, dtype=np.int64), chunk_bases)
            bc = max(1, int(batch_chunks))
            starts = [0] + [int(ends[k - 1]) for k in range(bc, len(ends), bc)]
            self.batches = [(a, b - a) for a, b in zip(starts, starts[1:] + [self.n_pairs]) if b > a]
        self.grp = AlignerGroup(self.anchor, device=device, inflight=inflight)
        for a in self.grp.aligners:
            a.pe.chunk_bases = chunk_bases
        nr = 2 * self.n_pairs
        z = lambda *shape, dt=torch.int32: torch.zeros(shape, dtype=dt, device=self.dev)  # noqa: E731
        self.out = {k: z(max(nr, 1)) for k in ("flag", "pos", "score", "n_cigar", "hits")}
        self.out["cigar"] = z(max(nr, 1), _lib.AF_MAX_CIGAR)
        self.s3 = (z(max(nr, 1)), z(max(nr, 1)), z(max(nr, 1)), z(3, dt=torch.int64))
        # the S4 + S5 queries, their SAM records, and the S6 queries (S5's survivors) with their rows
        self.n_q = z(1)
        self._alloc_queries(max(4096, int(nr * query_frac)))
        self.p_genome = _lib.default_params()  # bwa mem defaults (-k 19 -T 30), AF:188 / fn:716
        self.p_tail = _blat.params("split_tail")
        self.counts = None   # host (tmp1, tmp2, anchored, S4 pairs, S5 split reads) after run()
        self._npair = 0

    def _alloc_queries(self, cap):
        """The query buffers (S4 + S5 queries and their records) for cap queries; run() grows them
        when S3's counts need more."""
        import torch
        z = lambda *shape, dt=torch.int32: torch.zeros(shape, dtype=dt, device=self.dev)  # noqa: E731
        self.qcap = int(cap)
        self.q = z(self.qcap, self.L, dt=torch.uint8)
        self.q_lens, self.q_rows = z(self.qcap), z(self.qcap)
        self.q_recs = z(self.qcap * MAX_REC * _genome.REC_DTYPE.itemsize, dt=torch.uint8)
        self.q_nh = z(self.qcap)   # SAM records per query
        if getattr(self, "s6cap", 0) == 0:
            self._alloc_s6(4096)

    def _alloc_s6(self, cap):
        """The S6 rows for cap S5 queries, twice: `s6p` before the genome check (every QNAME-group
        leader's row, searched beside S5) and the survivors' (`s6`, `t_rows`, `t_nh`, `t_spill`:
        what the consumers read), each with its PSL rows and a spill pool for the rows past MAX_ROWS
        (BLAT prints them all; fn:630-649 reads every one); the pre set also counts its cap events
        per query, so that the summary counts the survivors' only."""
        import torch
        z = lambda *shape, dt=torch.int32: torch.zeros(shape, dtype=dt, device=self.dev)  # noqa: E731
        self.s6cap = int(cap)
        spill_cap = max(getattr(self, "spill_min", 1 << 16), self.s6cap // 2)
        psl = _blat.PSL_DTYPE.itemsize

        def rows_set():
            return dict(q=z(self.s6cap, _lib.AF_MAX_READ, dt=torch.uint8), lens=z(self.s6cap), src=z(self.s6cap), n=z(1),
                        rows=z(self.s6cap * _blat.MAX_ROWS * psl, dt=torch.uint8), n_rows=z(self.s6cap),
                        spill_rows=z(spill_cap * psl, dt=torch.uint8), spill_q=z(spill_cap), spill_n=z(1))
        self.s6p = rows_set()
        self.s6p.update(over=z(self.s6cap, dt=torch.uint8), caps=z(len(_blat.CAP_NAMES) * self.s6cap),
                        live=z(self.s6cap, dt=torch.uint8))
        f = rows_set()
        f["n_over"] = z(1)
        self.s6f = f
        # the survivors' set under the names the consumers read
        self.s6 = dict(q=f["q"], lens=f["lens"], src=f["src"], n=f["n"], over=f["n_over"])
        self.t_rows, self.t_nh = f["rows"], f["n_rows"]
        self.t_spill = dict(rows=f["spill_rows"], q=f["spill_q"], n=f["spill_n"])

    def _s6_pre(self, b, n5, stream, cont_t=None):
        """The S6 query rows of the S5 queries [b, b + n5) that lead a QNAME group (fn:506-528 on
        the rows the check can keep), before the check runs."""
        if n5 > self.s6cap:
            self._alloc_s6(int(n5 * 1.25) + 1024)
        _genome.s6_queries_device(self.tiles_ref.ctx, n5, self.q[b:], self.L, self.q_lens[b:], self.q_rows[b:],
                                  self.out, self.s6p, stream=stream, cont_t=cont_t)

    def _s6_search(self, stream):
        """S6 (`blat -minScore=20 genome split.fa`, fn:530) of the pre-check rows, its first part
        (af_blat_device_begin: every strand but the heavy ones searched; _s6_finish completes it for
        the survivors): MAX_ROWS per query in their row slots, the rest in their spill pool, cap
        events per query (registered for this search only: the tile reference may serve others)."""
        import torch
        sp = self.s6p
        with torch.cuda.stream(stream):
            sp["spill_n"].zero_()
            sp["caps"].zero_()
        self.tiles_ref.spill_to(sp["spill_rows"], sp["spill_q"], sp["spill_n"])
        self.tiles_ref.query_caps_to(sp["caps"], self.s6cap)
        try:
            self.tiles_ref.search_device_begin(sp["q"], sp["n"], _lib.AF_MAX_READ, sp["rows"], sp["n_rows"],
                                               lens_t=sp["lens"], p=self.p_tail, stream=stream)
            if _S6_HEAVY_EARLY:
                self.tiles_ref.search_device_end(None, stream=stream)
        finally:
            self.tiles_ref.spill_to()
            self.tiles_ref.query_caps_to()

    def _s6_check(self, b, n5, recs, stream, cont_t=None):
        """S5's genome check (fn:718-768) of the queries [b, b + n5): the pre rows' live flags."""
        w = MAX_REC * _genome.REC_DTYPE.itemsize // 4
        _genome.s6_check_device(self.tiles_ref.ctx, recs[b * w:], self.q_nh[b:], n5, self.q_rows[b:], self.out,
                                self.s6p, self.s6p["live"], stream=stream, cont_t=cont_t)

    def _s6_finish(self, stream):
        """The rest of the S6 search for the survivors (af_blat_device_end), then their S6 rows and
        BLAT rows compacted and renumbered in query order."""
        if not _S6_HEAVY_EARLY:
            self.tiles_ref.search_device_end(self.s6p["live"], stream=stream)
        _genome.s6_compact_device(self.tiles_ref.ctx, self.s6p, self.s6p["live"], self.s6f, stream=stream)

    def _s6_late(self, b, n5, recs, s0, s6, cont_t=None):
        """Round 4's order: S5's genome check and its survivors' S6 rows (af_s5_filter_device), then
        their BLAT on slot 1's stream."""
        import torch
        w = MAX_REC * _genome.REC_DTYPE.itemsize // 4
        if n5 > self.s6cap:
            self._alloc_s6(int(n5 * 1.25) + 1024)
        f = self.s6f
        _genome.s5_filter_device(self.ref.ctx, recs[b * w:], self.q_nh[b:], n5, self.q[b:], self.L, self.q_lens[b:],
                                 self.q_rows[b:], self.out, self.s6cap, f["q"], f["lens"], f["src"], f["n"],
                                 f["n_over"], stream=s0, cont_t=cont_t)
        s6.wait_stream(s0)
        with torch.cuda.stream(s6):
            f["spill_n"].zero_()
        self.tiles_ref.spill_to(f["spill_rows"], f["spill_q"], f["spill_n"])
        try:
            self.tiles_ref.search_device(f["q"], f["n"], _lib.AF_MAX_READ, f["rows"], f["n_rows"], lens_t=f["lens"],
                                         p=self.p_tail, stream=s6)
        finally:
            self.tiles_ref.spill_to()
        s0.wait_stream(s6)

    def s6_spilled(self):
        """{S6 query: [its rows past MAX_ROWS]} of the last search, in row order (synchronises)."""
        import torch
        torch.cuda.synchronize(self.dev)
        sp = self.t_spill
        n = min(int(sp["n"].item()), int(sp["q"].numel()))
        rows = sp["rows"][:n * _blat.PSL_DTYPE.itemsize].cpu().numpy().view(_blat.PSL_DTYPE)
        return _blat.spilled_rows(rows, sp["q"][:n].cpu().numpy())

    def _s4_ctx(self):
        """A second context for S4's genome call (its own pools and scratch; the index is shared)."""
        if getattr(self, "_ctx4", None) is None:
            import ctypes
            c = ctypes.c_void_p()
            _lib.check(None, _lib.lib().af_ctx_create(int(self.dev.index or 0), ctypes.byref(c)), "af_ctx_create")
            self._ctx4 = c
        return self._ctx4

    def close(self):
        self.grp.close()
        if getattr(self, "_ctx4", None) is not None:
            _lib.lib().af_ctx_destroy(self._ctx4)
            self._ctx4 = None

    def run(self, reads_t, k1_events=None, phase_events=None, lens_t=None):
        """One pass over reads_t (uint8 [2 n_pairs, read_len] on the device; lens_t: int32 [2 n_pairs]
        read lengths, or None when every read is read_len long).  k1_events: per group a pair of
        timing events around its K1 launches; phase_events: 4 events recorded on the first slot's
        stream after S2, S3, the gathers and the genome searches."""
        import torch
        G = self.grp.inflight
        s0 = self._s2(reads_t, lens_t, k1_events)
        # S6 runs on slot 1's stream (the tile index has its own context and scratch; slot 1 is
        # idle once S2 is done -- a stream of its own would share one of the 4 hardware queues
        # (GPU_MAX_HW_QUEUES) with a slot and serialise behind its S2 work) beside S4.
        s6 = self.grp.streams[1] if G > 1 else s0
        if _DEBUG:
            s0.synchronize()
            _log("S2 done")
        if phase_events:
            phase_events[0].record(s0)
        # S3: samtools sort + the three flag filters over every record
        al = self.grp.aligners[0]
        t1, t2, an, cnt = al.partition_device(self.out["flag"], self.out["pos"], outs=self.s3, stream=s0)
        if phase_events:
            phase_events[1].record(s0)
        s0.synchronize()
        n1, n2, na = (int(v) for v in cnt.cpu())
        if _DEBUG:
            _log(f"S3 done: tmp1 {n1}, tmp2 {n2}, anchored {na}")
        # S4 queries: tmp1 / tmp2 interleaved as bwa pairs its two FASTQs; S5: anchored split reads
        # (the buffers grow to S3's counts: at most 2 min(tmp1, tmp2) + anchored queries)
        need = 2 * min(n1, n2) + na
        if need > self.qcap:
            self._alloc_queries(int(need * 1.25) + 1024)
        npair = min(n1, n2, self.qcap // 2)
        al.gather_reads_device(reads_t, self.L, t1, npair, _lib.AF_GATHER_SEQUENCED, self.q, self.q_lens,
                               self.q_rows, None, lens_t=lens_t, first=0, step=2, stream=s0)
        al.gather_reads_device(reads_t, self.L, t2, npair, _lib.AF_GATHER_SEQUENCED, self.q, self.q_lens,
                               self.q_rows, self.n_q, lens_t=lens_t, first=1, step=2, stream=s0)
        al.gather_reads_device(reads_t, self.L, an, na, _lib.AF_GATHER_SPLIT_SAM, self.q, self.q_lens, self.q_rows,
                               self.n_q, out_t=self.out, lens_t=lens_t, first=2 * npair, step=1, stream=s0)
        if phase_events:
            phase_events[2].record(s0)
        s0.synchronize()   # the split-read count sizes S5
        nq_all = int(self.n_q.item())
        nq = min(nq_all, self.qcap)
        n5 = max(0, nq - 2 * npair)
        pe = _lib.default_pe(chunk_bases=self.chunk_bases, pair_base=0)
        recs = self.q_recs.view(torch.int32)
        w = MAX_REC * _genome.REC_DTYPE.itemsize // 4
        b = 2 * npair
        # S6's queries depend only on the S2 records (fn:506-528: deal_cigar's SEQ of the anchored
        # record); the genome check only decides which are kept.  So the rows of every query that
        # can be kept are written now and searched (fn:530) on slot 1's stream beside S4 / S5, and
        # compacted to the survivors once the check has run.
        if _S6_EARLY:
            self._s6_pre(b, n5, s0)
            s6.wait_stream(s0)
            self._s6_search(s6)
        # S4 (`bwa mem -M genome tmp1 tmp2`, AF:188: bwa's chunks over this input) and S5 (`bwa mem
        # -M genome split_reads.fa`, fn:716); S5's records on s0, S4's on slot 2's stream (idle
        # once S2 is done).  (Enqueued after S6's BLAT: enqueueing them first, so that their seed
        # kernels take the chip before k_blat's persistent grid, measured 222 vs 212 ms per step.)
        spe = self.grp.streams[2] if G > 2 else s0
        spe.wait_stream(s0)
        if _S4_SPLIT and spe is not s0:
            # S4's whole call on a second context of the same index, on its own stream, beside
            # S5's (each has its own seed / region launches, pools and scratch): S4's records
            # start once its 2 npair reads are seeded instead of after every read of both calls
            if npair:
                self.ref.align_pe_device(self.q, npair, self.L, self.q_lens, recs, self.q_nh, params=self.p_genome,
                                         pe=pe, stream=spe, ctx=self._s4_ctx())
            if n5:
                self.ref.align_se_device(self.q[b:], n5, self.L, recs[b * w:], self.q_nh[b:],
                                         lens_t=self.q_lens[b:], params=self.p_genome, pe=pe, id_base=0,
                                         stream=s0)
        elif npair or n5:
            self.ref.align_pe_se_device(self.q, npair, n5, self.L, self.q_lens, recs, self.q_nh,
                                        params=self.p_genome, pe_s4=pe, pe_s5=pe, se_id_base=0, stream=s0,
                                        stream_pe=spe)
        # S5's genome check (fn:718-768), then the rest of S6 (the survivors' heavy strands) and the
        # survivors' rows
        if _S6_EARLY:
            self._s6_check(b, n5, recs, s0)
            s0.wait_stream(s6)
            self._s6_finish(s0)
        else:
            self._s6_late(b, n5, recs, s0, s6)
        s0.wait_stream(spe)
        if _DEBUG:
            s0.synchronize()
            _log("genome calls done")
        if phase_events:
            phase_events[3].record(s0)
        self.counts = dict(tmp1=n1, tmp2=n2, anchored=na, s4_pairs=npair, s5_split_reads=n5,
                           s4_pairs_dropped=max(0, min(n1, n2) - npair), s5_dropped=max(0, nq_all - nq))
        self._npair = npair
        self._s4_ctx_used = bool(_S4_SPLIT and spe is not s0 and npair)
        return s0

    def _s2(self, reads_t, lens_t=None, k1_events=None):
        """S2 over every batch (K1s of a group back to back, then their K2 + K3 on the slots);
        returns slot 0's stream, which waits for all of it."""
        G = self.grp.inflight
        s0 = self.grp.streams[0]
        done = None
        for gi, k0 in enumerate(range(0, len(self.batches), G)):
            group = self.batches[k0:k0 + G]
            specs = []
            for p, n in group:
                r0, r1 = 2 * p, 2 * (p + n)
                specs.append((reads_t[r0:r1], n, self.L, {k: v[r0:r1] for k, v in self.out.items()},
                              None if lens_t is None else lens_t[r0:r1], self.pair_base + p))
            done = self.grp.run_device(specs, events=None if k1_events is None else k1_events[gi], wait=done)
        for e in done or ():
            s0.wait_event(e)
        return s0

    # ---- one rank of a sharded sample: the phases dist_discover drives --------------------------
    def attach(self, reads_t, lens_t=None, k1_events=None):
        """The reads (this rank's whole chunks, pairs pair_base ..) the phases below run on;
        k1_events as run() takes them."""
        self._in = (reads_t, lens_t, k1_events)
        return self

    def local_phase(self):
        """S2 + S3 + the gathers of this rank: tmp1 reads at query rows [0, n1), tmp2 at [n1, n1 +
        n2) (both as sequenced), the split reads (S5 queries, SAM orientation) after them."""
        import torch

        from .dist_discover import LocalQueries
        reads_t, lens_t, k1_events = self._in
        s0 = self._s2(reads_t, lens_t, k1_events)
        al = self.grp.aligners[0]
        t1, t2, an, cnt = al.partition_device(self.out["flag"], self.out["pos"], outs=self.s3, stream=s0)
        s0.synchronize()
        n1, n2, na = (int(v) for v in cnt.cpu())
        if n1 + n2 + na > self.qcap:
            self._alloc_queries(int((n1 + n2 + na) * 1.25) + 1024)
        al.gather_reads_device(reads_t, self.L, t1, n1, _lib.AF_GATHER_SEQUENCED, self.q, self.q_lens, self.q_rows,
                               None, lens_t=lens_t, first=0, step=1, stream=s0)
        al.gather_reads_device(reads_t, self.L, t2, n2, _lib.AF_GATHER_SEQUENCED, self.q, self.q_lens, self.q_rows,
                               None, lens_t=lens_t, first=n1, step=1, stream=s0)
        al.gather_reads_device(reads_t, self.L, an, na, _lib.AF_GATHER_SPLIT_SAM, self.q, self.q_lens, self.q_rows,
                               self.n_q, out_t=self.out, lens_t=lens_t, first=n1 + n2, step=1, stream=s0)
        s0.synchronize()
        b = n1 + n2
        n5 = max(0, min(int(self.n_q.item()), self.qcap) - b)
        self._lay = (n1, n2, n5)
        # the lists stay in HBM (dist_discover exchanges them over RCCL)
        rows = self.q_rows[:b + n5].long()
        pos = self.out["pos"][rows]
        key = pos.long() * 2 + ((self.out["flag"][rows] >> 4) & 1).long()
        seq, ql = self.q[:b + n5], self.q_lens[:b + n5]
        self.counts = dict(tmp1=n1, tmp2=n2, anchored=na, s5_split_reads=n5)
        return LocalQueries(
            dict(key=key[:n1], row=rows[:n1], seq=seq[:n1], len=ql[:n1]),
            dict(key=key[n1:b], row=rows[n1:b], seq=seq[n1:b], len=ql[n1:b]),
            dict(key=key[b:], row=rows[b:], pos=pos[b:], ncig=self.out["n_cigar"][rows[b:]],
                 cigar=self.out["cigar"][rows[b:]], seq=seq[b:], len=ql[b:]))

    def s5_s6_phase(self, ids, cont):
        """S5 with the queries' global ids, its genome check with the given QNAME groups, S6."""
        import torch
        n1, n2, n5 = self._lay
        b = n1 + n2
        s0 = self.grp.streams[0]
        pe = _lib.default_pe(chunk_bases=self.chunk_bases, pair_base=0)
        recs = self.q_recs.view(torch.int32)
        w = MAX_REC * _genome.REC_DTYPE.itemsize // 4
        ids_t = ids.to(self.dev, torch.int64).contiguous()
        cont_t = cont.to(self.dev, torch.uint8).contiguous()
        s0.wait_stream(torch.cuda.current_stream(self.dev))  # ids / cont were made on the current stream
        # S6's rows before the check, searched on slot 1's stream beside S5 (as in run())
        s6 = self.grp.streams[1] if self.grp.inflight > 1 else s0
        if _S6_EARLY:
            self._s6_pre(b, n5, s0, cont_t=cont_t)
            s6.wait_stream(s0)
            self._s6_search(s6)
        if n5:
            self.ref.align_se_ids_device(self.q[b:], n5, self.L, ids_t, recs[b * w:], self.q_nh[b:],
                                         lens_t=self.q_lens[b:], params=self.p_genome, pe=pe, stream=s0)
        if _S6_EARLY:
            self._s6_check(b, n5, recs, s0, cont_t=cont_t)
            s0.wait_stream(s6)
            self._s6_finish(s0)
        else:
            self._s6_late(b, n5, recs, s0, s6, cont_t=cont_t)
        s0.synchronize()
        n6 = int(self.s6["n"].item())
        self.counts["s6_queries"] = n6
        ns = min(int(self.t_spill["n"].item()), int(self.t_spill["q"].numel()))
        return dict(src=self.s6["src"][:n6], s6_seq=self.s6["q"][:n6], s6_len=self.s6["lens"][:n6],
                    psl=self.t_rows[:n6 * _blat.MAX_ROWS * _blat.PSL_DTYPE.itemsize].view(torch.int32),
                    n_psl=self.t_nh[:n6],
                    spill_psl=self.t_spill["rows"][:ns * _blat.PSL_DTYPE.itemsize].view(torch.int32),
                    spill_q=self.t_spill["q"][:ns])

    def s4_phase(self, q, ql, pair_base=0):
        """S4 over whole bwa chunks of the globally zipped pairs: reads q uint8 [2P, w] pair-major,
        lens ql; pair_base = the first pair's index in that stream (read ids, chunk grid)."""
        import torch
        P2 = int(q.shape[0])
        qt = q.to(self.dev, torch.uint8).contiguous()
        lt = ql.to(self.dev, torch.int32).contiguous()
        words = _genome.REC_DTYPE.itemsize // 4
        recs_t = torch.zeros((P2, MAX_REC, words), dtype=torch.int32, device=self.dev)
        nrec_t = torch.zeros(P2, dtype=torch.int32, device=self.dev)
        s0 = self.grp.streams[0]
        s0.wait_stream(torch.cuda.current_stream(self.dev))  # q / ql were made on the current stream
        self.ref.align_pe_device(qt, P2 // 2, int(qt.shape[1]), lt, recs_t, nrec_t, params=self.p_genome,
                                 pe=_lib.default_pe(chunk_bases=self.chunk_bases, pair_base=int(pair_base)), stream=s0)
        s0.synchronize()
        return recs_t, nrec_t

    def psl_lines(self, queries, rows, nrows, extra=None):
        return _blat.psl_lines(self.tiles_ref, queries, rows, nrows, extra=extra)

    def summary(self):
        """Host-side counts of the last pass (synchronises)."""
        import torch
        torch.cuda.synchronize(self.dev)
        nq = min(int(self.n_q.item()), self.qcap)
        n6 = int(self.s6["n"].item())
        tn = self.t_nh[:n6].cpu().numpy()
        rec = self.q_recs[:nq * MAX_REC * _genome.REC_DTYPE.itemsize].cpu().numpy().view(_genome.REC_DTYPE)
        rec = rec.reshape(nq, MAX_REC)
        first = rec[:, 0]["flag"] if nq else rec
        c = dict(self.counts or {})
        c.update(queries_s4_s5=nq, queries_placed=int(((first & 4) == 0).sum()) if nq else 0,
                 genome_records=int(self.q_nh[:nq].sum().item()), s6_queries=n6,
                 s6_placed=int((tn > 0).sum()), s6_at_row_cap=int((tn >= _blat.MAX_ROWS).sum()),
                 s6_rows_spilled=int(self.t_spill["n"].item()),
                 s6_clipped=int(self.s6["over"].item()),
                 mapped_reads=int(((self.out["flag"] & 4) == 0).sum().item()),
                 s2_overflow_reads=int(((self.out["flag"] & (_lib.AF_FLAG_MEM_OVERFLOW | _lib.AF_FLAG_CIGAR_OVERFLOW))
                                        != 0).sum().item()))
        gs = self.ref.stats()
        if getattr(self, "_ctx4", None) is not None and getattr(self, "_s4_ctx_used", False):
            # S4's call on its own context, when this pass made one (its counters are the last call's)
            for k, v in self.ref.stats(ctx=self._ctx4).items():
                gs[k] += v
        c.update({f"genome_{k}": v for k, v in gs.items()})
        c.update({f"blat_cap_{k}": v for k, v in self.tiles_ref.caps().items()})
        return c

    def s6_best_hits(self):
        """(read rows, row counts, best BLAT row per S6 query) of the last pass, on the host (synchronises)."""
        import torch
        torch.cuda.synchronize(self.dev)
        n6 = int(self.s6["n"].item())
        rows = self.t_rows[:n6 * _blat.MAX_ROWS * _blat.PSL_DTYPE.itemsize].cpu().numpy().view(_blat.PSL_DTYPE)
        src = self.s6["src"][:n6].long()
        read = self.q_rows[self._npair * 2:][src] if n6 else self.s6["src"][:0]
        return (read.cpu().numpy(), self.t_nh[:n6].cpu().numpy(),
                rows.reshape(n6, _blat.MAX_ROWS)[:, 0] if n6 else rows)
