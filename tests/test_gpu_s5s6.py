"""The genome check of the split reads and the S6 queries on the device (csrc/s5s6.hip,
af_s5_filter_device) against the host restatements the consumer stages use: genome_check
(`del_too_many_reads`, functions.py:705-768) over the SAM text of the same genome records, then
blocks.split_read_queries (`Find_fine_block`'s FASTA, fn:506-528).  Bit-exact: the survivors,
their order and deal_cigar's processed sequences.

World: tests/genome_world.py's repeat-rich genome; the anchor is three exons of chr1 joined;
pairs come from fusion transcripts (anchor exons + a partner segment elsewhere, some inside
Alu-like repeats) and from the anchor's own genomic locus (exon + intron: split on the anchor,
one operation on the genome -- the fn:749-751 drop), with substitutions and small indels (D / I
inside the anchored CIGAR exercise deal_cigar's sequence edits)."""
import numpy as np
import pytest

import afpkg  # noqa: F401
from genome_world import _mutate, _rc, make_genome

pytestmark = pytest.mark.gpu

EXONS = [(100_000, 100_300), (101_000, 101_250), (102_000, 102_400)]


def _indel(rng, s):
    i = int(rng.integers(40, len(s) - 40))
    if rng.random() < 0.5:
        return np.concatenate([s[:i], np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, int(rng.integers(1, 4)))],
                               s[i:]])
    return np.concatenate([s[:i], s[i + int(rng.integers(1, 4)):]])


def _world(n_pairs=3000, L=150, seed=31):
    contigs = make_genome()
    g = {n: np.frombuffer(s, np.uint8) for n, s in contigs}
    chr1 = g["chr1"]
    anchor = np.concatenate([chr1[a:b] for a, b in EXONS])
    rng = np.random.default_rng(seed)
    partners = []
    for k in range(12):
        c = ("chr2", "chr3")[k % 2]
        p = int(rng.integers(5_000, len(g[c]) - 5_000))
        partners.append(g[c][p:p + 600])
    locus = chr1[EXONS[0][0] - 400:EXONS[-1][1] + 400]  # the anchor gene with introns and flanks
    reads = np.zeros((2 * n_pairs, L), np.uint8)
    for i in range(n_pairs):
        u = rng.random()
        if u < 0.6:  # fusion: anchor[:a] + partner
            a = int(rng.integers(60, len(anchor) - 10))
            t = np.concatenate([anchor[:a], partners[int(rng.integers(0, len(partners)))]])
            j = int(rng.integers(max(0, a - 260), a - 20))
        elif u < 0.85:  # the anchor's genomic locus (crosses exon ends into introns)
            t, j = locus, int(rng.integers(0, len(locus) - 300))
        else:  # the anchor transcript itself
            t, j = anchor, int(rng.integers(0, len(anchor) - 300))
        f = t[j:j + 300]
        m1, m2 = _mutate(rng, f[:L], 0.01), _mutate(rng, _rc(f[-L:]), 0.01)
        if rng.random() < 0.25:
            m1 = _indel(rng, m1)
        m1 = np.resize(m1, L) if len(m1) >= L else np.concatenate([m1, np.full(L - len(m1), ord("A"), np.uint8)])
        if rng.random() < 0.5:
            m1, m2 = m2, m1
        reads[2 * i], reads[2 * i + 1] = m1, m2
    return contigs, anchor.tobytes(), reads


def host_s5_s6(reads, h, an_rows, rec_h, nrec_h, genome_names, gene="ANCHOR"):
    """The host chain over the same records: anchored.bam lines (pipeline.sam_line, read names
    r<pair>) -> genome_check.split_read_fasta -> the genome SAM text of the af_grec records
    (genome.sam_lines) -> genome_check.filter_genome_hits -> blocks.split_read_queries.
    Returns (S5 FASTA, split_sam lines, S6 FASTA)."""
    from anchored_fusion_amd import blocks, genome, genome_check
    from anchored_fusion_amd.align import AlignResult
    from anchored_fusion_amd.cigar import revcomp
    from anchored_fusion_amd.pipeline import sam_line
    res = AlignResult(h["flag"], h["pos"], h["score"], h["n_cigar"], h["cigar"].view(np.uint32), h["hits"])
    lines = []
    for r in an_rows:
        s = reads[r].tobytes().decode()
        f = int(h["flag"][r])
        lines.append(sam_line(f"r{r // 2}", f & 0xFFFF, gene, int(h["pos"][r]) + 1, res.cigar_str(r),
                              revcomp(s) if f & 0x10 else s))
    fasta = genome_check.split_read_fasta(lines)
    gsam = ["@HD\tVN:1.6\n"]
    for i, (name, sq) in enumerate(fasta):
        gsam += genome.sam_lines(genome_names, name, sq, rec_h[i], nrec_h[i])
    split_sam = genome_check.filter_genome_hits(gsam)
    _, s6_fa = blocks.split_read_queries(split_sam)
    return fasta, split_sam, s6_fa


def test_s5_check_and_s6_rows_equal_host():
    import torch

    from anchored_fusion_amd import _lib, genome
    from anchored_fusion_amd.align import AnchorAligner
    contigs, anchor, reads = _world()
    N, L = reads.shape[0] // 2, reads.shape[1]
    dev = torch.device("cuda:0")
    al = AnchorAligner(anchor, device=0)
    gi = genome.GenomeIndex(contigs, device=0)
    try:
        reads_t = torch.from_numpy(reads).to(dev)
        z = lambda *sh, dt=torch.int32: torch.zeros(sh, dtype=dt, device=dev)  # noqa: E731
        out = {k: z(2 * N) for k in ("flag", "pos", "score", "n_cigar", "hits")}
        out["cigar"] = z(2 * N, 32)
        al.align_pairs_device(reads_t, N, L, out)
        t1, t2, an, cnt = al.partition_device(out["flag"], out["pos"])
        na = int(cnt.cpu()[2])
        cap = 2 * N
        q, q_lens, q_rows, n_q = z(cap, L, dt=torch.uint8), z(cap), z(cap), z(1)
        al.gather_reads_device(reads_t, L, an, na, _lib.AF_GATHER_SPLIT_SAM, q, q_lens, q_rows, n_q, out_t=out)
        torch.cuda.synchronize()
        n5 = int(n_q.item())
        recs = z(cap * genome.MAX_REC * genome.REC_DTYPE.itemsize // 4)
        nrec = z(cap)
        gi.align_se_device(q, n5, L, recs, nrec, lens_t=q_lens)
        s6, s6_lens, s6_src, n6 = z(cap, _lib.AF_MAX_READ, dt=torch.uint8), z(cap), z(cap), z(1)
        genome.s5_filter_device(gi.ctx, recs, nrec, n5, q, L, q_lens, q_rows, out, cap, s6, s6_lens, s6_src, n6)
        torch.cuda.synchronize()
        # host: anchored.bam lines -> split-read FASTA -> genome SAM -> filter -> S6 FASTA
        h = {k: v.cpu().numpy() for k, v in out.items()}
        rec_h = recs.cpu().numpy().view(genome.REC_DTYPE)[:n5 * genome.MAX_REC].reshape(n5, genome.MAX_REC)
        fasta, split_sam, s6_fa = host_s5_s6(reads, h, an[:na].cpu().numpy(), rec_h, nrec[:n5].cpu().numpy(),
                                             gi.names)
        assert len(fasta) == n5 > 100
        qh, ql = q[:n5].cpu().numpy(), q_lens[:n5].cpu().numpy()
        assert all(qh[i, :ql[i]].tobytes().decode() == fasta[i][1] for i in range(n5))
        k6 = int(n6.item())
        assert k6 == len(split_sam) == len(s6_fa)
        assert 20 < k6 < n5, (k6, n5)  # both drop rules and survivors exercised
        rows, lens, src = s6[:k6].cpu().numpy(), s6_lens[:k6].cpu().numpy(), s6_src[:k6].cpu().numpy()
        for k in range(k6):
            assert split_sam[k].split("\t")[0] == fasta[src[k]][0].split("$")[0]
            assert lens[k] == len(s6_fa[k][1]) and rows[k, :lens[k]].tobytes().decode() == s6_fa[k][1], k
        # deal_cigar's sequence edits happened on some survivors (D -> N)
        assert any("D" in fasta[src[k]][0].split("$")[3] or "I" in fasta[src[k]][0].split("$")[3] for k in range(k6))
    finally:
        gi.close()
        al.close()


def test_s6_before_check_then_compact_equals_sequential():
    """af_s6_queries_device + af_blat_device_begin + af_s6_check_device + af_blat_device_end +
    af_s6_compact_device (S6 searched beside S5, discover.run) equals af_s5_filter_device + BLAT of
    its survivors byte for byte: the S6 rows, their S5 query
    index, the PSL rows (query field renumbered) and row counts, the spilled rows (max_rows 16:
    repeat-derived queries pass it), the clipped-row count and the cap counters."""
    import torch

    from anchored_fusion_amd import _lib, blat, genome
    from anchored_fusion_amd.align import AnchorAligner
    from anchored_fusion_amd.discover import CandidateDiscovery
    contigs, anchor, reads = _world(n_pairs=2000, seed=37)
    N, L = reads.shape[0] // 2, reads.shape[1]
    dev = torch.device("cuda:0")
    al = AnchorAligner(anchor, device=0)
    gi = genome.GenomeIndex(contigs, device=0)
    tiles = blat.TileReference([(n, s.decode()) for n, s in contigs], blat.TILE)
    try:
        reads_t = torch.from_numpy(reads).to(dev)
        z = lambda *sh, dt=torch.int32: torch.zeros(sh, dtype=dt, device=dev)  # noqa: E731
        out = {k: z(2 * N) for k in ("flag", "pos", "score", "n_cigar", "hits")}
        out["cigar"] = z(2 * N, 32)
        al.align_pairs_device(reads_t, N, L, out)
        _, _, an, cnt = al.partition_device(out["flag"], out["pos"])
        na = int(cnt.cpu()[2])
        cap = 2 * N
        q, q_lens, q_rows, n_q = z(cap, L, dt=torch.uint8), z(cap), z(cap), z(1)
        al.gather_reads_device(reads_t, L, an, na, _lib.AF_GATHER_SPLIT_SAM, q, q_lens, q_rows, n_q, out_t=out)
        torch.cuda.synchronize()
        n5 = int(n_q.item())
        recs = z(cap * genome.MAX_REC * genome.REC_DTYPE.itemsize // 4)
        nrec = z(cap)
        gi.align_se_device(q, n5, L, recs, nrec, lens_t=q_lens)
        torch.cuda.synchronize()
        p = blat.params("split_tail")
        psl = blat.PSL_DTYPE.itemsize
        # sequential: the check, then BLAT of its survivors
        s6, s6_lens, s6_src, n6, n_over = z(cap, _lib.AF_MAX_READ, dt=torch.uint8), z(cap), z(cap), z(1), z(1)
        genome.s5_filter_device(gi.ctx, recs, nrec, n5, q, L, q_lens, q_rows, out, cap, s6, s6_lens, s6_src, n6,
                                n_over_t=n_over)
        rows_a, nr_a = z(cap * blat.MAX_ROWS * psl, dt=torch.uint8), z(cap)
        nsp = 1 << 18  # both spill pools hold every row (a full pool drops rows in atomic order)
        sp_a = dict(rows=z(nsp * psl, dt=torch.uint8), q=z(nsp), n=z(1))
        tiles.caps(reset=True)
        tiles.spill_to(sp_a["rows"], sp_a["q"], sp_a["n"])
        try:
            tiles.search_device(s6, n6, _lib.AF_MAX_READ, rows_a, nr_a, lens_t=s6_lens, p=p)
        finally:
            tiles.spill_to()
        torch.cuda.synchronize()
        caps_a = tiles.caps(reset=True)
        # split: the leaders' rows, BLAT, the check + compaction (CandidateDiscovery's buffers)
        d = CandidateDiscovery.__new__(CandidateDiscovery)
        d.dev, d.tiles_ref, d.p_tail, d.L, d.s6cap, d.spill_min = dev, tiles, p, L, 0, nsp
        d.q, d.q_lens, d.q_rows, d.out, d.q_nh = q, q_lens, q_rows, out, nrec
        d._alloc_s6(64)  # grown by _s6_pre
        d._s6_pre(0, n5, torch.cuda.current_stream())
        d._s6_search(torch.cuda.current_stream())
        d._s6_check(0, n5, recs, torch.cuda.current_stream())
        d._s6_finish(torch.cuda.current_stream())
        torch.cuda.synchronize()
        caps_b = tiles.caps(reset=True)
        k6 = int(n6.item())
        assert int(d.s6["n"].item()) == k6 and 20 < k6 < int(d.s6p["n"].item()) <= n5
        assert torch.equal(d.s6["lens"][:k6], s6_lens[:k6]) and torch.equal(d.s6["src"][:k6], s6_src[:k6])
        for k in range(k6):
            ln = int(s6_lens[k])
            assert torch.equal(d.s6["q"][k, :ln], s6[k, :ln]), k
        assert torch.equal(d.t_nh[:k6], nr_a[:k6])
        ra = rows_a.cpu().numpy().view(blat.PSL_DTYPE).reshape(cap, blat.MAX_ROWS)
        rb = d.t_rows.cpu().numpy().view(blat.PSL_DTYPE).reshape(-1, blat.MAX_ROWS)
        nh = nr_a[:k6].cpu().numpy()
        for k in range(k6):
            m = min(int(nh[k]), blat.MAX_ROWS)
            assert ra[k, :m].tobytes() == rb[k, :m].tobytes(), k
        assert nh.sum() > 0
        ns_a, ns_b = int(sp_a["n"].item()), int(d.t_spill["n"].item())
        assert ns_a == ns_b and 0 < ns_a <= nsp
        ea = blat.spilled_rows(sp_a["rows"][:ns_a * psl].cpu().numpy().view(blat.PSL_DTYPE), sp_a["q"][:ns_a].cpu().numpy())
        eb = blat.spilled_rows(d.t_spill["rows"][:ns_b * psl].cpu().numpy().view(blat.PSL_DTYPE),
                               d.t_spill["q"][:ns_b].cpu().numpy())
        assert {k: sorted(r.tobytes() for r in v) for k, v in ea.items()} == {k: sorted(r.tobytes() for r in v) for k, v in eb.items()}
        assert int(d.s6["over"].item()) == int(n_over.item())
        assert caps_a == caps_b
    finally:
        tiles.close()
        gi.close()
        al.close()
