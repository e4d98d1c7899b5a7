"""End-to-end anchored fusion detection on the GPU path (the per-gene loop of
Anchored_Fusion.py:121-227 with its shell calls replaced).

| reference step | here |
|---|---|
| AF:58-80 gene names | `gene_names_from_fasta` / `gene_names_from_file` |
| AF:144-172 anchor FASTA + `bwa index` | `AnchorAligner(anchor)` (GPU index) |
| AF:182 `bwa mem -M anchor fq1 fq2 \\| samtools sort` | K1+K2+K3 per batch of bwa chunks (`discover.CandidateDiscovery`) |
| AF:186-194 samtools flag partitions | `af_partition_device` (S3 in HBM) |
| AF:173-178 `bwa index genome` | `genome.GenomeIndex` (suffix array + FM index built on the GPU) |
| AF:188 `bwa mem -M genome tmp1 tmp2` | `Searches.genome_sam_pe` (bwa-mem PE on the GPU, csrc/bwa_genome.hip) |
| AF:198 `Find_homo_genes` | `partner.homolog_genes` |
| AF:204 `del_too_many_reads` | S5 + `af_s5_filter_device` (the genome check in HBM) |
| AF:205 `Find_fine_block` BLAT (fn:530) | `af_blat_device` on the survivors |
| AF:205-206 `Find_blocks`, `Find_fine_block` | `blocks.spanning_blocks`, `blocks.add_fine_blocks` |
| AF:207 `Build_candidate_fasta` | `partner.candidate_targets` |
| AF:208 `contact_reads` | `splitreads.cluster_split_reads` |
| AF:209-210 `Find_Anchored_split`, `Find_candidate_genes` | `partner.*` |
| AF:227 `Final_fusion` | `report.write_predictions` |

By default a gene runs on the device path (`run_gene_device`): the reads are uploaded once,
S2-S6 run in HBM, and only the gathered queries (S4 pairs, S5's survivors and their S6 rows)
are rendered as the SAM / PSL text the host stages read (`device_products` ->
`consume_products`).  Searches and the S2 aligner are injectable: tests pass the CPU oracle,
which takes the host path (`run_gene` -> `consume_gene`: the same stages over host buffers).
The oracle is test infrastructure and never a fallback.

The false-positive filter (AF:212-225) runs when `filt` names a model file
(`--model_file` without `--not_filter_false_positive`): `filter_model.score_candidates` builds the
windows (get_test_reads), scores them on PyTorch-ROCm (Test_model) and Final_fusion writes the
Natural_score layout; a missing model file falls back to the no-filter tables, as in the reference.
"""
import os
import time
import re

from . import blocks as blk
from . import genome_check, partner, report, splitreads
from .annotation import ExonIndex
from .io import read_fasta, read_pairs

_COMP = str.maketrans("ACGTNacgtn", "TGCANtgcan")


def revcomp(s):
    return s.translate(_COMP)[::-1]


def gene_names_from_fasta(path):
    """AF:58-73: the first header token that is neither an accession (`NM_004327.4`) nor a
    descriptive word (gene/specie/trans/for/homo/sapiens, any case)."""
    names = []
    with open(path) as fh:
        for line in fh:
            if not line.startswith(">"):
                continue
            toks = line.rstrip()[1:].split(" ")
            keep = [t for t in toks if not re.match(r"[a-zA-Z]+_\d+\.\d+", t)
                    and not re.search(r"gene|specie|trans|for|homo|sapiens", t, re.IGNORECASE)]
            names.append(keep[0])
    return names


def gene_names_from_file(path):
    with open(path) as fh:
        return [ln.rstrip() for ln in fh if ln.rstrip() != ""]


def sam_line(name, flag, rname, pos1, cigar, seq):
    return f"{name}\t{flag}\t{rname}\t{pos1}\t60\t{cigar}\t*\t0\t0\t{seq}\t*\n"


class Searches:
    """The search services the partner stages need, on the GPU by default.

    `place(targets, queries, preset)` -> PSL lines (partner.py callback; BLAT restatement);
    `genome_sam_se(queries)` -> per query the SAM lines of `bwa mem -M genome q.fa` (fn:716, S5);
    `genome_sam_pe(pairs)` -> the SAM lines of `bwa mem -M genome fq1 fq2` (AF:188, S4), per pair
    mate 1's records then mate 2's.
    The genome calls run bwa-mem restated on the GPU over `bwa index` of the genome
    (genome.GenomeIndex, built once); genome_factory(contigs) may supply another engine with the
    same interface (the CPU oracle in tests)."""

    def __init__(self, genome_contigs, device=0, placer=None, chunk_bases=10_000_000, genome_factory=None):
        from . import _lib
        from .place import Placer
        self.genome = genome_contigs
        self.place = placer or Placer(device=device)
        self.chunk_bases = int(chunk_bases)
        self._gfac = genome_factory
        self._device = device
        self._gidx = None
        self.params = _lib.default_params()  # bwa mem defaults (-k 19 -T 30), as AF:188 / fn:716 run it

    @property
    def on_device(self):
        """True when every search runs on the GPU engines (the device path can use them)."""
        return self._gfac is None and getattr(self.place, "on_device", False)

    def genome_index(self):
        if self._gidx is None:
            if self._gfac is not None:
                self._gidx = self._gfac(self.genome)
            else:
                from .genome import GenomeIndex
                self._gidx = GenomeIndex(self.genome, device=self._device)
        return self._gidx

    def _pe(self):
        from . import _lib
        return _lib.default_pe(chunk_bases=self.chunk_bases)

    def genome_sam_se(self, queries):
        from .genome import sam_lines
        from .place import pack_queries
        if not queries:
            return []
        g = self.genome_index()
        buf, lens = pack_queries([s for _, s in queries])
        recs, nrec = g.align_se(buf, lens, self.params, self._pe(), id_base=0)
        return [sam_lines(g.names, n, s, recs[i], nrec[i]) for i, (n, s) in enumerate(queries)]

    def genome_sam_pe(self, pairs):
        from .genome import sam_lines
        from .place import pack_queries
        if not pairs:
            return []
        g = self.genome_index()
        buf, lens = pack_queries([s for _, a, b in pairs for s in (a, b)])
        recs, nrec = g.align_pe(buf, lens, self.params, self._pe())
        out = []
        for i, (name, a, b) in enumerate(pairs):
            out += sam_lines(g.names, name, a, recs[2 * i], nrec[2 * i])
            out += sam_lines(g.names, name, b, recs[2 * i + 1], nrec[2 * i + 1])
        return out

    def getfasta(self, rows):
        """bedtools getfasta -name: rows (chrom, start, end, name) -> [(name::chrom:start-end, seq)];
        intervals outside the contig are skipped, as bedtools does."""
        contigs = dict(self.genome)
        out = []
        for chrom, s, e, name in rows:
            seq = contigs.get(chrom)
            if seq is None or s < 0 or e > len(seq) or s >= e:
                continue
            out.append((f"{name}::{chrom}:{s}-{e}", seq[s:e]))
        return out


def homolog_rows(path, gtf, genome, gene, anchor, place):
    """<G>_homo_genes.bed (`Find_homo_genes`, fn:336-373), made once: AF:196 searches only when the
    file is absent, and reads it (column 4, the gene id) either way.  Rows (chrom, start, end,
    gene_id, gene_name, strand) as strings; the file is written whole or not at all."""
    if os.path.exists(path):
        with open(path) as fh:
            return [ln.rstrip("\n").split("\t") for ln in fh if ln.strip()]
    rows = partner.homolog_genes(gtf, genome, [(gene, anchor)], place)
    tmp = path + ".tmp"
    with open(tmp, "w") as fh:
        fh.writelines("\t".join(str(v) for v in r) + "\n" for r in rows)
    os.replace(tmp, path)
    return rows


def align_anchor(anchor, reads, lens, aligner_factory):
    """S1 + S2 for one anchor (AF:167-182): index it and align every pair."""
    aligner = aligner_factory(anchor.encode())
    try:
        return aligner.align_pairs(reads, lens)
    finally:
        close = getattr(aligner, "close", None)
        if close:
            close()


def run_gene(gene, anchor, names, reads, lens, index, homo_rows, searches, aligner_factory, out_prefix, log=print,
             filt=None):
    """One anchored gene (the body of AF:121-227).  Returns the candidate list."""
    res = align_anchor(anchor, reads, lens, aligner_factory)
    return consume_gene(gene, anchor, names, reads, lens, res, index, homo_rows, searches, out_prefix, log=log,
                        filt=filt)


def consume_gene(gene, anchor, names, reads, lens, res, index, homo_rows, searches, out_prefix, log=print, filt=None):
    """S3-S8 + Final_fusion (AF:183-227) on the S2 records ``res`` of ``reads`` (host buffers;
    the searches through ``searches``).  filt: None (`--not_filter_false_positive`) or
    dict(model_file=..., device=...)."""
    s4, split_sam, psl = host_products(gene, names, reads, lens, res, searches, log=log)
    return consume_products(gene, anchor, index, homo_rows, searches, out_prefix, s4, split_sam, psl, log=log,
                            filt=filt)


def host_products(gene, names, reads, lens, res, searches, log=print):
    """S3 -> S6 over host buffers: (the SAM lines of S4, the split_sam lines S5's check keeps,
    S6's PSL lines), the texts consume_products reads."""
    width = reads.shape[1]

    def seq(r):  # only the reads the partitions select are decoded
        return bytes(reads[r, : (lens[r] if lens is not None else width)]).decode()

    tmp1, tmp2, anchored = res.partition()
    log(f"[{gene}] S2: {res.n_mapped()} of {res.n_reads} reads on the anchor; "
        f"{len(tmp1)} one-end-anchored pairs; {len(anchored)} anchored records")
    n_ovf = res.n_overflow() if hasattr(res, "n_overflow") else 0
    if n_ovf:
        log(f"[{gene}] WARNING: {n_ovf} reads hit a per-read cap of the S2 restatement and are reported "
            f"unmapped (AF_FLAG_MEM_OVERFLOW / AF_FLAG_CIGAR_OVERFLOW; bwa has no caps)")
    # S4: one-end-anchored pairs on the genome, paired as bwa pairs tmp1.fq / tmp2.fq (samtools
    # fastq restores the sequenced orientation of both ends)
    q4 = [(names[a // 2], seq(a), seq(b)) for a, b in zip(tmp1, tmp2)]
    s4 = searches.genome_sam_pe(q4) if q4 else []
    # anchored.bam as `samtools view` prints it (SEQ reverse-complemented for 0x10)
    anch_lines = []
    for r in anchored:
        cig, f = res.cigar_str(r), res.flag_at(r)
        sq = revcomp(seq(r)) if f & 0x10 else seq(r)
        anch_lines.append(sam_line(names[r // 2], f & 0xFFFF, gene, res.pos_at(r) + 1, cig, sq))
    # S5: split reads vs the genome, the genome check
    fasta = genome_check.split_read_fasta(anch_lines)
    gsam = ["@HD\tVN:1.6\n"] + [ln for recs in (searches.genome_sam_se(fasta) if fasta else []) for ln in recs]
    split_sam = genome_check.filter_genome_hits(gsam)
    log(f"[{gene}] S5: {len(fasta)} split reads, {len(split_sam)} kept")
    # S6: the survivors' BLAT on the genome
    _, tail_fa = blk.split_read_queries(split_sam)
    psl = searches.place(searches.genome, tail_fa, "split_tail") if tail_fa else []
    return s4, split_sam, psl


def consume_products(gene, anchor, index, homo_rows, searches, out_prefix, s4, split_sam, psl, log=print, filt=None):
    """S6 consumer -> S7 / S8 -> Final_fusion (AF:205-227) from the texts the genome searches
    produce: s4 = the SAM lines of `bwa mem -M genome tmp1 tmp2` (AF:188), split_sam = the lines
    `del_too_many_reads` keeps (fn:735, 760), psl = the PSL of S6's BLAT of their processed
    sequences (fn:530; empty when there is none).  Both the host path (consume_gene) and the
    device path (run_gene_device) end here."""
    anchor_rec = [(gene, anchor)]
    homo = [row[3] for row in homo_rows]
    if isinstance(s4, blk.S4Records):
        blocks_chr = blk.spanning_blocks_records(s4, index, homo)
    else:
        blocks_chr = blk.spanning_blocks(s4, index, homo)
    tails, tail_fa = blk.split_read_queries(split_sam)
    if tail_fa:
        blk.add_fine_blocks(blocks_chr, tails, psl, index, homo)
    # the reference's widening can leave a non-integer end; its next step would raise
    for c in list(blocks_chr):
        blocks_chr[c] = [b for b in blocks_chr[c] if isinstance(b.start, int) and isinstance(b.end, int)]
    cand_recs = partner.candidate_targets(blocks_chr, searches.getfasta, searches.place, anchor_rec)
    bps = splitreads.cluster_split_reads(split_sam)
    good = partner.anchored_split_placement(cand_recs, blocks_chr, bps, index, searches.place, anchor_rec)
    cands, cnt_max = partner.candidate_genes(good, bps, blocks_chr, searches.place, searches.genome)
    log(f"[{gene}] blocks {sum(len(v) for v in blocks_chr.values())}, breakpoints {len(bps)}, "
        f"placed {len(good)}, candidates {len(cands)}")
    scores, no_filter = [], True
    if filt is not None and len(cands) != 0:
        from .filter_model import score_candidates
        scores, no_filter = score_candidates(cands, anchor, index, searches.getfasta, filt["model_file"], out_prefix,
                                             device=filt.get("device", "cpu"), log=log)
    report.write_predictions(out_prefix, cands, gene, index, scores, cnt_max, no_filter)
    return cands


_OPS = "MIDNSHP=X"


def device_products(d, gene, names, genome_names, s4_text=False):
    """What consume_products reads, from a discover.CandidateDiscovery pass: S4's records
    (blocks.S4Records: the fields Find_blocks reads, no text; the SAM lines of genome.sam_lines
    with s4_text), the pseudo-SAM lines of S5's survivors (the `del_too_many_reads` output
    format, fn:735/760) and the PSL lines of S6.  Only the gathered queries reach the host."""
    import numpy as np
    import torch

    from . import blat
    from .genome import MAX_REC, REC_DTYPE, sam_lines
    torch.cuda.synchronize(d.dev)
    nq = min(int(d.n_q.item()), d.qcap)
    npair = d._npair
    q, ql, rows = d.q[:nq].cpu().numpy(), d.q_lens[:nq].cpu().numpy(), d.q_rows[:nq].cpu().numpy()
    recs = d.q_recs[:nq * MAX_REC * REC_DTYPE.itemsize].cpu().numpy().view(REC_DTYPE).reshape(nq, MAX_REC)
    nrec = d.q_nh[:nq].cpu().numpy()

    def seq(i):
        return q[i, :ql[i]].tobytes().decode()
    pair_names = [names[int(r) // 2] for r in rows[0:2 * npair:2]]
    if s4_text:
        s4 = []
        for k in range(npair):
            s4 += sam_lines(genome_names, pair_names[k], seq(2 * k), recs[2 * k], nrec[2 * k])
            s4 += sam_lines(genome_names, pair_names[k], seq(2 * k + 1), recs[2 * k + 1], nrec[2 * k + 1])
    else:
        s4 = blk.S4Records(pair_names, recs[:2 * npair], nrec[:2 * npair], genome_names)
    n6 = int(d.s6["n"].item())
    split_sam, psl = [], []
    if n6:
        src = d.s6["src"][:n6].cpu().numpy()
        r = rows[2 * npair + src]
        rr = torch.from_numpy(r.astype(np.int64)).to(d.dev)
        pos = d.out["pos"][rr].cpu().numpy()
        ncig = d.out["n_cigar"][rr].cpu().numpy()
        cig = d.out["cigar"][rr].cpu().numpy().view(np.uint32)
        for k in range(n6):
            c = "".join(f"{int(v) >> 4}{_OPS[int(v) & 15]}" for v in cig[k, :ncig[k]])
            split_sam.append(f"{names[int(r[k]) // 2]}\t0\t{gene}\t{int(pos[k]) + 1}\t60\t{c}\t=\t1111\t0\t"
                             f"{seq(2 * npair + int(src[k]))}\tA\n")
        s6q, s6l = d.s6["q"][:n6].cpu().numpy(), d.s6["lens"][:n6].cpu().numpy()
        t_rows = d.t_rows[:n6 * blat.MAX_ROWS * blat.PSL_DTYPE.itemsize].cpu().numpy().view(blat.PSL_DTYPE)
        psl = ["psLayout version 3\n", "\n"] + blat.psl_lines(
            d.tiles_ref, [(str(k), s6q[k, :s6l[k]].tobytes().decode()) for k in range(n6)],
            t_rows.reshape(n6, blat.MAX_ROWS), d.t_nh[:n6].cpu().numpy(), extra=d.s6_spilled())
    return s4, split_sam, psl


def run_gene_device(gene, anchor, names, reads_t, lens_t, pair_bases, index, homo_rows, searches, out_prefix,
                    device=0, chunk_bases=10_000_000, log=print, filt=None, inflight=4, batch_chunks=240):
    """One anchored gene on the device path: S2 (K1 + K2 + K3 per batch of bwa chunks), S3, the
    gathers, S4 / S5, S5's genome check and S6 in HBM (discover.CandidateDiscovery), then the host
    stages on the gathered queries only (consume_products)."""
    from . import blat
    from .discover import CandidateDiscovery
    t0 = time.perf_counter()
    gidx = searches.genome_index()
    tiles = searches.place.tiles(searches.genome, blat.params("split_tail").step_size)
    log(f"[{gene}] genome index and tiles ready ({time.perf_counter() - t0:.1f} s)")
    t0 = time.perf_counter()
    n_pairs, stride = reads_t.shape[0] // 2, reads_t.shape[1]
    d = CandidateDiscovery(anchor.encode(), gidx, tiles, n_pairs, stride, device=device, inflight=inflight,
                           batch_chunks=batch_chunks, chunk_bases=chunk_bases, pair_bases=pair_bases)
    try:
        d.run(reads_t, lens_t=lens_t)
        c = d.summary()
        log(f"[{gene}] S2: {c['mapped_reads']} of {2 * n_pairs} reads on the anchor; {c['tmp1']} one-end-anchored "
            f"pairs; {c['anchored']} anchored records; S5: {c['s5_split_reads']} split reads, {c['s6_queries']} kept")
        if c["s2_overflow_reads"]:
            log(f"[{gene}] WARNING: {c['s2_overflow_reads']} reads hit a per-read cap of the S2 restatement and "
                f"are reported unmapped (AF_FLAG_MEM_OVERFLOW / AF_FLAG_CIGAR_OVERFLOW; bwa has no caps)")
        caps = {k: v for k, v in c.items() if k in ("genome_cap_overflow", "genome_pool_overflow",
                                                     "genome_record_overflow", "s6_clipped", "s4_pairs_dropped",
                                                     "s5_dropped") or (k.startswith("blat_cap_") and v)}
        if any(caps.values()):
            log(f"[{gene}] WARNING: caps reached: {caps}")
        s4, split_sam, psl = device_products(d, gene, names, gidx.names)
        log(f"[{gene}] S2-S6 on the device and the products on the host ({time.perf_counter() - t0:.1f} s)")
    finally:
        d.close()
    return consume_products(gene, anchor, index, homo_rows, searches, out_prefix, s4, split_sam, psl, log=log,
                            filt=filt)


def upload_reads(reads, lens, device):
    """The reads in HBM for the device path: rows padded to a multiple of 8 bytes (every bwa
    chunk's batch then starts on a 16-byte boundary), their lengths, and the pairs' base counts."""
    import numpy as np
    import torch
    n, width = reads.shape
    stride = max(8, -(-width // 8) * 8)
    ln = np.full(n, width, np.int32) if lens is None else np.ascontiguousarray(lens, dtype=np.int32)
    dev = torch.device("cuda", device)
    # the rows go up as read (no padded host copy: 15 GB at configs[2]) and are padded in HBM
    reads_t = torch.full((n, stride), ord("N"), dtype=torch.uint8, device=dev)
    step = max(1, (1 << 30) // max(1, width))  # 1 GiB per host-to-device copy
    for a in range(0, n, step):
        reads_t[a:a + step, :width] = torch.from_numpy(np.ascontiguousarray(reads[a:a + step])).to(dev)
    lens_t = torch.from_numpy(ln).to(dev)
    pair_bases = ln.astype(np.int64).reshape(-1, 2).sum(axis=1)
    torch.cuda.synchronize(dev)
    return reads_t, lens_t, pair_bases


def dist_world(group=None):
    """(rank, world) of the torch.distributed job this process is in, (0, 1) outside one."""
    try:
        import torch.distributed as dist
    except ImportError:  # pragma: no cover - torch is part of the image
        return 0, 1
    if not (dist.is_available() and dist.is_initialized()):
        return 0, 1
    return dist.get_rank(group), dist.get_world_size(group)


def run(anchored_cds, fastq1, fastq2, ref_seq, ref_ann, out_folder, gene_names=None, device=0, searches=None,
        aligner_factory=None, log=print, group=None, filt=None, chunk_bases=10_000_000, backend_factory=None):
    """All genes of --file_anchored_cds; writes <out>/<G>_fusion/<G>_fusion_predictions*.txt.

    Inside a torch.distributed job of N > 1 ranks (cli --gpus N: one process per GPU, `device`
    = this rank's GPU), S2 is sharded: every rank aligns whole bwa chunks of the pairs and the
    candidate records are all-gathered on the device (shard.align_sharded); rank 0 then runs
    S3-S8 and writes the tables, the other ranks return {}.

    chunk_bases: bwa's input chunk, 10,000,000 x --thread (AF:182/188 `bwa mem -t T`): S2 and S4
    estimate insert sizes per chunk, so the records depend on it as the reference's do.
    backend_factory (sharded runs): the per-rank dist_discover backend, default gpu_backend."""
    rank, world = dist_world(group)
    if world > 1:
        return _run_sharded(anchored_cds, fastq1, fastq2, ref_seq, ref_ann, out_folder, gene_names, device,
                            searches, aligner_factory, log, group, rank, world, filt, chunk_bases, backend_factory)
    genes = gene_names_from_file(gene_names) if gene_names and os.path.exists(gene_names) \
        else gene_names_from_fasta(anchored_cds)
    anchors = [s.decode().upper() for _, s in read_fasta(anchored_cds)]
    t0 = time.perf_counter()
    genome = [(h.split()[0], s.decode().upper()) for h, s in read_fasta(ref_seq)]
    with open(ref_ann) as fh:
        gtf = fh.readlines()
    index = ExonIndex.from_lines(gtf)
    log(f"genome and annotation read: {len(genome)} contigs, {sum(len(s) for _, s in genome)} bp, "
        f"{len(gtf)} GTF lines ({time.perf_counter() - t0:.1f} s)")
    t0 = time.perf_counter()
    names, reads, lens = read_pairs(fastq1, fastq2)
    log(f"ingest: {reads.shape[0] // 2} pairs ({time.perf_counter() - t0:.1f} s)")
    # the device path (S2-S6 in HBM) unless a test injects host backends
    on_device = aligner_factory is None and (searches is None or getattr(searches, "on_device", False))
    if searches is None:
        searches = Searches(genome, device=device, chunk_bases=chunk_bases)
    if aligner_factory is None:
        aligner_factory = _default_aligner(device, chunk_bases)
    dev_reads = upload_reads(reads, lens, device) if on_device and reads.shape[0] else None
    if dev_reads is not None:
        reads = lens = None  # the device copy is the one the genes read (15 GB at configs[2])
    results = {}
    for gene, anchor in zip(genes, anchors):
        folder = os.path.join(out_folder, gene + "_fusion")
        os.makedirs(os.path.join(folder, "work_dir"), exist_ok=True)
        t0 = time.perf_counter()
        homo_rows = homolog_rows(os.path.join(folder, "work_dir", gene + "_fusion_homo_genes.bed"), gtf, genome, gene,
                                 anchor, searches.place)
        log(f"[{gene}] homologs: {len(homo_rows)} gene rows ({time.perf_counter() - t0:.1f} s)")
        prefix = os.path.join(folder, gene + "_fusion")
        if dev_reads is not None:
            results[gene] = run_gene_device(gene, anchor, names, *dev_reads, index, homo_rows, searches, prefix,
                                            device=device, chunk_bases=chunk_bases, log=log, filt=filt)
        else:
            results[gene] = run_gene(gene, anchor, names, reads, lens, index, homo_rows, searches, aligner_factory,
                                     prefix, log=log, filt=filt)
    return results



def _default_aligner(device, chunk_bases):
    from .align import AnchorAligner

    def factory(anchor):
        a = AnchorAligner(anchor, device=device)
        a.pe.chunk_bases = int(chunk_bases)
        return a
    return factory


def gpu_backend(device, chunk_bases=10_000_000, inflight=4, batch_chunks=240):
    """The default per-rank backend of dist_discover: discover.CandidateDiscovery over the rank's
    reads uploaded to its GPU (once per rank: the upload is kept for every anchor gene), with the
    rank's genome index and tiles (built once per rank)."""
    held = {}

    def make(anchor, reads, lens, lo, searches, gene):
        from . import blat
        from .discover import CandidateDiscovery
        if held.get("src") is not reads:
            held.update(src=reads, up=upload_reads(reads, lens, device))
        reads_t, lens_t, pair_bases = held["up"]
        d = CandidateDiscovery(anchor.encode(), searches.genome_index(),
                               searches.place.tiles(searches.genome, blat.params("split_tail").step_size),
                               reads_t.shape[0] // 2, reads_t.shape[1], device=device, inflight=inflight,
                               batch_chunks=batch_chunks, pair_base=lo, chunk_bases=chunk_bases, pair_bases=pair_bases)
        return d.attach(reads_t, lens_t)
    return make


def _run_sharded(anchored_cds, fastq1, fastq2, ref_seq, ref_ann, out_folder, gene_names, device, searches,
                 aligner_factory, log, group, rank, world, filt=None, chunk_bases=10_000_000, backend_factory=None):
    """cli --gpus N: every rank ingests its share of the FASTQ pair (shard.read_pairs_sharded:
    BGZF parts, whole bwa chunks per rank) and runs S2-S6 on it with the global order of one run
    (dist_discover: S5's read ids and QNAME groups from all-gathered sort keys, S4 per rank on whole chunks of
    the globally zipped tmp1 / tmp2 lists); rank 0 renders the texts and runs the host stages."""
    import torch
    import torch.distributed as dist
    from . import dist_discover, shard
    genes = gene_names_from_file(gene_names) if gene_names and os.path.exists(gene_names) \
        else gene_names_from_fasta(anchored_cds)
    anchors = [s.decode().upper() for _, s in read_fasta(anchored_cds)]
    on_gpu = torch.cuda.is_available() and dist.get_backend(group) == "nccl"
    host_group = dist.new_group(backend="gloo") if on_gpu else group
    names, reads, lens, lo, n_pairs = shard.read_pairs_sharded(fastq1, fastq2, rank, world, group=host_group,
                                                               chunk_bases=chunk_bases)
    log(f"[rank {rank}] ingested pairs {lo} .. {lo + reads.shape[0] // 2} of {n_pairs}")
    genome = [(h.split()[0], s.decode().upper()) for h, s in read_fasta(ref_seq)]
    gtf = index = None
    if rank == 0:
        with open(ref_ann) as fh:
            gtf = fh.readlines()
        index = ExonIndex.from_lines(gtf)
    if searches is None:
        searches = Searches(genome, device=device, chunk_bases=chunk_bases)
    make = backend_factory or gpu_backend(device, chunk_bases)
    dev = torch.device("cuda", device) if on_gpu else torch.device("cpu")
    results = {}
    for gene, anchor in zip(genes, anchors):
        backend = make(anchor, reads, lens, lo, searches, gene)
        try:
            res, counts = dist_discover.search(backend, lo, rank, world, group=group, device=dev, names=names,
                                               host_group=host_group)
            log(f"[{gene}] rank {rank}: {counts}")
            if rank == 0:
                s4, split_sam, psl = dist_discover.render(res, backend, gene, [n for n, _ in genome], s4_text=False)
        finally:
            close = getattr(backend, "close", None)
            if close:
                close()
        if rank == 0:
            folder = os.path.join(out_folder, gene + "_fusion")
            os.makedirs(os.path.join(folder, "work_dir"), exist_ok=True)
            homo_rows = homolog_rows(os.path.join(folder, "work_dir", gene + "_fusion_homo_genes.bed"), gtf, genome,
                                     gene, anchor, searches.place)
            results[gene] = consume_products(gene, anchor, index, homo_rows, searches,
                                             os.path.join(folder, gene + "_fusion"), s4, split_sam, psl, log=log,
                                             filt=filt)
    # the end-of-run sync on the CPU group (rank 0 may be busy long after the others finish)
    dist.barrier(host_group)
    return results
