"""Single-cell fusion detection (Anchored_Fusion_singlecell.py, SURVEY.md §8 f rank 3).

The reference runs the whole bulk pipeline once per cell and per anchored gene, each cell
through its own `bwa mem` (SC:205-256), then merges the per-cell prediction tables
(SC:258-287).  Here the cells are batched: every cell's FASTQ pair is ingested once
(native reader), and per gene the pairs of whole cells are concatenated into batches of up to
``batch_pairs`` pairs: one H2D copy per batch and one device call per cell (each cell is its own
``bwa mem`` run, so read ids and insert-size chunks restart per cell).  The records are then
split back per cell and each cell runs S3-S8 + Final_fusion on its own records, exactly as a
separate run on that cell would (the S3 sort and every consumer see only the cell's reads).

| reference step | here |
|---|---|
| SC:86-113 cell FASTQ discovery | `discover_cells` |
| SC:172-203 anchor FASTA, index, `Find_homo_genes` once per gene | `partner.homolog_genes` once per gene |
| SC:205-217 per-cell `bwa mem` vs the anchor | one `align_pairs` per batch of cells |
| SC:218-256 per-cell S3-S8, `Final_fusion` | `pipeline.consume_gene` per cell |
| SC:258-287 merge by the first five columns, count cells | `merge_cell_tables` |

The merge reads the span/split counts from columns 6 and 7 of each cell's `_predictions.txt`,
as SC:277-283 does: that is the filter-model layout (column 5 = Natural_score), the default
mode whenever the model file exists.  With `--not_filter_false_positive` (or a missing model
file, which the reference also turns into the no-filter tables) the counts are columns 5 and 6
and column 7 holds read names, on which the reference's `int()` raises; there, on purpose, the
merge reads columns 5 and 6.  Each cell table's header says which layout it has.
"""
import os
import re

import numpy as np

from . import partner
from .align import AlignResult
from .annotation import ExonIndex
from .io import read_fasta, read_pairs
from .pipeline import Searches, consume_gene, dist_world, gene_names_from_fasta, gene_names_from_file


def discover_cells(fastq_dir):
    """(cell, fq1, fq2) triples as SC:86-113 pairs them: directory entries in sorted order; an
    entry matching ``<cell>_1.fastq`` (then ``.fastq.gz``, ``.fq.gz``, ``.fq``) pairs with the
    NEXT entry if that is the same cell's ``_2`` file.  The patterns are the reference's
    regular expressions (unescaped dots included)."""
    entries = sorted(os.listdir(fastq_dir + "/"))
    cells = []
    for i, e in enumerate(entries):
        for sfx in ("fastq", "fastq.gz", "fq.gz", "fq"):
            m = re.findall(r"(\S+)_1." + sfx + "$", e)
            if m:
                name = m[0]
                if i + 1 >= len(entries):  # the reference indexes past the end here (IndexError)
                    raise ValueError(f"{fastq_dir}: {e} has no {name}_2.{sfx} after it")
                if re.match(r"" + name + "_2." + sfx + "$", entries[i + 1]):
                    cells.append((name, f"{name}_1.{sfx}", f"{name}_2.{sfx}"))
                break
    return cells


def slice_result(res, r0, r1):
    """Rows [r0, r1) of an AlignResult."""
    return AlignResult(res.flag[r0:r1], res.pos[r0:r1], res.score[r0:r1], res.n_cigar[r0:r1], res.cigar[r0:r1],
                       res.hits[r0:r1])


def _concat(cells):
    """Pair-major reads of several cells in one matrix (common stride; lens when ragged)."""
    stride = max(r.shape[1] for _, r, _ in cells)
    rows = sum(r.shape[0] for _, r, _ in cells)
    reads = np.full((rows, max(stride, 1)), ord("N"), np.uint8)
    lens = np.empty(rows, np.int32)
    o = 0
    for _, r, ln in cells:
        reads[o:o + r.shape[0], :r.shape[1]] = r
        lens[o:o + r.shape[0]] = r.shape[1] if ln is None else ln
        o += r.shape[0]
    return reads, (None if (lens == stride).all() else lens)


def _per_segment(aligner, reads, lens, seg_pairs):
    """align_segments for aligners without a device path (one align_pairs call per cell)."""
    parts, r0 = [], 0
    for n in seg_pairs:
        r1 = r0 + 2 * n
        parts.append(aligner.align_pairs(reads[r0:r1], None if lens is None else lens[r0:r1]))
        r0 = r1
    return AlignResult(*(np.concatenate([getattr(p, k) for p in parts])
                         for k in ("flag", "pos", "score", "n_cigar", "cigar", "hits")))


def merge_cell_tables(cells, work_folder, out_name, out_prefix):
    """SC:258-287: the per-cell `_predictions.txt` tables merged into
    `<out_prefix>_gene_cell_predictions{,_abridged}.txt` (rows keyed by the first five columns,
    in first-seen order; counts summed; cells listed).  A table whose header has Natural_score
    (the filter layout) gives its counts from columns 6-7, exactly as SC:277-283; a no-filter
    table from columns 5-6 (module docstring)."""
    head = ["Fusion_gene", "Anchored_gene_X", "X_clip_location", "Partner_gene_Y", "Y_clip_location"]
    merged = {}
    with open(out_prefix + "_gene_cell_predictions.txt", "w") as fo:
        fo.write("\t".join(["Cell_name"] + head + ["Spanning_read_count", "Breakpoint_read_count"]) + "\n")
        for cell, _, _ in cells:
            path = os.path.join(work_folder, cell, out_name + "_predictions.txt")
            with open(path) as fh:
                lines = fh.readlines()
            if len(lines) <= 1:
                continue
            c0 = 6 if "Natural_score" in lines[0].split("\t") else 5
            for line in lines[1:]:
                arr = line.split("\t")
                key = "$".join(arr[:5])
                span, split = int(arr[c0]), int(arr[c0 + 1])
                if key not in merged:
                    merged[key] = [span, split, 1, [cell]]
                else:
                    v = merged[key]
                    v[0] += span
                    v[1] += split
                    v[2] += 1
                    v[3].append(cell)
                fo.write(cell + "\t" + "\t".join(arr[0:5] + arr[c0:c0 + 2]) + "\n")
    with open(out_prefix + "_gene_cell_predictions_abridged.txt", "w") as fa:
        fa.write("\t".join(head + ["All_Spanning_read_count", "All_Breakpoint_read_count", "Single_cells_count",
                                   "Single_cells_name"]) + "\n")
        for key, v in merged.items():
            fa.write("\t".join(key.split("$")) + f"\t{v[0]}\t{v[1]}\t{v[2]}\t" + ";".join(v[3]) + "\n")
    return merged


def run(anchored_cds, fastq_dir, ref_seq, ref_ann, out_folder, gene_names=None, device=0, searches=None,
        aligner_factory=None, batch_pairs=1 << 22, log=print, filt=None, chunk_bases=10_000_000):
    """All genes x all cells; writes `<out>/<G>/<G>_fusion_gene_cell_predictions*.txt` and the
    per-cell tables under `<out>/<G>/work_dir/<cell>/`.  Returns {gene: merged rows}."""
    genes = gene_names_from_file(gene_names) if gene_names and os.path.exists(gene_names) \
        else gene_names_from_fasta(anchored_cds)
    anchors = [s.decode().upper() for _, s in read_fasta(anchored_cds)]
    genome = [(h.split()[0], s.decode().upper()) for h, s in read_fasta(ref_seq)]
    with open(ref_ann) as fh:
        gtf = fh.readlines()
    index = ExonIndex.from_lines(gtf)
    cells = discover_cells(fastq_dir)
    # one process per GPU (cli --gpus N): the cells are dealt out round-robin and every rank
    # ingests and runs S2-S8 on its own cells only (no data exchange: each cell is its own run,
    # SC:205-256); rank 0 merges the per-cell tables once every rank is done
    rank, world = dist_world()
    data = {k: read_pairs(os.path.join(fastq_dir, cells[k][1]), os.path.join(fastq_dir, cells[k][2]))
            for k in range(rank, len(cells), world)}
    if searches is None:
        searches = Searches(genome, device=device, chunk_bases=chunk_bases)
    if aligner_factory is None:
        from .pipeline import _default_aligner
        aligner_factory = _default_aligner(device, chunk_bases)
    # whole cells per GPU batch
    mine, cur, n = [], [], 0
    for k, (_, reads, _) in data.items():
        if cur and n + reads.shape[0] // 2 > batch_pairs:
            mine.append(cur)
            cur, n = [], 0
        cur.append(k)
        n += reads.shape[0] // 2
    if cur:
        mine.append(cur)
    results = {}
    for gene, anchor in zip(genes, anchors):
        out_name = gene + "_fusion"
        temp_folder = os.path.join(out_folder, gene)
        work = os.path.join(temp_folder, "work_dir")
        os.makedirs(work, exist_ok=True)
        homo_rows = partner.homolog_genes(gtf, genome, [(gene, anchor)], searches.place)
        aligner = aligner_factory(anchor.encode())
        try:
            for grp in mine:
                reads, lens = _concat([data[k] for k in grp])
                # every cell is its own bwa run (read ids and insert-size chunks restart per cell)
                seg = [data[k][1].shape[0] // 2 for k in grp]
                segs = getattr(aligner, "align_segments", None)
                res = segs(reads, lens, seg) if segs else _per_segment(aligner, reads, lens, seg)
                log(f"[{gene}] S2 batch of {len(grp)} cells, {reads.shape[0] // 2} pairs: "
                    f"{int(((res.flag & 4) == 0).sum())} reads on the anchor")
                row = 0
                for k in grp:
                    cell = cells[k][0]
                    names, creads, clens = data[k]
                    nr = creads.shape[0]
                    os.makedirs(os.path.join(work, cell), exist_ok=True)
                    consume_gene(gene, anchor, names, creads, clens, slice_result(res, row, row + nr), index,
                                 homo_rows, searches, os.path.join(work, cell, out_name), log=log, filt=filt)
                    row += nr
        finally:
            close = getattr(aligner, "close", None)
            if close:
                close()
        if world > 1:
            import torch.distributed as dist
            dist.barrier()
        if rank == 0:
            results[gene] = merge_cell_tables(cells, work, out_name, os.path.join(temp_folder, out_name))
    return results
