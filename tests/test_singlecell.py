"""Single-cell driver (anchored_fusion_amd.singlecell; Anchored_Fusion_singlecell.py).

* cell discovery restates SC:86-113 (sorted entries, a `_1` file pairs with the NEXT entry);
* the merge restates SC:258-287 on hand-written per-cell tables (no-filter column layout);
* end to end (CPU oracle backends, and the GPU path under `-m gpu`): a synthetic fusion sample
  split into three cells, aligned in batches of whole cells, gives per-cell tables identical to
  separate bulk runs of each cell, and a merged table with the planted fusion.
"""
import gzip
import os

import pytest

import afpkg  # noqa: F401
from anchored_fusion_amd import io as afio
from anchored_fusion_amd import pipeline, singlecell
from fusion_world import make_world


def _touch(d, names):
    os.makedirs(d, exist_ok=True)
    for n in names:
        open(os.path.join(d, n), "w").close()


def test_discover_cells(tmp_path):
    d = str(tmp_path / "fq")
    _touch(d, ["b_1.fq.gz", "b_2.fq.gz", "a_1.fastq", "a_2.fastq", "c_1.fq", "c_2.fastq", "d_1.fastq.gz",
               "d_2.fastq.gz", "notes.txt"])
    # sorted: a_1.fastq a_2.fastq b_1.fq.gz b_2.fq.gz c_1.fq c_2.fastq d_1.fastq.gz d_2.fastq.gz notes.txt
    assert singlecell.discover_cells(d) == [("a", "a_1.fastq", "a_2.fastq"), ("b", "b_1.fq.gz", "b_2.fq.gz"),
                                            ("d", "d_1.fastq.gz", "d_2.fastq.gz")]
    _touch(d, ["zz_1.fq"])  # a _1 file with no successor: the reference indexes past the end
    with pytest.raises(ValueError, match="no zz_2.fq"):
        singlecell.discover_cells(d)


def test_merge_cell_tables(tmp_path):
    work = str(tmp_path / "work")
    head = "Fusion_gene\tAnchored_gene_X\tX_clip_location\tPartner_gene_Y\tY_clip_location\t" \
           "Spanning_read_count\tBreakpoint_read_count\tSpanning_reads\tBreakpoint_reads\tHomo_genes\n"
    rows = {
        "c1": ["G--P\tG\tG:10\tP:p1\tchr2:500\t3\t4\tr1;r2;r3\ts1;s2;s3;s4\t\n",
               "G--Q\tG\tG:20\tQ:q1\tchr3:700\t1\t2\tr9\ts8;s9\t\n"],
        "c2": [],
        "c3": ["G--P\tG\tG:10\tP:p1\tchr2:500\t5\t6\tx\ty\t\n"],
    }
    for c, rs in rows.items():
        os.makedirs(os.path.join(work, c))
        with open(os.path.join(work, c, "G_fusion_predictions.txt"), "w") as fh:
            fh.write(head + "".join(rs))
    cells = [(c, "", "") for c in rows]
    merged = singlecell.merge_cell_tables(cells, work, "G_fusion", str(tmp_path / "G_fusion"))
    assert list(merged) == ["G--P$G$G:10$P:p1$chr2:500", "G--Q$G$G:20$Q:q1$chr3:700"]
    ab = open(str(tmp_path / "G_fusion_gene_cell_predictions_abridged.txt")).read().splitlines()
    assert ab[1:] == ["G--P\tG\tG:10\tP:p1\tchr2:500\t8\t10\t2\tc1;c3", "G--Q\tG\tG:20\tQ:q1\tchr3:700\t1\t2\t1\tc1"]
    full = open(str(tmp_path / "G_fusion_gene_cell_predictions.txt")).read().splitlines()
    assert full[0].startswith("Cell_name\tFusion_gene")
    assert full[1:] == ["c1\tG--P\tG\tG:10\tP:p1\tchr2:500\t3\t4", "c1\tG--Q\tG\tG:20\tQ:q1\tchr3:700\t1\t2",
                        "c3\tG--P\tG\tG:10\tP:p1\tchr2:500\t5\t6"]


def test_merge_cell_tables_filter_layout(tmp_path):
    """SC:277-283 on the filter-model layout (column 5 = Natural_score): counts from columns 6-7."""
    work = str(tmp_path / "work")
    head = "Fusion_gene\tAnchored_gene_X\tX_clip_location\tPartner_gene_Y\tY_clip_location\tNatural_score\t" \
           "Spanning_read_count\tBreakpoint_read_count\tSpanning_reads\tBreakpoint_reads\tHomo_genes\n"
    rows = {"c1": ["G--P\tG\tG:10\tP:p1\tchr2:500\t0.93\t3\t4\tr1;r2;r3\ts1;s2;s3;s4\t\n"],
            "c2": ["G--P\tG\tG:10\tP:p1\tchr2:500\t0.5\t1\t2\tr7\ts5;s6\t\n"]}
    for c, rs in rows.items():
        os.makedirs(os.path.join(work, c))
        with open(os.path.join(work, c, "G_fusion_predictions.txt"), "w") as fh:
            fh.write(head + "".join(rs))
    merged = singlecell.merge_cell_tables([(c, "", "") for c in rows], work, "G_fusion", str(tmp_path / "G_fusion"))
    assert merged["G--P$G$G:10$P:p1$chr2:500"][:3] == [4, 6, 2]
    full = open(str(tmp_path / "G_fusion_gene_cell_predictions.txt")).read().splitlines()
    assert full[1:] == ["c1\tG--P\tG\tG:10\tP:p1\tchr2:500\t3\t4", "c2\tG--P\tG\tG:10\tP:p1\tchr2:500\t1\t2"]


def test_singlecell_filter_model_cpu_backends(tmp_path):
    """singlecell.run with a filter model present (the default mode of SC:241-256): each cell's
    table has the Natural_score layout and the merge sums its span/split columns (SC:277-283)."""
    import torch
    from oracle_backends import OracleAligner, oracle_searches
    from anchored_fusion_amd import filter_model
    paths, _ = make_world(str(tmp_path / "world"))
    fqd = str(tmp_path / "cells")
    cells = _split_cells(paths, fqd, n_cells=2)
    genome = [(h.split()[0], s.decode().upper()) for h, s in pipeline.read_fasta(paths["genome"])]

    def searches():
        return oracle_searches(genome)
    torch.manual_seed(3)
    model = str(tmp_path / "model.pt")
    # the world's windows are 301 long (get_test_reads: 100 + left + 'H' + right + 100 pad)
    torch.save(filter_model.FusionFilter(301).double().state_dict(), model)
    out = str(tmp_path / "sc")
    singlecell.run(paths["anchor"], fqd, paths["genome"], paths["gtf"], out, searches=searches(),
                   aligner_factory=OracleAligner, batch_pairs=4000, log=lambda *_: None,
                   filt=dict(model_file=model, device="cpu"))
    sums, n_rows = {}, 0
    for c in cells:
        lines = open(os.path.join(out, "BCRX", "work_dir", c, "BCRX_fusion_predictions.txt")).read().splitlines()
        assert lines[0].split("\t")[5] == "Natural_score"
        for ln in lines[1:]:
            a = ln.split("\t")
            v = sums.setdefault("$".join(a[:5]), [0, 0])
            v[0] += int(a[6])
            v[1] += int(a[7])
            n_rows += 1
    assert n_rows > 0
    ab = [ln.split("\t") for ln in open(os.path.join(out, "BCRX", "BCRX_fusion_gene_cell_predictions_abridged.txt"))
          .read().splitlines()[1:]]
    assert {"$".join(r[:5]): [int(r[5]), int(r[6])] for r in ab} == sums
    full = open(os.path.join(out, "BCRX", "BCRX_fusion_gene_cell_predictions.txt")).read().splitlines()
    assert len(full) == 1 + n_rows


def _split_cells(paths, d, n_cells=3):
    """Writes the world's pairs as n_cells cells (contiguous slices) under d."""
    n1, s1 = afio.read_fastq(paths["fq1"])
    _, s2 = afio.read_fastq(paths["fq2"])
    os.makedirs(d, exist_ok=True)
    k = len(n1)
    for c in range(n_cells):
        lo, hi = c * k // n_cells, (c + 1) * k // n_cells
        for m, ss in ((1, s1), (2, s2)):
            with gzip.open(os.path.join(d, f"cell{c}_{m}.fastq.gz"), "wt") as fh:
                for i in range(lo, hi):
                    fh.write(f"@{n1[i]}/{m}\n{ss[i].decode()}\n+\n{'I' * len(ss[i])}\n")
    return [f"cell{c}" for c in range(n_cells)]


def _run_and_compare(tmp_path, searches_factory, aligner_factory):
    paths, truth = make_world(str(tmp_path / "world"))
    fqd = str(tmp_path / "cells")
    cells = _split_cells(paths, fqd)
    out = str(tmp_path / "sc_out")
    kw = {} if aligner_factory is None else dict(aligner_factory=aligner_factory)
    # two GPU batches: cells 0+1 together, cell 2 alone
    merged = singlecell.run(paths["anchor"], fqd, paths["genome"], paths["gtf"], out, searches=searches_factory(paths),
                            batch_pairs=2 * 2200 // 3 + 10, log=lambda *_: None, **kw)
    for c in cells:
        bulk = str(tmp_path / ("bulk_" + c))
        pipeline.run(paths["anchor"], os.path.join(fqd, f"{c}_1.fastq.gz"), os.path.join(fqd, f"{c}_2.fastq.gz"),
                     paths["genome"], paths["gtf"], bulk, searches=searches_factory(paths), log=lambda *_: None, **kw)
        a = open(os.path.join(out, "BCRX", "work_dir", c, "BCRX_fusion_predictions_abridged.txt")).read()
        b = open(os.path.join(bulk, "BCRX_fusion", "BCRX_fusion_predictions_abridged.txt")).read()
        assert a == b, c
    rows = [ln.split("\t") for ln in open(os.path.join(out, "BCRX", "BCRX_fusion_gene_cell_predictions_abridged.txt"))]
    hit = [r for r in rows[1:] if "ABLX" in r[0]]
    assert hit and abs(int(hit[0][2].split(":")[1]) - truth["anchor_junction"]) <= 3
    assert int(hit[0][7]) >= 2 and set(hit[0][8].strip().split(";")) <= set(cells)
    assert list(merged["BCRX"])


def test_singlecell_cpu_backends(tmp_path):
    from oracle_backends import OracleAligner, oracle_searches

    def searches(paths):
        genome = [(h.split()[0], s.decode().upper()) for h, s in pipeline.read_fasta(paths["genome"])]
        return oracle_searches(genome)
    _run_and_compare(tmp_path, searches, OracleAligner)


@pytest.mark.gpu
def test_singlecell_gpu(tmp_path):
    def searches(paths):
        genome = [(h.split()[0], s.decode().upper()) for h, s in pipeline.read_fasta(paths["genome"])]
        return pipeline.Searches(genome)
    _run_and_compare(tmp_path, searches, None)


@pytest.mark.gpu
def test_singlecell_gpu_tables_equal_oracle(tmp_path):
    """Single-cell on the GPU (cells batched, one device call per cell) vs the same driver with
    the CPU-oracle backends: every per-cell table and both merged tables identical."""
    from oracle_backends import OracleAligner, oracle_searches
    paths, truth = make_world(str(tmp_path / "world"))
    fqd = str(tmp_path / "cells")
    cells = _split_cells(paths, fqd, n_cells=4)
    genome = [(h.split()[0], s.decode().upper()) for h, s in pipeline.read_fasta(paths["genome"])]
    gpu, cpu = str(tmp_path / "gpu"), str(tmp_path / "cpu")
    singlecell.run(paths["anchor"], fqd, paths["genome"], paths["gtf"], gpu, searches=pipeline.Searches(genome),
                   batch_pairs=1200, log=lambda *_: None)
    singlecell.run(paths["anchor"], fqd, paths["genome"], paths["gtf"], cpu,
                   searches=oracle_searches(genome),
                   aligner_factory=OracleAligner, batch_pairs=1200, log=lambda *_: None)
    files = [os.path.join("BCRX", "work_dir", c, "BCRX_fusion_predictions" + x) for c in cells
             for x in (".txt", "_abridged.txt")]
    files += [os.path.join("BCRX", "BCRX_fusion_gene_cell_predictions" + x) for x in (".txt", "_abridged.txt")]
    for f in files:
        a = open(os.path.join(gpu, f), "rb").read()
        b = open(os.path.join(cpu, f), "rb").read()
        assert a == b, f
