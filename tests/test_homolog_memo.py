"""The homolog set is made once per output folder, as the reference makes it (Anchored_Fusion.py:196:
`Find_homo_genes` runs only when <G>_homo_genes.bed is absent, and the file is read either way):
pipeline.homolog_rows writes the rows whole (tmp + rename) and a second call reads them back
without a search."""
import afpkg  # noqa: F401
from anchored_fusion_amd import pipeline

GTF = [
    "##x\n",
    'chr1\tS\tgene\t100\t900\t.\t+\t.\tgene_id "ENSG0001.1"; gene_type "protein_coding"; gene_name "AAA"; x\n',
    'chr1\tS\tgene\t5000\t6000\t.\t-\t.\tgene_id "ENSG0002.3"; gene_type "protein_coding"; gene_name "BBB"; x\n',
]


def _psl(chrom, s, e):
    return "\t".join(["100", "0", "0", "0", "0", "0", "0", "0", "+", "ANC", "100", "0", "100", chrom, "9000",
                      str(s), str(e), "1", "100,", "0,", f"{s},"]) + "\n"


def test_homolog_rows_made_once(tmp_path):
    calls = []

    def place(targets, queries, preset):
        calls.append(preset)
        return ["psLayout version 3\n", "\n", _psl("chr1", 150, 250), _psl("chr1", 5100, 5200)]

    path = str(tmp_path / "G_fusion_homo_genes.bed")
    rows = pipeline.homolog_rows(path, GTF, [("chr1", "A" * 9000)], "G", "ACGT" * 100, place)
    assert calls == ["homologs"] and [r[3] for r in rows] == ["ENSG0001.1", "ENSG0002.3"]
    again = pipeline.homolog_rows(path, GTF, [("chr1", "A" * 9000)], "G", "ACGT" * 100, place)
    assert calls == ["homologs"] and again == rows
    assert not (tmp_path / "G_fusion_homo_genes.bed.tmp").exists()
