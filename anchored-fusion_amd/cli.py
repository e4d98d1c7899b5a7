"""Command line of the GPU pipeline, with the flags of Anchored_Fusion.py:15-30.

    python run_anchored_fusion.py --file_anchored_cds anchor.fa --fastq1 s_1.fq.gz --fastq2 s_2.fq.gz \
        --file_ref_seq genome.fa --file_ref_ann genes.gtf --out_folder out/

Outputs go to `<out_folder>/<G>_fusion/<G>_fusion_predictions{,_abridged}.txt`, as in
AF:138-141 and Final_fusion. Some flags are accepted only so that existing command lines keep
working, and do nothing:
- the filter-model flags (Model.py is outside SURVEY.md §8), so every run behaves as
  `--not_filter_false_positive`;
- `--thread` (host threads; the searches run on the GPU).
"""
import argparse
import sys

from . import pipeline


def parser():
    ap = argparse.ArgumentParser(description="Anchor Gene Fusion Detection on MI355X")
    ap.add_argument("--file_anchored_cds", type=str, required=True, help="Target gene fasta file of anchored transcript")
    ap.add_argument("--gene_names", type=str, default="", help="The file of target gene names")
    ap.add_argument("--fastq1", type=str, default="fastq_1.fastq", help="The fastq1 file to scan")
    ap.add_argument("--fastq2", type=str, default="fastq_2.fastq", help="The fastq2 file to scan")
    ap.add_argument("--out_folder", type=str, default="./", help="The folder of the output file")
    ap.add_argument("--file_ref_seq", type=str, required=True, help="The reference sequence file")
    ap.add_argument("--file_ref_ann", type=str, required=True, help="The reference annotation file")
    ap.add_argument("--not_filter_false_positive", action="store_true", help="(always on: no filter model)")
    ap.add_argument("--not_train_filter_model", action="store_true", help="(accepted, unused)")
    ap.add_argument("--model_file", type=str, default="./data/model.pt", help="(accepted, unused)")
    ap.add_argument("--positive_samples", type=str, default="./data/positive_samples.txt", help="(accepted, unused)")
    ap.add_argument("--homo_gene_file", type=str, default="./data/homo_gene.npy", help="(accepted, unused)")
    ap.add_argument("--negative_samples", type=str, default="./Model/negative_samples.txt", help="(accepted, unused)")
    ap.add_argument("--thread", type=str, default="1", help="(accepted, unused)")
    ap.add_argument("--gpu_number", type=str, default="-1", help="GPU index (-1: the first visible GPU)")
    return ap


def parser_singlecell():
    """The flags of Anchored_Fusion_singlecell.py:15-31 (--fastq_dir instead of --fastq1/2)."""
    ap = argparse.ArgumentParser(description="Anchor Gene Fusion Detection (single cell) on MI355X")
    ap.add_argument("--file_anchored_cds", type=str, required=True, help="Target gene fasta file of anchored transcript")
    ap.add_argument("--gene_names", type=str, default="", help="The file of target gene names")
    ap.add_argument("--fastq_dir", type=str, required=True, help="The fastq files to scan")
    ap.add_argument("--out_folder", type=str, default="./", help="The folder of the output file")
    ap.add_argument("--file_ref_seq", type=str, required=True, help="The reference sequence file")
    ap.add_argument("--file_ref_ann", type=str, required=True, help="The reference annotation file")
    ap.add_argument("--not_filter_false_positive", action="store_true", help="(always on: no filter model)")
    ap.add_argument("--not_train_filter_model", action="store_true", help="(accepted, unused)")
    ap.add_argument("--model_file", type=str, default="./data/model.pt", help="(accepted, unused)")
    ap.add_argument("--positive_samples", type=str, default="./data/positive_samples.txt", help="(accepted, unused)")
    ap.add_argument("--homo_gene_file", type=str, default="./data/homo_gene.npy", help="(accepted, unused)")
    ap.add_argument("--negative_samples", type=str, default="./Model/negative_samples.txt", help="(accepted, unused)")
    ap.add_argument("--thread", type=str, default="1", help="(accepted, unused)")
    ap.add_argument("--gpu_number", type=str, default="-1", help="GPU index (-1: the first visible GPU)")
    ap.add_argument("--batch_pairs", type=int, default=1 << 22, help="pairs of whole cells per GPU alignment batch")
    return ap


def main_singlecell(argv=None):
    from . import singlecell
    args = parser_singlecell().parse_args(argv)
    dev = int(args.gpu_number)
    singlecell.run(args.file_anchored_cds, args.fastq_dir, args.file_ref_seq, args.file_ref_ann, args.out_folder,
                   gene_names=args.gene_names or None, device=dev if dev >= 0 else 0, batch_pairs=args.batch_pairs)
    return 0


def main(argv=None):
    args = parser().parse_args(argv)
    dev = int(args.gpu_number)
    pipeline.run(args.file_anchored_cds, args.fastq1, args.fastq2, args.file_ref_seq, args.file_ref_ann,
                 args.out_folder, gene_names=args.gene_names or None, device=dev if dev >= 0 else 0)
    return 0


if __name__ == "__main__":
    sys.exit(main())
