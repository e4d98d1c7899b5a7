"""Command line of the GPU pipeline, with the flags of Anchored_Fusion.py:15-30.

    python run_anchored_fusion.py --file_anchored_cds anchor.fa --fastq1 s_1.fq.gz --fastq2 s_2.fq.gz \
        --file_ref_seq genome.fa --file_ref_ann genes.gtf --out_folder out/

Outputs go to `<out_folder>/<G>_fusion/<G>_fusion_predictions{,_abridged}.txt`, as in
AF:138-141 and Final_fusion. Some flags are accepted only so that existing command lines keep
working, and do nothing: `--not_train_filter_model`, `--positive_samples`, `--homo_gene_file`,
`--negative_samples` (training is outside SURVEY.md §8).  `--thread T` sets bwa's input chunk to
10,000,000 x T bases (`bwa mem -t T` at AF:182/188 estimates insert sizes per chunk, so the records
depend on it); the work itself runs on the GPU.  Without `--not_filter_false_positive` the filter model `--model_file` scores
the candidates (AF:212-225); a missing model file is reported and the run continues unfiltered,
as the reference does.

`--gpus N` (N > 1) runs one process per GPU: the command relaunches itself under
`torch.distributed.run` (a child process; this process never touches the GPU), each rank takes
GPU LOCAL_RANK and joins an RCCL process group; S2 is sharded over the ranks (pipeline.run,
shard.py) and single-cell batches are dealt out to them (singlecell.run).
"""
import argparse
import datetime
import os
import socket
import subprocess
import sys

from . import pipeline

_PG_TIMEOUT = datetime.timedelta(hours=12)


def parser():
    ap = argparse.ArgumentParser(description="Anchor Gene Fusion Detection on MI355X")
    ap.add_argument("--file_anchored_cds", type=str, required=True, help="Target gene fasta file of anchored transcript")
    ap.add_argument("--gene_names", type=str, default="", help="The file of target gene names")
    ap.add_argument("--fastq1", type=str, default="fastq_1.fastq", help="The fastq1 file to scan")
    ap.add_argument("--fastq2", type=str, default="fastq_2.fastq", help="The fastq2 file to scan")
    ap.add_argument("--out_folder", type=str, default="./", help="The folder of the output file")
    ap.add_argument("--file_ref_seq", type=str, required=True, help="The reference sequence file")
    ap.add_argument("--file_ref_ann", type=str, required=True, help="The reference annotation file")
    ap.add_argument("--not_filter_false_positive", action="store_true", help="Do not score candidates with the filter model")
    ap.add_argument("--not_train_filter_model", action="store_true", help="(accepted, unused)")
    ap.add_argument("--model_file", type=str, default="./data/model.pt", help="The filter model (Model.py state_dict)")
    ap.add_argument("--positive_samples", type=str, default="./data/positive_samples.txt", help="(accepted, unused)")
    ap.add_argument("--homo_gene_file", type=str, default="./data/homo_gene.npy", help="(accepted, unused)")
    ap.add_argument("--negative_samples", type=str, default="./Model/negative_samples.txt", help="(accepted, unused)")
    ap.add_argument("--thread", type=str, default="1", help="bwa threads: sets the 10,000,000 x T base input chunk")
    ap.add_argument("--gpu_number", type=str, default="-1", help="GPU index (-1: the first visible GPU)")
    ap.add_argument("--gpus", type=int, default=1, help="GPUs of this node to shard the pairs over (one process each)")
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
    ap.add_argument("--not_filter_false_positive", action="store_true", help="Do not score candidates with the filter model")
    ap.add_argument("--not_train_filter_model", action="store_true", help="(accepted, unused)")
    ap.add_argument("--model_file", type=str, default="./data/model.pt", help="The filter model (Model.py state_dict)")
    ap.add_argument("--positive_samples", type=str, default="./data/positive_samples.txt", help="(accepted, unused)")
    ap.add_argument("--homo_gene_file", type=str, default="./data/homo_gene.npy", help="(accepted, unused)")
    ap.add_argument("--negative_samples", type=str, default="./Model/negative_samples.txt", help="(accepted, unused)")
    ap.add_argument("--thread", type=str, default="1", help="bwa threads: sets the 10,000,000 x T base input chunk")
    ap.add_argument("--gpu_number", type=str, default="-1", help="GPU index (-1: the first visible GPU)")
    ap.add_argument("--batch_pairs", type=int, default=1 << 22, help="pairs of whole cells per GPU alignment batch")
    ap.add_argument("--gpus", type=int, default=1, help="GPUs of this node to deal the cell batches to (one process each)")
    return ap


def _chunk_bases(args):
    """bwa's input chunk for --thread T (bwa mem: 10,000,000 x T bases, no -K)."""
    t = int(args.thread)
    if t < 1:
        raise SystemExit("--thread must be >= 1")
    return 10_000_000 * t


def _launch(n, script, argv):
    """Runs `script argv` as n ranks under torch.distributed.run (127.0.0.1 rendezvous) in a
    child process and returns its exit code."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", script] + list(argv)
    return subprocess.call(cmd, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))


def _rank_device(args):
    """Inside a launched job: join the process group (RCCL on GPUs, gloo otherwise) and return
    this rank's GPU (LOCAL_RANK); outside one: --gpu_number."""
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        import torch
        import torch.distributed as dist
        local = int(os.environ.get("LOCAL_RANK", "0"))
        if torch.cuda.is_available():
            torch.cuda.set_device(local)
            # rank 0 runs S3-S8 of each gene while the others wait in the next collective: a
            # generous timeout instead of the watchdog default
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=_PG_TIMEOUT)
        else:
            dist.init_process_group("gloo", timeout=_PG_TIMEOUT)
        return local
    dev = int(args.gpu_number)
    return dev if dev >= 0 else 0


def _finish():
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()


def _filter(args, dev):
    """The filter step's settings (AF:212-225), None with --not_filter_false_positive."""
    if args.not_filter_false_positive:
        return None
    import torch
    return dict(model_file=args.model_file, device=f"cuda:{dev}" if torch.cuda.is_available() else "cpu")


def _script(name):
    return os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), name)


def main_singlecell(argv=None):
    from . import singlecell
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parser_singlecell().parse_args(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return _launch(args.gpus, _script("run_anchored_fusion_singlecell.py"), argv)
    dev = _rank_device(args)
    try:
        singlecell.run(args.file_anchored_cds, args.fastq_dir, args.file_ref_seq, args.file_ref_ann,
                       args.out_folder, gene_names=args.gene_names or None, device=dev, batch_pairs=args.batch_pairs,
                       filt=_filter(args, dev), chunk_bases=_chunk_bases(args))
    finally:
        _finish()
    return 0


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parser().parse_args(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return _launch(args.gpus, _script("run_anchored_fusion.py"), argv)
    dev = _rank_device(args)
    try:
        pipeline.run(args.file_anchored_cds, args.fastq1, args.fastq2, args.file_ref_seq, args.file_ref_ann,
                     args.out_folder, gene_names=args.gene_names or None, device=dev, filt=_filter(args, dev),
                     chunk_bases=_chunk_bases(args))
    finally:
        _finish()
    return 0


if __name__ == "__main__":
    sys.exit(main())
