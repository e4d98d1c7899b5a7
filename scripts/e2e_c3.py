"""End-to-end leg at BASELINE.json configs[2] size: FASTQ.gz pair -> Final_fusion tables through the
product path (pipeline.run: native BGZF ingest, genome + tile indexes built on the GPU, homologs,
S2-S6 in HBM via discover.CandidateDiscovery, host stages on the gathered queries).

The inputs are written to disk first, as the reference's user has them: the simworld genome
(hg38-sized contigs with repeat families, anchor + 8 partner genes as exons) as FASTA, a GTF of the
embedded genes, the anchor FASTA (the bundled BCR transcript), and `pairs` wgsim-style 2x150 pairs as
BGZF FASTQ (--fusion-frac of them from the anchor fusions, 0.1 % by default).  Then pipeline.run runs from those files alone; its log
lines carry each phase's time.  Prints one JSON line.

    python scripts/e2e_c3.py [--pairs 50000000] [--scale 1.0] [--out gpurun_out/e2e_c3.json]
"""
import argparse
import json
import os
import sys
import time
from multiprocessing import Pool

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import afpkg  # noqa: E402,F401
import numpy as np  # noqa: E402

CHUNK = 2_000_000  # pairs simulated / written per round trip


def fastq_records(first, mate, seqs):
    """'@c3<9-digit index>/<mate>' records of uint8 [n, L] sequences, one buffer (vectorised)."""
    n, L = seqs.shape
    idx = np.arange(first, first + n, dtype=np.int64)
    digits = np.empty((n, 9), np.uint8)
    for k in range(8, -1, -1):
        digits[:, k] = ord("0") + idx % 10
        idx //= 10
    head = np.frombuffer(b"@c3", np.uint8)
    tail = np.frombuffer(f"/{mate}\n".encode(), np.uint8)
    w = len(head) + 9 + len(tail)
    rec = np.empty((n, w + L + 3 + L + 1), np.uint8)
    rec[:, :3] = head
    rec[:, 3:12] = digits
    rec[:, 12:w] = tail
    rec[:, w:w + L] = seqs
    rec[:, w + L:w + L + 3] = np.frombuffer(b"\n+\n", np.uint8)
    rec[:, w + L + 3:w + 2 * L + 3] = ord("I")
    rec[:, -1] = ord("\n")
    return rec.tobytes()


def write_inputs(folder, n_pairs, scale, log, fusion_frac):
    import torch

    from anchored_fusion_amd import io as afio
    from anchored_fusion_amd.simworld import GenomeWorld
    from e2e_bench import _bgzf_block
    os.makedirs(folder, exist_ok=True)
    paths = {k: os.path.join(folder, v) for k, v in dict(
        fq1="c3_1.fastq.gz", fq2="c3_2.fastq.gz", genome="genome.fa", gtf="genes.gtf", anchor="anchor.fa").items()}
    src_fa = os.path.join(ROOT, "tests", "golden", "target_gene.fasta")
    with open(src_fa) as fh:
        header = fh.readline().rstrip()[1:]
    anchor = afio.anchor_sequence(src_fa)
    t0 = time.perf_counter()
    W = GenomeWorld(anchor, device=0, scale=scale)
    log(f"world built ({time.perf_counter() - t0:.1f} s)")
    # genome FASTA, 60 columns
    t0 = time.perf_counter()
    blob = W.blob.cpu().numpy()
    with open(paths["genome"], "wb") as fh:
        for name, off, L in zip(W.names, W.offsets, W.lens):
            fh.write(f">{name}\n".encode())
            s = blob[off:off + L]
            full = (L // 60) * 60
            lines = np.empty((L // 60, 61), np.uint8)
            lines[:, :60] = s[:full].reshape(-1, 60)
            lines[:, 60] = ord("\n")
            fh.write(lines.tobytes())
            if full < L:
                fh.write(s[full:].tobytes() + b"\n")
    del blob
    # GTF of the embedded genes (1-based closed), the anchor named as its FASTA header names it
    gene_name = header.split()[1]
    gtf = ["##description: simworld genes (scripts/e2e_c3.py)\n"]
    for k, (g, spans) in enumerate(W.loci.items()):
        name = gene_name if g == "anchor" else g.upper()
        gid = f"ENSG{90000000000 + k:011d}.1"
        c = spans[0][0]
        attrs = f'gene_id "{gid}"; gene_type "protein_coding"; gene_name "{name}"; level 2;'
        gtf.append("\t".join([c, "SIM", "gene", str(spans[0][1] + 1), str(spans[-1][2]), ".", "+", ".", attrs]) + "\n")
        ta = f'gene_id "{gid}"; transcript_id "{gid}-T"; transcript_type "protein_coding"; gene_name "{name}";'
        gtf.append("\t".join([c, "SIM", "transcript", str(spans[0][1] + 1), str(spans[-1][2]), ".", "+", ".", ta])
                   + "\n")
        for j, (_, a, b) in enumerate(spans):
            gtf.append("\t".join([c, "SIM", "exon", str(a + 1), str(b), ".", "+", ".", ta + f" exon_number {j + 1};"])
                       + "\n")
    with open(paths["gtf"], "w") as fh:
        fh.writelines(gtf)
    afio.write_fasta(paths["anchor"], [(header, anchor.decode())], width=70)
    log(f"genome FASTA, GTF, anchor written ({time.perf_counter() - t0:.1f} s)")
    # reads: simulated in HBM per chunk, BGZF-compressed on the host's cores
    t0 = time.perf_counter()
    dev = torch.device("cuda", 0)
    buf = torch.empty((2 * CHUNK, 150), dtype=torch.uint8, device=dev)
    with Pool(min(16, os.cpu_count() or 1)) as pool, open(paths["fq1"], "wb") as f1, open(paths["fq2"], "wb") as f2:
        for first in range(0, n_pairs, CHUNK):
            n = min(CHUNK, n_pairs - first)
            W.simulate_pairs(n, read_len=150, seed=20251015, pair_base=first, out=buf[:2 * n], fusion_frac=fusion_frac)
            r = buf[:2 * n].cpu().numpy()
            for fh, mate in ((f1, 1), (f2, 2)):
                data = fastq_records(first, mate, r[mate - 1::2])
                blocks = [data[i:i + 65280] for i in range(0, len(data), 65280)]
                for b in pool.imap(_bgzf_block, blocks, chunksize=64):
                    fh.write(b)
            log(f"reads: {first + n} of {n_pairs} pairs written ({time.perf_counter() - t0:.1f} s)")
        for fh in (f1, f2):
            fh.write(_bgzf_block(b""))
    junctions = list(W.junctions)
    del buf, W
    torch.cuda.empty_cache()
    return paths, gene_name, junctions, time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=50_000_000)
    ap.add_argument("--scale", type=float, default=1.0, help="genome scale (1.0 = hg38-sized contigs)")
    ap.add_argument("--fusion-frac", type=float, default=0.001,
                    help="pairs from the fusion transcripts (the bench's 5 %% puts ~10^5 split reads on each "
                         "junction, where the reference's split-read clustering, functions.py:771-951, is "
                         "quadratic in Python whatever the aligner)")
    ap.add_argument("--out", default=None)
    ap.add_argument("--folder", default=os.path.join(os.environ.get("TMPDIR", "/tmp"), "af_e2e_c3"))
    args = ap.parse_args()
    t_start = time.perf_counter()
    marks = []

    def log(msg):
        t = time.perf_counter() - t_start
        marks.append((round(t, 1), msg))
        print(f"[{t:8.1f} s] {msg}", flush=True)
    from anchored_fusion_amd import pipeline
    paths, gene, junctions, t_reads = write_inputs(args.folder, args.pairs, args.scale, log, args.fusion_frac)
    outdir = os.path.join(args.folder, "out")
    t0 = time.perf_counter()
    pipeline.run(paths["anchor"], paths["fq1"], paths["fq2"], paths["genome"], paths["gtf"], outdir, log=log)
    t_run = time.perf_counter() - t0
    tab = os.path.join(outdir, f"{gene}_fusion", f"{gene}_fusion_predictions_abridged.txt")
    rows = [ln.rstrip("\n").split("\t") for ln in open(tab)] if os.path.exists(tab) else []
    partners = sorted({r[0] for r in rows[1:]})
    res = {
        "leg": "end to end at configs[2] size: BGZF FASTQ pair + genome FASTA + GTF on disk -> pipeline.run "
               "(native ingest, GPU genome / tile indexes, homologs, S2-S6 in HBM, host stages) -> tables",
        "pairs": args.pairs, "read_len": 150, "genome_scale": args.scale, "fusion_frac": args.fusion_frac,
        "fastq_gz_bytes": os.path.getsize(paths["fq1"]) + os.path.getsize(paths["fq2"]),
        "wall_s": round(t_run, 1), "pairs_per_s": round(args.pairs / t_run, 1),
        "phases": [m for m in marks if m[0] >= round(t0 - t_start, 1)],
        "predictions": len(rows) - 1 if rows else 0, "partners": partners[:20],
        "planted_fusions": len(junctions), "inputs_written_s": round(t_reads, 1),
        "host_threads": int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or os.cpu_count(),
    }
    line = json.dumps(res)
    print(line, flush=True)
    if args.out:
        with open(args.out, "w") as fh:
            fh.write(line + "\n")


if __name__ == "__main__":
    main()
