"""End-to-end leg (FASTQ.gz -> candidate TSV) on a configs[1]-sized sample: 1 M 2x100 pairs.

The world (genome, GTF, anchor, planted BCRX-ABLX fusion) is tests/fusion_world.make_world's;
its background is scaled up with vectorised fragments of the same sources, written as BGZF
(bgzip's blocked gzip, which the native reader inflates block-parallel).  Times `io.read_pairs`
alone and `pipeline.run` (ingest -> S2 on the GPU -> S3-S8 -> Final_fusion tables) on the GPU
box's host CPU share.  Prints one JSON line.

    python scripts/e2e_bench.py [pairs] [out.json]
"""
import json
import os
import struct
import sys
import time
import zlib
from multiprocessing import Pool

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import afpkg  # noqa: E402,F401
import numpy as np  # noqa: E402


def _bgzf_block(data):
    c = zlib.compressobj(1, zlib.DEFLATED, -15)
    cd = c.compress(data) + c.flush()
    hdr = b"\x1f\x8b\x08\x04\x00\x00\x00\x00\x00\xff\x06\x00BC\x02\x00" + struct.pack("<H", len(cd) + 25)
    return hdr + cd + struct.pack("<II", zlib.crc32(data) & 0xFFFFFFFF, len(data))


def write_bgzf(path, data, pool):
    blocks = [data[i:i + 65280] for i in range(0, len(data), 65280)]
    with open(path, "wb") as fh:
        for b in pool.imap(_bgzf_block, blocks, chunksize=64):
            fh.write(b)
        fh.write(_bgzf_block(b""))  # EOF marker block


def fastq_bytes(tag, mate, seqs):
    """Fixed-width records '@{tag}{i:08d}/{mate}' of uint8 [n, L] sequences, as one buffer."""
    n, L = seqs.shape
    name = [f"@{tag}{i:08d}/{mate}\n".encode() for i in range(n)]
    w = len(name[0])
    rec = np.empty((n, w + L + 3 + L + 1), dtype=np.uint8)
    rec[:, :w] = np.frombuffer(b"".join(name), dtype=np.uint8).reshape(n, w)
    rec[:, w:w + L] = seqs
    rec[:, w + L:w + L + 3] = np.frombuffer(b"\n+\n", dtype=np.uint8)
    rec[:, w + L + 3:w + 2 * L + 3] = ord("I")
    rec[:, -1] = ord("\n")
    return rec.tobytes()


def main():
    n_pairs = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    out = sys.argv[2] if len(sys.argv) > 2 else None
    from fusion_world import make_world
    from anchored_fusion_amd import io as afio
    from anchored_fusion_amd import pipeline
    folder = os.path.join(os.environ.get("TMPDIR", "/tmp"), "af_e2e")
    t0 = time.perf_counter()
    paths, truth = make_world(folder, n_fusion=2000, n_anchor=1500, n_background=2000)
    # scale the background: fragments of the world's genome (all four contigs), 0.5 % errors
    rng = np.random.default_rng(7)
    genome = np.concatenate([np.frombuffer(s, dtype=np.uint8) for _, s in afio.read_fasta(paths["genome"])])
    names0, reads0, _ = afio.read_pairs(paths["fq1"], paths["fq2"])
    L = reads0.shape[1]
    m = n_pairs - reads0.shape[0] // 2
    F = rng.integers(220, 320, size=m)
    s = rng.integers(0, len(genome) - 320, size=m)
    idx = s[:, None] + np.arange(L)[None, :]
    r1 = genome[idx]
    r2 = genome[(s + F - L)[:, None] + np.arange(L)[None, :]][:, ::-1]
    comp = np.zeros(256, dtype=np.uint8)
    for a, b in zip(b"ACGTN", b"TGCAN"):
        comp[a] = b
    r2 = comp[r2]
    for r in (r1, r2):
        e = rng.random(r.shape) < 0.005
        r[e] = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, size=int(e.sum()))]
    fq = {}
    with Pool(min(16, os.cpu_count() or 1)) as pool:
        for mate, (small, big) in enumerate(((reads0[0::2], r1), (reads0[1::2], r2)), start=1):
            buf = fastq_bytes("w", mate, small) + fastq_bytes("bgx", mate, big)
            fq[mate] = os.path.join(folder, f"big_{mate}.fastq.gz")
            write_bgzf(fq[mate], buf, pool)
    t_gen = time.perf_counter() - t0
    # ingest alone, then the whole pipeline (its own ingest included)
    t0 = time.perf_counter()
    names, reads, lens = afio.read_pairs(fq[1], fq[2])
    t_ingest = time.perf_counter() - t0
    assert reads.shape[0] == 2 * n_pairs
    del names, reads, lens
    outdir = os.path.join(folder, "out")
    t0 = time.perf_counter()
    pipeline.run(paths["anchor"], fq[1], fq[2], paths["genome"], paths["gtf"], outdir, log=lambda *_: None)
    t_run = time.perf_counter() - t0
    rows = [ln.split("\t") for ln in open(os.path.join(outdir, "BCRX_fusion", "BCRX_fusion_predictions_abridged.txt"))]
    hit = [r for r in rows[1:] if "ABLX" in r[0]]
    res = {
        "leg": "end to end: BGZF FASTQ pair -> io ingest -> S2 on the GPU (host-buffer API) -> S3-S8 -> "
               "Final_fusion tables (pipeline.run, one anchor)",
        "pairs": n_pairs, "read_len": int(L), "fastq_gz_bytes": os.path.getsize(fq[1]) + os.path.getsize(fq[2]),
        "wall_s": round(t_run, 3), "pairs_per_s": round(n_pairs / t_run, 1),
        "ingest_only_s": round(t_ingest, 3), "ingest_pairs_per_s": round(n_pairs / t_ingest, 1),
        "host_threads": int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or os.cpu_count(),
        "fusion_found": bool(hit), "breakpoint": hit[0][2] if hit else None,
        "truth_junction": truth["anchor_junction"], "generate_s": round(t_gen, 1),
    }
    line = json.dumps(res)
    print(line, flush=True)
    if out:
        with open(out, "w") as fh:
            fh.write(line + "\n")


if __name__ == "__main__":
    main()
