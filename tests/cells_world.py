"""Single-cell inputs at configs[4] scale (TEST INFRASTRUCTURE): C cells x P pairs of 2x100 as
BGZF FASTQ pairs.  Each cell holds a slice of tests/fusion_world.make_world's fusion / anchor
pairs plus vectorised background fragments of the world genome (0.5 % substitutions)."""
import os
import struct
import zlib
from multiprocessing import Pool

import numpy as np


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


def write_cells(folder, n_cells, per_cell, seed=11, workers=16):
    """The world (make_world) under folder/world and the cells under folder/cells; returns
    (paths, truth, cells_dir, [cell names])."""
    from anchored_fusion_amd import io as afio
    from fusion_world import make_world
    paths, truth = make_world(os.path.join(folder, "world"), n_fusion=4000, n_anchor=3000, n_background=100)
    cells_dir = os.path.join(folder, "cells")
    os.makedirs(cells_dir, exist_ok=True)
    genome = np.concatenate([np.frombuffer(s, dtype=np.uint8) for _, s in afio.read_fasta(paths["genome"])])
    _, reads0, _ = afio.read_pairs(paths["fq1"], paths["fq2"])
    L = reads0.shape[1]
    k0 = reads0.shape[0] // 2
    rng = np.random.default_rng(seed)
    comp = np.zeros(256, dtype=np.uint8)
    for a, b in zip(b"ACGTN", b"TGCAN"):
        comp[a] = b
    names = []
    with Pool(max(1, min(workers, os.cpu_count() or 1))) as pool:
        for c in range(n_cells):
            lo, hi = c * k0 // n_cells, (c + 1) * k0 // n_cells
            m = max(0, per_cell - (hi - lo))
            F = rng.integers(220, 320, size=m)
            s = rng.integers(0, len(genome) - 320, size=m)
            r1 = genome[s[:, None] + np.arange(L)[None, :]]
            r2 = comp[genome[(s + F - L)[:, None] + np.arange(L)[None, :]][:, ::-1]]
            for r in (r1, r2):
                e = rng.random(r.shape) < 0.005
                r[e] = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, size=int(e.sum()))]
            for mate, (small, big) in enumerate(((reads0[2 * lo:2 * hi:2], r1), (reads0[2 * lo + 1:2 * hi:2], r2)),
                                                start=1):
                buf = fastq_bytes(f"c{c:04d}w", mate, small) + fastq_bytes(f"c{c:04d}b", mate, big)
                write_bgzf(os.path.join(cells_dir, f"cell{c:04d}_{mate}.fastq.gz"), buf, pool)
            names.append(f"cell{c:04d}")
    return paths, truth, cells_dir, names
