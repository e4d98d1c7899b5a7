"""Host-side sequence I/O: FASTA/FASTQ(.gz) -> the device layout used by the C-ABI.

Device layout: reads are pair-major, one byte per base (ASCII as read
from the FASTQ), row ``2p`` = mate 1 and row ``2p + 1`` = mate 2 of pair ``p``, packed at a
fixed ``stride`` (the longest read).  A ``lens`` vector is only materialised when the batch
is ragged, so a fixed-length Illumina batch streams exactly 2·L bytes per pair.

Read names follow bwa's convention: the name is the first whitespace-delimited token and a
trailing ``/1`` or ``/2`` is stripped (Anchored_Fusion.py:182 feeds FASTQs to ``bwa mem``,
whose QNAMEs are what ``Find_blocks`` / ``contact_reads`` compare, functions.py:399, 917).
"""
import gzip
import io as _io
import os

import numpy as np


def _open(path):
    with open(path, "rb") as fh:
        magic = fh.read(2)
    if magic == b"\x1f\x8b":
        return _io.BufferedReader(gzip.open(path, "rb"))
    return open(path, "rb")


def read_fasta(path):
    """Returns a list of (header_line_without_gt, sequence_bytes)."""
    recs = []
    name, chunks = None, []
    with _open(path) as fh:
        for line in fh:
            line = line.rstrip(b"\r\n")
            if line.startswith(b">"):
                if name is not None:
                    recs.append((name, b"".join(chunks)))
                name, chunks = line[1:].decode(), []
            elif name is not None:
                chunks.append(line.strip())
    if name is not None:
        recs.append((name, b"".join(chunks)))
    return recs


def qname(raw):
    """bwa's QNAME: first token, trailing /1 or /2 removed."""
    nm = raw.split()[0] if raw else raw
    if len(nm) > 2 and nm[-2] == "/" and nm[-1].isdigit():
        nm = nm[:-2]
    return nm


def read_fastq(path):
    """Returns (names, seqs) with names as bwa QNAMEs and seqs as bytes."""
    names, seqs = [], []
    with _open(path) as fh:
        while True:
            h = fh.readline()
            if not h:
                break
            s = fh.readline().rstrip(b"\r\n")
            fh.readline()
            fh.readline()
            h = h.rstrip(b"\r\n")
            if not h.startswith(b"@"):
                raise ValueError(f"{path}: malformed FASTQ record header {h[:40]!r}")
            names.append(qname(h[1:].decode()))
            seqs.append(s)
    return names, seqs


def pack_reads(seqs, stride=None):
    """Packs byte strings into a [n, stride] uint8 matrix; returns (mat, lens or None)."""
    n = len(seqs)
    lens = np.fromiter((len(s) for s in seqs), dtype=np.int32, count=n)
    if stride is None:
        stride = int(lens.max()) if n else 0
    mat = np.full((n, max(stride, 1)), ord("N"), dtype=np.uint8)
    if n:
        if (lens == stride).all():
            mat[:] = np.frombuffer(b"".join(seqs), dtype=np.uint8).reshape(n, stride)
            return mat, None
        for i, s in enumerate(seqs):
            mat[i, : len(s)] = np.frombuffer(s, dtype=np.uint8)
    return mat, lens


def read_pairs(fq1, fq2):
    """Reads a FASTQ pair into the pair-major layout.

    Returns ``(names, reads[2N, stride] uint8, lens[2N] int32 or None)``; ``names[p]`` is the
    QNAME of pair p (mates must agree, as bwa requires for paired input)."""
    n1, s1 = read_fastq(fq1)
    n2, s2 = read_fastq(fq2)
    if len(s1) != len(s2):
        raise ValueError(f"paired FASTQs differ in length: {len(s1)} vs {len(s2)}")
    inter = [None] * (2 * len(s1))
    inter[0::2] = s1
    inter[1::2] = s2
    mat, lens = pack_reads(inter)
    return n1, mat, lens


def anchor_sequence(path, index=0):
    """The ``index``-th record of an anchor FASTA as uppercase bytes (AF:154-163 writes each
    record of --file_anchored_cds to its own single-record FASTA)."""
    recs = read_fasta(path)
    if index >= len(recs):
        raise IndexError(f"{path}: no FASTA record {index}")
    return recs[index][1].upper()


def write_fasta(path, recs, width=60):
    tmp = path + ".tmp"
    with open(tmp, "w") as fh:
        for name, seq in recs:
            if isinstance(seq, (bytes, bytearray)):
                seq = seq.decode()
            fh.write(">" + name + "\n")
            for i in range(0, len(seq), width):
                fh.write(seq[i:i + width] + "\n")
    os.replace(tmp, path)
