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
    """Returns a list of (header_line_without_gt, sequence_bytes): sequence lines joined with
    their surrounding whitespace stripped, lines before the first header ignored.  Whole-buffer
    form (C-speed joins: a 3.1 Gbp genome in seconds); records whose sequence lines carry blanks
    or a CR outside a line end take the line-by-line rule."""
    with _open(path) as fh:
        data = fh.read()
    recs = []
    at = 0 if data.startswith(b">") else data.find(b"\n>") + 1
    if at == 0 and not data.startswith(b">"):
        return recs
    while at < len(data):
        nxt = data.find(b"\n>", at)
        end = len(data) if nxt < 0 else nxt + 1
        rec = data[at:end]
        nl = rec.find(b"\n")
        head, body = (rec, b"") if nl < 0 else (rec[:nl], rec[nl + 1:])
        name = head.rstrip(b"\r\n")[1:].decode()
        if any(c in body for c in (b" ", b"\t", b"\x0b", b"\x0c")) or body.count(b"\r") != body.count(b"\r\n"):
            seq = b"".join(ln.rstrip(b"\r\n").strip() for ln in body.split(b"\n"))
        else:
            seq = body.replace(b"\n", b"").replace(b"\r", b"")
        recs.append((name, seq))
        at = end
    return recs


def qname(raw):
    """bwa's QNAME: first token, trailing /1 or /2 removed."""
    nm = raw.split()[0] if raw else raw
    if len(nm) > 2 and nm[-2] == "/" and nm[-1].isdigit():
        nm = nm[:-2]
    return nm


def read_fastq(path):
    """Returns (names, seqs) with names as bwa QNAMEs and seqs as bytes (single-file reader for
    small inputs; paired input goes through the native reader, ``read_pairs``)."""
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


class Names:
    """QNAMEs of a batch of pairs, kept as one NUL-terminated arena plus an offset per pair
    (a 50 M-pair run holds no per-read Python objects); indexes like a list of str."""

    def __init__(self, arena, off):
        self.arena = arena  # bytes
        self.off = off      # int64 [n]

    def __len__(self):
        return len(self.off)

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[k] for k in range(*i.indices(len(self)))]
        o = int(self.off[i])
        return self.arena[o:self.arena.index(b"\0", o)].decode()

    def __iter__(self):
        return (self[k] for k in range(len(self)))

    def slice(self, a, b):
        """Names of pairs [a, b) (shares the arena)."""
        return Names(self.arena, self.off[a:b])

    @staticmethod
    def concat(parts):
        if len(parts) == 1:
            return parts[0]
        arenas, offs, base = [], [], 0
        for p in parts:
            arenas.append(p.arena)
            offs.append(p.off + base)
            base += len(p.arena)
        return Names(b"".join(arenas), np.concatenate(offs) if offs else np.zeros(0, np.int64))


def iter_pairs(fq1, fq2, batch_pairs=1 << 20, threads=0):
    """Streams a FASTQ(.gz) pair through the native reader (csrc/ingest.cpp, af_fastq_*):
    yields ``(names, reads[2n, stride] uint8, lens[2n] int32)`` per batch of <= batch_pairs
    pairs, with stride = the batch's longest read."""
    import ctypes

    from . import _lib
    L = _lib.lib()
    h = ctypes.c_void_p()
    rc = L.af_fastq_open(os.fsencode(fq1), os.fsencode(fq2), int(threads), ctypes.byref(h))
    try:
        if rc != 0:
            raise _lib.AFError(f"af_fastq_open failed (rc={rc}): {L.af_fastq_error(h).decode(errors='replace')}")
        while True:
            n, ml, nb = ctypes.c_int64(), ctypes.c_int32(), ctypes.c_int64()
            rc = L.af_fastq_next(h, int(batch_pairs), ctypes.byref(n), ctypes.byref(ml), ctypes.byref(nb))
            if rc != 0:
                raise ValueError(f"{fq1}, {fq2}: {L.af_fastq_error(h).decode(errors='replace')}")
            if n.value == 0:
                return
            stride = max(int(ml.value), 1)
            reads = np.empty((2 * n.value, stride), dtype=np.uint8)
            lens = np.empty(2 * n.value, dtype=np.int32)
            arena = np.empty(max(int(nb.value), 1), dtype=np.uint8)
            off = np.empty(n.value, dtype=np.int64)
            rc = L.af_fastq_export(h, stride, reads.ctypes.data, lens.ctypes.data, arena.ctypes.data,
                                   arena.size, off.ctypes.data)
            if rc != 0:
                raise _lib.AFError(f"af_fastq_export failed (rc={rc}): {L.af_fastq_error(h).decode()}")
            yield Names(arena.tobytes(), off), reads, lens
    finally:
        L.af_fastq_close(h)


class NotBGZF(ValueError):
    """A sharded read of input that is not BGZF (blocked gzip)."""


def read_part(path, part, parts, threads=0):
    """Part `part` of `parts` of ONE BGZF FASTQ file (af_fastq_part_read: the records whose header
    starts in that share of the compressed blocks): ``(names, seqs[n, stride] uint8, lens[n]
    int32)``.  Raises NotBGZF for other input."""
    import ctypes

    from . import _lib
    L = _lib.lib()
    h = ctypes.c_void_p()
    n, ml, nb = ctypes.c_int64(), ctypes.c_int32(), ctypes.c_int64()
    rc = L.af_fastq_part_read(os.fsencode(path), int(part), int(parts), int(threads), ctypes.byref(h), ctypes.byref(n),
                              ctypes.byref(ml), ctypes.byref(nb))
    try:
        if rc == _lib.AF_E_UNSUPPORTED:
            raise NotBGZF(L.af_fastq_part_error(h).decode(errors="replace"))
        if rc != 0:
            raise ValueError(L.af_fastq_part_error(h).decode(errors="replace"))
        stride = max(int(ml.value), 1)
        seqs = np.empty((n.value, stride), dtype=np.uint8)
        lens = np.empty(n.value, dtype=np.int32)
        arena = np.empty(max(int(nb.value), 1), dtype=np.uint8)
        off = np.empty(n.value, dtype=np.int64)
        rc = L.af_fastq_part_export(h, stride, seqs.ctypes.data, lens.ctypes.data, arena.ctypes.data, arena.size,
                                    off.ctypes.data)
        if rc != 0:
            raise _lib.AFError(f"af_fastq_part_export failed (rc={rc}): {L.af_fastq_part_error(h).decode()}")
        return Names(arena.tobytes(), off), seqs, lens
    finally:
        if h:
            L.af_fastq_part_free(h)


def read_pairs(fq1, fq2, threads=0):
    """Reads a FASTQ(.gz) pair into the pair-major layout (native reader, ``iter_pairs``).

    Returns ``(names, reads[2N, stride] uint8, lens[2N] int32 or None)``; ``names[p]`` is the
    QNAME of pair p (mates must agree, as bwa requires for paired input); ``lens`` is None when
    every read has length ``stride``."""
    parts = list(iter_pairs(fq1, fq2, threads=threads))
    if not parts:
        return Names(b"", np.zeros(0, np.int64)), np.full((0, 1), ord("N"), np.uint8), None
    stride = max(r.shape[1] for _, r, _ in parts)
    if all(r.shape[1] == stride for _, r, _ in parts):
        reads = np.concatenate([r for _, r, _ in parts]) if len(parts) > 1 else parts[0][1]
    else:
        reads = np.full((sum(r.shape[0] for _, r, _ in parts), stride), ord("N"), np.uint8)
        row = 0
        for _, r, _ in parts:
            reads[row:row + r.shape[0], :r.shape[1]] = r
            row += r.shape[0]
    lens = np.concatenate([x for _, _, x in parts]) if len(parts) > 1 else parts[0][2]
    names = Names.concat([nm for nm, _, _ in parts])
    return names, reads, (None if (lens == stride).all() else lens)


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
