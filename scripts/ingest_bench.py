"""Times the native paired-FASTQ ingest (af_fastq_*, csrc/ingest.cpp) on the bench workload's
reads written as FASTQ (plain and gzip level 1) under $TMPDIR.

usage: python3 scripts/ingest_bench.py [pairs]"""
import gzip
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import afpkg  # noqa: E402,F401
import numpy as np  # noqa: E402

from anchored_fusion_amd import io as afio  # noqa: E402
from anchored_fusion_amd import simulate as sim  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
anchor = afio.anchor_sequence(os.path.join(ROOT, "tests", "golden", "target_gene.fasta"))
_, reads, _, _ = sim.fusion_reads(anchor, n, read_len=100, fusion_frac=0.05, seed=20251015)
L = reads.shape[1]
d = tempfile.mkdtemp()


def fastq_bytes(mate):
    rows = reads[mate::2]
    head = np.frombuffer(b"".join(b"@p%d/%d\n" % (i, mate + 1) for i in range(n)), np.uint8)
    body = np.empty((n, L + 1 + 2 + L + 1), np.uint8)
    body[:, :L] = rows
    body[:, L] = ord("\n")
    body[:, L + 1:L + 3] = np.frombuffer(b"+\n", np.uint8)
    body[:, L + 3:2 * L + 3] = ord("I")
    body[:, 2 * L + 3] = ord("\n")
    # interleave header lines with bodies
    hl = np.array([len(b"@p%d/%d\n" % (i, mate + 1)) for i in range(n)])
    out = np.empty(head.size + body.size, np.uint8)
    ho = np.concatenate([[0], np.cumsum(hl)])
    pos = 0
    for i in range(n):
        out[pos:pos + hl[i]] = head[ho[i]:ho[i + 1]]
        pos += hl[i]
        out[pos:pos + body.shape[1]] = body[i]
        pos += body.shape[1]
    return out.tobytes()


def write_bgzf(p, data, block=65280):
    import struct
    import zlib
    with open(p, "wb") as fh:
        for o in list(range(0, len(data), block)) + [len(data)]:
            chunk = data[o:o + block] if o < len(data) else b""
            c = zlib.compressobj(1, zlib.DEFLATED, -15)
            cdata = c.compress(chunk) + c.flush()
            fh.write(b"\x1f\x8b\x08\x04\0\0\0\0\0\xff" + struct.pack("<H", 6) + b"BC" +
                     struct.pack("<HH", 2, 12 + 6 + len(cdata) + 8 - 1) + cdata +
                     struct.pack("<II", zlib.crc32(chunk) & 0xFFFFFFFF, len(chunk)))
            if o >= len(data):
                break


paths = {}
for kind in ("plain", "gzip-1", "bgzf-1"):
    ps = []
    for m in (0, 1):
        p = os.path.join(d, f"r_{kind}_{m + 1}.fq" + ("" if kind == "plain" else ".gz"))
        data = fastq_bytes(m)
        if kind == "gzip-1":
            with gzip.open(p, "wb", compresslevel=1) as fh:
                fh.write(data)
        elif kind == "bgzf-1":
            write_bgzf(p, data)
        else:
            with open(p, "wb") as fh:
                fh.write(data)
        ps.append(p)
    paths[kind] = ps
for gz, (p1, p2) in paths.items():
    afio.read_pairs(p1, p2)  # warm the page cache
    t0 = time.perf_counter()
    names, got, lens = afio.read_pairs(p1, p2)
    dt = time.perf_counter() - t0
    assert (got == reads).all() and names[n - 1] == f"p{n - 1}"
    size = os.path.getsize(p1) + os.path.getsize(p2)
    print(f"{gz}: {n} pairs in {dt:.2f} s = {n / dt / 1e6:.2f} M pairs/s "
          f"({size / dt / 1e6:.0f} MB/s of input files)")
for ps in paths.values():
    for p in ps:
        os.remove(p)
os.rmdir(d)
