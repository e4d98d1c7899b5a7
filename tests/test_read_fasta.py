"""io.read_fasta's whole-buffer form equals the line-by-line rule it replaces (each sequence line
stripped of its line end and surrounding whitespace, lines before the first header ignored) on
random FASTA text: CRLF and bare CR, blanks and tabs inside lines, empty records, headers with
descriptions, missing final newline, gzip."""
import gzip
import random

import afpkg  # noqa: F401
from anchored_fusion_amd import io as afio


def _line_rule(data):
    recs, name, chunks = [], None, []
    for line in _split_lf(data):  # binary file iteration: lines end at LF only
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


def _split_lf(data):
    parts = data.split(b"\n")
    return [p + b"\n" for p in parts[:-1]] + ([parts[-1]] if parts[-1] else [])


def test_read_fasta_matches_line_rule(tmp_path):
    rng = random.Random(7)
    cases = [b">a desc\nACGT\nAC\n>b\n\nGG\r\nTT\n", b"junk\n>x\nAC GT\n  TT \n>y\n", b"", b"nohdr\nACGT\n",
             b">only", b">h\nACGT", b">h\r\nAC\r\nGT\r\n>g x\r\n\r\n", b">a\nAC\tG\n\x0bT\n>b\nN\n"]
    for _ in range(300):
        parts = [rng.choice([b"", b"x\n"])]
        for _ in range(rng.randint(0, 4)):
            parts.append(b">" + bytes(rng.choice(b"abc ") for _ in range(rng.randint(0, 5))) +
                         rng.choice([b"\n", b"\r\n"]))
            for _ in range(rng.randint(0, 4)):
                parts.append(bytes(rng.choice(b"ACGTN \t\r") for _ in range(rng.randint(0, 8))) +
                             rng.choice([b"\n", b"\r\n", b""]))
        cases.append(b"".join(parts))
    for i, c in enumerate(cases):
        p = tmp_path / (f"c{i}.fa.gz" if i % 3 == 0 else f"c{i}.fa")
        if i % 3 == 0:
            with gzip.open(p, "wb") as fh:
                fh.write(c)
        else:
            p.write_bytes(c)
        assert afio.read_fasta(str(p)) == _line_rule(c), c
