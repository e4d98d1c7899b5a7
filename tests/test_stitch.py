"""Long BLAT queries stitched into one alignment (stitch.py; functions.py:341 / 966 hand BLAT the
whole anchor transcript).  CPU: the Placer over the BLAT restatement's CPU contract
(oracle/blat.c via tests/oracle_backends.OracleTileReference -- the kernel is bit-exact to it,
tests/test_gpu_blat.py), so the window rows are the kernel's; the stitching is host code.

The world: a three-exon gene (the anchor = its exons joined), a processed copy at 92 % identity,
a reverse-complement copy at 95 %, a diverged copy at 72 % (below -minIdentity=80 as a whole),
and a query whose six 30-nt pieces match a target colinearly: each window alone scores below
-minScore=50, the stitched alignment above it."""
import numpy as np
import pytest

import afpkg  # noqa: F401
from anchored_fusion_amd.place import Placer
from oracle_backends import OracleTileReference

ACGT = np.frombuffer(b"ACGT", np.uint8)
EXONS = [(20_000, 20_400), (22_000, 22_350), (25_000, 25_500)]


def _rand(rng, n):
    return ACGT[rng.integers(0, 4, n)]


def _subst(rng, s, frac):
    s = s.copy()
    idx = rng.choice(len(s), int(len(s) * frac), replace=False)
    s[idx] = ACGT[(np.searchsorted(ACGT, s[idx]) + rng.integers(1, 4, len(idx))) % 4]
    return s


def _rc(s):
    return np.frombuffer(s[::-1].tobytes().translate(bytes.maketrans(b"ACGT", b"TGCA")), np.uint8)


def make_world():
    rng = np.random.default_rng(5)
    chr1 = _rand(rng, 200_000)
    chr2 = _rand(rng, 200_000)
    anchor = np.concatenate([chr1[a:b] for a, b in EXONS])
    chr2[50_000:50_000 + len(anchor)] = _subst(rng, anchor, 0.08)
    chr2[150_000:150_000 + len(anchor)] = _rc(_subst(rng, anchor, 0.05))
    chr2[80_000:80_000 + len(anchor)] = _subst(rng, anchor, 0.28)
    # six 30-nt pieces of a random query, colinear on chr2 at 100 kb with 150-nt target gaps
    pq = _rand(rng, 1400)
    for k in range(6):
        chr2[100_000 + 180 * k:100_000 + 180 * k + 30] = pq[200 * k:200 * k + 30]
    genome = [("chr1", chr1.tobytes().decode()), ("chr2", chr2.tobytes().decode())]
    return genome, anchor.tobytes().decode(), pq.tobytes().decode(), Placer(tile_factory=OracleTileReference)


@pytest.fixture(scope="module")
def world():
    w = make_world()
    yield w
    w[3].close()


def _rows(lines):
    return [ln.rstrip("\n").split("\t") for ln in lines[2:]]


def _ints(field):
    return [int(v) for v in field.rstrip(",").split(",")]


def test_anchor_locus_is_one_stitched_alignment(world):
    genome, anchor, _, placer = world
    rows = _rows(placer(genome, [("ANC", anchor)], "homologs"))
    locus = [r for r in rows if r[13] == "chr1" and r[8] == "+"]
    assert len(locus) == 1
    r = locus[0]
    assert (int(r[0]), int(r[1]), int(r[10]), int(r[11]), int(r[12])) == (1250, 0, 1250, 0, 1250)
    assert (int(r[15]), int(r[16]), int(r[17])) == (20_000, 25_500, 3)
    assert _ints(r[18]) == [400, 350, 500] and _ints(r[19]) == [0, 400, 750]
    assert _ints(r[20]) == [a for a, _ in EXONS]
    assert (int(r[6]), int(r[7])) == (2, 1600 + 2650)  # the introns: target inserts
    # the copies: whole-anchor rows; the diverged copy fails -minIdentity=80 as a whole
    fwd = [r for r in rows if r[13] == "chr2" and r[8] == "+" and 49_000 < int(r[15]) < 51_000]
    rev = [r for r in rows if r[13] == "chr2" and r[8] == "-" and 149_000 < int(r[15]) < 151_000]
    assert len(fwd) == 1
    assert int(fwd[0][11]) < 20 and int(fwd[0][12]) > 1230 and int(fwd[0][0]) > 1100
    assert len(rev) == 1 and int(rev[0][11]) < 20 and int(rev[0][12]) > 1230 and int(rev[0][0]) > 1150
    assert not [r for r in rows if r[13] == "chr2" and 79_000 < int(r[15]) < 82_000]
    # rows sorted by score, best first (the kernel's per-query order)
    sc = [int(r[0]) - int(r[1]) - int(r[4]) - int(r[6]) for r in rows]
    assert sc == sorted(sc, reverse=True)


def test_min_score_judged_on_the_stitched_alignment(world):
    genome, _, pq, placer = world
    rows = _rows(placer(genome, [("PQ", pq)], "homologs"))
    hit = [r for r in rows if r[13] == "chr2" and 99_000 < int(r[15]) < 101_500]
    assert len(hit) == 1
    r = hit[0]
    # the six pieces (extensions may run a few bases into the random flanks)
    assert 6 <= int(r[17]) <= 8 and int(r[0]) - int(r[1]) - int(r[4]) - int(r[6]) >= 150
    assert int(r[15]) == 100_000 and abs(int(r[16]) - (100_000 + 180 * 5 + 30)) <= 20
    # no single 300-nt window holds more than two pieces (score < 50 < the stitched 170)
    assert max(sum(1 for k in range(6) if off <= 200 * k and 200 * k + 30 <= off + 300) for off in range(0, 1250, 150)) <= 2


def test_short_queries_unchanged(world):
    """Queries within the kernel's length limit keep the kernel's rows as they are."""
    genome, anchor, _, placer = world
    q = anchor[100:250]
    rows = _rows(placer(genome, [("S", q)], "homologs"))
    assert rows and rows[0][13] == "chr1" and int(rows[0][15]) == EXONS[0][0] + 100 and int(rows[0][0]) == 150
