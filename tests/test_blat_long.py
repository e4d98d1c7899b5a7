"""Long BLAT queries searched whole (functions.py:341 / 966 hand BLAT the whole anchor transcript):
afo_blat_long / af_blat_long, one query of kilobases with the short search's algorithm (tiles,
clumps, parts by banded extension, the chain DP) and rows of any block count.  CPU: the Placer over
the restatement's CPU contract (oracle/blat.c via tests/oracle_backends.OracleTileReference; the
kernel is bit-exact to it, tests/test_gpu_blat.py).

The world: a three-exon gene (the anchor = its exons joined), a processed copy at 92 % identity,
a reverse-complement copy at 95 %, a diverged copy at 72 % (below -minIdentity=80 as a whole),
and a query whose six 30-nt pieces match a target colinearly: each piece alone scores below
-minScore=50, their chained alignment above it."""
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


def test_anchor_locus_is_one_alignment(world):
    genome, anchor, _, placer = world
    rows = _rows(placer(genome, [("ANC", anchor)], "homologs"))
    locus = [r for r in rows if r[13] == "chr1" and r[8] == "+"]
    assert len(locus) == 1
    r = locus[0]
    # every anchor base aligned; an exon's extension may run a few bases into the next intron
    # when they happen to match the next exon's first bases (the later part is trimmed by them)
    assert int(r[0]) + int(r[1]) == 1250 and int(r[1]) <= 2 and (int(r[10]), int(r[11]), int(r[12])) == (1250, 0, 1250)
    assert (int(r[15]), int(r[16]), int(r[17])) == (20_000, 25_500, 3)
    assert sum(_ints(r[18])) == 1250 and _ints(r[19])[0] == 0
    assert all(abs(t - a) <= 8 for t, (a, _) in zip(_ints(r[20]), EXONS))
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


def test_min_score_judged_on_the_chained_alignment(world):
    genome, _, pq, placer = world
    rows = _rows(placer(genome, [("PQ", pq)], "homologs"))
    hit = [r for r in rows if r[13] == "chr2" and 99_000 < int(r[15]) < 101_500]
    assert len(hit) == 1
    r = hit[0]
    # the six pieces (extensions may run a few bases into the random flanks)
    assert 6 <= int(r[17]) <= 8 and int(r[0]) - int(r[1]) - int(r[4]) - int(r[6]) >= 150
    assert int(r[15]) == 100_000 and abs(int(r[16]) - (100_000 + 180 * 5 + 30)) <= 20
    # no row of a single piece (30 nt < -minScore=50): the pieces pass only chained
    assert not [r for r in rows if int(r[17]) == 1 and r[13] == "chr2" and 99_000 < int(r[15]) < 101_500]


def test_short_queries_unchanged(world):
    """Queries within a read's length keep the short search's rows as they are."""
    genome, anchor, _, placer = world
    q = anchor[100:250]
    rows = _rows(placer(genome, [("S", q)], "homologs"))
    assert rows and rows[0][13] == "chr1" and int(rows[0][15]) == EXONS[0][0] + 100 and int(rows[0][0]) == 150


def test_many_exon_anchor_row_keeps_every_block():
    """A 24-exon gene (more than the 16 blocks a short search's row holds): its locus is one row
    with 24 blocks and 23 introns as target inserts -- the case BCR (23 exons) hands fn:341."""
    from anchored_fusion_amd import blat
    rng = np.random.default_rng(9)
    chr1 = _rand(rng, 300_000)
    exons = [(10_000 + 9_000 * k, 10_000 + 9_000 * k + 120 + 7 * k) for k in range(24)]
    anchor = np.concatenate([chr1[a:b] for a, b in exons]).tobytes().decode()
    ref = OracleTileReference([("chr1", chr1.tobytes().decode())], 3)
    rows, n_all, blocks, off = ref.search_long(anchor, blat.params("homologs"))
    top = rows[0]
    nb = int(top["block_count"])
    assert n_all >= 1 and nb >= 24 and int(off[1] - off[0]) == nb  # (an exon edge may add a short block)
    assert int(top["matches"]) >= 0.99 * len(anchor) and int(top["t_num_insert"]) >= 23
    starts = [int(b["t_start"]) for b in blocks[off[0]:off[1]]]
    assert all(any(abs(t - a) <= 16 for t in starts) for a, _ in exons)  # a block at every exon
    assert abs(int(top["t_start"]) - exons[0][0]) <= 16 and abs(int(top["t_end"]) - exons[-1][1]) <= 16
    assert int(top["q_start"]) == 0 and int(top["q_end"]) == len(anchor)
