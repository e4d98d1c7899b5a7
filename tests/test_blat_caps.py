"""The BLAT restatement's fixed caps made visible (af_blat_caps, oracle afo_blat_caps): BLAT
prints every row at or above -minScore, the restatement keeps the first 32,768 tile hits of a
query strand, 4,096 clumps and max_rows rows per query, and counts each time one of them binds
(every clump whose seed lies in no earlier part is aligned: the parts have no cap of their own).  CPU: the oracle's counters on a world built so that each cap binds, and all
zero on unique sequence; tests/test_gpu_blat.py checks the kernel's counters against these."""
import ctypes

import numpy as np

import afpkg  # noqa: F401
from anchored_fusion_amd import blat
from oracle_backends import OracleTileReference

_B = np.frombuffer(b"ACGT", np.uint8)


def caps_world():
    """A random contig with a 13-nt unit tandem-repeated over 260 kb (every tile of the unit
    occurs thousands of times: hits and clumps bind), two exact copies of a 200-nt segment (two
    rows), queries of each kind."""
    rng = np.random.default_rng(17)
    unit = _B[rng.integers(0, 4, 13)].tobytes()
    a = _B[rng.integers(0, 4, 300_000)].tobytes()
    seg = a[50_000:50_200]
    b = bytearray(_B[rng.integers(0, 4, 300_000)].tobytes())
    b[200_000:200_200] = seg
    ctgs = [("a", a.decode()), ("b", b.decode()), ("rep", (unit * 20_000).decode())]
    qs = [(unit * 12)[:150].decode(), seg.decode(), a[120_000:120_150].decode()]
    return ctgs, qs


def test_caps_bind_and_are_counted():
    ctgs, qs = caps_world()
    p = blat.params("homologs")
    o = OracleTileReference(ctgs, p.step_size)
    rows, nr = o.search(qs[:1], p)
    c = o.caps()
    assert c["hits"] >= 1 and c["clumps"] >= 1 and c["parts"] == 0, c
    o.search(qs[1:2], p, 1)  # two exact copies, one row kept
    assert o.caps() == dict(hits=0, clumps=0, parts=0, rows=1)
    o.search(qs[1:], p)
    assert o.caps() == dict(hits=0, clumps=0, parts=0, rows=0)
    # counters accumulate until read with reset
    o.search(qs[:1], p)
    o.search(qs[:1], p)
    assert o.caps(reset=False)["hits"] == 2 * c["hits"]
    assert o.caps()["hits"] == 2 * c["hits"] and o.caps()["hits"] == 0


def family_world(copies=60, seed=23):
    """A 300-nt element in `copies` diverged copies (3 %) across a random contig, plus halves of it
    placed in order 2 kb apart (parts that chain across an intron-like gap)."""
    rng = np.random.default_rng(seed)
    elem = _B[rng.integers(0, 4, 300)]
    g = _B[rng.integers(0, 4, 600_000)].copy()
    at = np.sort(rng.choice(np.arange(1_000, 560_000, 4_000), copies, replace=False))
    for k, a in enumerate(at):
        e = elem.copy()
        mut = rng.random(300) < 0.03
        e[mut] = _B[rng.integers(0, 4, int(mut.sum()))]
        if k % 3 == 0:
            g[a:a + 150], g[a + 2150:a + 2300] = e[:150], e[150:]
        else:
            g[a:a + 300] = e
    return [("fam", g.tobytes().decode())], [elem.tobytes().decode(), elem[40:260].tobytes().decode()]


def test_many_parts_incremental_chain_equals_literal():
    """A query with dozens of aligned parts (a repeat family): the oracle's incremental chain DP
    (only parts whose predecessor path met a used part are recomputed) emits exactly the rows of
    the literal rule (every part recomputed each round); no cap binds except max_rows."""
    import oracle
    ctgs, qs = family_world()
    p = blat.params("split_tail")
    o = OracleTileReference(ctgs, p.step_size)
    L = oracle.lib()
    L.afo_blat_set_literal.argtypes = [ctypes.c_int]
    rows, nr = o.search(qs, p)
    c = o.caps()
    L.afo_blat_set_literal(1)
    try:
        rows_l, nr_l = o.search(qs, p)
    finally:
        L.afo_blat_set_literal(0)
    assert np.array_equal(nr, nr_l)
    for q in range(len(qs)):
        assert rows[q, :nr[q]].tobytes() == rows_l[q, :nr[q]].tobytes(), q
    assert c["hits"] == c["clumps"] == c["parts"] == 0 and c["rows"] == 2, c
    assert (nr == blat.MAX_ROWS).all()
    # the chained halves: rows with one target gap of 2 kb
    assert any(int(r["t_num_insert"]) >= 1 and int(r["t_base_insert"]) >= 1_900 for r in rows[0, :nr[0]]) or \
        any(int(r["block_count"]) >= 2 for r in rows[0, :nr[0]])
