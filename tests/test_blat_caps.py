"""The BLAT restatement's fixed caps made visible (af_blat_caps, oracle afo_blat_caps): BLAT
prints every row at or above -minScore, the restatement keeps the first 32,768 tile hits of a
query strand, 4,096 clumps, 16 aligned parts and max_rows rows per query, and counts each time
one of them binds.  CPU: the oracle's counters on a world built so that each cap binds, and all
zero on unique sequence; tests/test_gpu_blat.py checks the kernel's counters against these."""
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
    assert c["hits"] >= 1 and c["clumps"] >= 1 and c["parts"] >= 1, c
    o.search(qs[1:2], p, 1)  # two exact copies, one row kept
    assert o.caps() == dict(hits=0, clumps=0, parts=0, rows=1)
    o.search(qs[1:], p)
    assert o.caps() == dict(hits=0, clumps=0, parts=0, rows=0)
    # counters accumulate until read with reset
    o.search(qs[:1], p)
    o.search(qs[:1], p)
    assert o.caps(reset=False)["hits"] == 2 * c["hits"]
    assert o.caps()["hits"] == 2 * c["hits"] and o.caps()["hits"] == 0
