"""One long query searched whole on the GPU (af_blat_long, csrc/blat_long.hip) vs the CPU contract
(oracle/blat.c afo_blat_long): every row field, every block, the row count and the caps, for the
homolog search of functions.py:341 and the candidate veto of fn:966.

Worlds: tests/test_blat_long.py's (an exon-structured anchor with copies at 92 / 95 / 72 %
identity and a query of six short pieces), a 24-exon gene (a row of more than 16 blocks), long
random and repeat-derived queries on tests/test_gpu_blat.py's repeat world (thousands of clumps,
the hit cap), and the configs[2] world at 2 % (62 Mbp, the simulator's repeat families) with the
anchor transcript itself against the genome (step 3, -repMatch=10000) and against candidate
blocks around its partners' loci."""
import numpy as np
import pytest

import oracle
from oracle_backends import OracleTileReference

pytestmark = pytest.mark.gpu


def _same(g, o, ctx):
    rg, ng, bg, og = g
    ro, no, bo, oo = o
    assert ng == no, (ctx, ng, no)
    assert len(rg) == len(ro)
    for i in range(len(rg)):
        assert rg[i].tobytes() == ro[i].tobytes(), (ctx, i, rg[i], ro[i])
    assert np.array_equal(og, oo), ctx
    assert bg.tobytes() == bo.tobytes(), ctx


def _check(ctgs, queries, presets, step=None):
    from anchored_fusion_amd import blat
    refs = {}
    try:
        for preset in presets:
            p = blat.params(preset)
            key = p.step_size
            if key not in refs:
                refs[key] = (blat.TileReference(ctgs, key), OracleTileReference(ctgs, key))
            g, o = refs[key]
            g.caps(reset=True)
            o.caps(reset=True)
            for qi, q in enumerate(queries):
                _same(g.search_long(q, p), o.search_long(q, p), (preset, qi))
            assert g.caps() == o.caps(), preset
    finally:
        for g, _ in refs.values():
            g.close()


def test_long_exon_world_equals_oracle():
    from test_blat_long import make_world
    genome, anchor, pq, _ = make_world()
    _check(genome, [anchor, pq, anchor[::-1]], ["homologs", "candidate_homolog", "split_tail"])


def test_long_many_exons_equals_oracle():
    rng = np.random.default_rng(9)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    chr1 = acgt[rng.integers(0, 4, 300_000)]
    exons = [(10_000 + 9_000 * k, 10_000 + 9_000 * k + 120 + 7 * k) for k in range(24)]
    anchor = np.concatenate([chr1[a:b] for a, b in exons]).tobytes().decode()
    ctgs = [("chr1", chr1.tobytes().decode())]
    _check(ctgs, [anchor], ["homologs", "candidate_homolog"])


def test_long_repeat_world_equals_oracle():
    from test_gpu_blat import _world
    ctgs, rep = _world(11)
    rng = np.random.default_rng(21)
    qs = []
    for k in range(6):
        c = ctgs[k % len(ctgs)][1]
        ln = int(rng.integers(400, 3000))
        p = int(rng.integers(0, len(c) - ln))
        q = bytearray(c[p:p + ln].encode())
        for j in np.nonzero(rng.random(ln) < 0.03)[0]:
            q[j] = b"ACGT"[(b"ACGT".index(q[j]) + 1) % 4] if q[j] in b"ACGT" else q[j]
        qs.append(q.decode())
    qs.append((rep * 10).decode())  # repeat-derived: thousands of clumps per strand
    _check(ctgs, qs, ["homologs", "candidate_homolog"])


def test_long_c3_world_anchor_equals_oracle(anchor):
    """The anchor transcript (6,783 nt) against the 2 % configs[2] genome at step 3 (fn:341) and
    against candidate blocks around the partners' loci (fn:966)."""
    from anchored_fusion_amd import blat, simworld
    W = simworld.GenomeWorld(anchor, device=0, seed=20251015, scale=0.02)
    blob = W.blob.cpu().numpy()
    ctgs = [(nm, blob[o:o + ln].tobytes().decode()) for nm, o, ln in zip(W.names, W.offsets, W.lens)]
    q = anchor.decode() if isinstance(anchor, bytes) else anchor
    p = blat.params("homologs")
    g = W.tiles(p.step_size)
    o = OracleTileReference(ctgs, p.step_size)
    try:
        rg = g.search_long(q, p)
        _same(rg, o.search_long(q, p), "homologs")
        assert rg[1] >= 1
        assert g.caps() == o.caps()
    finally:
        g.close()
    # candidate blocks: 5 kb around each partner locus and the anchor's own exons
    blocks = []
    for name, spans in W.loci.items():
        c, s, e = spans[0]
        seq = ctgs[W.names.index(c)][1]
        a = max(0, s - 2500)
        blocks.append((f"{len(blocks)}::{c}:{a}-{a + 5000}", seq[a:a + 5000]))
    _check(blocks, [q], ["candidate_homolog"])
