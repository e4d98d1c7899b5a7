"""The BLAT restatement's CPU contract (oracle/blat.c) and the PSL rendering (blat.psl_lines)."""
import numpy as np

import afpkg  # noqa: F401
import oracle
from anchored_fusion_amd.place import pack_queries

_B = np.frombuffer(b"ACGT", np.uint8)


def _genome(seed=1, n=200_000):
    return _B[np.random.default_rng(seed).integers(0, 4, n)].tobytes()


def test_short_tail_needs_two_tiles():
    g = _genome()
    t = oracle.OracleTiles(g, 3)
    p = oracle.blat_params(step_size=3, min_score=12, min_identity=90)
    buf, lens = pack_queries([g[1000:1014].decode(), g[3002:3017].decode()])
    rows, n = t.blat(buf, lens, p)
    assert n[0] == 0  # 1000 % 3 == 1: only one tile (offset 2) lies inside 14 nt
    assert n[1] == 1 and rows[1, 0]["t_start"] == 3002 and rows[1, 0]["score"] == 15


def test_junction_is_one_stitched_row():
    g = _genome()
    q = g[70000:70060] + g[72000:72040]
    comp = bytes.maketrans(b"ACGT", b"TGCA")
    buf, lens = pack_queries([q.decode(), q[::-1].translate(comp).decode()])
    for step in (3, 11):
        rows, n = oracle.OracleTiles(g, step).blat(buf, lens, oracle.blat_params(step_size=step, min_score=20))
        for i, strand in ((0, 0), (1, 1)):
            r = rows[i, 0]
            assert n[i] == 1 and r["strand"] == strand and r["block_count"] == 2
            assert (r["t_start"], r["t_end"], r["t_num_insert"], r["t_base_insert"]) == (70000, 72040, 1, 1940)
            assert r["score"] == 99 and r["matches"] == 100  # PSL score: one target insert


def test_identity_filter_uses_millibad():
    g = bytearray(_genome())
    q = bytearray(g[90_000:90_125])
    for j in range(27, 27 + 6 * 13, 6):  # 13 mismatches between exact 27 / 26-nt ends
        q[j] = b"ACGT"[(b"ACGT".index(q[j]) + 1) % 4]
    t = oracle.OracleTiles(bytes(g), 3)
    buf, lens = pack_queries([q.decode()])
    _, n = t.blat(buf, lens, oracle.blat_params(step_size=3, min_score=20, min_identity=90, min_match=3))
    assert n[0] == 0  # milliBad 1000 * 13 / 125 = 104 > 100
    rows, n = t.blat(buf, lens, oracle.blat_params(step_size=3, min_score=20, min_identity=0))
    assert n[0] == 1 and rows[0, 0]["mismatches"] == 13 and rows[0, 0]["score"] == 112 - 13


def test_psl_lines_layout():
    from anchored_fusion_amd import blat

    class Ref:
        names, lens, offsets = ["c1"], [200_000], [0]

        def locate(self, ts, te):
            return (0, int(ts), int(te))
    g = _genome()
    q = (g[70000:70060] + g[72000:72040]).decode()
    buf, lens = pack_queries([q])
    rows, n = oracle.OracleTiles(g, 11).blat(buf, lens, oracle.blat_params(min_score=20))
    f = blat.psl_lines(Ref(), [("q", q)], rows.view(blat.PSL_DTYPE), n)[0].rstrip("\n").split("\t")
    assert len(f) == 21
    assert f[:9] == ["100", "0", "0", "0", "0", "0", "1", "1940", "+"]
    assert f[9:17] == ["q", "100", "0", "100", "c1", "200000", "70000", "72040"]
    assert f[17:] == ["2", "60,40,", "0,60,", "70000,72000,"]
