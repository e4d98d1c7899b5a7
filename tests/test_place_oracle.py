"""CPU tests of the placement oracle (afo_place, the multi-hit form of the S2 algorithm used
for the genome / BLAT searches of the partner stages)."""
import numpy as np

import afpkg  # noqa: F401
import oracle
from anchored_fusion_amd.place import concat_contigs, pack_queries
from place_cases import contigs, queries


def test_place_recovers_tails():
    ctgs = contigs()
    blob, offs = concat_contigs(ctgs)
    ix = oracle.OracleIndex(blob)
    qs = queries(ctgs, 300)
    buf, lens = pack_queries([q for _, q, _ in qs])
    p = oracle.default_params()
    p.T, p.min_seed_len = 20, 16
    hits, nh = ix.place(buf, lens, p, max_hits=8, threads=4)
    names = [n for n, _ in ctgs]
    found = total = 0
    for i, (_, q, truth) in enumerate(qs):
        got = set()
        for k in range(max(nh[i], 0)):
            h = hits[i, k]
            c = int(np.searchsorted(offs, h["t_start"], side="right")) - 1
            got.add((names[c], int(h["t_start"]) - offs[c]))
            assert h["q_start"] < h["q_end"] <= len(q) and h["matches"] <= h["q_end"] - h["q_start"]
            assert h["score"] >= p.T
        for name, s, e in truth:
            if e - s < 30:
                continue
            total += 1
            found += any(g[0] == name and abs(g[1] - s) <= 8 for g in got)
        if i and nh[i] > 1:  # best first
            assert hits[i, 0]["score"] >= hits[i, 1]["score"]
    assert found >= 0.95 * total, (found, total)


