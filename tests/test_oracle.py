"""CPU tests of the oracle (oracle/af_oracle.c) against the reference's own test data.

Parity pinning: bwa/BLAT are absent, so the oracle is pinned by
(1) the wgsim truth encoded in the bundled FASTQ read names (test/test_sample_*.fastq.gz,
copied to tests/golden/), and (2) the junction known-answers of SURVEY.md §4 for BCR.
"""
import collections

import numpy as np
import pytest

import oracle
from cases import edge_pairs, ragged, synthetic_pairs


@pytest.fixture(scope="module")
def oidx(anchor):
    return oracle.OracleIndex(anchor)


@pytest.fixture(scope="module")
def bundled_out(oidx, bundled_pairs):
    names, reads, lens = bundled_pairs
    return oidx.align_pairs(reads, lens, threads=4)


def junctions(out):
    bp = collections.Counter()
    for r in np.nonzero((out["flag"] & 4) == 0)[0]:
        ops = [(int(c >> 4), "MIDNSHP"[c & 15]) for c in out["cigar"][r][: out["n_cigar"][r]]]
        if len(ops) == 2 and ops[0][1] == "S" and ops[1][1] == "M" and ops[0][0] >= 15:
            bp[("SM", int(out["pos"][r]) + 1)] += 1
        elif len(ops) == 2 and ops[0][1] == "M" and ops[1][1] == "S" and ops[1][0] >= 15:
            bp[("MS", int(out["pos"][r]) + ops[0][0])] += 1
    return bp


def test_bundled_only_bcr_fusion_reads_map(bundled_pairs, bundled_out):
    names = bundled_pairs[0]
    mapped = (bundled_out["flag"] & 4) == 0
    src = collections.Counter(names[r // 2].split("_")[0] for r in np.nonzero(mapped)[0])
    # every mapped read comes from the BCR-ABL1 transcript (EU216071.1); none from the 5 others
    assert set(src) == {"EU216071.1"}
    assert src["EU216071.1"] == 1261  # = the 20-mer-seeded read count of SURVEY.md §4 item 2


def test_bundled_junction_known_answers(bundled_out):
    top = [k for k, _ in junctions(bundled_out).most_common(3)]
    # MS 3235 (BCR->ABL1), MS 1848 and SM 2568 (splice variants inside BCR)
    assert top == [("MS", 3235), ("MS", 1848), ("SM", 2568)]


def test_filter_is_superset_of_seeded(oidx, bundled_out):
    mapped = (bundled_out["flag"] & 4) == 0
    assert (bundled_out["hits"][mapped] > 0).all()


def test_pair_flags_consistent(bundled_out):
    f = bundled_out["flag"]
    assert ((f & 1) == 1).all()
    assert ((f[0::2] & 0x40) != 0).all() and ((f[1::2] & 0x80) != 0).all()
    m1, m2 = (f[0::2] & 4) == 0, (f[1::2] & 4) == 0
    assert (((f[0::2] & 8) != 0) == ~m2).all() and (((f[1::2] & 8) != 0) == ~m1).all()
    # an unmapped read with a mapped mate is placed at its mate's position
    p = bundled_out["pos"]
    one = m1 & ~m2
    assert (p[1::2][one] == p[0::2][one]).all()


def test_synthetic_truth_positions(anchor, oidx):
    """Reads whose whole fragment lies in the anchor part of a fusion map at the true spot."""
    reads, truth, world = synthetic_pairs(anchor, 3000, 100, seed=11, err=0.0, indel_frac=0.0, n_rate=0.0,
                                          fusion_frac=1.0)
    out = oidx.align_pairs(reads)
    nf = len(world["fusions"])
    checked = 0
    for p in range(len(truth["tid"])):
        t = truth["tid"][p]
        if t >= nf:
            continue
        a = world["fusion_bp"][t][0]
        s, fr = truth["start"][p], truth["frag"][p]
        if s + fr > a:
            continue
        fwd, rev = 2 * p + int(truth["flip"][p]), 2 * p + 1 - int(truth["flip"][p])
        assert out["flag"][fwd] & 0x14 == 0 and out["pos"][fwd] == s
        assert out["flag"][rev] & 0x14 == 0x10 and out["pos"][rev] == s + fr - 100
        checked += 1
    assert checked > 200


def test_edge_cases_run(anchor, oidx):
    reads, lens = edge_pairs(anchor)
    out = oidx.align_pairs(reads, lens)
    f = out["flag"]
    assert f[0] & 0x14 == 0 and out["pos"][0] == 0 and out["n_cigar"][0] == 1   # exact, start
    assert f[1] & 0x14 == 0x10 and out["pos"][1] == len(anchor) - 100           # exact rc, end
    assert f[22] & 4  # all-N read: no seed, unmapped


def test_ragged_runs(anchor, oidx):
    reads, _, _ = synthetic_pairs(anchor, 500, 150, seed=3)
    rr, lens = ragged(reads, 5)
    out = oidx.align_pairs(rr, lens)
    assert ((out["flag"] & 4) == 0).sum() > 0
