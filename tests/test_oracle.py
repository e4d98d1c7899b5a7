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
    f, sc = bundled_out["flag"], bundled_out["score"]
    mapped = (f & 4) == 0
    src = collections.Counter(names[r // 2].split("_")[0] for r in np.nonzero(mapped)[0])
    # every mapped read comes from the BCR-ABL1 transcript (EU216071.1); none from the 5 others
    assert set(src) == {"EU216071.1"}
    # 1,261 reads seed and map on their own (the 20-mer-seeded count of SURVEY.md §4 item 2);
    # mate rescue (mem_matesw) adds 3 mates whose anchor part is too short or too mismatched to
    # seed: they score below -T 30 and are printed only because they pair properly
    assert int((mapped & (sc >= 30)).sum()) == 1261
    rescued = np.nonzero(mapped & (sc < 30))[0]
    assert len(rescued) == 3
    for r in rescued:
        assert f[r] & 0x2 and not (f[r ^ 1] & 0x4) and bundled_out["hits"][r] >= 0


def test_bundled_junction_known_answers(bundled_out):
    top = [k for k, _ in junctions(bundled_out).most_common(3)]
    # MS 3235 (BCR->ABL1), MS 1848 and SM 2568 (splice variants inside BCR)
    assert top == [("MS", 3235), ("MS", 1848), ("SM", 2568)]


def test_filter_is_superset_of_seeded(oidx, bundled_out):
    mapped = (bundled_out["flag"] & 4) == 0
    assert (bundled_out["hits"][mapped] > 0).all()


def test_pair_flags_consistent(bundled_out):
    """mem_aln2sam's flag rules for one primary record per read."""
    f = bundled_out["flag"]
    assert ((f & 1) == 1).all()
    assert ((f[0::2] & 0x40) != 0).all() and ((f[1::2] & 0x80) != 0).all()
    m1, m2 = (f[0::2] & 4) == 0, (f[1::2] & 4) == 0
    assert (((f[0::2] & 8) != 0) == ~m2).all() and (((f[1::2] & 8) != 0) == ~m1).all()
    # an unmapped read with a mapped mate is placed at its mate's position and strand
    p = bundled_out["pos"]
    one = m1 & ~m2
    assert (p[1::2][one] == p[0::2][one]).all()
    assert ((f[1::2][one] & 0x10) == (f[0::2][one] & 0x10)).all()
    # ... and the mapped read copies its own strand to the mate: 0x20 iff 0x10
    assert (((f[0::2][one] & 0x20) != 0) == ((f[0::2][one] & 0x10) != 0)).all()
    # the proper-pair bit only on pairs with both ends mapped; no secondary primary records
    assert ((f & 0x2) == 0)[~np.repeat(m1 & m2, 2)].all()
    assert ((f & 0x100) == 0).all()


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


def test_mate_rescue_changes_s3_partitions(anchor, oidx):
    """A mate too mismatched to seed (no exact 19-mer, K1 hits 0) at the proper insert distance is
    rescued by mem_matesw, so the pair leaves S3's one-end-anchored sets (-f 8 / -f 4,
    Anchored_Fusion.py:186-187) and both reads reach anchored.bam (-F 772)."""
    from anchored_fusion_amd.align import AlignResult, partition
    from cases import rescue_pairs
    reads, probe = rescue_pairs(anchor)
    out = oidx.align_pairs(reads)
    f = out["flag"]
    r1, r2 = 2 * probe, 2 * probe + 1
    assert out["hits"][r2] == 0                         # the mate cannot seed
    assert not f[r1] & 4 and not f[r2] & 4 and f[r1] & 2  # ... yet maps, properly paired
    res = AlignResult(**out)
    tmp1, tmp2, anchored = partition(res)
    assert r1 not in tmp1 and r2 not in tmp2 and r2 in anchored
    # without a proper-pair model (too few pairs in the chunk) the same mate stays unmapped
    lone = oidx.align_pairs(reads[2 * probe:2 * probe + 2])
    assert lone["flag"][1] & 4 and lone["flag"][0] & 8
    t1, t2, _ = partition(AlignResult(**lone))
    assert 0 in t1 and 1 in t2


def test_tie_break_follows_read_ids(anchor):
    """A read matching two copies of a segment equally well: mem_mark_primary_se picks by
    hash_64(read id), so the primary copy depends on the pair's global index (pair_base)."""
    from cases import repeat_anchor_pairs
    anc2, reads = repeat_anchor_pairs(anchor)
    ix = oracle.OracleIndex(anc2)
    picks = set()
    for base in (0, 1, 7, 1000, 123456):
        out = ix.align_pairs(reads, pair_base=base)
        picks.add(tuple(out["pos"][0::2]))
    assert len(picks) > 1


def test_chunks_change_insert_stats(anchor, oidx):
    """Insert-size statistics are per bwa chunk (bseq_read: >= chunk_bases bases): a rescue that
    needs its chunk's pairs fails when the chunk is cut smaller."""
    from cases import rescue_pairs
    reads, probe = rescue_pairs(anchor)
    big = oidx.align_pairs(reads)
    small = oidx.align_pairs(reads, chunk_bases=200 * 6)   # 6 pairs of 2x100 per chunk
    assert not big["flag"][2 * probe + 1] & 4 and small["flag"][2 * probe + 1] & 4


def test_tandem_repeat_runs(anchor, oidx):
    """The oracle aligns (CGC)n reads against the anchor's own CGC repeat (many equal regions)."""
    from cases import tandem_pairs
    reads = tandem_pairs(anchor)
    out = oidx.align_pairs(reads, threads=4)
    assert len(out["flag"]) == reads.shape[0]
