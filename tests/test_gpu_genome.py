"""The genome calls S4 / S5 on the GPU (csrc/fmindex.hip, csrc/bwa_genome.hip) against the CPU
restatement (oracle/bwa_pe.c, FM mode) -- bit-exact.

* the index: bns_fasta2bntseq's text (lrand48 for ambiguous bases) and the suffix array, equal
  row for row on a repeat-rich genome (young Alu-like subfamily above max_occ, a satellite array,
  an exact 3 kb duplication, N runs);
* S5 (`bwa mem -M genome reads.fa`, functions.py:716): regions after mem_align1_core and every
  SAM record (flags, contigs, positions, CIGARs with -M hard clips, SEQ slices) on chimeric and
  plain reads with errors, indels and N;
* S4 (`bwa mem -M genome fq1 fq2`, AF:188): every record of every pair, with the per-chunk
  insert-size statistics, mate rescue and pairing.
"""
import numpy as np
import pytest

import afpkg  # noqa: F401
import oracle
from genome_world import make_genome, sample_pairs, sample_reads

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def world():
    contigs = make_genome()
    from anchored_fusion_amd.genome import GenomeIndex
    return contigs, oracle.OracleGenome(contigs), GenomeIndex(contigs, device=0)


def test_index_equals_oracle(world):
    _, og, gg = world
    assert gg.l_pac == og.l_pac
    assert np.array_equal(gg.text(), og.text())
    assert gg.primary() == og.primary()
    sa_o, sa_g = og.sa(), gg.sa()
    bad = np.nonzero(sa_o != sa_g)[0]
    assert bad.size == 0, f"{bad.size} suffix-array rows differ, first {bad[:5]}"


def _rec_equal(a, b, n):
    for k in range(n):
        x, y = a[k], b[k]
        for f in ("flag", "rid", "mrid", "pos", "mpos", "score", "n_cigar", "seq_b", "seq_e"):
            if int(x[f]) != int(y[f]):
                return f"record {k} field {f}: {int(x[f])} != {int(y[f])}"
        nc = int(x["n_cigar"])
        if not np.array_equal(x["cigar"][:nc], y["cigar"][:nc]):
            return f"record {k} cigar"
    return None


def test_se_regions_equal_oracle(world):
    contigs, og, gg = world
    reads, lens = sample_reads(contigs, 400, seed=21)
    ro, no = og.regions(reads, lens, max_reg=64, threads=8)
    rg, ng = gg.regions(reads, lens, max_reg=64)
    assert np.array_equal(no, ng), np.nonzero(no != ng)[0][:10]
    for r in range(len(no)):
        for k in range(min(no[r], 64)):
            o = ro[r, k]
            g = rg[r, k]
            want = (o["rb"], o["re"], o["qb"], o["qe"], o["rid"], o["score"], o["truesc"], o["w"], o["seedcov"],
                    o["seedlen0"])
            assert tuple(int(v) for v in want) == tuple(int(v) for v in g[:10]), (r, k)


def test_se_records_equal_oracle(world):
    contigs, og, gg = world
    reads, lens = sample_reads(contigs, 600, seed=22, chimeric=0.4)
    ro, no = og.align_se(reads, lens, id_base=7, threads=8)
    rg, ng = gg.align_se(reads, lens, id_base=7)
    assert np.array_equal(no, ng)
    for r in range(len(no)):
        msg = _rec_equal(ro[r], rg[r], min(no[r], 8))
        assert msg is None, (r, msg)
    assert gg.stats()["cap_overflow"] == 0
    n_supp = int(((rg["flag"] & 0x100) != 0).sum())
    assert n_supp > 20 and int(((rg[:, 0]["flag"] & 4) == 0).sum()) > 500


def test_pe_records_equal_oracle(world):
    contigs, og, gg = world
    reads = sample_pairs(contigs, 1500, seed=23)
    lens = np.full(reads.shape[0], reads.shape[1], np.int32)
    # two bwa chunks (insert-size statistics per chunk) at 300 kbase
    pe_o = oracle.default_pe(chunk_bases=300_000, pair_base=4)
    ro, no = og.align_pe(reads, lens, pe=pe_o, threads=8)
    from anchored_fusion_amd import _lib
    rg, ng = gg.align_pe(reads, lens, pe=_lib.default_pe(chunk_bases=300_000, pair_base=4))
    assert np.array_equal(no, ng)
    for r in range(len(no)):
        msg = _rec_equal(ro[r], rg[r], min(no[r], 8))
        assert msg is None, (r, msg)
    assert int(((rg[:, 0]["flag"] & 2) != 0).sum()) > 1500  # proper pairs found


def test_pe_rescue_case_equals_oracle():
    """tests/test_genome_rescue_blocks.py's crafted pairs (a mate placeable only by mem_matesw,
    2.5 kb inserts): the kernel's records equal the oracle's with rescue on and off."""
    from anchored_fusion_amd import _lib
    from anchored_fusion_amd.genome import GenomeIndex
    from test_genome_rescue_blocks import L, crafted
    contigs, reads, _ = crafted()
    og, gg = oracle.OracleGenome(contigs), GenomeIndex(contigs, device=0)
    try:
        lens = np.full(reads.shape[0], L, np.int32)
        for matesw in (50, 0):
            pe_o = oracle.default_pe()
            pe_o.max_matesw = matesw
            pe_g = _lib.default_pe()
            pe_g.max_matesw = matesw
            ro, no = og.align_pe(reads, lens, pe=pe_o, pair_base=0, threads=8)
            rg, ng = gg.align_pe(reads, lens, pe=pe_g)
            assert np.array_equal(no, ng), matesw
            for r in range(len(no)):
                msg = _rec_equal(ro[r], rg[r], min(no[r], 8))
                assert msg is None, (matesw, r, msg)
            probe = rg[len(reads) - 1, 0]
            assert bool(probe["flag"] & 4) == (matesw == 0)
    finally:
        gg.close()
