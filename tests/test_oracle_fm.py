"""The genome side of the bwa restatement (oracle/bwa_pe.c, FM mode) -- CPU tests.

* bns_fasta2bntseq: contigs joined without separators, every non-ACGT base replaced by
  lrand48() & 3 after srand48(11), then the reverse complement;
* the suffix array of the bwa text ('$' smallest) against a brute-force sort;
* seeds: mem_collect_intv restated twice -- bwt_smem1 / bwt_seed_strategy1 on the FM index, and
  the MEM-set restatement that S2's GPU kernels follow -- give the same seed walk (intervals,
  counts, max_occ sampling and suffix-array order of the occurrences) on the anchor and on a
  repeat-rich genome where intervals exceed max_occ.
"""
import numpy as np
import pytest

import afpkg  # noqa: F401
import oracle
from genome_world import make_genome, sample_reads


def _lrand48_codes(n):
    x = (11 << 16) | 0x330E
    out = []
    for _ in range(n):
        x = (0x5DEECE66D * x + 0xB) & ((1 << 48) - 1)
        out.append((x >> 17) & 3)
    return out


def test_bwa_text_and_suffix_array():
    rng = np.random.default_rng(3)
    contigs = []
    for k, L in enumerate((257, 130, 311)):
        s = bytearray(rng.choice(list(b"ACGT"), L).astype(np.uint8).tobytes())
        s[5:9] = b"NNNN"
        s[L - 3] = ord("R")  # IUPAC codes are ambiguous bases too
        contigs.append((f"c{k}", bytes(s)))
    g = oracle.OracleGenome(contigs)
    pac = []
    rnd = iter(_lrand48_codes(100))
    for _, s in contigs:
        for ch in s:
            pac.append("ACGT".index(chr(ch)) if chr(ch) in "ACGT" else next(rnd))
    T = np.array(pac + [3 - c for c in pac[::-1]], dtype=np.uint8)
    assert np.array_equal(g.text(), T)
    N = len(T)
    tb = bytes(T)
    want = [N] + sorted(range(N), key=lambda i: tb[i:])
    sa = g.sa()
    assert sa.tolist() == want
    assert sa[g.primary()] == 0


def _seed_tuples(g, read, memset):
    rb, qb, ln = g.seeds(read, memset=memset)
    return list(zip(rb.tolist(), qb.tolist(), ln.tolist()))


def test_fm_seeds_equal_memset_seeds_anchor(anchor, bundled_pairs):
    """On the anchor text (one contig), bwt_smem1 over the FM index gives exactly the seeds of
    the MEM-set restatement (S2's contract) for every read that seeds."""
    g = oracle.OracleGenome([("anchor", anchor)], memset_too=True)
    _, reads, lens = bundled_pairs
    n_seeded = 0
    for r in range(0, reads.shape[0], 3):
        rd = bytes(reads[r, :reads.shape[1] if lens is None else lens[r]])
        a, b = _seed_tuples(g, rd, False), _seed_tuples(g, rd, True)
        assert a == b, r
        n_seeded += bool(a)
    assert n_seeded > 300


@pytest.fixture(scope="module")
def repeat_genome():
    contigs = make_genome()
    return contigs, oracle.OracleGenome(contigs, memset_too=True)


def test_fm_seeds_equal_memset_seeds_repeats(repeat_genome):
    contigs, g = repeat_genome
    reads, lens = sample_reads(contigs, 300, seed=11)
    big = 0
    for r in range(reads.shape[0]):
        rd = bytes(reads[r, :lens[r]])
        a, b = _seed_tuples(g, rd, False), _seed_tuples(g, rd, True)
        assert a == b, r
        if a:
            _, counts = np.unique([q for _, q, _ in a], return_counts=True)
            big += int((counts >= 500).any())
    assert big > 0, "no read had an interval sampled at max_occ"


def test_genome_align_se_records(repeat_genome):
    """S5 records: every read yields >= 1 record; mapped records are placed on their contig with
    a CIGAR spanning the read; -M parts carry 0x100 and hard clips."""
    contigs, g = repeat_genome
    reads, lens = sample_reads(contigs, 200, seed=5)
    recs, nrec = g.align_se(reads, lens, threads=4)
    assert (nrec >= 1).all()
    n_supp = n_mapped = 0
    for r in range(len(nrec)):
        for k in range(min(nrec[r], recs.shape[1])):
            e = recs[r, k]
            if e["flag"] & 4:
                continue
            n_mapped += 1
            ops = [(int(c) >> 4, int(c) & 15) for c in e["cigar"][:e["n_cigar"]]]
            qlen = sum(n for n, o in ops if o in (0, 1, 4, 5))
            assert qlen == lens[r]
            assert 0 <= e["pos"] < len(contigs[e["rid"]][1])
            if k:
                assert e["flag"] & 0x100
                n_supp += any(o == 5 for _, o in ops)
    assert n_mapped > 150 and n_supp > 10
