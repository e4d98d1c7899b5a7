"""CPU tests of the host restatements of the split-read consumer stages (SURVEY.md §8 a4-a8,
a11, a12, a14) against golden fixtures produced by the reference's own functions.py
(tests/golden/make_fixtures.py, canned tool outputs; see its docstring).
"""
import json
import os

import pytest

import afpkg  # noqa: F401
from anchored_fusion_amd import annotation, blocks, cigar, genome_check, report, splitreads

FX_PATH = os.path.join(os.path.dirname(__file__), "golden", "consumers.json")


@pytest.fixture(scope="module")
def fx():
    with open(FX_PATH) as fh:
        return json.load(fh)


@pytest.fixture(scope="module")
def index(fx):
    return annotation.ExonIndex.from_lines(fx["gtf"])


def _plain(x):
    """tuples -> lists, recursively (JSON has no tuples)."""
    if isinstance(x, (list, tuple)):
        return [_plain(v) for v in x]
    if isinstance(x, dict):
        return {k: _plain(v) for k, v in x.items()}
    return x


def test_annotation_table(fx, index):
    assert _plain(index.dic) == fx["gene_co"]


def test_find_exon(fx, index):
    for chrom, s, e, gene, k in fx["find_exon"]:
        assert _plain(index.find_exon(chrom, s, e)) == [gene, k], (chrom, s, e)


def test_find_positions(fx, index):
    for chrom, p, ln, want, err in fx["find_positions"]:
        assert err is None
        assert _plain(index.walk(chrom, p, ln)) == want, (chrom, p, ln)


def test_deal_cigar(fx):
    for cig, seq, ops, seq2 in fx["deal_cigar"]:
        got_ops, got_seq = cigar.normalize(cig, seq)
        assert (got_ops, got_seq) == (ops, seq2), cig


def test_reverse(fx):
    for s, r in fx["reverse"]:
        assert cigar.revcomp(s) == r


def test_contact_reads(fx):
    for lines, want in fx["contact_reads"]:
        got = [list(r.as_tuple()) for r in splitreads.cluster_split_reads(lines)]
        assert got == want


def _dump(bc):
    return {c: [list(b.as_tuple()) for b in bl] for c, bl in bc.items()}


def test_find_blocks(fx, index):
    homo = fx["homo_genes"]
    for recs, want, err in fx["find_blocks"]:
        assert err is None
        assert _plain(_dump(blocks.spanning_blocks(recs, index, homo))) == want


def test_find_fine_block(fx, index):
    homo = fx["homo_genes"]
    for lines, psl, base_recs, want, err in fx["find_fine_block"]:
        assert err is None
        base = blocks.spanning_blocks(base_recs, index, homo) if base_recs else {}
        tails, fasta = blocks.split_read_queries(lines)
        got = blocks.add_fine_blocks(base, tails, psl, index, homo)
        assert _plain(_dump(got)) == want


def test_del_too_many_reads(fx):
    for anch, gsam, want in fx["del_too_many_reads"]:
        fasta = genome_check.split_read_fasta(anch)
        names = [n for n, _ in fasta]
        # the genome SAM's queries are exactly the FASTA the function sends to bwa
        assert {ln.split("\t")[0] for ln in gsam if not ln.startswith("@")} <= set(names)
        assert genome_check.filter_genome_hits(gsam) == want


def _split_row(row, n_fixed):
    f = row.rstrip("\n").split("\t")
    head, rest = f[:n_fixed], f[n_fixed:]
    return head, [set(x.split(";")) - {""} for x in rest]


def test_final_fusion(fx, index, tmp_path):
    for case in fx["final_fusion"]:
        cands = []
        for c in case["spec"]:
            obj = report.Candidate(c["type"])
            for a in c["adds"]:
                obj.add_reads(a["target"], list(a["other"]), a["left"], a["right"], a["mid"], a["cnt"],
                              list(a["spanning"]), list(a["split"]))
            obj.score = c["score"]
            cands.append(obj)
        for obj, want in zip(cands, case["maxpos"]):
            pos, best = obj.find_max_pos()
            assert list(pos) + [best] == want
        scores = [c["score"] for c in case["spec"]]
        prefix = str(tmp_path / "pred")
        report.write_predictions(prefix, cands, "BCR", index, scores, case["cnt_max"], case["no_filter"])
        with open(prefix + "_predictions_abridged.txt") as fa:
            assert fa.readlines() == case["abridged"]
        n_fixed = 7 if case["no_filter"] else 8   # read-name columns follow; order = set order
        with open(prefix + "_predictions.txt") as fo:
            got = fo.readlines()
        assert len(got) == len(case["full"]) and got[0] == case["full"][0]
        for g, w in zip(got[1:], case["full"][1:]):
            assert _split_row(g, n_fixed) == _split_row(w, n_fixed)


def test_partner_chain():
    """a9 -> a10 -> a11 -> a13 -> a14 replayed against the reference's outputs (and the
    exact sequence of tool queries it issued), in a PYTHONHASHSEED=0 subprocess."""
    import subprocess
    import sys
    env = dict(os.environ, PYTHONHASHSEED="0")
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "partner_chain.py")],
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]


def test_partition_matches_full_sort():
    # align.partition (S3, AF:183-194) sorts only placed records; check it against sorting every
    # record by samtools' key (placed by (pos, strand), ties in input order, unplaced last)
    import numpy as np
    from anchored_fusion_amd.align import AlignResult, partition
    rng = np.random.default_rng(5)
    n = 20000
    flag = np.zeros(n, np.int32)
    pos = np.full(n, -1, np.int32)
    for p in range(n // 2):
        m = rng.random(2) < 0.3
        rv = rng.random(2) < 0.5
        x = rng.integers(0, 300, 2)
        for k in (0, 1):
            r = 2 * p + k
            f = 0x1 | (0x40 if k == 0 else 0x80)
            if m[k]:
                f |= 0x10 if rv[k] else 0
                pos[r] = x[k]
            else:
                f |= 0x4
            if not m[1 - k]:
                f |= 0x8
            elif rv[1 - k]:
                f |= 0x20
            flag[r] = f
        for k in (0, 1):  # unmapped mate of a mapped read: the mate's position
            if not m[k] and m[1 - k]:
                pos[2 * p + k] = pos[2 * p + 1 - k]
    z = np.zeros(n, np.int32)
    res = AlignResult(flag, pos, z, z, np.zeros((n, 32), np.uint32), z)
    key = np.where(pos >= 0, pos.astype(np.int64) * 2 + ((flag & 0x10) != 0), np.int64(1) << 62)
    order = np.argsort(key, kind="stable")
    f = flag[order]
    want = (order[((f & 0x8) != 0) & ((f & 260) == 0)], order[((f & 0x4) != 0) & ((f & 264) == 0)],
            order[(f & 772) == 0])
    for a, b in zip(partition(res), want):
        assert np.array_equal(a, b)
