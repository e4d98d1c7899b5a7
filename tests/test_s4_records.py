"""The S4 consumer over records (blocks.S4Records / spanning_blocks_records: no SAM text) equals
`spanning_blocks` over the SAM lines of the same records (Find_blocks, functions.py:376-496):
the genome records of the one-end-anchored pairs of a fusion world (S2 + S3 + S4 on the CPU
oracle, through dist_discover's driver), plus crafted groups -- unmapped mates, duplicate QNAMEs
of consecutive pairs, reads without records, mates on one contig within and beyond 2,000 nt."""
import numpy as np

import afpkg  # noqa: F401
from anchored_fusion_amd import blocks, genome, pipeline
from anchored_fusion_amd.annotation import ExonIndex
from fusion_world import make_world

CHUNK = 300_000
GENE = "BCRX"


def _as_tuples(bc):
    return {c: [b.as_tuple() for b in bl] for c, bl in bc.items()}


def _texts(names, recs, nrec, contigs, seqs):
    lines = []
    for k in range(len(nrec) // 2):
        for m in (0, 1):
            r = 2 * k + m
            lines += genome.sam_lines(contigs, names[k], seqs[r], recs[r], nrec[r])
    return lines


def test_records_path_equals_text_path(tmp_path):
    import oracle
    from anchored_fusion_amd import dist_discover
    from anchored_fusion_amd import io as afio
    from oracle_discovery import OracleDiscovery, tiles_for
    paths, _ = make_world(str(tmp_path / "w"), n_fusion=600, n_anchor=500, n_background=2500)
    names, reads, lens = afio.read_pairs(paths["fq1"], paths["fq2"])
    contigs = [(h.split()[0], s.decode().upper()) for h, s in pipeline.read_fasta(paths["genome"])]
    anchor = afio.anchor_sequence(paths["anchor"])
    with open(paths["gtf"]) as fh:
        index = ExonIndex.from_lines(fh.readlines())
    og = oracle.OracleGenome(contigs)
    ln = np.full(reads.shape[0], reads.shape[1], np.int32) if lens is None else lens
    backend = OracleDiscovery(anchor, og, tiles_for(contigs), reads, ln, 0, CHUNK, GENE)
    res, _ = dist_discover.search(backend, 0, 0, 1, names=names, s4_reads=True)
    q, ql, recs, nrec, g1 = (x.numpy() for x in res["s4"])
    recs = recs.view(genome.REC_DTYPE).reshape(recs.shape[0], recs.shape[1])
    pn = [res["names"][int(g)] for g in g1]
    seqs = [q[r, :ql[r]].tobytes().decode() for r in range(len(ql))]
    homo = ["ENSG00000186716.21"]
    want = blocks.spanning_blocks(_texts(pn, recs, nrec, og.names, seqs), index, homo)
    got = blocks.spanning_blocks_records(blocks.S4Records(pn, recs, nrec, og.names), index, homo)
    assert sum(len(v) for v in want.values()) > 0
    assert _as_tuples(got) == _as_tuples(want)
    # crafted: duplicate names of consecutive pairs, reads without records, unmapped mates,
    # mates far apart on one contig
    rng = np.random.default_rng(3)
    P = len(nrec) // 2
    pn2 = list(pn)
    for k in rng.choice(np.arange(1, P), P // 10, replace=False):
        pn2[k] = pn2[k - 1]
    nrec2 = nrec.copy()
    nrec2[rng.choice(len(nrec2), len(nrec2) // 20, replace=False)] = 0
    recs2 = recs.copy()
    un = rng.choice(len(nrec2), len(nrec2) // 10, replace=False)
    recs2["flag"][un, 0] = 4
    recs2["rid"][un, 0] = -1
    recs2["n_cigar"][un, 0] = 0
    far = rng.choice(len(nrec2), len(nrec2) // 10, replace=False)
    recs2["pos"][far, 0] += 2500
    want = blocks.spanning_blocks(_texts(pn2, recs2, nrec2, og.names, seqs), index, homo)
    got = blocks.spanning_blocks_records(blocks.S4Records(pn2, recs2, nrec2, og.names), index, homo)
    assert _as_tuples(got) == _as_tuples(want)


def test_records_path_empty():
    from anchored_fusion_amd.annotation import ExonIndex
    R = blocks.S4Records([], None, np.zeros(0, np.int32), ["chr1"])
    assert blocks.spanning_blocks_records(R, ExonIndex({}), []) == {}
