"""dist_discover on CPU with gloo: S3-S6 of a sample sharded over 1-3 ranks, each rank on its own
whole bwa chunks (S5 with the global read ids and QNAME groups, S4 per rank on whole chunks of the globally
zipped tmp1 / tmp2 lists), equal to the one-process host path (pipeline.host_products) text for
text -- S4's SAM lines, the split_sam lines S5's check keeps, S6's PSL lines.  The backend is the
CPU oracle (tests/oracle_discovery.py); the GPU backend is discover.CandidateDiscovery."""
import json
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import afpkg  # noqa: F401
from anchored_fusion_amd import pipeline
from fusion_world import make_world

CHUNK = 300_000
GENE = "BCRX"


def _inputs(paths):
    from anchored_fusion_amd import io as afio
    names, reads, lens = afio.read_pairs(paths["fq1"], paths["fq2"])
    genome = [(h.split()[0], s.decode().upper()) for h, s in pipeline.read_fasta(paths["genome"])]
    anchor = afio.anchor_sequence(paths["anchor"])
    return names, reads, lens, genome, anchor


def _worker(rank, world, port, paths, out, chunk):
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    import torch.distributed as dist

    import oracle
    from anchored_fusion_amd import dist_discover, shard
    from oracle_discovery import OracleDiscovery, tiles_for
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    names, reads, lens, genome, anchor = _inputs(paths)
    ln = np.full(reads.shape[0], reads.shape[1], np.int32) if lens is None else lens
    lo, hi = shard.shard_pairs(ln.astype(np.int64).reshape(-1, 2).sum(axis=1), rank, world, chunk)
    og = oracle.OracleGenome(genome)
    backend = OracleDiscovery(anchor, og, tiles_for(genome), reads[2 * lo:2 * hi], ln[2 * lo:2 * hi], lo, chunk, GENE)
    res, counts = dist_discover.search(backend, lo, rank, world, names=names.slice(lo, hi), s4_reads=True)
    if rank == 0:
        texts = dist_discover.render(res, backend, GENE, og.names)
        with open(os.path.join(out, f"texts{world}.json"), "w") as fh:
            json.dump(texts, fh)
    dist.barrier()
    dist.destroy_process_group()


def _run(paths, out, world, chunk=CHUNK):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.start_processes(_worker, args=(world, port, paths, out, chunk), nprocs=world, join=True, start_method="spawn")
    with open(os.path.join(out, f"texts{world}.json")) as fh:
        return json.load(fh)


@pytest.fixture(scope="module")
def world_and_host(tmp_path_factory):
    from oracle_backends import OracleAligner, oracle_searches
    d = tmp_path_factory.mktemp("dd")
    paths, _ = make_world(str(d / "world"), n_fusion=600, n_anchor=500, n_background=2500)
    names, reads, lens, genome, anchor = _inputs(paths)
    res = OracleAligner(anchor, chunk_bases=CHUNK).align_pairs(reads, lens)
    host = pipeline.host_products(GENE, names, reads, lens, res, oracle_searches(genome, CHUNK), log=lambda *_: None)
    return paths, str(d), [list(x) for x in host]


@pytest.mark.parametrize("world", [1, 2, 3])
def test_dist_discover_equals_host_path(world_and_host, world):
    paths, d, host = world_and_host
    got = _run(paths, d, world)
    s4, split_sam, psl = host
    assert len(split_sam) > 10 and len(s4) > 10 and len(psl) > 10
    assert got[0] == s4
    assert got[1] == split_sam
    assert got[2] == psl


def test_dist_discover_s4_over_several_chunks(world_and_host, tmp_path):
    """bwa chunks of 20 kbases: S4's stream spans several chunks, so each of 3 ranks aligns its
    share of them (pair_base = its first S4 pair) and rank 0 collects the records."""
    from oracle_backends import OracleAligner, oracle_searches
    paths, _, _ = world_and_host
    chunk = 20_000
    names, reads, lens, genome, anchor = _inputs(paths)
    res = OracleAligner(anchor, chunk_bases=chunk).align_pairs(reads, lens)
    host = pipeline.host_products(GENE, names, reads, lens, res, oracle_searches(genome, chunk), log=lambda *_: None)
    s4_bases = sum(len(ln.split("\t")[9]) for ln in host[0] if int(ln.split("\t")[1]) & 0x900 == 0)
    assert s4_bases > 3 * chunk  # every rank gets S4 work
    got = _run(paths, str(tmp_path), 3, chunk)
    assert [list(x) for x in host] == got


def test_dist_discover_one_process_without_group(world_and_host):
    """world 1 needs no process group: the driver is also the one-GPU form of the step."""
    import oracle
    from anchored_fusion_amd import dist_discover
    from oracle_discovery import OracleDiscovery, tiles_for
    paths, _, host = world_and_host
    names, reads, lens, genome, anchor = _inputs(paths)
    og = oracle.OracleGenome(genome)
    ln = np.full(reads.shape[0], reads.shape[1], np.int32) if lens is None else lens
    backend = OracleDiscovery(anchor, og, tiles_for(genome), reads, ln, 0, CHUNK, GENE)
    res, _ = dist_discover.search(backend, 0, 0, 1, names=names, s4_reads=True)
    assert [list(x) for x in dist_discover.render(res, backend, GENE, og.names)] == host
