"""The multi-GPU configs at one rank's shape, on one GPU.

* configs[3] (50 M 2x150 pairs over 8 GPUs): rank 3's shard -- 6.25 M pairs starting at its bwa
  chunk (pair_base) -- through discover.CandidateDiscovery as bench.py's ranks run it: S2
  bit-exact vs the oracle on the shard's first two chunks (the read ids and insert-size chunks of
  the global input), the S4 / S5 records equal to the genome engine's own host-buffer calls,
  S5's genome check and the S6 queries equal to the host chain, and the product's multi-GPU step
  (dist_discover.search on the rank's lo) through a one-rank RCCL group, its all-gathers and
  all-to-alls on device tensors, giving the same counts, S4 records and survivors with global
  read rows.  The genome is
  the configs[2] world at full size (3.09 Gbp: the index and tiles the bench's ranks build).
* configs[4] (1,000 cells x 100 k pairs over 8 GPUs): one rank's 125 cells through
  singlecell.run, the planted fusion merged from the cells, and three sampled cells' tables
  byte-identical to the CPU-oracle backends on the same cells (SC:205-287)."""
import os

import numpy as np
import pytest

import oracle
from helpers import assert_records_equal

pytestmark = pytest.mark.gpu


def test_configs3_rank3_shape(anchor):
    import socket

    import torch
    import torch.distributed as dist

    from anchored_fusion_amd import discover, simworld
    from anchored_fusion_amd.align import AlignResult, partition
    from anchored_fusion_amd.shard import chunk_pairs, shard_range
    from test_gpu_c3 import _check_genome_records, _check_s5_s6
    N, L, world, rank = 50_000_000, 150, 8, 3
    lo, hi = shard_range(N, rank, world, L)
    n = hi - lo
    assert lo % chunk_pairs(L) == 0 and 6_000_000 < n < 6_500_000
    W = simworld.GenomeWorld(anchor, device=0, seed=20251015, scale=1.0)
    gidx, tiles = W.genome_index(), W.tiles()
    reads_t = W.simulate_pairs(n, read_len=L, seed=20251015, pair_base=lo)
    torch.cuda.synchronize()
    W.blob = None
    rank_chunks = -(-n // chunk_pairs(L))
    d = discover.CandidateDiscovery(anchor, gidx, tiles, n, L, device=0, inflight=4,
                                    batch_chunks=max(1, min(240, -(-rank_chunks // 4))), pair_base=lo)
    try:
        d.run(reads_t)
        summ = d.summary()
        assert summ["anchored"] > 50_000 and summ["s4_pairs"] > 1000 and summ["s6_queries"] > 1000
        assert summ["s4_pairs_dropped"] == 0 and summ["s5_dropped"] == 0 and summ["s6_clipped"] == 0
        # S2 bit-exact on the shard's first two bwa chunks (global read ids / chunks via pair_base)
        m = 2 * chunk_pairs(L)
        sub = reads_t[:2 * m].cpu().numpy()
        got = {k: v[:2 * m].cpu().numpy() for k, v in d.out.items()}
        got["cigar"] = got["cigar"].view(np.uint32)
        assert_records_equal(got, oracle.OracleIndex(anchor).align_pairs(sub, threads=8, pair_base=lo), sub)
        # S3 on the device == the host rule over the whole shard
        reads = reads_t.cpu().numpy()
        full = {k: v.cpu().numpy() for k, v in d.out.items()}
        full["cigar"] = full["cigar"].view(np.uint32)
        res = AlignResult(full["flag"], full["pos"], full["score"], full["n_cigar"], full["cigar"], full["hits"])
        t1, t2, an = partition(res)
        c = d.counts
        assert (c["tmp1"], c["tmp2"], c["anchored"]) == (len(t1), len(t2), len(an))
        assert np.array_equal(d.s3[2][:len(an)].cpu().numpy(), an)
        # the genome calls and S5's check / S6 queries
        nq = int(d.n_q.item())
        _check_genome_records(d, gidx, d.q[:nq].cpu().numpy(), nq, c["s4_pairs"])
        _check_s5_s6(d, gidx, reads, full, an, c["s4_pairs"], nq)
        # the product's multi-GPU step (dist_discover.search) on the rank's lo, its exchanges through a
        # one-rank RCCL group on device tensors (AF_DIST_COLLECTIVES=1): the same counts, S4 records
        # and survivors, global read rows inside the shard
        npair = c["s4_pairs"]
        rec_bytes = 2 * npair * discover.MAX_REC * discover._genome.REC_DTYPE.itemsize
        s4_n0, s4_r0 = d.q_nh[:2 * npair].cpu().numpy(), d.q_recs[:rec_bytes].cpu().numpy()
        from anchored_fusion_amd import dist_discover
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), AF_DIST_COLLECTIVES="1")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        try:
            out, cnt = dist_discover.search(d.attach(reads_t, None), lo, 0, 1, device="cuda:0")
            torch.cuda.synchronize()
        finally:
            dist.destroy_process_group()
            os.environ.pop("AF_DIST_COLLECTIVES", None)
        for k in ("tmp1", "tmp2", "s5_split_reads", "s6_queries", "s4_pairs"):
            assert cnt[k] == summ[k], (k, cnt[k], summ[k])
        _, _, recs, nrec, g1 = out["s4"]
        assert np.array_equal(nrec.cpu().numpy(), s4_n0)
        got_r = recs.cpu().numpy().view(np.uint8).reshape(2 * npair, -1)
        want_r = s4_r0.reshape(2 * npair, -1)
        live = np.arange(discover.MAX_REC)[None, :] < s4_n0[:, None]
        per = want_r.shape[1] // discover.MAX_REC
        assert np.array_equal(got_r.reshape(2 * npair, discover.MAX_REC, per)[live],
                              want_r.reshape(2 * npair, discover.MAX_REC, per)[live])
        surv = out["surv"].cpu().numpy()
        assert surv.shape[0] == summ["s6_queries"]
        grow = surv[:, -2].view(np.uint32).astype(np.int64) | (surv[:, -1].astype(np.int64) << 32)
        assert (grow >= 2 * lo).all() and (grow < 2 * (lo + n)).all()
        g1 = g1.cpu().numpy()
        assert (g1 >= 2 * lo).all() and (g1 < 2 * (lo + n)).all()
    finally:
        d.close()
        gidx.close()
        tiles.close()


def test_configs4_rank_125_cells(tmp_path):
    from anchored_fusion_amd import pipeline, singlecell
    from cells_world import write_cells
    from oracle_backends import OracleAligner, oracle_searches
    paths, truth, cells_dir, cells = write_cells(str(tmp_path), 125, 100_000)
    gpu = str(tmp_path / "gpu")
    merged = singlecell.run(paths["anchor"], cells_dir, paths["genome"], paths["gtf"], gpu, log=lambda *_: None)
    rows = [k for k in merged.get("BCRX", {}) if "ABLX" in k]
    assert rows, "the planted fusion is not in the merged table"
    assert merged["BCRX"][rows[0]][2] >= 50  # cells that support it
    assert abs(int(rows[0].split("$")[2].split(":")[1]) - truth["anchor_junction"]) <= 3
    # three sampled cells through the CPU-oracle backends: per-cell tables byte-identical
    sample = [cells[0], cells[62], cells[124]]
    sub = str(tmp_path / "sample")
    os.makedirs(sub)
    for c in sample:
        for m in (1, 2):
            f = f"{c}_{m}.fastq.gz"
            os.symlink(os.path.join(cells_dir, f), os.path.join(sub, f))
    genome = [(h.split()[0], s.decode().upper()) for h, s in pipeline.read_fasta(paths["genome"])]
    cpu = str(tmp_path / "cpu")
    singlecell.run(paths["anchor"], sub, paths["genome"], paths["gtf"], cpu, searches=oracle_searches(genome),
                   aligner_factory=OracleAligner, log=lambda *_: None)
    for c in sample:
        for x in (".txt", "_abridged.txt"):
            f = os.path.join("BCRX", "work_dir", c, "BCRX_fusion_predictions" + x)
            a = open(os.path.join(gpu, f), "rb").read()
            b = open(os.path.join(cpu, f), "rb").read()
            assert a == b, f
