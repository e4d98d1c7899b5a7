#!/usr/bin/env python3
"""Benchmark of the anchored split-read alignment hot path (BASELINE.json metric: paired reads/sec
through anchored split-read align on 1/2/4/8 MI355X).

Default workload (--config c3, BASELINE.json configs[2]; configs[3] at N > 1): 50 M distinct
synthetic 2x150 bp pairs against one anchor transcript (the bundled BCR NM_004327.4) with an
hg38-scale genome index resident in HBM.  The world is made on the device by libafsim.so
(simworld.py): 3.09 Gbp in hg38's 24 contig sizes with repeat families, satellites and segmental
duplications, the anchor and 8 partner genes embedded as exons; 5 % of the pairs come from the
anchor fusions, the rest from the genome (wgsim's read model, seeded per pair).  A step is one
pass of discover.CandidateDiscovery over the resident pairs:
  S2  K1 + K2 + K3 per batch of 240 bwa chunks (8 M pairs; `bwa mem -M anchor fq1 fq2`,
      Anchored_Fusion.py:182), 4 batches in flight;
  S3  the samtools coordinate sort and the -f 8 / -f 4 / -F 772 partitions (AF:182, 186-194);
  S4  the one-end-anchored pairs (tmp1 / tmp2) and S5 the anchored split reads placed on the genome
      (`bwa mem -M genome`, AF:188 and functions.py:716);
  S5 check  `del_too_many_reads`' genome check of the split reads (fn:718-768) on the device;
  S6  the survivors searched on the genome with the BLAT restatement (-minScore=20, fn:530;
      11-mer tile index of the genome);
  and at N > 1 the all-gatherv of the breakpoint candidates (RCCL).
Inputs are resident in HBM before timing starts.  At N > 1 the 50 M pairs are sharded on bwa's
10 Mbase chunk grid (strong scaling, configs[3]).

--config c2 is configs[1]: 1 M synthetic 2x100 pairs per GPU, the step S2 + split-tail placement on
the workload's transcripts, 8 batches in flight (round-1 headline; weak scaling).

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 the driver uses
torch.distributed.run, one rank per GPU.  The time is the max over ranks.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--config", choices=("c3", "c2"), default="c3")
    ap.add_argument("--steps", type=int, default=None, help="default 12 (c3) / 20 (c2)")
    ap.add_argument("--warmup", type=int, default=None, help="default 2 (c3) / 3 (c2)")
    ap.add_argument("--pairs", type=int, default=None, help="c3: total pairs (50 M); c2: pairs per GPU (1 M)")
    ap.add_argument("--read-len", type=int, default=None, help="default 150 (c3) / 100 (c2)")
    ap.add_argument("--genome-scale", type=float, default=1.0, help="c3: genome size as a fraction of hg38")
    ap.add_argument("--batch-chunks", type=int, default=0,
                    help="c3: bwa chunks per S2 batch; 0 = min(240, the rank's chunks / batches in flight), so a "
                         "rank's share is at least one full group (240 x 33,334 pairs = 8 M pairs; sweep in DESIGN.md)")
    ap.add_argument("--fusion-frac", type=float, default=0.05)
    ap.add_argument("--cpu-sample", type=int, default=1_000_000, help="pairs timed on the CPU oracle (rank 0, N=1)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="repeat the CPU sample until this much wall time")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = the host CPU share (OMP_NUM_THREADS, else all cores)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-placement", action="store_true", help="skip the S2 + partner placement leg")
    ap.add_argument("--no-kernel-events", action="store_true", help="diagnostic: no timing events in the timed region")
    ap.add_argument("--inflight", type=int, default=None,
                    help="batches in flight (AlignerGroup): their K1s back to back, then their K2s at once "
                         "(default 4 for c3, 8 for c2)")
    a = ap.parse_args()
    c3 = a.config == "c3"
    a.steps = a.steps if a.steps is not None else (12 if c3 else 20)
    a.warmup = a.warmup if a.warmup is not None else (2 if c3 else 3)
    a.pairs = a.pairs if a.pairs is not None else (50_000_000 if c3 else 1_000_000)
    a.read_len = a.read_len if a.read_len is not None else (150 if c3 else 100)
    a.inflight = a.inflight if a.inflight is not None else (4 if c3 else 8)
    return a


def pmc_traffic(pairs, read_len):
    """HBM bytes per K1 launch of this batch shape from the committed counter passes
    (profiles/pmc_seed_filter.json: rocprofv3 FETCH_SIZE + WRITE_SIZE, gfx950-corrected), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_seed_filter.json")
    try:
        pm = json.load(open(path))
    except (OSError, ValueError):
        return None
    for e in pm.get("entries", [pm]):
        if e.get("pairs") == pairs and e.get("read_len") == read_len:
            return e.get("hbm_bytes_per_launch")
    return None


PROF = os.path.join("profiles", "r05")  # this round's committed rocprofv3 summaries (scripts/summarize_prof.py)


def rocprof_k1(bytes_per_launch, n_launch):
    """K1's roofline fraction from the committed rocprofv3 kernel trace of the same command
    (profiles/r05/kernel_stats_c3.csv: average k_seed_stream duration over every launch of the
    traced steps, the same mix of full and remainder batches), beside the live HIP-event figure."""
    import csv
    path = os.path.join(ROOT, PROF, "kernel_stats_c3.csv")
    try:
        for r in csv.DictReader(open(path)):
            if "k_seed_stream" in r["Name"]:
                calls, avg_ns = int(r["Calls"]), float(r["AverageNs"])
                if calls % max(1, n_launch):
                    return None  # a different batch shape
                gbs = bytes_per_launch / avg_ns
                return {"source": f"{PROF}/kernel_stats_c3.csv", "launches": calls,
                        "avg_us": round(avg_ns / 1e3, 1), "achieved": round(gbs, 1),
                        "frac": round(gbs / HBM_PEAK_GBS, 4)}
    except (OSError, KeyError, ValueError):
        return None
    return None


def issue_roofline():
    """The step's compute / latency-bound kernels against their VALU issue roofline and HBM
    traffic, from this round's committed counter passes of the same command (profiles/r05/
    pmc_c3.json: SQ issue / wait counters and FETCH_SIZE per launch), or None."""
    try:
        pm = json.load(open(os.path.join(ROOT, PROF, "pmc_c3.json")))
    except (OSError, ValueError):
        return None
    keep = ("avg_duration_us", "unit", "valu_issue_frac", "wait_any_frac", "avg_resident_waves_per_simd",
            "fetch_gbs_x2", "fetch_bytes_per_unit_x2")
    return {"source": f"{PROF}/pmc_c3.json", "model": pm.get("issue_model"),
            "kernels": {k: {f: e[f] for f in keep if f in e} for k, e in pm.get("kernels", {}).items()
                        if any(k.startswith(p) for p in ("k_g_", "k_blat", "k_s2_", "k_s5"))}}


def cpu_threads(args):
    """The host CPU share: OMP_NUM_THREADS (16 per GPU on the box, where os.cpu_count() shows the
    whole machine), else every core."""
    if args.cpu_threads:
        return args.cpu_threads
    env = os.environ.get("OMP_NUM_THREADS")
    return int(env) if env and env.isdigit() and int(env) > 0 else (os.cpu_count() or 1)


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import afpkg  # noqa: F401

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; AF_BENCH_BACKEND=gloo rehearses N ranks on fewer GPUs (ranks share
    # devices round-robin) -- the driver's runs use RCCL ("nccl") with one GPU per rank
    backend = os.environ.get("AF_BENCH_BACKEND", "nccl")
    gpu = local % max(1, torch.cuda.device_count()) if backend == "gloo" else local
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    ctx = dict(world=world, rank=rank, gpu=gpu, dev=dev, backend=backend)
    if args.config == "c3":
        bench_c3(args, **ctx)
    else:
        bench_c2(args, **ctx)
    if world > 1:
        dist.destroy_process_group()


def max_over_ranks(t, world, dev, backend):
    import torch
    import torch.distributed as dist
    if world == 1:
        return t
    tt = torch.tensor([t], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    return float(tt.item())


def bench_c2(args, world, rank, gpu, dev, backend):
    """configs[1]: S2 + split-tail placement on 1 M 2x100 pairs per GPU (weak scaling)."""
    import torch
    import torch.distributed as dist

    from anchored_fusion_amd import io as afio
    from anchored_fusion_amd import simulate as sim
    from anchored_fusion_amd.align import AlignerGroup
    anchor = afio.anchor_sequence(os.path.join(ROOT, "tests", "golden", "target_gene.fasta"))
    L = args.read_len
    _, reads, _, fworld = sim.fusion_reads(anchor, args.pairs, read_len=L, fusion_frac=args.fusion_frac,
                                      seed=20251015 + 7919 * rank)
    nr = reads.shape[0]
    reads_t = torch.from_numpy(reads).to(dev)
    G = max(1, args.inflight)

    def outs():
        o = {k: torch.zeros(nr, dtype=torch.int32, device=dev) for k in ("flag", "pos", "score", "n_cigar", "hits")}
        o["cigar"] = torch.zeros((nr, 32), dtype=torch.int32, device=dev)
        return o

    bufs = [outs() for _ in range(G)]
    grp = AlignerGroup(anchor, device=gpu, inflight=G)

    post = None if args.no_placement else Placement(fworld, anchor, nr, L, G, dev)

    def run(n_batches, evs=None, with_placement=True):
        """n_batches steps (one batch each), G at a time; every group waits for the last.
        evs: per group a pair of timing events around its back-to-back K1 launches."""
        done = None
        for k0 in range(0, n_batches, G):
            g = min(G, n_batches - k0)
            pl = with_placement and post is not None
            done = grp.run_device([(reads_t, args.pairs, L, bufs[j]) for j in range(g)],
                                  events=None if evs is None else evs[k0 // G], wait=done,
                                  tails=post.tails if pl else None, before=post.before if pl else None)
            if pl:
                post.end_group()
        if with_placement and post is not None:
            s0 = grp.streams[0]
            for e in done:
                s0.wait_event(e)
            post.flush(s0)
            torch.cuda.current_stream(dev).wait_stream(s0)
        return done

    run(args.warmup)
    torch.cuda.synchronize(dev)
    n_cand = grp.aligners[0].last_candidates()
    out = bufs[0]
    mapped = int(((out["flag"] & 4) == 0).sum().item())

    # timing events around each group's K1 launches only (they run back to back on one
    # stream): markers between the overlapped K2s would cost time
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range((args.steps + G - 1) // G)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    run(args.steps, None if args.no_kernel_events else evs)
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    elapsed = t1 - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    k1_ms = float("nan") if args.no_kernel_events else sum(e[0].elapsed_time(e[1]) for e in evs) / args.steps
    k23_ms = elapsed / args.steps * 1e3 - k1_ms  # the rest of the step: K2 + K3 (+ launch gaps)

    bytes_per_launch = nr * L + 4 * nr  # 2L bases + 2 x int32 per pair (SURVEY.md §8 d)
    achieved = bytes_per_launch / (k1_ms * 1e-3) / 1e9
    traffic = pmc_traffic(args.pairs, L)

    total_pairs = args.pairs * world * args.steps
    value = total_pairs / elapsed
    res = {
        "metric": "paired reads/sec through anchored split-read align",
        "value": round(value, 1),
        "unit": "pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic (wgsim-style simulator, seed 20251015 + rank)",
        "config": {
            "workload": f"configs[1] (--config c2): {args.pairs} synthetic 2x{L} bp pairs per GPU, one anchor "
                        f"(BCR NM_004327.4, {len(anchor)} nt), {args.fusion_frac:.0%} fusion pairs"
                        + ("" if args.no_placement else "; S2 + partner placement of the split-read tails"),
            "pairs_per_gpu": args.pairs, "read_len": L, "anchor_len": len(anchor),
            "parallelism": f"dp{world}", "candidates_per_step": n_cand, "mapped_reads_per_step": mapped,
        },
        "inflight": G,
        "kernels_ms": {"seed_filter": round(k1_ms, 5), "align_candidates_and_pairs": round(k23_ms, 5),
                       "note": "seed_filter: HIP events around each group's back-to-back K1 launches on their "
                               "stream, per batch; "
                               "align_candidates_and_pairs: ms_per_step minus that"},
        "roofline": {
            "kernel": "k_seed_filter", "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "bytes_per_launch": bytes_per_launch,
        },
    }
    if post is not None:
        res["partner_placement"] = post.report()
        # the same steps without the placement (S2 alone), for reference
        run(G, with_placement=False)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        run(args.steps, with_placement=False)
        torch.cuda.synchronize(dev)
        t_s2 = time.perf_counter() - t0
        if world > 1:
            tt = torch.tensor([t_s2], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            t_s2 = float(tt.item())
        res["s2_only"] = {"value": round(args.pairs * world * args.steps / t_s2, 1), "unit": "pairs/s",
                          "ms_per_step": round(t_s2 / args.steps * 1e3, 4)}
    if rank == 0 and world == 1:
        # the host-buffer API on the same batch: H2D of the reads + the three kernels + D2H of
        # the records (reported beside `value`, never as it)
        al = grp.aligners[0]
        al.align_pairs(reads)
        t0 = time.perf_counter()
        al.align_pairs(reads)
        dt = time.perf_counter() - t0
        res["pcie_inclusive"] = {"value": round(args.pairs / dt, 1), "unit": "pairs/s",
                                 "note": "af_align_pairs with host buffers (H2D reads, D2H records), 1 call"}
    if rank == 0 and world == 1 and not args.no_cpu:
        res["cpu_baseline"] = cpu_baseline(anchor, reads, args, None if args.no_placement else fworld)
    if rank == 0:
        print(json.dumps(res), flush=True)
    grp.close()


def bench_c3(args, world, rank, gpu, dev, backend):
    """configs[2] (N = 1) / configs[3] (N > 1): S2 + S3 + the S4/S5/S6 genome searches over 50 M
    2x150 pairs with an hg38-scale genome index resident (strong scaling across ranks)."""
    import torch
    import torch.distributed as dist

    from anchored_fusion_amd import discover, dist_discover, simworld
    from anchored_fusion_amd import io as afio
    from anchored_fusion_amd.shard import shard_range
    anchor = afio.anchor_sequence(os.path.join(ROOT, "tests", "golden", "target_gene.fasta"))
    L, N = args.read_len, args.pairs

    def log(msg):
        if rank == 0:
            print(f"[bench c3] {msg}", file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    W = simworld.GenomeWorld(anchor, device=gpu, seed=20251015, scale=args.genome_scale)
    t_gen = time.perf_counter() - t0
    log(f"genome {W.total / 1e9:.2f} Gbp made in {t_gen:.1f} s")
    subset = genome_subset(W) if rank == 0 and world == 1 and not args.no_cpu else None
    t0 = time.perf_counter()
    ref = W.genome_index()
    torch.cuda.synchronize(dev)
    t_bwa = time.perf_counter() - t0
    tiles = W.tiles()
    torch.cuda.synchronize(dev)
    t_idx = time.perf_counter() - t0
    log(f"genome indexes built: bwa index (suffix array + FM occ) {t_bwa:.1f} s, BLAT 11-mer tiles "
        f"{t_idx - t_bwa:.1f} s")
    lo, hi = shard_range(N, rank, world, L)
    from anchored_fusion_amd.shard import chunk_pairs
    rank_chunks = -(-(hi - lo) // chunk_pairs(L))
    # at most 240 bwa chunks (8 M pairs of 2x150) per batch, at least `inflight` batches per rank
    # (profiles/r02/c3_n1_batch_sweep.txt, c3_n8_batch_sweep.txt)
    batch_chunks = args.batch_chunks or max(1, min(240, -(-rank_chunks // max(1, args.inflight))))
    n = hi - lo
    reads_t = torch.empty((2 * max(n, 1), L), dtype=torch.uint8, device=dev)
    if n:
        W.simulate_pairs(n, read_len=L, seed=20251015, pair_base=lo, out=reads_t[:2 * n])
    torch.cuda.synchronize(dev)
    log(f"{n} pairs simulated")
    W.blob = None  # the index keeps its own copy
    torch.cuda.empty_cache()
    disc = discover.CandidateDiscovery(anchor, ref, tiles, n, L, device=gpu, inflight=max(1, args.inflight),
                                       batch_chunks=batch_chunks, pair_base=lo)
    genome_bp = sum(W.lens)
    G = disc.grp.inflight
    n_groups = (len(disc.batches) + G - 1) // G

    step_counts = {}

    def step(k1=None, ph=None):
        if world > 1:
            # the product's multi-GPU step (dist_discover): S2-S6 on this rank's chunks with the
            # global read ids and QNAME groups, S4 on whole chunks of the globally zipped stream per rank, the
            # survivors and their S6 rows all-gathered over RCCL
            _, c = dist_discover.search(disc.attach(reads_t, None, k1), lo, rank, world, device=dev)
            step_counts.update(c)
        else:
            disc.run(reads_t, k1_events=k1, phase_events=ph)

    for w in range(args.warmup):
        t0 = time.perf_counter()
        step()
        torch.cuda.synchronize(dev)
        log(f"warm-up pass {w}: {time.perf_counter() - t0:.3f} s, "
            f"{disc.summary() if world == 1 else step_counts}")
    free, total = torch.cuda.mem_get_info(dev)
    E = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    k1 = [[[E(), E()] for _ in range(n_groups)] for _ in range(args.steps)]
    ph = [[E() for _ in range(5)] for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    disc.tiles_ref.caps(reset=True)  # BLAT cap counters: from the timed steps only
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        s0 = disc.grp.streams[0]
        if world == 1:
            ph[k][0].record(s0)
        step(None if args.no_kernel_events else k1[k], ph[k][1:] if world == 1 else None)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    elapsed = max_over_ranks(elapsed, world, dev, backend)
    ms = elapsed / args.steps * 1e3
    summ = disc.summary() if world == 1 else dict(step_counts)
    if world == 1:  # af_blat_caps accumulates over the timed steps: per step
        summ.update({k: v / args.steps for k, v in summ.items() if k.startswith("blat_cap_")})
    n_launch = len(disc.batches)
    k1_ms = float("nan") if args.no_kernel_events else \
        sum(e[0].elapsed_time(e[1]) for st in k1 for e in st) / args.steps
    phase = lambda a, b: sum(p[a].elapsed_time(p[b]) for p in ph) / args.steps  # noqa: E731
    bp = max(b for _, b in disc.batches) if disc.batches else 0
    # SURVEY §8 d: 2L bases + 2 x int32 per pair, one batch per K1 launch; the average launch
    # over the step (the batches are equal up to the last chunk's remainder)
    k1_bytes = sum(b for _, b in disc.batches) * (2 * L + 8)
    bytes_per_launch = k1_bytes / max(1, n_launch)
    k1_launch_ms = k1_ms / max(1, n_launch)
    achieved = bytes_per_launch / (k1_launch_ms * 1e-3) / 1e9
    traffic = pmc_traffic(bp, L)
    if traffic is not None:
        traffic = round(traffic * bytes_per_launch / (bp * (2 * L + 8)))
    res = {
        "metric": "paired reads/sec through anchored split-read align",
        "value": round(N / elapsed * args.steps, 1),
        "unit": "pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic, made on the device (simworld.py / libafsim.so, seed 20251015): hg38-sized genome with "
                "repeat families, 5% anchor-fusion pairs, wgsim read model, every pair distinct",
        "config": {
            "workload": f"configs[{2 if world == 1 else 3}]: {N} synthetic 2x{L} bp pairs"
                        + (f" sharded over {world} GPUs" if world > 1 else "")
                        + f", bwa genome index {genome_bp / 1e9:.2f} Gbp HBM-resident, one anchor (BCR NM_004327.4); "
                          "step = S2 + S3 sort/partition + S4/S5 genome bwa mem + S5 genome check + S6 BLAT"
                        + (" per rank with the global order (dist_discover: keys all-gathered, S4 sharded by its chunk grid, "
                           "survivors and S4 records gathered to rank 0 over RCCL)" if world > 1 else ""),
            "pairs_total": N, "pairs_per_gpu": n, "read_len": L, "genome_bp": genome_bp, "anchor_len": len(anchor),
            "parallelism": f"dp{world}", "batches": n_launch, "pairs_per_batch": bp, "inflight": G,
        },
        "counts_per_step": summ,
        "phases_ms": None if world > 1 else {
            "s2": round(phase(0, 1), 3), "s3_partition": round(phase(1, 2), 3),
            "gather_queries": round(phase(2, 3), 3), "genome_bwa_s4_s5": round(phase(3, 4), 3),
            "note": "HIP events on the first slot's stream; s2 includes every batch's K1 + K2 + K3; "
                    "genome_bwa_s4_s5 = the gathers' end to the join of: S4 (bwa PE, its own context, slot 2's "
                    "stream), S5 (bwa SE, slot 0) then its genome check, and S6 BLAT of every S5 query that can "
                    "be kept (slot 1, from the gathers on; its heavy strands after the check, survivors only), "
                    "compacted to the survivors on slot 0"},
        "genome_phase": None if world > 1 else genome_phase(summ, phase(3, 4)),
        "kernels_ms": {"seed_filter_per_launch": round(k1_launch_ms, 5), "seed_filter_per_step": round(k1_ms, 4)},
        "roofline": {
            "kernel": "k_seed_filter", "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "bytes_per_launch": round(bytes_per_launch),
            "note": "HIP events on K1's stream around each group's back-to-back K1 launches (distinct read "
                    "ranges, no reuse; a group's K1s start once the previous group is done, so no other kernel shares the chip); "
                    "traffic: the committed FETCH_SIZE + WRITE_SIZE passes of this batch shape",
            "rocprof_check": rocprof_k1(bytes_per_launch, n_launch),
        },
        "setup_s": {"genome": round(t_gen, 2), "bwa_index": round(t_bwa, 2), "blat_tiles": round(t_idx - t_bwa, 2)},
        "hbm_in_use_gib": round((total - free) / 2**30, 1),
    }
    issue = issue_roofline()
    if issue:
        res["issue_roofline"] = issue
    if rank == 0 and world == 1 and not args.no_cpu:
        res["cpu_baseline"] = cpu_baseline_c3(anchor, reads_t, args, subset)
    if rank == 0:
        print(json.dumps(res), flush=True)
    disc.close()
    ref.close()
    tiles.close()


def genome_phase(summ, ms):
    """The genome phase's rates: bwa-mem genome reads (S4's both ends + S5's split reads, one
    seed / region launch) and BLAT queries (S6) over the phase's wall time, and the HBM bytes per
    genome read of its kernels from the committed FETCH_SIZE pass (profiles/r05/pmc_c3.json)."""
    q, n6 = summ.get("queries_s4_s5", 0), summ.get("s6_queries", 0)
    out = {"ms": round(ms, 3), "bwa_genome_reads": q, "blat_queries": n6,
           "bwa_genome_reads_per_s": round(q / (ms * 1e-3), 1) if ms else None,
           "blat_queries_per_s": round(n6 / (ms * 1e-3), 1) if ms else None}
    try:
        pm = json.load(open(os.path.join(ROOT, PROF, "pmc_c3.json")))["kernels"]
        per = {k: e["fetch_bytes_per_unit_x2"] for k, e in pm.items() if "fetch_bytes_per_unit_x2" in e}
        if per:
            out["fetch_bytes_per_unit_x2"] = per
            out["fetch_source"] = f"{PROF}/pmc_c3.json"
    except (OSError, ValueError, KeyError):
        pass
    return out


def genome_subset(W, flank=250_000):
    """The CPU baseline's genome: a window of each embedded gene's locus +- flank (host copies,
    taken before the bench frees the world's blob).  The step's S4/S5 queries and S6 tails come
    from these loci (anchor reads, their mates in the partner genes or the anchor's introns)."""
    spans = {}
    for name, ex in W.loci.items():
        c = ex[0][0]
        a, b = min(s for _, s, _ in ex), max(e for _, _, e in ex)
        spans.setdefault(c, []).append((max(0, a - flank), min(W.lens[W.names.index(c)], b + flank)))
    out = []
    for c, iv in spans.items():
        iv.sort()
        merged = [list(iv[0])]
        for a, b in iv[1:]:
            if a <= merged[-1][1]:
                merged[-1][1] = max(merged[-1][1], b)
            else:
                merged.append([a, b])
        off = W.offsets[W.names.index(c)]
        for a, b in merged:
            out.append((f"{c}:{a}-{b}", W.blob[off + a:off + b].cpu().numpy().tobytes()))
    return out


def _host_queries(sample, rec, res, partition):
    """S3's lists of the sample and the genome searches' queries as the reference makes them:
    S4 tmp1 / tmp2 interleaved as sequenced (AF:186-188), S5 the split-read FASTA of the anchored
    records (genome_check.split_read_fasta over their SAM lines, fn:705-715)."""
    import numpy as np

    from anchored_fusion_amd import genome_check
    from anchored_fusion_amd.cigar import revcomp
    from anchored_fusion_amd.pipeline import sam_line
    t1, t2, an = partition(res)
    npair = min(len(t1), len(t2))
    s4 = np.empty((2 * npair, sample.shape[1]), np.uint8)
    s4[0::2], s4[1::2] = sample[t1[:npair]], sample[t2[:npair]]
    lines = []
    for r in an:
        s = sample[r].tobytes().decode()
        f = int(rec["flag"][r])
        lines.append(sam_line(f"r{r // 2}", f & 0xFFFF, "ANCHOR", int(rec["pos"][r]) + 1, res.cigar_str(r),
                              revcomp(s) if f & 0x10 else s))
    return s4, genome_check.split_read_fasta(lines)


def _host_s6_queries(names, fasta, recs, nrec):
    """S5's genome check (genome_check.filter_genome_hits, fn:718-768) over the SAM text of the
    S5 records and the S6 FASTA of the survivors (blocks.split_read_queries, fn:506-528)."""
    from anchored_fusion_amd import blocks, genome, genome_check
    gsam = ["@HD\tVN:1.6\n"]
    for i, (name, sq) in enumerate(fasta):
        gsam += genome.sam_lines(names, name, sq, recs[i], nrec[i])
    return blocks.split_read_queries(genome_check.filter_genome_hits(gsam))[1]


def cpu_baseline_c3(anchor, reads_t, args, subset):
    """The CPU oracle on a bounded sample of the same pairs, over the stages of the GPU step: S2
    (oracle/bwa_pe.c, bwa-mem PE restated) + S3 (samtools order and filters) + the queries'
    gathers + S4 / S5 (the same restatement's genome calls, FM index) + S5's genome check + S6
    (oracle/blat.c, -minScore=20, 11-mer tiles, on S5's survivors), repeated for --cpu-seconds.  The genome of S4/S5/S6 is `subset`
    (genome_subset: the gene loci +- 250 kb) -- an oracle index of the whole 3.1 Gbp takes longer to
    build than the bench runs."""
    import numpy as np

    import oracle
    from anchored_fusion_amd import place
    from anchored_fusion_amd.align import AlignResult, partition
    threads = cpu_threads(args)
    n = min(args.cpu_sample, reads_t.shape[0] // 2)
    sample = reads_t[: 2 * n].cpu().numpy()
    ix = oracle.OracleIndex(anchor)
    t0 = time.perf_counter()
    og = oracle.OracleGenome(subset)
    blob, _ = place.concat_contigs([(nm, sq.decode()) for nm, sq in subset])
    tiles = oracle.OracleTiles(blob, 11)
    t_index = time.perf_counter() - t0
    po = oracle.blat_params(min_score=20)
    pe = oracle.default_pe()
    ix.align_pairs(sample[: 2 * min(n, 20000)], threads=threads)  # warm-up
    passes, dt = 0, 0.0
    st = dict(s2_s3=0.0, gather=0.0, s4=0.0, s5=0.0, s5_check=0.0, s6=0.0)
    counts = {}
    names = [nm for nm, _ in subset]
    while passes == 0 or dt < args.cpu_seconds:
        t0 = time.perf_counter()
        rec = ix.align_pairs(sample, threads=threads)
        res = AlignResult(rec["flag"], rec["pos"], rec["score"], rec["n_cigar"], rec["cigar"], rec["hits"])
        t1 = time.perf_counter()
        s4, fasta = _host_queries(sample, rec, res, partition)
        t2 = time.perf_counter()
        if len(s4):
            og.align_pe(s4, np.full(len(s4), s4.shape[1], np.int32), pe=pe, threads=threads)
        t3 = time.perf_counter()
        s6q = []
        if fasta:
            buf, ln = place.pack_queries([sq for _, sq in fasta])
            r5, n5 = og.align_se(buf, ln, threads=threads)
            t4 = time.perf_counter()
            s6q = _host_s6_queries(names, fasta, r5, n5)
        else:
            t4 = time.perf_counter()
        t5 = time.perf_counter()
        if s6q:
            buf, ln = place.pack_queries([sq for _, sq in s6q])
            tiles.blat(buf, ln, po, 16, threads=threads)
        t6 = time.perf_counter()
        for k, v in zip(st, (t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4, t6 - t5)):
            st[k] += v
        dt += t6 - t0
        passes += 1
        counts = dict(s4_pairs=len(s4) // 2, s5_split_reads=len(fasta), s6_queries=len(s6q))
    s2s3 = st["s2_s3"] + st["gather"]
    gen = st["s4"] + st["s5"] + st["s5_check"] + st["s6"]
    rate = n * passes / dt
    ncpu = os.cpu_count() or threads
    return {"value": round(rate, 1), "unit": "pairs/s", "cores": threads, "kind": "port",
            "host_cpus_visible": ncpu,
            "cores_note": f"{threads} OpenMP threads = the GPU's host CPU share (OMP_NUM_THREADS); "
                          f"host_cpus_visible = the whole machine",
            "per_core": round(rate / threads, 1),
            "all_cores_extrapolated": {
                "value": round(rate / threads * ncpu, 1), "cores": ncpu, "measured": False,
                "note": "per-core rate x host_cpus_visible (linear, an upper bound for the port): the GPU pool "
                        "shares the machine and caps a one-GPU job's host threads at its CPU share, so the "
                        "all-core run is not made"},
            "legs": {
                "s2_s3": {"pairs_per_s": round(n * passes / s2s3, 1), "s_per_pass": round(s2s3 / passes, 3),
                          "comparable": True,
                          "note": "S2 + S3 + the query gathers: the same pairs and anchor as the GPU step"},
                "genome": {"s_per_pass": round(gen / passes, 3), "comparable": False,
                           "queries_per_s": round(passes * (counts.get("s4_pairs", 0) * 2 + counts.get("s5_split_reads", 0)
                                                            + counts.get("s6_queries", 0)) / gen, 1) if gen else None,
                           "note": f"S4/S5 bwa-mem + S5 check + S6 BLAT on the gene loci +- 250 kb only "
                                   f"({sum(len(q) for _, q in subset) / 1e6:.1f} Mbp, not the GPU's 3.09 Gbp: far "
                                   f"fewer repeat occurrences per seed, so not a like-for-like rate)"}},
            "stages_s_per_pass": {k: round(v / passes, 3) for k, v in st.items()},
            "queries_per_pass": counts,
            "sample": f"first {n} pairs of the batch x {passes} passes ({dt:.1f} s): S2 + S3 + gathers + S4/S5 "
                      f"genome bwa mem + S5 genome check + S6 BLAT on the oracle (C restatements: oracle/bwa_pe.c, oracle/blat.c; "
                      f"bwa, BLAT and samtools are absent), OpenMP {threads} threads = the GPU's host CPU share "
                      f"(OMP_NUM_THREADS; host_cpus_visible is the whole machine's count); S4/S5/S6 genome = "
                      f"the {len(subset)} gene-locus windows +- 250 kb ({sum(len(q) for _, q in subset) / 1e6:.1f} Mbp, "
                      f"oracle indexes built in {t_index:.1f} s, untimed)"}


class Placement:
    """Partner placement inside the step (SURVEY §8 d: S2 + partner placement).  Each batch's K3
    (af_align_candidates_tails_device) appends the split reads' soft-clipped tails (clip >= 20)
    to a group-wide buffer; one af_blat_device launch per group searches them (the BLAT
    restatement with -minScore=20, functions.py:530) on a reference of the workload's
    transcripts (anchor, fusion partners, background; hash index) -- the bench workload has no
    genome.  A group's placement is enqueued in the next group, after its K1s and ahead of
    its first K2, so it runs beside that group's other K2s instead of idling the chip between
    groups; the last group's placement is flushed at the end of the timed steps.  Two tail
    buffers are used in turn."""

    MIN_CLIP, MAX_HITS = 20, 16

    def __init__(self, fworld, anchor, n_reads, L, G, dev):
        import torch

        from anchored_fusion_amd import blat
        ctgs = [("anchor", anchor.decode())] + [(f"partner{k}", t.decode()) for k, t in enumerate(fworld["partners"])]
        ctgs += [(f"bg{k}", t.decode()) for k, t in enumerate(fworld["background"])]
        self.ref = blat.TileReference(ctgs, 11, device=dev.index)
        self.params = blat.params("split_tail")
        self.row_bytes = blat.PSL_DTYPE.itemsize * blat.MAX_ROWS
        self.n_reads, self.L = n_reads, L
        self.cap = G * max(1024, n_reads // 100)
        z = lambda *shape, dt=torch.int32: torch.zeros(shape, dtype=dt, device=dev)  # noqa: E731
        self.buf = [dict(tails=z(self.cap, L, dt=torch.uint8), tl=z(self.cap), tr=z(self.cap), nt=z(1),
                         hits=z(self.cap * self.row_bytes, dt=torch.uint8),
                         nh=z(self.cap)) for _ in range(2)]
        self.nt_last = z(1)
        self.fill, self.to_place, self.g, self.last, self.last_g = 0, None, 0, None, 1

    def tails(self, j):
        """Batch j's tails spec: appended (in its K3) to the buffer this group fills."""
        b = self.buf[self.fill]
        self.g = max(self.g, j + 1)
        return dict(tails=b["tails"], lens=b["tl"], read=b["tr"], n=b["nt"], min_clip=self.MIN_CLIP,
                    read_base=j * self.n_reads, append=True)

    def _place(self, k, stream):
        import torch
        b = self.buf[k]
        # the TileReference's own context (queue heads, scratch): one search at a time
        self.ref.search_device(b["tails"], b["nt"], self.L, b["hits"], b["nh"], lens_t=b["tl"], p=self.params,
                               stream=stream)
        with torch.cuda.stream(stream):
            self.nt_last.copy_(b["nt"])
            b["nt"].zero_()
        self.last = b

    def before(self, j, aligner, stream):
        """Ahead of the first K2 of a group: the previous group's placement."""
        if j == 0 and self.to_place is not None:
            self._place(self.to_place[0], stream)
            self.last_g = self.to_place[1]
            self.to_place = None

    def end_group(self):
        self.to_place = (self.fill, self.g)
        self.fill ^= 1
        self.g = 0

    def flush(self, stream):
        """The last group's placement (stream must follow every batch of that group)."""
        if self.to_place is not None:
            self._place(self.to_place[0], stream)
            self.last_g = self.to_place[1]
            self.to_place = None

    def report(self):
        n_t = int(self.nt_last.item())
        placed = int((self.last["nh"][:min(n_t, self.cap)] > 0).sum().item())
        self.ref.close()
        return {"split_tails_per_batch": round(n_t / self.last_g, 1), "placed_fraction": round(placed / max(n_t, 1), 4),
                "min_clip": self.MIN_CLIP,
                "reference": "the workload's transcripts (anchor, 8 partners, 400 background), hash index",
                "params": "BLAT restatement, -minScore=20 (functions.py:530), 11-mer tiles, one launch per group"}


def _split_tails(reads, rec, min_clip):
    """Host form of the split-read tail rule (af_emit_tail): mapped, CIGAR exactly S+M / M+S,
    clip >= min_clip; the clipped part of SEQ (reverse-complemented read for 0x10)."""
    import numpy as np
    comp = bytes.maketrans(b"ACGTNacgtn", b"TGCANTGCAN")
    rows = np.nonzero(((rec["flag"] & 4) == 0) & (rec["n_cigar"] == 2))[0]
    out = []
    for r in rows:
        c0, c1 = int(rec["cigar"][r, 0]), int(rec["cigar"][r, 1])
        if (c0 & 15, c1 & 15) == (4, 0):
            clip, head = c0 >> 4, True
        elif (c0 & 15, c1 & 15) == (0, 4):
            clip, head = c1 >> 4, False
        else:
            continue
        n = reads.shape[1]
        if clip < min_clip or clip > n:
            continue
        seq = reads[r].tobytes()
        if rec["flag"][r] & 0x10:
            seq = seq[::-1].translate(comp)
        out.append(seq[:clip] if head else seq[n - clip:])
    return out


def cpu_baseline(anchor, reads, args, fworld=None):
    """The CPU oracle (a port of the same algorithm; bwa and BLAT themselves are absent) timed on
    a bounded sample of this rank's batch: the first --cpu-sample pairs, repeated until
    --cpu-seconds.  With fworld, each pass also cuts the split-read tails and searches them
    (afo_blat, -minScore=20) on the same transcripts reference as the GPU step."""
    import numpy as np

    import oracle
    from anchored_fusion_amd import place
    threads = cpu_threads(args)
    n = min(args.cpu_sample, reads.shape[0] // 2)
    sample = reads[: 2 * n]
    ix = oracle.OracleIndex(anchor)
    ref_ix = po = None
    if fworld is not None:
        ctgs = [("anchor", anchor.decode())] + [(f"p{k}", t.decode()) for k, t in enumerate(fworld["partners"])]
        ctgs += [(f"bg{k}", t.decode()) for k, t in enumerate(fworld["background"])]
        ref_ix = oracle.OracleTiles(place.concat_contigs(ctgs)[0], 11)
        po = oracle.blat_params(min_score=20)
    ix.align_pairs(sample, threads=threads)  # untimed warm-up pass (thread pool, first-touch pages)
    passes, dt, n_tails = 0, 0.0, 0
    while passes == 0 or dt < args.cpu_seconds:
        t0 = time.perf_counter()
        rec = ix.align_pairs(sample, threads=threads)
        if ref_ix is not None:
            tails = _split_tails(sample, rec, Placement.MIN_CLIP)
            n_tails = len(tails)
            if tails:
                buf, ln = place.pack_queries(tails)
                ref_ix.blat(buf, ln, po, 16, threads=threads)
        dt += time.perf_counter() - t0
        passes += 1
    what = "S2 + tail placement" if ref_ix is not None else "S2"
    return {"value": round(n * passes / dt, 1), "unit": "pairs/s", "cores": threads, "kind": "port",
            "sample": f"first {n} pairs of rank 0's batch x {passes} passes ({dt:.1f} s), {what}"
                      + (f" ({n_tails} tails per pass)" if ref_ix is not None else "")
                      + f", oracle/af_oracle.c (C restatement of bwa-mem's algorithm; bwa and BLAT are absent), "
                        f"OpenMP {threads} threads"}


if __name__ == "__main__":
    main()
