"""BASELINE.json configs[2] (C3) on one GPU: 50 M synthetic 2x150 bp pairs resident in HBM, aligned
by the S2 path (K1 + K2 + K3) in one step, with a 3.1 Gbp genome index (af_index_build_genome)
resident beside them.

The simulator makes `--unique` distinct pairs (8 s per million on the host); the batch is those
pairs tiled to `--pairs` on the device, so per-pair work has the same distribution as a fully
simulated batch.  Prints one JSON line like bench.py (not the driver's bench: that is C2).

usage: python3 scripts/c3_bench.py [--pairs 50e6] [--unique 1e6] [--read-len 150] [--genome 3.1e9]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import afpkg  # noqa: E402,F401
import numpy as np  # noqa: E402
import torch  # noqa: E402

from anchored_fusion_amd import io as afio  # noqa: E402
from anchored_fusion_amd import place  # noqa: E402
from anchored_fusion_amd import simulate as sim  # noqa: E402
from anchored_fusion_amd.align import AnchorAligner  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--pairs", type=float, default=50e6)
ap.add_argument("--unique", type=float, default=1e6)
ap.add_argument("--read-len", type=int, default=150)
ap.add_argument("--genome", type=float, default=3.1e9)
ap.add_argument("--steps", type=int, default=3)
args = ap.parse_args()
N, U, L = int(args.pairs), int(args.unique), args.read_len
dev = torch.device("cuda:0")
anchor = afio.anchor_sequence(os.path.join(ROOT, "tests", "golden", "target_gene.fasta"))
t0 = time.perf_counter()
_, uniq, _, world = sim.fusion_reads(anchor, U, read_len=L, fusion_frac=0.05, seed=20251015)
print(f"simulated {U} pairs in {time.perf_counter() - t0:.0f} s", flush=True)
genome_ref = None
if args.genome > 0:
    rng = np.random.default_rng(7)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    ctgs = [(f"chr{k + 1}", acgt[rng.integers(0, 4, int(args.genome) // 24, dtype=np.uint8)].tobytes().decode())
            for k in range(24)]
    # the fusion partners (and the anchor) live in the genome: partner k at chr(k+2):PLACE0
    PLACE0 = 1_000_000
    loci = {}
    for k, seq in enumerate([anchor] + world["partners"]):
        name, c = ctgs[k + 1]
        ctgs[k + 1] = (name, c[:PLACE0] + seq.decode() + c[PLACE0 + len(seq):])
        loci[name] = (PLACE0, PLACE0 + len(seq))
    t0 = time.perf_counter()
    genome_ref = place.Reference(ctgs)
    del ctgs
    print(f"genome index ({genome_ref.kind}, {genome_ref.total / 1e9:.2f} Gbp) built in "
          f"{time.perf_counter() - t0:.1f} s", flush=True)
u_t = torch.from_numpy(uniq).to(dev)
reads_t = torch.empty((2 * N, L), dtype=torch.uint8, device=dev)
for o in range(0, 2 * N, 2 * U):
    k = min(2 * U, 2 * N - o)
    reads_t[o:o + k] = u_t[:k]
del u_t
out = {k: torch.zeros(2 * N, dtype=torch.int32, device=dev) for k in ("flag", "pos", "score", "n_cigar", "hits")}
out["cigar"] = torch.zeros((2 * N, 32), dtype=torch.int32, device=dev)
al = AnchorAligner(anchor, device=0)
s = torch.cuda.current_stream(dev)
free, total = torch.cuda.mem_get_info(dev)
print(f"HBM in use {(total - free) / 2**30:.1f} GiB of {total / 2**30:.0f} GiB", flush=True)


def step(ev=None):
    if ev:
        ev[0].record(s)
    al.seed_filter_device(reads_t, 2 * N, L, out["hits"], stream=s)
    if ev:
        ev[1].record(s)
    al.align_candidates_device(reads_t, N, L, out, stream=s)
    if ev:
        ev[2].record(s)


step()
torch.cuda.synchronize()
evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
t0 = time.perf_counter()
for k in range(args.steps):
    step(evs[k])
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / args.steps
k1 = sum(e[0].elapsed_time(e[1]) for e in evs) / args.steps
mapped = int(((out["flag"] & 4) == 0).sum().item())
bpp = 2 * L + 8
print(json.dumps({
    "metric": "paired reads/sec through anchored split-read align", "value": round(N / dt, 1), "unit": "pairs/s",
    "n_gpus": 1, "steps": args.steps, "ms_per_step": round(dt * 1e3, 3), "dtype": "int32",
    "data": f"synthetic: {U} simulated 2x{L} pairs tiled to {N}",
    "config": {"workload": f"configs[2]: {N} x 2x{L} pairs, genome index {args.genome / 1e9:.1f} Gbp resident",
               "candidates_per_step": al.last_candidates(), "mapped_reads_per_step": mapped},
    "kernels_ms": {"seed_filter": round(k1, 4)},
    "roofline": {"kernel": "k_seed_filter", "bound": "hbm", "achieved": round(bpp * N / (k1 * 1e-3) / 1e9, 1),
                 "peak": 8000.0, "unit": "GB/s", "frac": round(bpp * N / (k1 * 1e-3) / 8e12, 4),
                 "bytes_per_launch": bpp * N}}), flush=True)
if genome_ref is not None:
    # partner placement (S6-S8's genome search) of the split reads' soft-clipped tails with
    # af_place on the resident genome index: the tails of the U distinct pairs (checked against
    # the embedded loci), then those tails tiled N/U times = the whole batch's tails, one call
    from anchored_fusion_amd.align import AlignResult
    h = {k: v[:2 * U].cpu().numpy() for k, v in out.items()}
    h["cigar"] = h["cigar"].view(np.uint32)
    res = AlignResult(**h)
    tails = []
    for r in np.nonzero(res.mapped())[0]:
        ops = res.cigar_ops(r)
        if len(ops) != 2 or "S" not in (ops[0][1], ops[1][1]):
            continue
        seq = uniq[r].tobytes()
        if res.flag[r] & 0x10:
            seq = seq[::-1].translate(bytes.maketrans(b"ACGTN", b"TGCAN"))
        n_clip = ops[0][0] if ops[0][1] == "S" else ops[1][0]
        if n_clip < 20:
            continue
        tails.append(seq[:n_clip] if ops[0][1] == "S" else seq[-n_clip:])
    genome_ref.raw_hits(tails[:1000])
    t0 = time.perf_counter()
    hits, nh = genome_ref.raw_hits(tails)
    t_place = time.perf_counter() - t0
    # the tails of the whole N-pair batch (the U-pair tails tiled N/U times) in one call
    t0 = time.perf_counter()
    genome_ref.raw_hits(tails * (N // U))
    t_place_n = time.perf_counter() - t0
    on_partner = 0
    for q in range(len(tails)):
        if nh[q] > 0:
            loc = genome_ref.locate(hits[q, 0]["t_start"], hits[q, 0]["t_end"])
            if loc is not None:
                name = genome_ref.names[loc[0]]
                if name in loci and loci[name][0] <= loc[1] < loci[name][1]:
                    on_partner += 1
    print(json.dumps({
        "placement": {"split_tails": len(tails), "of_pairs": U, "seconds": round(t_place, 4),
                      "tails_per_s": round(len(tails) / t_place, 1),
                      "best_hit_on_embedded_partner_or_anchor": on_partner,
                      "note": "af_place host API (H2D queries, D2H hits) on the 3.1 Gbp genome index; soft clip >= 20"},
        "s2_plus_placement": {"value": round(N / (dt + t_place_n), 1), "unit": "pairs/s",
                              "note": f"N / (S2 step + one af_place call on the {len(tails) * (N // U)} tails "
                                      f"of the N pairs = {t_place_n:.4f} s)"}}),
          flush=True)
    genome_ref.close()
al.close()
