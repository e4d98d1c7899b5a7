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
# partner placement buffers: tails of split reads (S6's queries) placed on the genome index
MIN_CLIP, MAX_HITS = 20, 16
CAP = max(1024, 2 * N // 200)
if genome_ref is not None:
    tails_t = torch.zeros((CAP, L), dtype=torch.uint8, device=dev)
    tl_t = torch.zeros(CAP, dtype=torch.int32, device=dev)
    tr_t = torch.zeros(CAP, dtype=torch.int32, device=dev)
    nt_t = torch.zeros(1, dtype=torch.int32, device=dev)
    hits_t = torch.zeros(CAP * MAX_HITS * place.HIT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    nh_t = torch.zeros(CAP, dtype=torch.int32, device=dev)
    pp = place.preset_params("split_tail")  # BLAT -minScore=20 (functions.py:530)
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
    if genome_ref is not None:
        al.split_tails_device(reads_t, L, out, tails_t, tl_t, tr_t, nt_t, min_clip=MIN_CLIP, stream=s)
        genome_ref.place_device(tails_t, nt_t, L, hits_t, nh_t, lens_t=tl_t, params=pp, max_hits=MAX_HITS, stream=s)
    if ev:
        ev[3].record(s)


step()
torch.cuda.synchronize()
evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(args.steps)]
t0 = time.perf_counter()
for k in range(args.steps):
    step(evs[k])
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / args.steps
k1 = sum(e[0].elapsed_time(e[1]) for e in evs) / args.steps
k23 = sum(e[1].elapsed_time(e[2]) for e in evs) / args.steps
kpl = sum(e[2].elapsed_time(e[3]) for e in evs) / args.steps
mapped = int(((out["flag"] & 4) == 0).sum().item())
bpp = 2 * L + 8
res = {
    "metric": "paired reads/sec through anchored split-read align", "value": round(N / dt, 1), "unit": "pairs/s",
    "n_gpus": 1, "steps": args.steps, "ms_per_step": round(dt * 1e3, 3), "dtype": "int32",
    "data": f"synthetic: {U} simulated 2x{L} pairs tiled to {N}",
    "config": {"workload": f"configs[2]: {N} x 2x{L} pairs, genome index {args.genome / 1e9:.1f} Gbp resident"
                           + (", S2 + partner placement of the split-read tails" if genome_ref is not None else ""),
               "candidates_per_step": al.last_candidates(), "mapped_reads_per_step": mapped},
    "kernels_ms": {"seed_filter": round(k1, 4), "align_candidates_and_pairs": round(k23, 4),
                   "split_tails_and_place": round(kpl, 4)},
    "roofline": {"kernel": "k_seed_filter", "bound": "hbm", "achieved": round(bpp * N / (k1 * 1e-3) / 1e9, 1),
                 "peak": 8000.0, "unit": "GB/s", "frac": round(bpp * N / (k1 * 1e-3) / 8e12, 4),
                 "bytes_per_launch": bpp * N}}
if genome_ref is not None:
    n_t = int(nt_t.item())
    n_q = min(n_t, CAP)
    nh = nh_t[:n_q].cpu().numpy()
    best = hits_t.view(-1)[:n_q * MAX_HITS * place.HIT_DTYPE.itemsize].cpu().numpy().view(place.HIT_DTYPE)
    best = best.reshape(n_q, MAX_HITS)[:, 0]
    on = 0
    for q in np.nonzero(nh > 0)[0]:
        loc = genome_ref.locate(best[q]["t_start"], best[q]["t_end"])
        if loc is not None:
            name = genome_ref.names[loc[0]]
            on += name in loci and loci[name][0] <= loc[1] < loci[name][1]
    res["placement"] = {"split_tails_per_step": n_t, "placed": int((nh > 0).sum()),
                        "best_hit_in_embedded_partner_or_anchor": int(on), "min_clip": MIN_CLIP,
                        "params": "T=20 (BLAT -minScore=20, functions.py:530), up to 16 hits per tail"}
print(json.dumps(res), flush=True)
if genome_ref is not None:
    genome_ref.close()
al.close()
