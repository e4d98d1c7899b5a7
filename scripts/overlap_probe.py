"""Two batches in flight: the bench step (K1 -> K2+K3) on one stream vs consecutive batches
alternating over two contexts and two streams, so the next batch's K1 and K2 waves fill the
CUs the current K2's tail leaves idle.  Prints ms per batch for both and checks the records
of the overlapped run equal the serial run's.

usage: python3 scripts/overlap_probe.py [steps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import afpkg  # noqa: E402,F401
import torch  # noqa: E402

from anchored_fusion_amd import io as afio  # noqa: E402
from anchored_fusion_amd import simulate as sim  # noqa: E402
from anchored_fusion_amd.align import AnchorAligner  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
n, L = 1_000_000, 100
anchor = afio.anchor_sequence(os.path.join(ROOT, "tests", "golden", "target_gene.fasta"))
_, reads, _, _ = sim.fusion_reads(anchor, n, read_len=L, fusion_frac=0.05, seed=20251015)
dev = torch.device("cuda", 0)
reads_t = torch.from_numpy(reads).to(dev)
nr = reads.shape[0]


def outs():
    o = {k: torch.zeros(nr, dtype=torch.int32, device=dev) for k in ("flag", "pos", "score", "n_cigar", "hits")}
    o["cigar"] = torch.zeros((nr, 32), dtype=torch.int32, device=dev)
    return o


G = 4
als = [AnchorAligner(anchor, device=0) for _ in range(G)]
streams = [torch.cuda.Stream(dev) for _ in range(G)]
bufs = [outs() for _ in range(G)]


def group(g):
    """g batches: their K1 launches back to back (each after the previous one, on its own
    stream), then their K2+K3 on g streams at once, so each K2's tail overlaps the next K2's
    start; the next group's K1s wait for all of this group's K2s."""
    done = []
    prev = None
    for j in range(g):
        s = streams[j]
        if prev is not None:
            s.wait_event(prev)
        als[j].seed_filter_device(reads_t, nr, L, bufs[j]["hits"], stream=s)
        prev = torch.cuda.Event()
        prev.record(s)
    for j in range(g):
        s = streams[j]
        s.wait_event(prev)  # every K1 of the group done: K2s start together
        als[j].align_candidates_device(reads_t, n, L, bufs[j], stream=s)
        e = torch.cuda.Event()
        e.record(s)
        done.append(e)
    for j in range(g):
        for e in done:
            streams[j].wait_event(e)


for g in (1, 2, 4, 1, 2, 4):
    for k in range(2):
        group(g)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    reps = max(1, steps // g)
    for k in range(reps):
        group(g)
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    nb = reps * g
    print(f"group of {g}: {dt / nb * 1e3:.4f} ms per batch = {n * nb / dt / 1e9:.3f} G pairs/s", flush=True)
same = all(torch.equal(bufs[0][k], b[k]) for b in bufs[1:] for k in bufs[0])
print("records equal across contexts:", same)
