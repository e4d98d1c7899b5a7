"""Split-read tails on the device (af_split_tails_device, and fused into K3 by
af_align_candidates_tails_device), the queries of the S6 BLAT: the tails equal a host
restatement of the split-read rule over the same records (deal_cigar's two-operation M/S case,
functions.py:713; SAM-orientation clipped part, fn:1001-1005).  Integer work: bit-exact."""
import numpy as np
import pytest

from cases import ragged, synthetic_pairs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def aligner(anchor):
    from anchored_fusion_amd.align import AnchorAligner
    a = AnchorAligner(anchor, device=0)
    yield a
    a.close()


_COMP = bytes.maketrans(b"ACGTNacgtn", b"TGCANTGCAN")


def host_tails(reads, lens, res, min_clip):
    """{read row: tail bytes} from host records (AlignResult)."""
    out = {}
    for r in np.nonzero(res.mapped())[0]:
        ops = res.cigar_ops(r)
        if len(ops) != 2 or sorted(op for _, op in ops) != ["M", "S"]:
            continue
        n = int(lens[r]) if lens is not None else reads.shape[1]
        clip = ops[0][0] if ops[0][1] == "S" else ops[1][0]
        if clip < min_clip or clip > n:
            continue
        seq = reads[r, :n].tobytes()
        if res.flag[r] & 0x10:
            seq = seq[::-1].translate(_COMP)
        out[int(r)] = seq[:clip] if ops[0][1] == "S" else seq[n - clip:]
    return out


def _device_records(aligner, reads, lens, dev):
    import torch
    nr = reads.shape[0]
    rt = torch.from_numpy(reads).to(dev)
    lt = None if lens is None else torch.from_numpy(lens).to(dev)
    out = {k: torch.zeros(nr, dtype=torch.int32, device=dev) for k in ("flag", "pos", "score", "n_cigar", "hits")}
    out["cigar"] = torch.zeros((nr, 32), dtype=torch.int32, device=dev)
    aligner.align_pairs_device(rt, nr // 2, reads.shape[1], out, lens_t=lt)
    return rt, lt, out


def _tails(aligner, rt, lt, out, stride, cap, min_clip, dev):
    import torch
    tails = torch.zeros((cap, stride), dtype=torch.uint8, device=dev)
    tl = torch.zeros(cap, dtype=torch.int32, device=dev)
    tr = torch.zeros(cap, dtype=torch.int32, device=dev)
    nt = torch.zeros(1, dtype=torch.int32, device=dev)
    aligner.split_tails_device(rt, stride, out, tails, tl, tr, nt, min_clip=min_clip, lens_t=lt)
    return tails, tl, tr, nt


@pytest.mark.parametrize("ragged_lens", [False, True])
def test_split_tails_match_host_rule(aligner, anchor, ragged_lens):
    import torch
    dev = torch.device("cuda:0")
    reads, _, _ = synthetic_pairs(anchor, 4000, 100, seed=51)
    lens = None
    if ragged_lens:
        reads, lens = ragged(reads, seed=52)
    res = aligner.align_pairs(reads, lens)
    want = host_tails(reads, lens, res, 20)
    assert len(want) > (5 if ragged_lens else 50)  # the fusion-rich synthetic set has split reads
    rt, lt, out = _device_records(aligner, reads, lens, dev)
    tails, tl, tr, nt = _tails(aligner, rt, lt, out, reads.shape[1], 2 * len(want), 20, dev)
    torch.cuda.synchronize()
    n = int(nt.item())
    assert n == len(want)
    t, ln, rd = tails.cpu().numpy(), tl.cpu().numpy(), tr.cpu().numpy()
    got = {int(rd[i]): t[i, :ln[i]].tobytes() for i in range(n)}
    assert got == want


def test_split_tails_capacity(aligner, anchor):
    """cap below the number of split reads: the count is still exact, only cap rows written."""
    import torch
    dev = torch.device("cuda:0")
    reads, _, _ = synthetic_pairs(anchor, 2000, 100, seed=53)
    res = aligner.align_pairs(reads)
    want = host_tails(reads, None, res, 20)
    rt, lt, out = _device_records(aligner, reads, None, dev)
    cap = max(1, len(want) // 3)
    tails, tl, tr, nt = _tails(aligner, rt, lt, out, reads.shape[1], cap, 20, dev)
    torch.cuda.synchronize()
    assert int(nt.item()) == len(want)
    t, ln, rd = tails.cpu().numpy(), tl.cpu().numpy(), tr.cpu().numpy()
    for i in range(cap):
        assert t[i, :ln[i]].tobytes() == want[int(rd[i])]


def test_fused_tails_and_append(aligner, anchor):
    """af_align_candidates_tails_device (tails cut in K3) gives the same tails as the host rule;
    two batches appended into one buffer keep their read_base offsets."""
    import torch
    dev = torch.device("cuda:0")
    batches = [synthetic_pairs(anchor, 3000, 100, seed=56 + k)[0] for k in range(2)]
    want = {}
    for k, reads in enumerate(batches):
        for r, t in host_tails(reads, None, aligner.align_pairs(reads), 20).items():
            want[k * 100_000 + r] = t
    cap = 2 * len(want) + 16
    tb = dict(tails=torch.zeros((cap, 100), dtype=torch.uint8, device=dev),
              lens=torch.zeros(cap, dtype=torch.int32, device=dev), read=torch.zeros(cap, dtype=torch.int32, device=dev),
              n=torch.full((1,), 12345, dtype=torch.int32, device=dev), min_clip=20)
    for k, reads in enumerate(batches):
        nr = reads.shape[0]
        rt = torch.from_numpy(reads).to(dev)
        out = {f: torch.zeros(nr, dtype=torch.int32, device=dev) for f in ("flag", "pos", "score", "n_cigar", "hits")}
        out["cigar"] = torch.zeros((nr, 32), dtype=torch.int32, device=dev)
        aligner.seed_filter_device(rt, nr, 100, out["hits"])
        aligner.align_candidates_tails_device(rt, nr // 2, 100, out, dict(tb, read_base=k * 100_000, append=k > 0))
        torch.cuda.synchronize()
    n = int(tb["n"].item())
    assert n == len(want)
    t, ln, rd = tb["tails"].cpu().numpy(), tb["lens"].cpu().numpy(), tb["read"].cpu().numpy()
    assert {int(rd[i]): t[i, :ln[i]].tobytes() for i in range(n)} == want
