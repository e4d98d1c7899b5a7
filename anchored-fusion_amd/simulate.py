"""Seeded synthetic inputs: a wgsim-style paired-read simulator and fusion worlds.

The reference simulates its benchmark reads with ``wgsim -d 200 -1 101 -2 101 -N n`` from
fusion transcripts (utils/simulate_reads.py:4-20); wgsim is not in this image and there is
no network, so this module restates wgsim's read model with numpy:

* a fragment of length ~ N(frag_mean, frag_sd) is drawn uniformly from a transcript chosen
  with probability proportional to weight x length;
* mate 1 is the first ``read_len`` bases of the fragment, mate 2 the reverse complement of
  its last ``read_len`` bases; with probability 1/2 the pair is flipped (mate 1 from the
  reverse strand), as wgsim does;
* sequencing errors are substitutions at rate ``err`` (wgsim -e, default 0.02); a small
  fraction of reads carries a 1-3 nt insertion or deletion and a few bases are ``N``.

Read names follow wgsim's ``<contig>_<start>_<end>_<e1>:0:<i1>_<e2>:0:<i2>_<idx>`` layout so
that tests can recover the truth exactly as the bundled test FASTQ allows.
"""
import numpy as np

_COMP = bytes.maketrans(b"ACGTNacgtn", b"TGCANtgcan")
_BASES = np.frombuffer(b"ACGT", dtype=np.uint8)


def revcomp(s: bytes) -> bytes:
    return s.translate(_COMP)[::-1]


def random_seq(rng, n, gc=0.5) -> bytes:
    p = np.array([(1 - gc) / 2, gc / 2, gc / 2, (1 - gc) / 2])
    return _BASES[rng.choice(4, size=n, p=p)].tobytes()


_RC_LUT = np.zeros(256, dtype=np.uint8)
for _a, _b in zip(b"ACGTNacgtn", b"TGCANtgcan"):
    _RC_LUT[_a] = _b


def simulate_pairs(transcripts, n_pairs, read_len=100, frag_mean=200, frag_sd=20, err=0.02, indel_frac=0.01,
                   n_rate=0.0005, weights=None, names=None, seed=20251015, with_names=True):
    """Returns (qnames or None, reads uint8 [2*n_pairs, read_len] pair-major, truth dict)."""
    rng = np.random.default_rng(seed)
    T = np.frombuffer(b"".join(transcripts), dtype=np.uint8)
    lens = np.array([len(t) for t in transcripts], dtype=np.int64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]])
    if (lens < read_len + 8).any():
        raise ValueError("every transcript must be longer than read_len + 8")
    w = np.ones(len(transcripts)) if weights is None else np.asarray(weights, dtype=np.float64)
    pr = w * lens
    pr = pr / pr.sum()
    tid = rng.choice(len(transcripts), size=n_pairs, p=pr)
    frag = np.rint(rng.normal(frag_mean, frag_sd, size=n_pairs)).astype(np.int64)
    frag = np.clip(frag, read_len, lens[tid])
    start = (rng.random(n_pairs) * (lens[tid] - frag + 1)).astype(np.int64)
    ar = np.arange(read_len, dtype=np.int64)
    g1 = offs[tid][:, None] + start[:, None] + ar[None, :]
    g2 = offs[tid][:, None] + (start + frag - read_len)[:, None] + ar[None, :]
    r1 = T[g1]
    r2 = _RC_LUT[T[g2][:, ::-1]]
    flip = rng.random(n_pairs) < 0.5
    m1 = np.where(flip[:, None], r2, r1)
    m2 = np.where(flip[:, None], r1, r2)
    reads = np.empty((2 * n_pairs, read_len), dtype=np.uint8)
    reads[0::2] = m1
    reads[1::2] = m2
    # substitutions
    sub = rng.random(reads.shape) < err
    shift = rng.integers(1, 4, size=int(sub.sum()), dtype=np.uint8)
    code = np.searchsorted(_BASES, reads[sub])
    code = np.clip(code, 0, 3)
    reads[sub] = _BASES[(code + shift) % 4]
    nerr = sub.sum(axis=1)
    # small indels on a fraction of reads (python loop over the few affected reads)
    nind = np.zeros(2 * n_pairs, dtype=np.int64)
    if indel_frac > 0:
        hit = np.nonzero(rng.random(2 * n_pairs) < indel_frac)[0]
        for r in hit:
            L = read_len
            s = bytearray(reads[r].tobytes())
            k = int(rng.integers(1, 4))
            p = int(rng.integers(10, L - 10))
            if rng.random() < 0.5:  # insertion
                s = s[:p] + bytearray(random_seq(rng, k)) + s[p:]
                s = s[:L]
            else:  # deletion: drop k bases, refill the tail with random bases
                s = s[:p] + s[p + k:] + bytearray(random_seq(rng, k))
            reads[r] = np.frombuffer(bytes(s), dtype=np.uint8)
            nind[r] = 1
    if n_rate > 0:
        nmask = rng.random(reads.shape) < n_rate
        reads[nmask] = ord("N")
    qn = None
    if with_names:
        tn = names or [f"t{i}" for i in range(len(transcripts))]
        qn = [f"{tn[t]}_{s + 1}_{s + f}_{nerr[2 * i]}:0:{nind[2 * i]}_{nerr[2 * i + 1]}:0:{nind[2 * i + 1]}_{i:x}"
              for i, (t, s, f) in enumerate(zip(tid.tolist(), start.tolist(), frag.tolist()))]
    truth = dict(tid=tid, start=start, frag=frag, flip=flip)
    return qn, reads, truth


def fusion_world(anchor: bytes, n_partners=8, n_background=400, bg_len=(800, 3000), seed=20251015):
    """One anchor transcript fused to random partners, plus a random background transcriptome.

    Returns dict(fusions=[bytes], fusion_bp=[(anchor_bp, partner_bp)], background=[bytes]).
    Each fusion joins anchor[:a] with partner[b:] at a random junction."""
    rng = np.random.default_rng(seed)
    n = len(anchor)
    fusions, bps, partners = [], [], []
    for _ in range(n_partners):
        partner = random_seq(rng, int(rng.integers(1500, 4000)))
        a = int(rng.integers(n // 4, 3 * n // 4))
        b = int(rng.integers(200, len(partner) - 800))
        fusions.append(anchor[:a] + partner[b:])
        bps.append((a, b))
        partners.append(partner)
    bg = [random_seq(rng, int(rng.integers(*bg_len))) for _ in range(n_background)]
    return dict(fusions=fusions, fusion_bp=bps, partners=partners, background=bg)


def fusion_reads(anchor: bytes, n_pairs, read_len=100, fusion_frac=0.05, seed=20251015, with_names=False, **kw):
    """Config-2 style input: ``fusion_frac`` of pairs from anchor fusions, rest background."""
    wd = fusion_world(anchor, seed=seed)
    tr = wd["fusions"] + wd["background"]
    nf, nb = len(wd["fusions"]), len(wd["background"])
    lf = sum(len(t) for t in wd["fusions"])
    lb = sum(len(t) for t in wd["background"])
    # per-transcript weights so that the fusion share of pairs is fusion_frac
    w = np.array([fusion_frac / lf] * nf + [(1 - fusion_frac) / lb] * nb)
    names = [f"fusion{i}" for i in range(nf)] + [f"bg{i}" for i in range(nb)]
    qn, reads, truth = simulate_pairs(tr, n_pairs, read_len=read_len, weights=w, names=names, seed=seed + 1,
                                      with_names=with_names, **kw)
    return qn, reads, truth, wd
