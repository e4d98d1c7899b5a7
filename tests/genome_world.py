"""A small repeat-rich multi-contig genome and reads from it (TEST INFRASTRUCTURE ONLY).

The genome calls S4/S5 (`bwa mem -M genome ...`, Anchored_Fusion.py:188, functions.py:716) are
decided by repeats: bwa samples at most max_occ = 500 occurrences of an interval in suffix-array
order, and the chain filter and dedup act on the copies that survive.  This world has what
makes those paths matter, at a size the CPU oracle indexes in seconds:

- contigs joined as bwa joins them (no separators), N runs at the contig ends and one inside;
- an Alu-like family (300 nt, both strands): old copies 2-15 % diverged and a young subfamily
  of > 500 copies within 1 %, so that intervals exceed max_occ; an L1-like family of 5' truncated copies; a satellite array
  (171-nt monomer); simple tandem repeats;
- a segmental duplication (1 % diverged) and an exact 3 kb duplication (deep suffix sorting).

`sample_reads` draws single reads (some chimeric: two loci joined, as split reads are) and
`sample_pairs` paired reads (wgsim-like, some discordant) with substitutions and small indels.
"""
import numpy as np

_B = np.frombuffer(b"ACGT", dtype=np.uint8)
_RC = np.zeros(256, dtype=np.uint8)
for _a, _b in zip(b"ACGTN", b"TGCAN"):
    _RC[_a] = _b


def _rand(rng, n, gc=0.41):
    p = np.array([(1 - gc) / 2, gc / 2, gc / 2, (1 - gc) / 2])
    return _B[rng.choice(4, size=n, p=p)]


def _mutate(rng, s, d):
    s = s.copy()
    m = rng.random(len(s)) < d
    s[m] = _B[(np.searchsorted(_B, s[m]) + rng.integers(1, 4, m.sum())) & 3]
    return s


def _rc(s):
    return _RC[s[::-1]]


def make_genome(seed=7, n_ctg=3, ctg_len=(300_000, 220_000, 160_000), alu_copies=420, young_copies=660,
                l1_copies=40):
    rng = np.random.default_rng(seed)
    alu = _rand(rng, 300, 0.55)
    alu_sub = [_mutate(rng, alu, 0.04) for _ in range(3)]
    l1 = _rand(rng, 2400, 0.38)
    sat = _rand(rng, 171, 0.38)
    contigs = []
    for k in range(n_ctg):
        L = ctg_len[k % len(ctg_len)]
        g = _rand(rng, L)
        # interspersed copies
        n_alu = alu_copies // n_ctg
        for j in range(n_alu + young_copies // n_ctg):
            young = j >= n_alu  # a young subfamily: > max_occ copies share most 19-mers
            src = alu if young else alu_sub[rng.integers(0, 3)]
            cp = _mutate(rng, src, rng.uniform(0.002, 0.012) if young else rng.uniform(0.02, 0.15))
            if rng.random() < 0.5:
                cp = _rc(cp)
            at = int(rng.integers(1000, L - 1000))
            g[at:at + len(cp)] = cp
        for _ in range(l1_copies // n_ctg):
            ln = int(rng.integers(300, len(l1)))
            cp = _mutate(rng, l1[len(l1) - ln:], rng.uniform(0.05, 0.2))
            if rng.random() < 0.5:
                cp = _rc(cp)
            at = int(rng.integers(1000, L - 3000))
            g[at:at + len(cp)] = cp
        # satellite array
        at = L // 3
        for m in range(60):
            g[at + m * 171: at + (m + 1) * 171] = _mutate(rng, sat, rng.uniform(0.02, 0.1))
        # simple tandem repeats
        for _ in range(6):
            unit = _rand(rng, int(rng.integers(1, 7)))
            rep = np.tile(unit, 200 // len(unit) + 1)[:int(rng.integers(40, 200))]
            at = int(rng.integers(1000, L - 1000))
            g[at:at + len(rep)] = _mutate(rng, rep, 0.03)
        # N runs: the ends and one gap
        g[:int(rng.integers(0, 400))] = ord("N")
        g[L - int(rng.integers(0, 400)):] = ord("N")
        mid = int(L * 0.6)
        g[mid:mid + 500] = ord("N")
        contigs.append([f"chr{k + 1}", g])
    # a segmental duplication (1 % diverged) and an exact 3 kb duplication across contigs
    a, b = contigs[0][1], contigs[1 % n_ctg][1]
    b[50_000:60_000] = _mutate(rng, a[120_000:130_000], 0.01)
    b[80_000:83_000] = a[200_000:203_000]
    return [(n, bytes(g)) for n, g in contigs]


def _sample_frag(rng, contigs, length):
    for _ in range(100):
        k = int(rng.integers(0, len(contigs)))
        s = contigs[k][1]
        if len(s) <= length + 2:
            continue
        p = int(rng.integers(0, len(s) - length))
        f = s[p:p + length]
        if b"N" not in f:
            return np.frombuffer(f, dtype=np.uint8).copy()
    raise RuntimeError("no N-free fragment")


def _noisy(rng, s, err=0.02, indel=0.1):
    s = _mutate(rng, s, err)
    if rng.random() < indel:
        i = int(rng.integers(10, len(s) - 10))
        if rng.random() < 0.5:
            s = np.concatenate([s[:i], _rand(rng, int(rng.integers(1, 4))), s[i:]])
        else:
            s = np.concatenate([s[:i], s[i + int(rng.integers(1, 4)):]])
    return s


def sample_reads(contigs, n, read_len=150, seed=1, chimeric=0.3, n_rate=0.002):
    """Single reads [n, read_len] (uint8 ASCII) and their lengths (ragged by indels)."""
    rng = np.random.default_rng(seed)
    out = np.full((n, read_len + 4), ord("N"), dtype=np.uint8)
    lens = np.zeros(n, np.int32)
    for i in range(n):
        if rng.random() < chimeric:
            c = int(rng.integers(25, read_len - 25))
            r = np.concatenate([_sample_frag(rng, contigs, c), _sample_frag(rng, contigs, read_len - c)])
        else:
            r = _sample_frag(rng, contigs, read_len)
        if rng.random() < 0.5:
            r = _rc(r)
        r = _noisy(rng, r)
        r[rng.random(len(r)) < n_rate] = ord("N")
        lens[i] = len(r)
        out[i, :len(r)] = r
    return out, lens


def sample_pairs(contigs, n_pairs, read_len=150, seed=2, frag_mean=320, frag_sd=30, discordant=0.15):
    """Pair-major reads [2 n_pairs, read_len]: mate 1 forward from the fragment start, mate 2 the
    reverse complement of its end (flipped half the time); some pairs join two loci."""
    rng = np.random.default_rng(seed)
    out = np.zeros((2 * n_pairs, read_len), dtype=np.uint8)
    for i in range(n_pairs):
        fl = int(np.clip(rng.normal(frag_mean, frag_sd), read_len + 10, 3 * frag_mean))
        if rng.random() < discordant:
            m1 = _sample_frag(rng, contigs, read_len)
            m2 = _rc(_sample_frag(rng, contigs, read_len))
        else:
            f = _sample_frag(rng, contigs, fl)
            m1, m2 = f[:read_len], _rc(f[-read_len:])
        m1, m2 = _mutate(rng, m1, 0.02), _mutate(rng, m2, 0.02)
        if rng.random() < 0.5:
            m1, m2 = m2, m1
        out[2 * i], out[2 * i + 1] = m1, m2
    return out
