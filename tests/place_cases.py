"""Synthetic multi-contig references and tail queries for the placement tests."""
import numpy as np

COMP = str.maketrans("ACGTN", "TGCAN")


def rc(s):
    return s.translate(COMP)[::-1]


def contigs(seed=7, n=4, length=20000):
    rng = np.random.default_rng(seed)
    out = []
    for k in range(n):
        s = "".join(rng.choice(list("ACGT"), length + 1000 * k))
        out.append((f"chr{k + 1}", s))
    return out


def mutate(rng, s, rate):
    b = list(s)
    for i in range(len(b)):
        if rng.random() < rate:
            b[i] = "ACGT"[rng.integers(4)]
    return "".join(b)


def queries(ctgs, n, seed=11, lens=(20, 40, 60, 100, 150)):
    """(name, seq, truth) triples: plain tails, reverse strand, chimeras of two contigs, noise."""
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        L = int(rng.choice(lens))
        kind = rng.random()
        k = int(rng.integers(len(ctgs)))
        name, seq = ctgs[k]
        p = int(rng.integers(0, len(seq) - L))
        q = mutate(rng, seq[p:p + L], 0.02)
        truth = [(name, p, p + L)]
        if kind < 0.3:
            q = rc(q)
        elif kind < 0.55:
            k2 = int(rng.integers(len(ctgs)))
            n2, s2 = ctgs[k2]
            cut = int(rng.integers(L // 4, 3 * L // 4))
            p2 = int(rng.integers(0, len(s2) - L))
            q = q[:cut] + mutate(rng, s2[p2:p2 + L - cut], 0.02)
            truth = [(name, p, p + cut), (n2, p2, p2 + L - cut)]
        elif kind < 0.6:
            q = "".join(rng.choice(list("ACGT"), L))
            truth = []
        out.append((f"q{i}", q, truth))
    return out
