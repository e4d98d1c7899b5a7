"""Deterministic read sets shared by the CPU oracle tests and the GPU parity tests."""
import numpy as np

from anchored_fusion_amd import simulate as sim


def _pad(seqs, stride):
    out = np.full((len(seqs), stride), ord("N"), dtype=np.uint8)
    lens = np.zeros(len(seqs), dtype=np.int32)
    for i, s in enumerate(seqs):
        s = s[:stride]
        out[i, : len(s)] = np.frombuffer(s, dtype=np.uint8)
        lens[i] = len(s)
    return out, lens


def edge_pairs(anchor: bytes, read_len=100, seed=7):
    """Hand-made pairs covering the edge cases of the aligner (returned pair-major)."""
    rng = np.random.default_rng(seed)
    n = len(anchor)
    L = read_len
    rc = sim.revcomp
    seqs = []
    # exact full-length matches at both anchor ends, both strands
    seqs += [anchor[:L], rc(anchor[n - L:])]
    seqs += [rc(anchor[:L]), anchor[n - L:]]
    # split reads: anchor part + random tail (MS) and random head + anchor part (SM)
    for cut in (20, 31, 45, 60, 75, 85):
        a = int(rng.integers(200, n - 300))
        seqs += [anchor[a:a + cut] + sim.random_seq(rng, L - cut), sim.random_seq(rng, L - cut) + anchor[a:a + cut]]
    # exon-skip-like read (two anchor segments), and its reverse complement
    a = 1500
    seqs += [anchor[a:a + 50] + anchor[a + 150:a + 200], rc(anchor[a:a + 55] + anchor[a + 400:a + 445])]
    # insertions / deletions inside a read
    a = 3000
    seqs += [anchor[a:a + 40] + b"GT" + anchor[a + 40:a + L - 2], anchor[a:a + 50] + anchor[a + 53:a + L + 3]]
    seqs += [rc(anchor[a:a + 30] + b"TTTA" + anchor[a + 30:a + L - 4]), rc(anchor[a:a + 60] + anchor[a + 66:a + L + 6])]
    # N handling: all-N, single N, N-dense
    s = bytearray(anchor[4000:4000 + L]); s[50] = ord("N")
    seqs += [b"N" * L, bytes(s)]
    s2 = bytearray(anchor[4200:4200 + L])
    for k in range(0, L, 9):
        s2[k] = ord("N")
    seqs += [bytes(s2), anchor[4300:4300 + L].lower()]
    # low complexity and random
    seqs += [b"AC" * (L // 2), sim.random_seq(rng, L)]
    # many mismatches (forces the global DP path)
    s3 = bytearray(anchor[5000:5000 + L])
    for k in range(5, L, 11):
        s3[k] = ord("A") if s3[k] != ord("A") else ord("C")
    seqs += [bytes(s3), rc(bytes(s3))]
    if len(seqs) % 2:
        seqs.append(sim.random_seq(rng, L))
    return _pad(seqs, L)


def synthetic_pairs(anchor: bytes, n_pairs, read_len, seed, err=0.02, indel_frac=0.03, n_rate=0.001, fusion_frac=0.6):
    _, reads, truth, world = sim.fusion_reads(anchor, n_pairs, read_len=read_len, fusion_frac=fusion_frac, seed=seed,
                                              err=err, indel_frac=indel_frac, n_rate=n_rate)
    return reads, truth, world


def ragged(reads, seed):
    """Random per-read lengths in [12, stride] with N padding (exercises the lens path)."""
    rng = np.random.default_rng(seed)
    n, stride = reads.shape
    lens = rng.integers(12, stride + 1, size=n).astype(np.int32)
    out = reads.copy()
    for i in range(n):
        out[i, lens[i]:] = ord("N")
    return out, lens


def rescue_pairs(anchor: bytes, n_normal=60, read_len=100, insert=250, seed=5):
    """n_normal proper FR pairs from the anchor (insert-size model) plus one probe pair whose
    mate 2 carries a mismatch every 12 bases: no exact 19-mer (K1 finds nothing) but a local
    alignment score far above min_seed_len at the right distance.  Returns (reads, probe pair)."""
    rng = np.random.default_rng(seed)
    rc = sim.revcomp
    seqs = []
    n = len(anchor)
    for k in range(n_normal):
        a = int(rng.integers(0, n - insert - 1))
        ins = insert + int(rng.integers(-15, 16))
        frag = anchor[a:a + ins]
        seqs += [frag[:read_len], rc(frag[-read_len:])]
    a = 2000
    frag = anchor[a:a + insert]
    m2 = bytearray(rc(frag[-read_len:]))
    for k in range(6, read_len, 12):
        m2[k] = ord("A") if m2[k] != ord("A") else ord("G")
    seqs += [frag[:read_len], bytes(m2)]
    reads, _ = _pad(seqs, read_len)
    return reads, n_normal


def repeat_anchor_pairs(anchor: bytes, read_len=100, n=12, seed=9):
    """An anchor with a 400-nt segment duplicated at its end, and pairs whose mate 1 lies inside
    the segment (two equal-score hits) with mate 2 in unique sequence far away (no pairing
    decides between the copies)."""
    seg = anchor[1000:1400]
    anc2 = anchor + b"ACGTTGCA" * 4 + seg
    rng = np.random.default_rng(seed)
    rc = sim.revcomp
    seqs = []
    for k in range(n):
        a = 1000 + int(rng.integers(0, 400 - read_len))
        b = 4000 + int(rng.integers(0, 1000))
        seqs += [anchor[a:a + read_len], rc(anchor[b:b + read_len])]
    return anc2, _pad(seqs, read_len)[0]


# A pair from the configs[2] world whose mate 1 opens with 41 bases of (CGC)n against the anchor's
# CGCCGCCGCCGCCGCCGC (BCR 5' UTR): nine regions on the same repeat, three left after dedup with
# equal scores -- the input that exposed the introsort else-branch and the unbounded partition scan
# (K2 hung on it).
TANDEM_PAIR = (
    b"CGCCGCCGCCGCCGCCGCCGCCGCCGCCGCCGCCGCCGCCGGATCGTAAATAACAATTTAATATATTTCCGTTTAACCCACGCAGGAAATCGGGCATACTA"
    b"TTGAAAAGCTGTAATGCGCCATAGGATGGCTATCTCTCAAGAATCGACG",
    b"GAATGCAGGTGGGCTCTTGGGTGGGAAGTTTGCAAAAGTTTACTTAATTTGGAACAATGCATCCGTCGATTCTTGAGAGATAGCCCGCCTATAGCGCGCTAC"
    b"AGCTTTGCAATAGTATGCCCAATTTCCTGCGTGGGTTAAACGGAAATA",
)


def tandem_pairs(anchor: bytes, n_extra=40, seed=11):
    """TANDEM_PAIR, then (CGC)n / (GCC)n reads of several phases and lengths around the anchor's
    repeat, paired with random mates, after some ordinary pairs."""
    rng = np.random.default_rng(seed)
    reads, _, _ = synthetic_pairs(anchor, n_extra, 150, seed=seed)
    rows = [r.tobytes() for r in reads]
    rows += list(TANDEM_PAIR)
    tail = TANDEM_PAIR[0][41:]
    for ph in range(3):
        for k in (14, 20, 30, 45):
            rep = (b"CGC" * 40)[ph:ph + 3 * k][:3 * k]
            r1 = (rep + tail)[:150]
            r2 = sim.random_seq(rng, 150)
            rows += [r1.ljust(150, b"N"), r2]
    return np.frombuffer(b"".join(rows), np.uint8).reshape(-1, 150).copy()
