"""Size-independent checks of a bwa index (the text T = pac ++ revcomp(pac), its suffix array and
the FM occurrence table of fmindex.hip) read back through three accessors, so that an index too
large for the oracle (the 3.09 Gbp configs[2] genome: 6.18 G suffix-array rows) is validated by
its defining properties on samples:

* totals: the last occurrence block's counts equal the base counts of T ('$' not counted);
* blocks: sampled blocks' BWT codes equal T[SA[r] - 1] of their rows, and consecutive blocks'
  counts differ by the block's own histogram;
* LF: for sampled rows r with p = SA[r] > 0 and c = T[p - 1], SA[C[c] + Occ(c, r)] == p - 1 (the
  suffix array and the occurrence table agree on the step bwt_smem1 walks; this also makes SA a
  consistent permutation on the sample);
* order: sampled adjacent rows hold suffixes in strictly increasing order ('$' = end of T
  smallest), compared over `window` bases (longer when a repeat makes the window equal).

text(first, n) -> uint8 codes; sa(first, n) -> int64 rows; occ(first_blk, n_blk) -> uint64 [n, 8].
"""
import numpy as np

BLK = 128


def base_counts(text, l_pac, piece=1 << 28):
    """A/C/G/T counts of T from its forward half (the second half is its reverse complement)."""
    cnt = np.zeros(4, np.int64)
    for a in range(0, l_pac, piece):
        t = text(a, min(piece, l_pac - a))
        cnt += np.bincount(t, minlength=4)[:4]
    return cnt + cnt[::-1]


def block_codes(words):
    """The 128 BWT codes of one occurrence block (words 4..7)."""
    w = np.asarray(words[4:8], np.uint64)
    sh = (2 * np.arange(32)).astype(np.uint64)
    return ((w[:, None] >> sh[None, :]) & np.uint64(3)).astype(np.int64).reshape(-1)


def occ_at(occ, primary, c, r):
    """bwt_occ(c, r): occurrences of c among BWT rows [0, r)."""
    b = r // BLK
    blk = occ(b, 1)[0]
    codes = block_codes(blk)[: r - b * BLK]
    n = int(blk[c]) + int((codes == c).sum())
    if c == 0 and b * BLK <= primary < r:
        n -= 1  # '$' is stored as A
    return n


def compare_suffixes(text, N, p, q, window):
    """-1 / 0 / 1: suffix p vs suffix q over `window` bases (end of T smallest)."""
    a = text(p, min(window, N - p))
    b = text(q, min(window, N - q))
    m = min(len(a), len(b))
    d = np.nonzero(a[:m] != b[:m])[0]
    if d.size:
        return -1 if a[d[0]] < b[d[0]] else 1
    if len(a) != len(b):
        return -1 if len(a) < len(b) else 1
    return 0


def check_index(text, sa, occ, l_pac, primary, seed=1, n_rows=400, n_blocks=24, window=4096, max_window=1 << 18):
    """Runs the four checks; returns a summary dict (raises AssertionError on a violation)."""
    N = 2 * l_pac
    rng = np.random.default_rng(seed)
    nblk = (N + 1 + BLK - 1) // BLK + 1
    tot = base_counts(text, l_pac)
    last = occ(nblk - 1, 1)[0]
    assert [int(v) for v in last[:4]] == [int(v) for v in tot], (last[:4], tot)
    C = np.zeros(4, np.int64)
    C[0] = 1
    for c in range(1, 4):
        C[c] = C[c - 1] + tot[c - 1]
    assert int(sa(0, 1)[0]) == N
    # blocks
    blocks = np.unique(np.concatenate([[0, nblk - 2], rng.integers(0, nblk - 1, n_blocks)]))
    for b in blocks:
        r0, r1 = int(b) * BLK, min(int(b) * BLK + BLK, N + 1)
        rows = sa(r0, r1 - r0)
        w = occ(int(b), 2)
        codes = block_codes(w[0])[: r1 - r0]
        want = np.array([0 if p == 0 else int(text(int(p) - 1, 1)[0]) for p in rows], np.int64)
        assert np.array_equal(codes, want), ("BWT codes", int(b))
        h = np.bincount(want[rows != 0], minlength=4)[:4]
        assert np.array_equal(w[1, :4].astype(np.int64) - w[0, :4].astype(np.int64), h), ("block counts", int(b))
        if (rows == 0).any():
            assert int(r0 + np.nonzero(rows == 0)[0][0]) == primary
    # LF and order on sampled rows (both strands: rows whose suffix starts in the reverse half
    # lie above l_pac, i.e. above 2^31 at hg38 size)
    rows = rng.integers(1, N, n_rows)
    high = 0
    undecided = 0
    for r in rows:
        r = int(r)
        p, q = (int(v) for v in sa(r, 2))
        high += p >= 1 << 31
        if p > 0:
            c = int(text(p - 1, 1)[0])
            lf = int(C[c]) + occ_at(occ, primary, c, r)
            assert int(sa(lf, 1)[0]) == p - 1, ("LF", r, p, lf)
        w = window
        while True:
            o = compare_suffixes(text, N, p, q, w)
            if o != 0 or w >= max_window:
                break
            w *= 8
        if o == 0:
            undecided += 1
        else:
            assert o < 0, ("order", r, p, q)
    return dict(rows=len(rows), blocks=len(blocks), rows_above_2_31=high, undecided=undecided, totals=tot.tolist())


def occ_from_sa(T, sa):
    """numpy occurrence table of (T, sa) in fmindex.hip's layout (CPU tests of the checker)."""
    N = len(T)
    nblk = (N + 1 + BLK - 1) // BLK + 1
    codes = np.zeros(nblk * BLK, np.uint64)
    codes[:N + 1] = np.where(sa > 0, T[np.maximum(sa - 1, 0)], 0)
    counted = np.full(nblk * BLK, 4, np.int64)
    counted[:N + 1] = np.where(sa > 0, codes[:N + 1].astype(np.int64), 4)
    occ = np.zeros((nblk, 8), np.uint64)
    sh = (2 * np.arange(32)).astype(np.uint64)
    occ[:, 4:] = np.bitwise_or.reduce(codes.reshape(nblk, 4, 32) << sh[None, None, :], axis=2)
    per = np.stack([(counted.reshape(nblk, BLK) == c).sum(1) for c in range(4)], 1).astype(np.uint64)
    occ[1:, :4] = np.cumsum(per, 0)[:-1]
    return occ
