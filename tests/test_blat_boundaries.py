"""Where the BLAT restatement's alignments of a split read end, at the resolution S6's consumer
reads them (Find_fine_block, /root/reference/functions.py:632-649): a row counts as a partner
block when its qStart / qEnd fall within 5 nt of the junction (left_length), as "bad" or "good"
by qStart <= 5 / qEnd >= qSize - 5 and the other half's extent.  oracle/blat.c aligns as Kent
2002 publishes it: the hits of one diagonal whose tiles touch form a range, a range is extended
without gaps into an HSP (+1 / -1, an end stops XDOWN = 10 positions after its last new best), and
gaps appear only where HSPs are stitched.  So on a chimeric read each partner's row is one gapless
block that ends where the running match score along its diagonal peaks: at the junction, or past
it when chance matches lift the score to a new best within 10 positions, or before it when the
last bases mismatch.

CPU tests (the oracle; tests/test_gpu_blat.py holds the GPU to the oracle): 1,000 chimeric reads
(left part on chrA, right part on chrB, 1 % substitutions away from the junction, mismatches
planted at junction - 1 .. - 3 in half of them) -- every partner row is the HSP of its first
range, no partner row holds a gap, and fn:632-649's windows hold for the reads without planted
mismatches.  The round-5 gapped extension (afo_blat_set_gapped) is measured beside it."""
import ctypes

import numpy as np

from anchored_fusion_amd import blat
from oracle_backends import OracleTileReference

ACGT = np.frombuffer(b"ACGT", np.uint8)


def _world(seed=5):
    rng = np.random.default_rng(seed)
    a = ACGT[rng.integers(0, 4, 400_000)]
    b = ACGT[rng.integers(0, 4, 400_000)]
    return rng, a, b


XDOWN = 10  # oracle/blat.c: an HSP end stops 10 positions after its last new best


def _walk(q, t):
    """Bases an HSP end takes along q / t (aligned arrays from the range's end outwards): the
    first best running score (+1 / -1), the walk stopped XDOWN positions after its last new best."""
    s = best = nb = 0
    for i in range(1, min(len(q), len(t)) + 1):
        s += 1 if q[i - 1] == t[i - 1] else -1
        if s > best:
            best, nb = s, i
        elif i - nb > XDOWN:
            break
    return nb


def _first_hsp(q, g, t0, step=11):
    """(qb, qe) of the HSP of the first range of query q on the diagonal where q[i] pairs with
    g[t0 + i] (t0: the blob coordinate of q[0]; tiles start at multiples of step)."""
    hits = [i for i in range(len(q) - 10) if (t0 + i) % step == 0 and 0 <= t0 + i and
            bytes(q[i:i + 11]) == bytes(g[t0 + i:t0 + i + 11])]
    if not hits:
        return None
    q0 = hits[0]
    q1 = q0 + 11
    for h in hits[1:]:
        if h > q1:
            break
        q1 = h + 11
    left = _walk(q[:q0][::-1], g[max(t0, 0):t0 + q0][::-1])
    right = _walk(q[q1:], g[t0 + q1:t0 + len(q)])
    return q0 - left, q1 + right


def _peak(q, t, start):
    """The first position after which the running match score (+1 / -1) from start peaks (no
    stopping rule): the end of the round-5 extension's gapless rows."""
    s = best = 0
    end = start
    for x in range(start, len(q)):
        s += 1 if q[x] == t[x] else -1
        if s > best:
            best, end = s, x + 1
    return end


def _reads(rng, a, b, n=400):
    out = []
    for k in range(n):
        left = int(rng.integers(40, 111))
        pa = int(rng.integers(1000, len(a) - 1000))
        pb = int(rng.integers(1000, len(b) - 1000))
        q = np.concatenate([a[pa:pa + left], b[pb:pb + 150 - left]]).copy()
        for j in np.nonzero(rng.random(150) < 0.01)[0]:
            if abs(int(j) - left) > 8:
                q[j] = ACGT[(int(np.nonzero(ACGT == q[j])[0][0]) + 1) % 4]
        # some reads: mismatches planted just before the junction (the extension stops early)
        planted = []
        if k % 4 == 1:
            planted = [left - 1 - int(rng.integers(0, 3))]
        elif k % 4 == 2:
            planted = [left - 1, left - 2]
        for j in planted:
            q[j] = ACGT[(int(np.nonzero(ACGT == a[pa + j])[0][0]) + 1) % 4]
        out.append((q, left, pa, pb))
    return out


def _classify(reads, rows, nr, off_b):
    """Per read: (gapless, missing, gapped, within) of the first chrA / chrB rows."""
    out = []
    for i, (q, left, pa, pb) in enumerate(reads):
        ra = [r for r in rows[i, :nr[i]] if r["strand"] == 0 and r["t_start"] < off_b]
        rb = [r for r in rows[i, :nr[i]] if r["strand"] == 0 and r["t_start"] >= off_b]
        if not ra or not rb:
            out.append(("missing", None, None))
            continue
        x, y = ra[0], rb[0]
        gapped = int(x["q_num_insert"]) + int(x["t_num_insert"]) + int(y["q_num_insert"]) + int(y["t_num_insert"]) > 0
        out.append(("gapped" if gapped else "gapless", x, y))
    return out


def test_split_read_rows_end_where_the_score_peaks():
    """Every partner row is one gapless HSP: the HSP of its first range on the partner's diagonal;
    no partner row holds a gap (the round-5 gapped extension put 1.2 % of them across the junction
    with a gap and lost 1 % under -minIdentity); fn:632-649's +-5 windows hold for >= 90 % of the
    reads without planted mismatches."""
    import oracle
    rng, a, b = _world()
    ctgs = [("chrA", a.tobytes().decode()), ("chrB", b.tobytes().decode())]
    o = OracleTileReference(ctgs, 11)
    reads = _reads(rng, a, b, 1000)
    rows, nr = o.search([r[0].tobytes().decode() for r in reads], blat.params("split_tail"), 16)
    off_b = o.offsets[1]
    blob = np.concatenate([a, np.frombuffer(b"N" * off_b, np.uint8)[:off_b - len(a)], b])
    n = gapless = missing = gapped = within = plain = 0
    for i, (kind, x, y) in enumerate(_classify(reads, rows, nr, off_b)):
        q, left, pa, pb = reads[i]
        n += 1
        if kind == "missing":
            missing += 1
            continue
        if kind == "gapped":
            gapped += 1
            continue
        gapless += 1
        assert int(x["t_start"]) - int(x["q_start"]) == pa and int(y["t_start"]) - off_b - int(y["q_start"]) == pb - left
        assert (int(x["q_start"]), int(x["q_end"])) == _first_hsp(q, blob, pa), i
        assert (int(y["q_start"]), int(y["q_end"])) == _first_hsp(q, blob, off_b + pb - left), i
        if i % 4 in (0, 3):  # no mismatch planted at the junction: fn:632-649's +-5 windows
            plain += 1
            within += abs(int(x["q_end"]) - left) <= 5 and abs(int(y["q_start"]) - left) <= 5
    assert gapped == 0 and missing <= 0.02 * n and gapless == n - missing, (n, gapless, missing, gapped)
    assert within >= 0.9 * plain, (within, plain)
    # the round-5 extension on the same reads: gapped partner rows and reads without both rows
    L = oracle.lib()
    L.afo_blat_set_gapped.argtypes = [ctypes.c_int]
    L.afo_blat_set_gapped(1)
    try:
        rows5, nr5 = o.search([r[0].tobytes().decode() for r in reads], blat.params("split_tail"), 16)
    finally:
        L.afo_blat_set_gapped(0)
    kinds5 = [k for k, _, _ in _classify(reads, rows5, nr5, off_b)]
    print("round-5 extension: gapped", kinds5.count("gapped"), "missing", kinds5.count("missing"), "| HSPs: missing", missing)
    assert kinds5.count("gapped") > 0, kinds5.count("gapped")


def test_consumer_windows_on_planted_junction_mismatches():
    """Reads whose last 1-2 bases before the junction mismatch the left partner: the left row is
    the HSP of its first range -- it ends before the junction when no chance match within 10
    positions pays the mismatches back, past it when one does."""
    rng, a, b = _world(11)
    ctgs = [("chrA", a.tobytes().decode()), ("chrB", b.tobytes().decode())]
    o = OracleTileReference(ctgs, 11)
    reads = [r for k, r in enumerate(_reads(rng, a, b, 200)) if k % 4 in (1, 2)]
    rows, nr = o.search([r[0].tobytes().decode() for r in reads], blat.params("split_tail"), 16)
    off_b = o.offsets[1]
    blob = np.concatenate([a, np.frombuffer(b"N" * off_b, np.uint8)[:off_b - len(a)], b])
    seen = before = 0
    for i, (q, left, pa, pb) in enumerate(reads):
        xs = [r for r in rows[i, :nr[i]] if r["strand"] == 0 and r["t_start"] < off_b]
        if not xs:
            continue
        seen += 1
        assert int(xs[0]["block_count"]) == 1
        assert (int(xs[0]["q_start"]), int(xs[0]["q_end"])) == _first_hsp(q, blob, pa), i
        before += int(xs[0]["q_end"]) < left
    assert seen >= 0.95 * len(reads) and before > 0
