"""Where the BLAT restatement's alignments of a split read end, at the resolution S6's consumer
reads them (Find_fine_block, /root/reference/functions.py:632-649): a row counts as a partner
block when its qStart / qEnd fall within 5 nt of the junction (left_length), as "bad" or "good"
by qStart <= 5 / qEnd >= qSize - 5 and the other half's extent.  oracle/blat.c extends a clump
with ksw_extend2 (match 1, mismatch 1, gaps 3 + 1, band 16, z-drop 20) where BLAT extends hits
gaplessly and stitches (DESIGN.md §2 lists the departures).  Both stop an extension at its best
running score, so on a chimeric read the part of each partner ends where the match score along
the diagonal peaks: at the junction, or past it when the running score (a walk with drift -1/2
per base after the junction) climbs back above the junction's value -- net +1 suffices, however
many bases later: 1/3 of junctions, 6+ nt past it in ~11 % -- or before it when the last bases
mismatch.

CPU tests (the oracle; tests/test_gpu_blat.py holds the GPU to the oracle): 1,000 chimeric reads
(left part on chrA, right part on chrB, 1 % substitutions away from the junction, mismatches
planted at junction - 1 .. - 3 in half of them) -- every gapless row's junction end is where that
rule puts it; fn:632-649's windows hold for the reads without planted mismatches; the gapped
departures are counted and bounded."""
import numpy as np

from anchored_fusion_amd import blat
from oracle_backends import OracleTileReference

ACGT = np.frombuffer(b"ACGT", np.uint8)


def _world(seed=5):
    rng = np.random.default_rng(seed)
    a = ACGT[rng.integers(0, 4, 400_000)]
    b = ACGT[rng.integers(0, 4, 400_000)]
    return rng, a, b


def _peak(q, t, start):
    """The first position after which the running match score (+1 / -1) from start peaks: the
    end of a gapless extension that keeps its best score (first strict maximum)."""
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


def test_split_read_rows_end_where_the_score_peaks():
    """Every gapless partner row ends exactly where the gapless peak rule puts it (BLAT's own
    gapless extension stops there too); the departures -- a gapped extension into the other
    partner's bases (a 1-base gap buying chance matches), which can also sink the row under
    -minIdentity -- are counted and bounded (measured: 1.2 % gapped, 1 % missing per half)."""
    rng, a, b = _world()
    ctgs = [("chrA", a.tobytes().decode()), ("chrB", b.tobytes().decode())]
    o = OracleTileReference(ctgs, 11)
    reads = _reads(rng, a, b, 1000)
    rows, nr = o.search([r[0].tobytes().decode() for r in reads], blat.params("split_tail"), 16)
    off_b = o.offsets[1]
    n = gapless = missing = gapped = within = plain = 0
    for i, (q, left, pa, pb) in enumerate(reads):
        ra = [r for r in rows[i, :nr[i]] if r["strand"] == 0 and r["t_start"] < off_b]
        rb = [r for r in rows[i, :nr[i]] if r["strand"] == 0 and r["t_start"] >= off_b]
        n += 1
        if not ra or not rb:
            missing += 1
            continue
        x, y = ra[0], rb[0]
        if x["block_count"] == 1 and y["block_count"] == 1:
            # on the partners' diagonals
            assert int(x["t_start"]) - int(x["q_start"]) == pa and int(y["t_start"]) - off_b - int(y["q_start"]) == pb - left
            # chrA's half from the read start to the peak after (or before) the junction; chrB's
            # half from the peak of the reversed walk to the read end
            assert int(x["q_start"]) <= 5 and int(x["q_end"]) == _peak(q, a[pa:pa + 150], 0), i
            tb = b[pb - left:pb - left + 150]
            assert int(y["q_end"]) >= 145 and int(y["q_start"]) == 150 - _peak(q[::-1], tb[::-1], 0), i
            gapless += 1
        else:
            gapped += 1
        if i % 4 in (0, 3):  # no mismatch planted at the junction: fn:632-649's +-5 windows hold
            plain += 1
            within += abs(int(x["q_end"]) - left) <= 5 and abs(int(y["q_start"]) - left) <= 5
    assert gapless >= 0.95 * n and missing <= 0.03 * n and gapped <= 0.03 * n, (n, gapless, missing, gapped)
    # the peak rule itself moves ~11 % of clean junctions out of the windows: the running score
    # passes the junction's value again after a few chance matches (net +1 suffices, however far)
    assert within >= 0.85 * plain, (within, plain)


def test_consumer_windows_on_planted_junction_mismatches():
    """Reads whose last 1-2 bases before the junction mismatch the left partner: the left row ends
    by the peak rule -- before the junction when no chance match after it pays the mismatches
    back, past it when one does (overshoots of 6+ nt then move the read out of fn:632-649's
    windows, as they would under BLAT's gapless extension)."""
    rng, a, b = _world(11)
    ctgs = [("chrA", a.tobytes().decode()), ("chrB", b.tobytes().decode())]
    o = OracleTileReference(ctgs, 11)
    reads = [r for k, r in enumerate(_reads(rng, a, b, 200)) if k % 4 in (1, 2)]
    rows, nr = o.search([r[0].tobytes().decode() for r in reads], blat.params("split_tail"), 16)
    off_b = o.offsets[1]
    seen = 0
    for i, (q, left, pa, pb) in enumerate(reads):
        xs = [r for r in rows[i, :nr[i]] if r["strand"] == 0 and r["t_start"] < off_b]
        if not xs or xs[0]["block_count"] != 1:
            continue
        seen += 1
        assert int(xs[0]["q_end"]) == _peak(q, a[pa:pa + 150], 0), i
    assert seen >= 0.9 * len(reads)
