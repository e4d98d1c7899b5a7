"""bwa mem -M record rules for the genome searches (bwa_records): host logic on crafted hits."""
import numpy as np

import afpkg  # noqa: F401
from anchored_fusion_amd import bwa_records as br
from anchored_fusion_amd.place import HIT_DTYPE


class Ref:
    """Two contigs of 10 kb joined with 512 N (place.concat_contigs layout)."""
    names, lens, offsets = ["c1", "c2"], [10_000, 10_000], [0, 10_512]
    total = 20_512

    def locate(self, ts, te):
        k = 0 if ts < 10_512 else 1
        s, e = int(ts) - self.offsets[k], int(te) - self.offsets[k]
        return (k, s, e) if 0 <= s < e <= self.lens[k] else None


def cig(*ops):
    code = {"M": 0, "I": 1, "D": 2, "S": 4}
    return [n << 4 | code[o] for n, o in ops]


def hits_row(specs):
    """specs: (score, q_start, q_end, t_start, rev, cigar ops)"""
    h = np.zeros(16, HIT_DTYPE)
    for k, (sc, qs, qe, ts, rev, ops) in enumerate(specs):
        c = cig(*ops)
        alen = sum(n for n, o in ops if o in "MD")
        h[k]["score"], h[k]["q_start"], h[k]["q_end"] = sc, qs, qe
        h[k]["t_start"], h[k]["t_end"], h[k]["flag"] = ts, ts + alen, 0x10 if rev else 0
        h[k]["n_cigar"] = len(c)
        h[k]["cigar"][:len(c)] = c
    return h, len(specs)


SEQ = "ACGT" * 25  # 100 nt


def test_hash_64_matches_bwa():
    # values of bwa's utils.h hash_64 (compiled C, 64-bit wrap)
    assert br.hash_64(0) == 0x6a396cd39c352659
    assert br.hash_64(12345) == 0xced1fe8e61c2d2b1


def test_chimeric_part_is_a_minus_M_record_with_hard_clips():
    # 60M40S at c1:1000 (score 60), 60S40M at c2:2000 reverse (score 40): no query overlap
    h, n = hits_row([(60, 0, 60, 1000, False, [(60, "M"), (40, "S")]),
                     (40, 60, 100, 10_512 + 2000, True, [(60, "S"), (40, "M")])])
    lines = br.se_records(Ref(), "r", SEQ, h, n, 0, 30)
    f = [ln.split("\t") for ln in lines]
    assert [x[1] for x in f] == ["0", str(0x100 | 0x10)]
    assert f[0][2:6] == ["c1", "1001", "60", "60M40S"] and f[0][9] == SEQ
    assert f[1][2:4] == ["c2", "2001"] and f[1][5] == "60H40M"
    rc = SEQ.translate(str.maketrans("ACGT", "TGCA"))[::-1]
    assert f[1][9] == rc[60:]


def test_overlapping_alternative_is_not_printed():
    # two placements of the same query span: the lower one is secondary (XA), not a record;
    # a third one below T is dropped as well
    h, n = hits_row([(90, 0, 95, 100, False, [(95, "M"), (5, "S")]),
                     (80, 2, 100, 5000, False, [(2, "S"), (98, "M")]),
                     (25, 0, 30, 7000, False, [(30, "M"), (70, "S")])])
    lines = br.se_records(Ref(), "r", SEQ, h, n, 7, 30)
    assert len(lines) == 1 and lines[0].split("\t")[3] == "101"


def test_equal_scores_break_by_hash():
    # two equal-score placements of the whole read: bwa's primary is the lower hash_64(id + i),
    # i being the region's place in (score, rb, qb) order
    h, n = hits_row([(100, 0, 100, 3000, False, [(100, "M")]), (100, 0, 100, 200, False, [(100, "M")])])
    for rid in range(6):
        lines = br.se_records(Ref(), "r", SEQ, h, n, rid, 30)
        assert len(lines) == 1
        first = 201 if br.hash_64(rid + 0) < br.hash_64(rid + 1) else 3001  # region 0 = rb 200
        assert lines[0].split("\t")[3] == str(first)


def test_unmapped_record():
    h, n = hits_row([(20, 0, 20, 100, False, [(20, "M"), (80, "S")])])
    f = br.se_records(Ref(), "q", SEQ, h, n, 0, 30)[0].split("\t")
    assert f[1] == "4" and f[2] == "*" and f[5] == "*"


def test_pestat_and_pairing():
    # 40 FR pairs on c1 with insert ~300: pestat succeeds for FR; a probe pair whose mate 2 has
    # two placements (one consistent with the insert size) is paired on the consistent one
    ref = Ref()
    pairs, rows = [], []
    rng = np.random.default_rng(3)
    for i in range(40):
        a = 500 + 100 * i
        ins = 300 + int(rng.integers(-20, 21))
        rows.append(hits_row([(100, 0, 100, a, False, [(100, "M")])]))
        rows.append(hits_row([(100, 0, 100, a + ins - 100, True, [(100, "M")])]))
        pairs.append((f"p{i}", SEQ, SEQ))
    rows.append(hits_row([(100, 0, 100, 6000, False, [(100, "M")])]))
    rows.append(hits_row([(95, 0, 100, 6200, True, [(100, "M")]), (99, 0, 100, 10_512 + 4000, True, [(100, "M")])]))
    pairs.append(("probe", SEQ, SEQ))
    hits = np.stack([r[0] for r in rows])
    nh = np.array([r[1] for r in rows], np.int32)
    raw = [(br.regions(ref, hits[2 * i], nh[2 * i]), br.regions(ref, hits[2 * i + 1], nh[2 * i + 1]))
           for i in range(len(pairs))]
    pes = br.pestat(raw, ref.total)
    assert not pes[1].failed and pes[0].failed and pes[2].failed and pes[3].failed
    assert 250 < pes[1].avg < 350
    lines = br.pe_records(ref, pairs, hits, nh, 30)
    probe = [ln.split("\t") for ln in lines if ln.startswith("probe\t")]
    assert len(probe) == 2
    f1, f2 = (int(x[1]) for x in probe)
    assert f1 & 0x2 and f2 & 0x2 and f1 & 0x40 and f2 & 0x80 and f2 & 0x10 and f1 & 0x20
    assert probe[1][2:4] == ["c1", "6201"]  # the consistent placement, not the higher-scoring c2 one
    normal = [ln.split("\t") for ln in lines if ln.startswith("p0\t")]
    assert len(normal) == 2 and all(int(x[1]) & 0x2 for x in normal)


def test_unpaired_run_prints_every_record_with_mate_fields():
    # too few pairs for insert statistics: each end printed as single-end records with mate fields
    ref = Ref()
    r1 = hits_row([(60, 0, 60, 1000, False, [(60, "M"), (40, "S")]),
                   (40, 60, 100, 10_512 + 2000, True, [(60, "S"), (40, "M")])])
    r2 = hits_row([])
    hits = np.stack([r1[0], r2[0]])
    nh = np.array([r1[1], 0], np.int32)
    lines = [ln.split("\t") for ln in br.pe_records(ref, [("x", SEQ, SEQ)], hits, nh, 30)]
    assert [int(x[1]) for x in lines] == [0x1 | 0x40 | 0x8, 0x1 | 0x40 | 0x8 | 0x10 | 0x20 | 0x100,
                                          0x1 | 0x80 | 0x4]
    assert lines[2][2:4] == ["c1", "1001"]  # the unmapped end sits at its mate's position
