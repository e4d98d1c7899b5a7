"""The per-query rules of csrc/s5s6.hip (k_s5_check's keep flag, k_s6_rows' processed SEQ),
compiled for the host too and exported as af_s5_rules_host, against the consumer-stage
restatements on CPU: genome_check.filter_genome_hits over the SAM text of the same af_grec
records (`del_too_many_reads`, functions.py:705-768) and cigar.normalize (`deal_cigar`,
fn:656-702).  Random CIGARs reach the corner cases the GPU worlds rarely produce: leading D / I
(Python's ops[-1]), N / H ops, reverse records, unmapped records, QNAME groups of several queries
(mates with the same POS and CIGAR), caller-given group flags, clipped output rows.  The same
source is what runs on the device (tests/test_gpu_s5s6.py checks that)."""
import ctypes

import numpy as np
import pytest

import afpkg  # noqa: F401
from anchored_fusion_amd import _lib, genome, genome_check
from anchored_fusion_amd.cigar import normalize

_OPS = "MIDNSHP=X"
NAMES = ["chrA", "chrB", "chrC"]


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def rules_host(recs, nrec, q_rows, pos, ncig, cig, cont, q, qlens, out_stride):
    n = len(q_rows)
    keep = np.zeros(n, np.uint8)
    rows = np.zeros((n, out_stride), np.uint8)
    olens = np.zeros(n, np.int32)
    over = np.zeros(n, np.uint8)
    rc = _lib.lib().af_s5_rules_host(_ptr(recs), _ptr(nrec), n, _ptr(q_rows), _ptr(pos), _ptr(ncig), _ptr(cig),
                                     _ptr(cont), _ptr(q), q.shape[1], _ptr(qlens), _ptr(keep), _ptr(rows), out_stride,
                                     _ptr(olens), _ptr(over))
    assert rc == 0
    return keep, rows, olens, over


def _cigar(rng, ops, n):
    return [(int(rng.integers(1, 60)) << 4) | _OPS.index(ops[int(rng.integers(0, len(ops)))]) for _ in range(n)]


def _cstr(words):
    return "".join(f"{w >> 4}{_OPS[w & 15]}" for w in words) or "*"


def _world(seed, n_pairs=400, L=120):
    rng = np.random.default_rng(seed)
    n_rows = 2 * n_pairs
    pos = rng.integers(0, 5000, n_rows).astype(np.int32)
    ncig = np.zeros(n_rows, np.int32)
    cig = np.zeros((n_rows, _lib.AF_MAX_CIGAR), np.uint32)
    for r in range(n_rows):
        u = rng.random()
        if u < 0.5:  # split-read shaped: S+M / M+S with the odd I / D inside
            a = int(rng.integers(10, L - 10))
            w = [(a << 4) | 4, ((L - a) << 4)] if rng.random() < 0.5 else [(a << 4), ((L - a) << 4) | 4]
            if rng.random() < 0.4:
                w.insert(int(rng.integers(0, 3)), (int(rng.integers(1, 6)) << 4) | int(rng.choice([1, 2])))
        else:
            w = _cigar(rng, "MIDNSH", int(rng.integers(1, 7)))
        ncig[r] = len(w)
        cig[r, :len(w)] = w
    # mates share POS and CIGAR now and then: QNAME groups of two queries
    for i in range(0, n_rows, 2):
        if rng.random() < 0.3:
            pos[i + 1], ncig[i + 1], cig[i + 1] = pos[i], ncig[i], cig[i]
    # queries: some rows, in row order (both mates often), each with a unique random sequence
    q_rows = np.sort(rng.choice(n_rows, int(n_rows * 0.8), replace=False)).astype(np.int32)
    n = len(q_rows)
    qlens = rng.integers(L - 20, L + 1, n).astype(np.int32)
    q = np.full((n, L), ord("N"), np.uint8)
    for k in range(n):
        q[k, :qlens[k]] = np.frombuffer(b"ACGTN", np.uint8)[rng.integers(0, 5, qlens[k])]
    recs = np.zeros((n, genome.MAX_REC), genome.REC_DTYPE)
    nrec = rng.integers(1, genome.MAX_REC + 1, n).astype(np.int32)
    for k in range(n):
        for j in range(nrec[k]):
            e = recs[k, j]
            if rng.random() < 0.05 and j == 0:
                e["flag"], e["rid"], e["pos"], e["n_cigar"] = 4, -1, -1, 0
            else:
                e["flag"] = int(rng.choice([0, 16])) | (0 if j == 0 else 256)
                e["rid"], e["pos"] = int(rng.integers(0, 3)), int(rng.integers(0, 10_000))
                w = _cigar(rng, "MMMSSHID", int(rng.integers(1, 6)))
                e["n_cigar"] = len(w)
                e["cigar"][:len(w)] = w
            e["mrid"], e["seq_b"], e["seq_e"] = -1, 0, qlens[k]
    return dict(recs=recs, nrec=nrec, q_rows=q_rows, pos=pos, ncig=ncig, cig=cig, q=q, qlens=qlens)


def _expected_keep(w, names):
    """filter_genome_hits over the SAM text of the records, QNAMEs `names[k]`; the emitted lines
    carry the group's first query's (unique) sequence, which maps them back to their query."""
    lines = ["@HD\tVN:1.6\n"]
    for k, nm in enumerate(names):
        lines += genome.sam_lines(NAMES, nm, w["q"][k, :w["qlens"][k]].tobytes().decode(), w["recs"][k], w["nrec"][k])
    out = genome_check.filter_genome_hits(lines)
    emitted = {ln.split("\t")[9] for ln in out}
    assert len(emitted) == len(out)
    keep = np.zeros(len(names), np.uint8)
    for k, nm in enumerate(names):
        start = k == 0 or names[k - 1] != nm
        keep[k] = start and w["q"][k, :w["qlens"][k]].tobytes().decode() in emitted
    return keep, len(out)


def _qname(w, k):
    r = int(w["q_rows"][k])
    return f"p{r >> 1}$GENE${int(w['pos'][r]) + 1}${_cstr(w['cig'][r, :w['ncig'][r]].tolist())}"


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_rules_match_genome_check_and_deal_cigar(seed):
    w = _world(seed)
    n = len(w["q_rows"])
    keep, rows, olens, over = rules_host(w["recs"], w["nrec"], w["q_rows"], w["pos"], w["ncig"], w["cig"], None,
                                         w["q"], w["qlens"], _lib.AF_MAX_READ)
    names = [_qname(w, k) for k in range(n)]
    want, n_out = _expected_keep(w, names)
    assert 20 < n_out < n
    assert np.array_equal(keep, want)
    assert any(names[k] == names[k - 1] for k in range(1, n))  # multi-query groups present
    assert _check_rows(w, rows, olens, over, _lib.AF_MAX_READ) < n // 10


def _check_rows(w, rows, olens, over, stride):
    """deal_cigar's SEQ exactly, unless the row is counted as over (a byte was dropped on the
    way: the edits then run on the clipped row, the result is not deal_cigar's); every row whose
    SEQ exceeds the stride is counted.  Returns the over count."""
    n_over = 0
    for k in range(len(w["q_rows"])):
        r = int(w["q_rows"][k])
        _, seq = normalize(_cstr(w["cig"][r, :w["ncig"][r]].tolist()), w["q"][k, :w["qlens"][k]].tobytes().decode())
        got = rows[k, :olens[k]].tobytes().decode()
        if over[k]:
            n_over += 1
            assert olens[k] <= stride, k
        else:
            assert got == seq, k
        if len(seq) > stride:
            assert over[k], k
    return n_over


def test_rules_with_caller_groups():
    """d_cont given (a rank's share of a sharded list): groups are the caller's, whatever the QNAMEs."""
    w = _world(7)
    n = len(w["q_rows"])
    rng = np.random.default_rng(8)
    cont = (rng.random(n) < 0.35).astype(np.uint8)
    cont[0] = 0
    keep, _, _, _ = rules_host(w["recs"], w["nrec"], w["q_rows"], w["pos"], w["ncig"], w["cig"], cont, w["q"],
                               w["qlens"], _lib.AF_MAX_READ)
    gid = np.zeros(n, np.int64)
    for k in range(1, n):
        gid[k] = gid[k - 1] if cont[k] else k
    # the group's QNAME carries the CIGAR the check reads: the first query's
    names = [f"g{gid[k]}$GENE$1${_qname(w, int(gid[k])).split('$')[3]}" for k in range(n)]
    want, n_out = _expected_keep(w, names)
    assert 10 < n_out < n and np.array_equal(keep, want)


def test_rules_clipped_rows():
    """Rows longer than the output stride are counted as over; the others are exact."""
    w = _world(11)
    n = len(w["q_rows"])
    stride = 100
    _, rows, olens, over = rules_host(w["recs"], w["nrec"], w["q_rows"], w["pos"], w["ncig"], w["cig"], None, w["q"],
                                      w["qlens"], stride)
    assert _check_rows(w, rows, olens, over, stride) > 10
