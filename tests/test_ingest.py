"""Native paired FASTQ ingest (csrc/ingest.cpp, af_fastq_*; the fq1/fq2 inputs of `bwa mem` at
Anchored_Fusion.py:182).  Host-only: runs without a GPU.  The reference is bwa's reader
(kseq + trim_readno): the bundled test/ FASTQs are checked against a plain Python
four-line parser, and the record syntax edge cases against hand-written expectations."""
import gzip
import os
import re

import numpy as np
import pytest

from anchored_fusion_amd import io as afio

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _write(path, text, gz=False):
    data = text.encode()
    if gz:
        with gzip.open(path, "wb") as fh:
            fh.write(data)
    else:
        with open(path, "wb") as fh:
            fh.write(data)
    return str(path)


def _fq(recs, sep="\n"):
    return "".join(f"@{n}{sep}{s}{sep}+{sep}{'I' * len(s)}{sep}" for n, s in recs)


def test_bundled_pair_matches_python_reader():
    f1, f2 = (os.path.join(GOLDEN, f"test_sample_{m}.fastq.gz") for m in (1, 2))
    names, reads, lens = afio.read_pairs(f1, f2)
    n1, s1 = afio.read_fastq(f1)
    n2, s2 = afio.read_fastq(f2)
    assert n1 == n2 and len(names) == len(n1) == 11258
    inter = [None] * (2 * len(s1))
    inter[0::2], inter[1::2] = s1, s2
    want, wlens = afio.pack_reads(inter)
    assert lens is None and wlens is None
    assert reads.shape == want.shape and (reads == want).all()
    assert list(names) == n1


def test_batches_and_compression_agree(tmp_path):
    rng = np.random.default_rng(7)
    recs1, recs2 = [], []
    for i in range(3000):
        la, lb = int(rng.integers(0, 160)), int(rng.integers(1, 160))
        recs1.append((f"r{i}/1 extra", "".join(rng.choice(list("ACGTN"), la))))
        recs2.append((f"r{i}/2\tx", "".join(rng.choice(list("acgt"), lb))))
    p1 = _write(tmp_path / "a_1.fq.gz", _fq(recs1), gz=True)
    p2 = _write(tmp_path / "a_2.fq", _fq(recs2))
    names, reads, lens = afio.read_pairs(p1, p2)
    assert lens is not None and reads.shape == (6000, int(lens.max()))
    for i in (0, 1, 1234, 2999):
        for m, recs in enumerate((recs1, recs2)):
            s = recs[i][1].encode()
            assert lens[2 * i + m] == len(s)
            assert bytes(reads[2 * i + m, :len(s)]) == s
            assert (reads[2 * i + m, len(s):] == ord("N")).all()
        assert names[i] == f"r{i}"
    parts = list(afio.iter_pairs(p1, p2, batch_pairs=777))
    assert [len(nm) for nm, _, _ in parts] == [777] * 3 + [3000 - 3 * 777]
    row = 0
    for nm, r, ln in parts:
        k = r.shape[0]
        assert (ln == lens[row:row + k]).all()
        assert (r == reads[row:row + k, :r.shape[1]]).all()
        row += k


def test_record_syntax(tmp_path):
    # CRLF, blank lines between records, multi-line sequence and quality (kseq), a quality line
    # starting with '@', "/<digit>" trimmed only at the end of the first token
    t1 = ("@p1/1 c\r\nACGT\r\nAC\r\n+\r\n@III\r\nII\r\n\r\n"
          "@p2/x\nGG\n+p2\nII\n"
          "@p3/12\nT\n+\n@\n")
    t2 = "@p1/2\nCCCCCC\n+\nIIIIII\n@p2/x\nA\n+\nI\n\n\n@p3/12\nTT\n+\nII\n"
    names, reads, lens = afio.read_pairs(_write(tmp_path / "1.fq", t1), _write(tmp_path / "2.fq", t2))
    assert list(names) == ["p1", "p2/x", "p3/12"]  # "/12" is not a /<digit> suffix
    assert list(lens) == [6, 6, 2, 1, 1, 2]
    assert bytes(reads[0]) == b"ACGTAC" and bytes(reads[1]) == b"CCCCCC"
    assert bytes(reads[2]) == b"GGNNNN" and bytes(reads[5]) == b"TTNNNN"


def test_fasta_records(tmp_path):
    t1 = ">a/1\nAC\nGT\n>b\nTT\n"
    t2 = ">a/2\nCCC\n>b desc\nG\n"
    names, reads, lens = afio.read_pairs(_write(tmp_path / "1.fa", t1), _write(tmp_path / "2.fa", t2))
    assert list(names) == ["a", "b"] and list(lens) == [4, 3, 2, 1]
    assert bytes(reads[0]) == b"ACGT" and bytes(reads[3]) == b"GNNN"


def test_empty_input(tmp_path):
    names, reads, lens = afio.read_pairs(_write(tmp_path / "1.fq", ""), _write(tmp_path / "2.fq", "\n"))
    assert len(names) == 0 and reads.shape[0] == 0 and lens is None


@pytest.mark.parametrize("t1,t2,msg", [
    (_fq([("a", "AC"), ("b", "GG")]), _fq([("a", "AC")]), "differ in length"),
    (_fq([("a", "AC")]), _fq([("c", "AC")]), "different names"),
    ("@a\nACGT\n+\nII\n", _fq([("a", "AC")]), "quality shorter"),
    ("@a\nACGT\n", _fq([("a", "AC")]), "no '+' line"),
    ("xyz\n", _fq([("a", "AC")]), "record header"),
])
def test_malformed_pairs_raise(tmp_path, t1, t2, msg):
    with pytest.raises(ValueError, match=re.escape(msg)):
        afio.read_pairs(_write(tmp_path / "1.fq", t1), _write(tmp_path / "2.fq", t2))


def test_missing_file_raises(tmp_path):
    with pytest.raises(Exception, match="cannot open"):
        afio.read_pairs(str(tmp_path / "nope_1.fq"), str(tmp_path / "nope_2.fq"))


def _write_bgzf(path, text, block=60000, level=6):
    """BGZF as bgzip writes it: raw-deflate members of <= 64 KiB input with a 'BC' extra
    subfield holding the member size - 1, then the empty end-of-file member."""
    import struct
    import zlib
    data = text.encode()
    with open(path, "wb") as fh:
        for o in list(range(0, len(data), block)) + [len(data)]:
            chunk = data[o:o + block] if o < len(data) else b""
            c = zlib.compressobj(level, zlib.DEFLATED, -15)
            cdata = c.compress(chunk) + c.flush()
            bsize = 12 + 6 + len(cdata) + 8
            fh.write(b"\x1f\x8b\x08\x04" + b"\0\0\0\0" + b"\0\xff" + struct.pack("<H", 6) + b"BC" +
                     struct.pack("<HH", 2, bsize - 1) + cdata +
                     struct.pack("<II", zlib.crc32(chunk) & 0xFFFFFFFF, len(chunk)))
            if o >= len(data):
                break
    return str(path)


def test_bgzf_block_parallel(tmp_path):
    # BGZF input takes the block-parallel inflate path; records identical to the plain files,
    # including records that straddle block boundaries (small blocks force many of them)
    rng = np.random.default_rng(3)
    recs1 = [(f"b{i}/1", "".join(rng.choice(list("ACGTN"), int(rng.integers(1, 151))))) for i in range(5000)]
    recs2 = [(f"b{i}/2", "".join(rng.choice(list("ACGT"), 100))) for i in range(5000)]
    t1, t2 = _fq(recs1), _fq(recs2)
    plain = afio.read_pairs(_write(tmp_path / "p_1.fq", t1), _write(tmp_path / "p_2.fq", t2))
    for block in (997, 65280):
        b1 = _write_bgzf(tmp_path / f"b{block}_1.fq.gz", t1, block)
        b2 = _write_bgzf(tmp_path / f"b{block}_2.fq.gz", t2, block)
        assert gzip.open(b1).read().decode() == t1  # a valid multi-member gzip file as well
        for threads in (1, 8):
            names, reads, lens = afio.read_pairs(b1, b2, threads=threads)
            assert list(names) == list(plain[0])
            assert (reads == plain[1]).all() and (lens == plain[2]).all()


def test_bgzf_corrupt_block_raises(tmp_path):
    t = _fq([(f"c{i}", "ACGT" * 20) for i in range(3000)])
    b1 = _write_bgzf(tmp_path / "c_1.fq.gz", t, 4000)
    raw = bytearray(open(b1, "rb").read())
    raw[len(raw) // 2] ^= 0x55  # inside some member's deflate data
    open(b1, "wb").write(bytes(raw))
    b2 = _write_bgzf(tmp_path / "c_2.fq.gz", t, 4000)
    with pytest.raises(ValueError, match="BGZF"):
        afio.read_pairs(b1, b2)


def test_bgzf_corrupt_isize_raises(tmp_path):
    # a member whose ISIZE field claims more than BGZF's 64 KiB maximum is rejected as corrupt
    # before any allocation is sized from it (no std::bad_alloc escaping the reader thread)
    import struct
    t = _fq([(f"s{i}", "ACGT" * 20) for i in range(300)])
    b1 = _write_bgzf(tmp_path / "s_1.fq.gz", t, 4000)
    raw = bytearray(open(b1, "rb").read())
    bsize = struct.unpack_from("<H", raw, 16)[0] + 1  # first member
    struct.pack_into("<I", raw, bsize - 4, 0xFFFFFFF0)
    open(b1, "wb").write(bytes(raw))
    b2 = _write_bgzf(tmp_path / "s_2.fq.gz", t, 4000)
    with pytest.raises(ValueError, match="ISIZE"):
        afio.read_pairs(b1, b2)
