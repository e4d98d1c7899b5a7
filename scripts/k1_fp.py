"""K1 Bloom design study (CPU, numpy): candidate counts on the bench workload for the exact
16-mer membership test and for Bloom variants.  Not used by the product or tests."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import afpkg  # noqa: E402,F401
from anchored_fusion_amd import io as afio  # noqa: E402
from anchored_fusion_amd import simulate as sim  # noqa: E402

n = int(os.environ.get("PAIRS", "1000000"))
anchor = afio.anchor_sequence(os.path.join(ROOT, "tests", "golden", "target_gene.fasta"))
_, reads, _, _ = sim.fusion_reads(anchor, n, read_len=100, fusion_frac=0.05, seed=20251015)
R, L = reads.shape
code = lambda b: (np.uint32(0x8340) >> (2 * (b.astype(np.uint32) & 7))) & 3


def keys_at(buf, starts):
    k = np.zeros(len(starts), dtype=np.uint32)
    for j in range(16):
        k |= code(buf[starts + j]) << np.uint32(8 * (j & 3) + 2 * (j >> 2))
    return k


flat = reads.reshape(-1)
offs = np.arange(0, L - 15, 4)          # stride 100 is a multiple of 4: offsets 0,4,..,84
starts = (np.arange(R)[:, None] * L + offs[None, :]).reshape(-1)
qk = keys_at(flat, starts)
rid = np.repeat(np.arange(R), len(offs))
A = np.frombuffer(anchor, dtype=np.uint8)
rcl = np.zeros(256, np.uint8)
for a, b in zip(b"ACGTN", b"TGCAN"):
    rcl[a] = b
D = np.concatenate([A, rcl[A[::-1]]])
ok = np.array([all(c in b"ACGT" for c in D[p:p + 16]) for p in range(len(D) - 15)])
ak = np.unique(keys_at(D, np.nonzero(ok)[0]))
nd = len(ak)
member = np.isin(qk, ak)
print(f"reads {R}  probes {len(qk)}  anchor keys {nd}")
print(f"exact: positive probes {member.sum()}  candidate reads {len(np.unique(rid[member]))}")


def run(name, hashf, nbits_words, fields):
    """fields(h) -> list of (word index array, mask array)"""
    W = np.zeros(1 << nbits_words, dtype=np.uint32)
    for wi, m in fields(hashf(ak)):
        np.bitwise_or.at(W, wi, m)
    ok = np.ones(len(qk), bool)
    for wi, m in fields(hashf(qk)):
        ok &= (W[wi] & m) == m
    fp = ok & ~member
    print(f"{name:40s} FP/probe {fp.sum() / len(qk):.2e}  candidate reads {len(np.unique(rid[ok]))}")


def mask(v):
    one = np.uint32(1)
    return (one << ((v >> 8) & 31)) | (one << ((v >> 16) & 31)) | (one << ((v >> 24) & 31))


def rot4(v):
    return (v >> np.uint32(4)) | (v << np.uint32(28))


bits = 15
MUL = np.uint64(0x9E3779B1)
h_mix = lambda k: (k ^ (k >> np.uint32(16))).astype(np.uint64) * MUL
h_raw = lambda k: k.astype(np.uint64) * MUL


def two_word(h):
    lo = (h & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    hi = (h >> np.uint64(32)).astype(np.uint32)
    return [(hi >> np.uint32(32 - bits), mask(lo)), ((hi >> np.uint32(2)) & np.uint32((1 << bits) - 1), mask(rot4(lo)))]


run("2 words x 3 bits, premix", h_mix, bits, two_word)
run("2 words x 3 bits, no premix", h_raw, bits, two_word)


def fld(v, b):
    return np.uint32(1) << ((v >> np.uint32(8 * b)) & np.uint32(31))


def split_hl(h):
    return (h & np.uint64(0xFFFFFFFF)).astype(np.uint32), (h >> np.uint64(32)).astype(np.uint32)


def w22(h):   # 2 + 2 bits, fields = lo bytes 0..3
    lo, hi = split_hl(h)
    return [(hi >> np.uint32(32 - bits), fld(lo, 0) | fld(lo, 1)),
            ((hi >> np.uint32(2)) & np.uint32((1 << bits) - 1), fld(lo, 2) | fld(lo, 3))]


def w33h(h):  # 3 + 3 bits: word 1 from hi bytes 0,1 + lo byte 3; word 2 from lo bytes 0..2
    lo, hi = split_hl(h)
    return [(hi >> np.uint32(32 - bits), fld(hi, 0) | fld(hi, 1) | fld(lo, 3)),
            ((hi >> np.uint32(2)) & np.uint32((1 << bits) - 1), fld(lo, 0) | fld(lo, 1) | fld(lo, 2))]


def w32(h):   # 3 + 2 bits
    lo, hi = split_hl(h)
    return [(hi >> np.uint32(32 - bits), fld(hi, 0) | fld(hi, 1) | fld(lo, 3)),
            ((hi >> np.uint32(2)) & np.uint32((1 << bits) - 1), fld(lo, 0) | fld(lo, 1))]


run("2 words x 2 bits (lo bytes)", h_raw, bits, w22)
run("2 words x 3 bits (hi+lo bytes)", h_raw, bits, w33h)
run("3 + 2 bits (hi+lo bytes)", h_raw, bits, w32)

BYTEBIT = np.array([1 << i for i in range(8)], dtype=np.uint32)


def pmask(v):  # v_perm of one-bit bytes: byte i of the mask = 1 << (byte i of v & 7)
    out = np.zeros_like(v)
    for b in range(4):
        out |= BYTEBIT[(v >> np.uint32(8 * b)) & np.uint32(7)] << np.uint32(8 * b)
    return out


def wp_a(h):  # word1 = hi[31:17] mask(lo), word2 = lo[31:17] mask(hi)
    lo, hi = split_hl(h)
    return [(hi >> np.uint32(32 - bits), pmask(lo)), (lo >> np.uint32(32 - bits), pmask(hi))]


def wp_b(h):  # word1 = hi[16:2] mask(lo), word2 = hi[31:17] mask(lo >> 4)
    lo, hi = split_hl(h)
    return [((hi >> np.uint32(2)) & np.uint32((1 << bits) - 1), pmask(lo)),
            (hi >> np.uint32(32 - bits), pmask(lo >> np.uint32(4)))]


run("perm masks A (hi/lo addresses)", h_raw, bits, wp_a)
run("perm masks B (hi addresses)", h_raw, bits, wp_b)


def wp_a2(h):  # word1 = hi[16:2] mask(lo), word2 = lo[31:17] mask(hi)
    lo, hi = split_hl(h)
    return [((hi >> np.uint32(2)) & np.uint32((1 << bits) - 1), pmask(lo)), (lo >> np.uint32(32 - bits), pmask(hi))]


run("perm masks A' (hi[16:2] / lo[31:17])", h_raw, bits, wp_a2)
