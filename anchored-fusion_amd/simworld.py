"""Device-side synthetic world for BASELINE.json configs[2]-[4]: an hg38-scale genome with repeat
families, the anchored gene and its fusion partners embedded as exons, and 50 M distinct wgsim-style
2x150 pairs, all generated in HBM by libafsim.so (csrc/sim.hip).  Bench and test infrastructure: the
product path (libafgpu.so) never imports this module.

The reference benchmarks on `wgsim -d 200` reads of fusion transcripts (utils/simulate_reads.py:4-20)
aligned against hg38 (Anchored_Fusion.py:172-188).  Neither is available offline; this world keeps
the properties the hot path is sensitive to:

- contig sizes of hg38 chr1-22, X, Y (3.09 Gbp), telomere and centromere N gaps;
- repeats: Alu-, L1-, MIR-, L2-, LTR- and DNA-transposon-like families with subfamilies and per-copy
  divergence, simple tandem repeats, 171-bp satellite arrays around each centromere and 16 kb
  segmental duplications -- so 16-mer occurrence counts span 1 to 10^5 and placement hits the MEM cap
  and re-seeding paths as hg38's repeats would;
- the anchor (the bundled BCR transcript) as exons on chr22 near BCR's hg38 locus, 8 random partner
  genes as exons elsewhere, each carrying a diverged Alu-like copy in its 3' part (multi-mapping
  tails); fusion transcripts join an anchor exon end to a partner exon start, as real fusions do.
"""
import ctypes
import os

import numpy as np

from . import _lib

HERE = os.path.dirname(os.path.abspath(__file__))
SIM_PATH = os.path.join(HERE, "libafsim.so")
MAX_CTG, MAX_FAM = 64, 16

HG38 = [("chr1", 248956422), ("chr2", 242193529), ("chr3", 198295559), ("chr4", 190214555), ("chr5", 181538259),
        ("chr6", 170805979), ("chr7", 159345973), ("chr8", 145138636), ("chr9", 138394717), ("chr10", 133797422),
        ("chr11", 135086622), ("chr12", 133275309), ("chr13", 114364328), ("chr14", 107043718),
        ("chr15", 101991189), ("chr16", 90338345), ("chr17", 83257441), ("chr18", 80373285), ("chr19", 58617616),
        ("chr20", 64444167), ("chr21", 46709983), ("chr22", 50818468), ("chrX", 156040895), ("chrY", 57227415)]


class Family(ctypes.Structure):
    _fields_ = [("cons_off", ctypes.c_int32), ("cons_len", ctypes.c_int32), ("n_sub", ctypes.c_int32),
                ("min_len", ctypes.c_int32), ("max_len", ctypes.c_int32), ("kind", ctypes.c_int32),
                ("div_lo", ctypes.c_float), ("div_hi", ctypes.c_float), ("div_step", ctypes.c_float),
                ("prob", ctypes.c_float)]


class GenomeSpec(ctypes.Structure):
    _fields_ = [("n_ctg", ctypes.c_int32), ("n_fam", ctypes.c_int32), ("off", ctypes.c_int64 * MAX_CTG),
                ("len", ctypes.c_int64 * MAX_CTG), ("fam", Family * MAX_FAM), ("sat_off", ctypes.c_int32),
                ("sat_len", ctypes.c_int32), ("telomere", ctypes.c_int32), ("cen_gap", ctypes.c_int32),
                ("sat_flank", ctypes.c_int32), ("cen_at", ctypes.c_float), ("segdup_prob", ctypes.c_float),
                ("gc", ctypes.c_float), ("seed", ctypes.c_uint64)]


class ReadSpec(ctypes.Structure):
    _fields_ = [("genome", ctypes.c_void_p), ("n_genome", ctypes.c_int64), ("n_ctg", ctypes.c_int32),
                ("off", ctypes.c_int64 * MAX_CTG), ("len", ctypes.c_int64 * MAX_CTG),
                ("cum", ctypes.c_int64 * (MAX_CTG + 1)), ("tx", ctypes.c_void_p), ("tx_off", ctypes.c_void_p),
                ("tx_cum", ctypes.c_void_p), ("n_tx", ctypes.c_int32), ("L", ctypes.c_int32),
                ("fusion_frac", ctypes.c_float), ("frag_mean", ctypes.c_float), ("frag_sd", ctypes.c_float),
                ("err", ctypes.c_float), ("indel_frac", ctypes.c_float), ("n_rate", ctypes.c_float),
                ("seed", ctypes.c_uint64), ("pair_base", ctypes.c_int64)]


_S = None


def simlib():
    global _S
    if _S is None:
        if not os.path.exists(SIM_PATH):
            raise _lib.AFError(f"{SIM_PATH} is missing: run __graft_entry__.build()")
        S = ctypes.CDLL(SIM_PATH)
        S.afs_genome.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(GenomeSpec), ctypes.c_void_p,
                                 ctypes.c_void_p]
        S.afs_pairs.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(ReadSpec), ctypes.c_void_p,
                                ctypes.c_void_p]
        S.afs_spec_sizes.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        g, r = ctypes.c_int32(), ctypes.c_int32()
        S.afs_spec_sizes(ctypes.byref(g), ctypes.byref(r))
        if (g.value, r.value) != (ctypes.sizeof(GenomeSpec), ctypes.sizeof(ReadSpec)):
            raise _lib.AFError(f"libafsim struct sizes {g.value}/{r.value} != binding "
                               f"{ctypes.sizeof(GenomeSpec)}/{ctypes.sizeof(ReadSpec)}")
        _S = S
    return _S


_BASES = np.frombuffer(b"ACGT", np.uint8)

# (name, consensus length, subfamilies, copy length range, divergence lo/hi, step per subfamily,
#  slot probability, kind)
FAMILIES = [
    ("Alu", 300, 4, (120, 300), (0.02, 0.10), 0.03, 0.36, 0),
    ("L1", 6000, 4, (150, 1000), (0.03, 0.12), 0.04, 0.17, 0),
    ("MIR", 260, 2, (80, 260), (0.22, 0.30), 0.0, 0.06, 0),
    ("L2", 3000, 2, (100, 800), (0.24, 0.34), 0.0, 0.05, 0),
    ("LTR", 500, 3, (150, 500), (0.08, 0.18), 0.03, 0.05, 0),
    ("DNA", 1000, 2, (100, 900), (0.15, 0.25), 0.0, 0.04, 0),
    ("simple", 1, 1, (20, 90), (0.0, 0.0), 0.0, 0.08, 1),
]
SAT_LEN = 171


def repeat_library(seed=20251015):
    """Consensus sequences (codes 0-3): per family `n_sub` subfamilies diverged 6 % apart from a
    random root, then the satellite monomer.  Returns (codes uint8, [Family], sat_off)."""
    rng = np.random.default_rng([seed, 1])  # its own stream: the genes must not copy the consensi
    parts, fams, off = [], [], 0
    for name, clen, nsub, (lo, hi), (dlo, dhi), step, prob, kind in FAMILIES:
        root = rng.integers(0, 4, clen, dtype=np.uint8)
        for k in range(nsub):
            s = root.copy()
            m = rng.random(clen) < 0.06 * k
            s[m] = (s[m] + rng.integers(1, 4, int(m.sum()), dtype=np.uint8)) % 4
            parts.append(s)
        fams.append(Family(off, clen, nsub, lo, min(hi, clen) if kind == 0 else hi, kind, dlo, dhi, step, prob))
        off += clen * nsub
    sat = rng.integers(0, 4, SAT_LEN, dtype=np.uint8)
    parts.append(sat)
    return np.concatenate(parts), fams, off


def _exons(rng, seq_len, lo=80, hi=250):
    """Exon lengths covering a transcript of seq_len bases."""
    out, left = [], seq_len
    while left > 0:
        e = int(rng.integers(lo, hi + 1))
        if left - e < lo:
            e = left
        out.append(e)
        left -= e
    return out


def _mutate(rng, codes, d):
    s = codes.copy()
    m = rng.random(len(s)) < d
    s[m] = (s[m] + rng.integers(1, 4, int(m.sum()), dtype=np.uint8)) % 4
    return s


class GenomeWorld:
    """The configs[2] world in HBM.  `blob` (torch uint8 tensor) is the joined genome (contigs with
    place.SEP N's between them; the indexes read the contigs at `offsets`); `loci[name]` lists each embedded
    gene's exons as (contig, start, end) 0-based; `fusions` the fusion transcripts with their
    junctions (anchor exon end, partner exon start)."""

    def __init__(self, anchor: bytes, device=0, seed=20251015, scale=1.0, n_partners=8):
        import torch

        from . import place
        self.device = device
        dev = torch.device("cuda", device)
        rng = np.random.default_rng([seed, 2])
        self.contigs = [(n, max(1 << 20, int(L * scale))) for n, L in HG38]
        self.names = [n for n, _ in self.contigs]
        self.lens = [L for _, L in self.contigs]
        self.offsets, off = [], 0
        for k, L in enumerate(self.lens):
            if k:
                off += place.SEP
            self.offsets.append(off)
            off += L
        self.total = off
        codes, fams, sat_off = repeat_library(seed)
        self.lib_codes = codes
        spec = GenomeSpec()
        spec.n_ctg, spec.n_fam = len(self.lens), len(fams)
        for k in range(len(self.lens)):
            spec.off[k], spec.len[k] = self.offsets[k], self.lens[k]
        for k, f in enumerate(fams):
            spec.fam[k] = f
        spec.sat_off, spec.sat_len = sat_off, SAT_LEN
        spec.telomere = min(10000, self.lens[-1] // 64)
        spec.cen_gap, spec.sat_flank = int(300_000 * min(1.0, scale)), int(150_000 * min(1.0, scale))
        spec.cen_at, spec.segdup_prob, spec.gc, spec.seed = 0.4, 0.035, 0.41, seed
        self.spec = spec
        lib_t = torch.from_numpy(codes).to(dev)
        self.blob = torch.empty(self.total, dtype=torch.uint8, device=dev)
        s = torch.cuda.current_stream(dev)
        rc = simlib().afs_genome(self.blob.data_ptr(), self.total, ctypes.byref(spec), lib_t.data_ptr(), s.cuda_stream)
        if rc:
            raise _lib.AFError(f"afs_genome failed (hipError {rc})")
        torch.cuda.synchronize(dev)
        del lib_t
        # genes: the anchor on chr22 (BCR's hg38 neighbourhood), partners on other chromosomes
        anchor = bytes(anchor).upper()
        alu = codes[fams[0].cons_off:fams[0].cons_off + fams[0].cons_len]
        self.partners = []
        for k in range(n_partners):
            body = rng.integers(0, 4, int(rng.integers(1500, 4000)), dtype=np.uint8)
            cut = int(len(body) * 0.7)
            rep = _mutate(rng, alu, 0.10)
            body = np.concatenate([body[:cut], rep, body[cut:]])
            self.partners.append(_BASES[body].tobytes())
        genes = [("anchor", "chr22", int(23_180_000 * min(1.0, scale)), anchor)]
        hosts = ["chr9", "chr1", "chr2", "chr3", "chr5", "chr7", "chr11", "chr12", "chr17", "chr4"]
        for k, p in enumerate(self.partners):
            c = hosts[k % len(hosts)]
            L = self.lens[self.names.index(c)]
            genes.append((f"partner{k}", c, int(L * (0.55 + 0.03 * k)), p))
        self.loci, self.exon_ends = {}, {}
        for gname, c, start, seq in genes:
            ci = self.names.index(c)
            ex, pos, cur = _exons(rng, len(seq)), start, 0
            spans, ends = [], []
            for e in ex:
                a = self.offsets[ci] + pos
                self.blob[a:a + e] = torch.from_numpy(np.frombuffer(seq[cur:cur + e], np.uint8).copy()).to(dev)
                spans.append((c, pos, pos + e))
                cur += e
                ends.append(cur)
                pos += e + int(rng.integers(300, 3000))
            self.loci[gname] = spans
            self.exon_ends[gname] = ends
        self.anchor = anchor
        # fusion transcripts: anchor exons 1..i joined to partner exons j..
        self.fusions, self.junctions = [], []
        ae = self.exon_ends["anchor"]
        for k, p in enumerate(self.partners):
            a = ae[int(rng.integers(len(ae) // 4, max(len(ae) // 4 + 1, 3 * len(ae) // 4)))]
            pe = [0] + self.exon_ends[f"partner{k}"][:-1]
            b = pe[int(rng.integers(1, max(2, len(pe) - 2)))]
            self.fusions.append(anchor[:a] + p[b:])
            self.junctions.append((a, b))
        torch.cuda.synchronize(dev)

    def contig_list(self):
        """(name, length) per contig."""
        return list(zip(self.names, self.lens))

    def genome_index(self):
        """genome.GenomeIndex (`bwa index`, csrc/fmindex.hip) over the contigs in HBM."""
        from .genome import GenomeIndex
        return GenomeIndex.from_device(self.blob, self.names, self.offsets, self.lens, device=self.device)

    def tiles(self, step_size=11):
        """blat.TileReference over the genome in HBM (af_tile_index_build_device)."""
        from . import blat
        return blat.TileReference.from_device(self.blob, self.names, self.lens, self.offsets, step_size,
                                              device=self.device)

    def simulate_pairs(self, n_pairs, read_len=150, seed=20251015, fusion_frac=0.05, frag_mean=200, frag_sd=20,
                       err=0.02, indel_frac=0.01, n_rate=0.0005, pair_base=0, out=None, src=None):
        """n_pairs distinct pairs into out (torch uint8 [2 n_pairs, read_len] on the device; made if
        None).  src (optional int32 [n_pairs]): fusion transcript index, len(fusions) + contig, or -1."""
        import torch
        dev = torch.device("cuda", self.device)
        if out is None:
            out = torch.empty((2 * n_pairs, read_len), dtype=torch.uint8, device=dev)
        if tuple(out.shape) != (2 * n_pairs, read_len) or not out.is_contiguous():
            raise ValueError("out must be a contiguous [2 n_pairs, read_len] tensor")
        if not hasattr(self, "_tx"):
            tx = b"".join(self.fusions)
            toff = np.concatenate([[0], np.cumsum([len(t) for t in self.fusions])]).astype(np.int64)
            w = np.array([len(t) for t in self.fusions], np.float64)
            cum = np.cumsum(w / w.sum())
            cum[-1] = 1.0
            self._tx = (torch.from_numpy(np.frombuffer(tx, np.uint8).copy()).to(dev), torch.from_numpy(toff).to(dev),
                        torch.from_numpy(cum).to(dev))
        tx_t, toff_t, cum_t = self._tx
        r = ReadSpec()
        r.genome, r.n_genome, r.n_ctg = self.blob.data_ptr(), self.total, len(self.lens)
        c = 0
        for k in range(len(self.lens)):
            r.off[k], r.len[k], r.cum[k] = self.offsets[k], self.lens[k], c
            c += self.lens[k]
        r.cum[len(self.lens)] = c
        r.tx, r.tx_off, r.tx_cum, r.n_tx, r.L = tx_t.data_ptr(), toff_t.data_ptr(), cum_t.data_ptr(), len(self.fusions), \
            read_len
        r.fusion_frac, r.frag_mean, r.frag_sd = fusion_frac, frag_mean, frag_sd
        r.err, r.indel_frac, r.n_rate, r.seed, r.pair_base = err, indel_frac, n_rate, seed, pair_base
        s = torch.cuda.current_stream(dev)
        rc = simlib().afs_pairs(out.data_ptr(), n_pairs, ctypes.byref(r), None if src is None else src.data_ptr(),
                                s.cuda_stream)
        if rc:
            raise _lib.AFError(f"afs_pairs failed (hipError {rc})")
        return out

    def host_contigs(self):
        """[(name, str)] copied to the host (tests at reduced scale only)."""
        b = self.blob.cpu().numpy().tobytes()
        return [(n, b[o:o + L].decode()) for n, o, L in zip(self.names, self.offsets, self.lens)]
