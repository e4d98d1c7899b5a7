"""TEST INFRASTRUCTURE ONLY -- ctypes binding of the CPU oracle (oracle/af_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module.  The product path (anchored-fusion_amd/) never loads it.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libafo.so")
MAX_CIGAR = 32
FLAG_MEM_OVERFLOW = 0x10000
FLAG_CIGAR_OVERFLOW = 0x20000


class Params(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "a", "b", "o_del", "e_del", "o_ins", "e_ins", "pen_clip5", "pen_clip3", "w", "zdrop",
        "min_seed_len", "max_occ", "T", "max_ext", "max_mems")]


class Pe(ctypes.Structure):
    """bwa mem paired-end options + the batch's place in bwa's input stream (afo_pe)."""
    _fields_ = [("pen_unpaired", ctypes.c_int32), ("max_ins", ctypes.c_int32), ("max_matesw", ctypes.c_int32),
                ("split_width", ctypes.c_int32), ("max_mem_intv", ctypes.c_int32), ("max_chain_gap", ctypes.c_int32),
                ("chunk_bases", ctypes.c_int64), ("pair_base", ctypes.c_int64)]


class _Out(ctypes.Structure):
    _fields_ = [("flag", ctypes.c_void_p), ("pos", ctypes.c_void_p), ("score", ctypes.c_void_p),
                ("n_cigar", ctypes.c_void_p), ("hits", ctypes.c_void_p), ("cigar", ctypes.c_void_p)]


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        L.afo_index_build.restype = ctypes.c_void_p
        L.afo_index_build.argtypes = [ctypes.c_char_p, ctypes.c_int64]
        L.afo_index_free.argtypes = [ctypes.c_void_p]
        L.afo_filter_words.restype = ctypes.c_int32
        L.afo_filter_words.argtypes = [ctypes.c_void_p]
        L.afo_filter_table.restype = ctypes.c_void_p
        L.afo_filter_table.argtypes = [ctypes.c_void_p]
        L.afo_params_default.argtypes = [ctypes.POINTER(Params)]
        L.afo_seed_filter.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                      ctypes.c_void_p, ctypes.c_void_p]
        L.afo_align_pairs.restype = ctypes.c_int
        L.afo_align_pairs.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                      ctypes.c_void_p, ctypes.POINTER(Params), ctypes.POINTER(Pe), ctypes.c_int,
                                      ctypes.POINTER(_Out)]
        L.afo_pe_default.argtypes = [ctypes.POINTER(Pe)]
        _lib = L
    return _lib


def default_params():
    p = Params()
    lib().afo_params_default(ctypes.byref(p))
    return p


def default_pe(**kw):
    pe = Pe()
    lib().afo_pe_default(ctypes.byref(pe))
    for k, v in kw.items():
        setattr(pe, k, v)
    return pe


class OracleIndex:
    def __init__(self, anchor: bytes):
        self.anchor = bytes(anchor)
        self.h = lib().afo_index_build(self.anchor, len(self.anchor))
        if not self.h:
            raise ValueError("empty anchor")

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.afo_index_free(self.h)
            self.h = None

    def filter_table(self):
        nw = lib().afo_filter_words(self.h)
        ptr = lib().afo_filter_table(self.h)
        return np.ctypeslib.as_array((ctypes.c_uint32 * nw).from_address(ptr)).copy()

    def seed_filter(self, reads, lens=None):
        reads = np.ascontiguousarray(reads, dtype=np.uint8)
        n = reads.shape[0]
        hits = np.zeros(n, dtype=np.int32)
        lp = None if lens is None else np.ascontiguousarray(lens, dtype=np.int32)
        lib().afo_seed_filter(self.h, reads.ctypes.data, n, reads.shape[1],
                              None if lp is None else lp.ctypes.data, hits.ctypes.data)
        return hits

    def align_pairs(self, reads, lens=None, params=None, threads=0, pe=None, pair_base=None, chunk_bases=None):
        """bwa mem -M paired-end restatement (bwa_pe.c).  reads: [2N, stride] uint8 pair-major,
        starting at a bwa chunk boundary; pair_base = global index of the first pair.
        Returns a dict of per-read arrays (one primary record per read)."""
        reads = np.ascontiguousarray(reads, dtype=np.uint8)
        nr = reads.shape[0]
        assert nr % 2 == 0
        out = {k: np.zeros(nr, dtype=np.int32) for k in ("flag", "pos", "score", "n_cigar", "hits")}
        out["cigar"] = np.zeros((nr, MAX_CIGAR), dtype=np.uint32)
        o = _Out(*(out[k].ctypes.data for k in ("flag", "pos", "score", "n_cigar", "hits", "cigar")))
        p = params or default_params()
        e = pe or default_pe()
        if pair_base is not None:
            e.pair_base = int(pair_base)
        if chunk_bases is not None:
            e.chunk_bases = int(chunk_bases)
        lp = None if lens is None else np.ascontiguousarray(lens, dtype=np.int32)
        rc = lib().afo_align_pairs(self.h, reads.ctypes.data, nr // 2, reads.shape[1],
                                   None if lp is None else lp.ctypes.data, ctypes.byref(p), ctypes.byref(e),
                                   int(threads), ctypes.byref(o))
        if rc != 0:
            raise RuntimeError(f"afo_align_pairs failed: {rc}")
        return out


PSL_DTYPE = np.dtype([(n, "<i4") for n in (
    "query", "strand", "score", "matches", "mismatches", "n_count", "q_num_insert", "q_base_insert", "t_num_insert",
    "t_base_insert", "q_start", "q_end", "q_size", "block_count")] + [
    ("t_start", "<i8"), ("t_end", "<i8"), ("block_sizes", "<i4", (16,)), ("q_starts", "<i4", (16,)),
    ("t_starts", "<i8", (16,))])
assert PSL_DTYPE.itemsize == 328


class BlatParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ("step_size", "min_match", "rep_match", "min_score", "min_identity",
                                                "max_gap", "max_intron")]


def blat_params(**kw):
    L = lib()
    L.afo_blat_params_default.argtypes = [ctypes.POINTER(BlatParams)]
    p = BlatParams()
    L.afo_blat_params_default(ctypes.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


BLOCK_DTYPE = np.dtype([("size", "<i4"), ("q_start", "<i4"), ("t_start", "<i8")])  # afo_psl_block


class OracleTiles:
    """BLAT restatement (blat.c): the tile index of `seq` and its searches."""

    def __init__(self, seq: bytes, step_size=11):
        L = lib()
        L.afo_tiles_build.restype = ctypes.c_void_p
        L.afo_tiles_build.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_int32]
        L.afo_tiles_free.argtypes = [ctypes.c_void_p]
        L.afo_blat_caps.restype = ctypes.c_int
        L.afo_blat_caps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p,
                                    ctypes.POINTER(BlatParams), ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_int, ctypes.c_void_p]
        self.caps = np.zeros(4, np.int32)  # af_blat_caps' counters, cumulative (caps_read resets)
        self.seq = bytes(seq)
        self.step = int(step_size)
        self.h = L.afo_tiles_build(self.seq, len(self.seq), self.step)
        if not self.h:
            raise ValueError("reference shorter than a tile or bad step")

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.afo_tiles_free(self.h)
            self.h = None

    def blat(self, queries, lens=None, params=None, max_rows=16, threads=0):
        """(rows [n, max_rows] PSL_DTYPE, n_rows [n])."""
        q = np.ascontiguousarray(queries, dtype=np.uint8)
        n = q.shape[0]
        rows = np.zeros((n, max_rows), dtype=PSL_DTYPE)
        nr = np.zeros(n, dtype=np.int32)
        p = params or blat_params(step_size=self.step)
        lp = None if lens is None else np.ascontiguousarray(lens, dtype=np.int32)
        rc = lib().afo_blat_caps(self.h, q.ctypes.data, n, q.shape[1], None if lp is None else lp.ctypes.data,
                                 ctypes.byref(p), max_rows, rows.ctypes.data, nr.ctypes.data, int(threads),
                                 self.caps.ctypes.data)
        if rc != 0:
            raise RuntimeError(f"afo_blat failed: {rc}")
        return rows, nr

    def blat_long(self, query, params=None, max_rows=4096):
        """afo_blat_long: one long query searched whole -> (rows [k] PSL_DTYPE, n_rows (all rows),
        blocks [m] BLOCK_DTYPE, block_off [k + 1]): row i's blocks are blocks[off[i]:off[i + 1]]."""
        L = lib()
        L.afo_blat_long.restype = ctypes.c_int
        L.afo_blat_long.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int32, ctypes.POINTER(BlatParams),
                                    ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        q = bytes(query)
        p = params or blat_params(step_size=self.step)
        rows = np.zeros(max_rows, dtype=PSL_DTYPE)
        nr = np.zeros(1, np.int32)
        off = np.zeros(max_rows + 1, np.int64)
        nb = np.zeros(1, np.int64)
        cap, caps0 = 1 << 16, self.caps.copy()
        while True:
            self.caps[:] = caps0  # a rerun with a larger block arena counts the caps once
            blocks = np.zeros(cap, dtype=BLOCK_DTYPE)
            rc = L.afo_blat_long(self.h, q, len(q), ctypes.byref(p), max_rows, rows.ctypes.data, nr.ctypes.data,
                                 blocks.ctypes.data, cap, off.ctypes.data, nb.ctypes.data, self.caps.ctypes.data)
            if rc == -3:
                cap = int(nb[0])
                continue
            if rc != 0:
                raise RuntimeError(f"afo_blat_long failed: {rc}")
            k = min(int(nr[0]), max_rows)
            return rows[:k].copy(), int(nr[0]), blocks[:int(off[k])].copy(), off[:k + 1].copy()

    def caps_read(self, reset=True):
        out = self.caps.copy()
        if reset:
            self.caps[:] = 0
        return out


# ---- the genome calls S4 / S5 (bwa_pe.c, FM mode) ---------------------------------------
G_MAX_REC = 8
GREC_DTYPE = np.dtype([("read", "<i4"), ("flag", "<i4"), ("rid", "<i4"), ("mrid", "<i4"), ("pos", "<i8"),
                       ("mpos", "<i8"), ("score", "<i4"), ("n_cigar", "<i4"), ("seq_b", "<i4"), ("seq_e", "<i4"),
                       ("cigar", "<u4", (MAX_CIGAR,))])
assert GREC_DTYPE.itemsize == 176
REG_DTYPE = np.dtype([("rb", "<i8"), ("re", "<i8"), ("qb", "<i4"), ("qe", "<i4"), ("rid", "<i4"), ("score", "<i4"),
                      ("truesc", "<i4"), ("w", "<i4"), ("seedcov", "<i4"), ("seedlen0", "<i4")])
assert REG_DTYPE.itemsize == 48


def _glib():
    L = lib()
    if not getattr(L, "_genome_bound", False):
        vp, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
        L.afo_genome_build.restype = vp
        L.afo_genome_build.argtypes = [ctypes.c_char_p, vp, vp, ctypes.c_int, ctypes.c_int]
        L.afo_genome_free.argtypes = [vp]
        L.afo_genome_lpac.restype = i64
        L.afo_genome_lpac.argtypes = [vp]
        L.afo_genome_text.restype = vp
        L.afo_genome_text.argtypes = [vp]
        L.afo_genome_sa.restype = vp
        L.afo_genome_sa.argtypes = [vp]
        L.afo_genome_primary.restype = i64
        L.afo_genome_primary.argtypes = [vp]
        L.afo_genome_seeds.restype = ctypes.c_int
        L.afo_genome_seeds.argtypes = [vp, vp, i32, ctypes.POINTER(Params), ctypes.POINTER(Pe), ctypes.c_int, vp, vp,
                                       vp, i32]
        L.afo_genome_intervals.restype = ctypes.c_int
        L.afo_genome_intervals.argtypes = [vp, vp, i64, i32, vp, ctypes.POINTER(Params), ctypes.POINTER(Pe),
                                           ctypes.c_int, i32, vp, vp]
        L.afo_genome_regions.restype = ctypes.c_int
        L.afo_genome_regions.argtypes = [vp, vp, i64, i32, vp, ctypes.POINTER(Params), ctypes.POINTER(Pe),
                                         ctypes.c_int, i32, vp, vp]
        L.afo_genome_align_se.restype = ctypes.c_int
        L.afo_genome_align_se.argtypes = [vp, vp, i64, i32, vp, ctypes.POINTER(Params), ctypes.POINTER(Pe), i64,
                                          ctypes.c_int, i32, vp, vp]
        L.afo_genome_align_se_ids.restype = ctypes.c_int
        L.afo_genome_align_se_ids.argtypes = [vp, vp, i64, i32, vp, ctypes.POINTER(Params), ctypes.POINTER(Pe), vp,
                                              ctypes.c_int, i32, vp, vp]
        L.afo_genome_align_pe.restype = ctypes.c_int
        L.afo_genome_align_pe.argtypes = [vp, vp, i64, i32, vp, ctypes.POINTER(Params), ctypes.POINTER(Pe),
                                          ctypes.c_int, i32, vp, vp]
        L._genome_bound = True
    return L


class OracleGenome:
    """bwa's index of a multi-contig genome (bns_fasta2bntseq + the FM index) and the genome calls
    S4 (`bwa mem -M genome fq1 fq2`, AF:188) and S5 (`bwa mem -M genome reads.fa`, fn:716).

    contigs: [(name, seq)].  memset_too: also build the MEM-set seeding structures (the anchor's
    restatement) for the seed cross-check."""

    def __init__(self, contigs, memset_too=False):
        self.names = [n for n, _ in contigs]
        self.lens = [len(s) for _, s in contigs]
        blob = b"".join(s.encode() if isinstance(s, str) else bytes(s) for _, s in contigs)
        off = np.concatenate([[0], np.cumsum(self.lens)[:-1]]).astype(np.int64)
        ln = np.asarray(self.lens, dtype=np.int64)
        self._blob = blob
        self.h = _glib().afo_genome_build(blob, off.ctypes.data, ln.ctypes.data, len(contigs), int(bool(memset_too)))
        if not self.h:
            raise ValueError("empty genome")
        self.l_pac = int(_glib().afo_genome_lpac(self.h))

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.afo_genome_free(self.h)
            self.h = None

    def text(self):
        p = _glib().afo_genome_text(self.h)
        return np.ctypeslib.as_array((ctypes.c_uint8 * (2 * self.l_pac)).from_address(p)).copy()

    def sa(self):
        p = _glib().afo_genome_sa(self.h)
        return np.ctypeslib.as_array((ctypes.c_int64 * (2 * self.l_pac + 1)).from_address(p)).copy()

    def primary(self):
        return int(_glib().afo_genome_primary(self.h))

    def seeds(self, read, params=None, pe=None, memset=False, cap=1 << 16):
        """mem_chain's seed walk for one read: (rbeg int64, qbeg, len) arrays."""
        r = np.frombuffer(read.encode() if isinstance(read, str) else bytes(read), dtype=np.uint8).copy()
        rb = np.zeros(cap, np.int64)
        qb = np.zeros(cap, np.int32)
        ln = np.zeros(cap, np.int32)
        n = _glib().afo_genome_seeds(self.h, r.ctypes.data, len(r), ctypes.byref(params or default_params()),
                                     ctypes.byref(pe or default_pe()), int(memset), rb.ctypes.data, qb.ctypes.data,
                                     ln.ctypes.data, cap)
        if n < 0:
            raise OverflowError(f"afo_genome_seeds: {n}")
        return rb[:n], qb[:n], ln[:n]

    def intervals(self, reads, lens=None, params=None, pe=None, max_iv=512, threads=0):
        """mem_collect_intv per read: int64 [n, max_iv, 4] {sa_k, s, qb, qe} in mem_chain's order,
        counts [n] (-1: past the interval cap)."""
        reads = np.ascontiguousarray(reads, dtype=np.uint8)
        n = reads.shape[0]
        out = np.zeros((n, max_iv, 4), np.int64)
        niv = np.zeros(n, np.int32)
        lp = None if lens is None else np.ascontiguousarray(lens, dtype=np.int32)
        rc = _glib().afo_genome_intervals(self.h, reads.ctypes.data, n, reads.shape[1],
                                          None if lp is None else lp.ctypes.data,
                                          ctypes.byref(params or default_params()), ctypes.byref(pe or default_pe()),
                                          int(threads), max_iv, out.ctypes.data, niv.ctypes.data)
        if rc != 0:
            raise RuntimeError(f"afo_genome_intervals failed: {rc}")
        return out, niv

    def regions(self, reads, lens=None, params=None, pe=None, max_reg=64, threads=0):
        reads = np.ascontiguousarray(reads, dtype=np.uint8)
        n = reads.shape[0]
        regs = np.zeros((n, max_reg), dtype=REG_DTYPE)
        nreg = np.zeros(n, dtype=np.int32)
        lp = None if lens is None else np.ascontiguousarray(lens, dtype=np.int32)
        rc = _glib().afo_genome_regions(self.h, reads.ctypes.data, n, reads.shape[1], None if lp is None else lp.ctypes.data,
                                        ctypes.byref(params or default_params()), ctypes.byref(pe or default_pe()),
                                        int(threads), max_reg, regs.ctypes.data, nreg.ctypes.data)
        if rc != 0:
            raise RuntimeError(f"afo_genome_regions failed: {rc}")
        return regs, nreg

    def align_se(self, reads, lens=None, params=None, pe=None, id_base=0, threads=0, max_rec=G_MAX_REC, ids=None):
        """S5: (records [n, max_rec] GREC_DTYPE, counts [n]); read ids id_base + r, or ids[r]."""
        reads = np.ascontiguousarray(reads, dtype=np.uint8)
        n = reads.shape[0]
        recs = np.zeros((n, max_rec), dtype=GREC_DTYPE)
        nrec = np.zeros(n, dtype=np.int32)
        lp = None if lens is None else np.ascontiguousarray(lens, dtype=np.int32)
        if ids is not None:
            ids = np.ascontiguousarray(ids, dtype=np.int64)
            rc = _glib().afo_genome_align_se_ids(self.h, reads.ctypes.data, n, reads.shape[1],
                                                 None if lp is None else lp.ctypes.data,
                                                 ctypes.byref(params or default_params()),
                                                 ctypes.byref(pe or default_pe()), ids.ctypes.data, int(threads),
                                                 max_rec, recs.ctypes.data, nrec.ctypes.data)
        else:
            rc = _glib().afo_genome_align_se(self.h, reads.ctypes.data, n, reads.shape[1],
                                             None if lp is None else lp.ctypes.data,
                                             ctypes.byref(params or default_params()),
                                             ctypes.byref(pe or default_pe()), int(id_base), int(threads), max_rec,
                                             recs.ctypes.data, nrec.ctypes.data)
        if rc != 0:
            raise RuntimeError(f"afo_genome_align_se failed: {rc}")
        return recs, nrec

    def align_pe(self, reads, lens=None, params=None, pe=None, pair_base=None, chunk_bases=None, threads=0,
                 max_rec=G_MAX_REC):
        """S4 on pair-major reads [2N, stride]: (records [2N, max_rec] GREC_DTYPE, counts [2N])."""
        reads = np.ascontiguousarray(reads, dtype=np.uint8)
        nr = reads.shape[0]
        assert nr % 2 == 0
        recs = np.zeros((nr, max_rec), dtype=GREC_DTYPE)
        nrec = np.zeros(nr, dtype=np.int32)
        e = pe or default_pe()
        if pair_base is not None:
            e.pair_base = int(pair_base)
        if chunk_bases is not None:
            e.chunk_bases = int(chunk_bases)
        lp = None if lens is None else np.ascontiguousarray(lens, dtype=np.int32)
        rc = _glib().afo_genome_align_pe(self.h, reads.ctypes.data, nr // 2, reads.shape[1],
                                         None if lp is None else lp.ctypes.data, ctypes.byref(params or default_params()),
                                         ctypes.byref(e), int(threads), max_rec, recs.ctypes.data, nrec.ctypes.data)
        if rc != 0:
            raise RuntimeError(f"afo_genome_align_pe failed: {rc}")
        return recs, nrec
