"""ctypes binding of libafgpu.so (include/afgpu.h).

The library is built in-tree (``csrc/Makefile`` -> ``anchored-fusion_amd/libafgpu.so``) and
loaded from there, so the GPU box sees exactly the code object that ``build()`` produced.
There is no CPU fallback: if the library is missing or no GPU is present, calls raise.

torch is imported first when available so that a process using both torch and this library
shares one HIP runtime (both link ``libamdhip64.so.7``).
"""
import ctypes
import os
import subprocess

try:  # one HIP runtime per process (see module docstring)
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the host-buffer API
    torch = None

HERE = os.path.dirname(os.path.abspath(__file__))
# AF_GPU_LIB selects an in-tree build variant (e.g. libafgpu_prof.so for scripts/s2_prof.py)
LIB_PATH = os.path.join(HERE, os.environ.get("AF_GPU_LIB", "libafgpu.so"))
CSRC = os.path.join(HERE, "csrc")

AF_OK = 0
AF_E_INVALID, AF_E_HIP, AF_E_CAPACITY, AF_E_NOMEM, AF_E_UNSUPPORTED = -1, -2, -3, -4, -5
AF_BLAT_LONG_MAX = 131072
AF_MAX_CIGAR = 32
AF_MAX_READ = 320
AF_K = 16
AF_FLAG_MEM_OVERFLOW = 0x10000
AF_FLAG_CIGAR_OVERFLOW = 0x20000
AF_GATHER_SEQUENCED, AF_GATHER_SPLIT_SAM = 0, 1

# every symbol include/afgpu.h declares (checked by tests/test_abi.py)
EXPORTS = (
    "af_ctx_create", "af_ctx_destroy", "af_last_error", "af_params_default", "af_pe_default", "af_index_build",
    "af_index_free", "af_index_anchor_len", "af_index_filter_words", "af_index_filter_table",
    "af_align_pairs", "af_align_pairs_device", "af_seed_filter_device", "af_align_candidates_device",
    "af_last_candidates", "af_split_tails_device", "af_partition_device", "af_align_candidates_tails_device", "af_gather_reads_device", "af_blat_params_default", "af_tile_index_build",
    "af_tile_index_build_device", "af_blat", "af_blat_device", "af_blat_device_range", "af_fastq_open", "af_fastq_next", "af_fastq_export", "af_fastq_error",
    "af_fastq_close", "af_fastq_part_read", "af_fastq_part_export", "af_fastq_part_error", "af_fastq_part_free",
    "af_genome_build", "af_genome_build_device", "af_genome_free", "af_genome_lpac",
    "af_genome_primary", "af_genome_read", "af_genome_align_se_device", "af_genome_align_pe_device",
    "af_genome_align_se", "af_genome_align_pe", "af_genome_regions", "af_genome_stats", "af_s5_filter_device",
    "af_genome_align_se_ids_device", "af_genome_align_pe_se_device", "af_genome_intervals", "af_s5_rules_host", "af_blat_caps", "af_blat_spill",
    "af_blat_query_caps", "af_s6_queries_device", "af_s6_check_device", "af_s6_compact_device",
    "af_blat_device_begin", "af_blat_device_end", "af_blat_long", "af_blat_heavy_stats",
)
AF_G_MAX_REC = 8
AF_GSTAT_N = 4


class AFError(RuntimeError):
    pass


class Params(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "a", "b", "o_del", "e_del", "o_ins", "e_ins", "pen_clip5", "pen_clip3", "w", "zdrop",
        "min_seed_len", "max_occ", "T", "max_ext", "max_mems")]


class Pe(ctypes.Structure):
    """af_pe: bwa mem paired-end options and the batch's place in bwa's input stream."""
    _fields_ = [("pen_unpaired", ctypes.c_int32), ("max_ins", ctypes.c_int32), ("max_matesw", ctypes.c_int32),
                ("split_width", ctypes.c_int32), ("max_mem_intv", ctypes.c_int32), ("max_chain_gap", ctypes.c_int32),
                ("chunk_bases", ctypes.c_int64), ("pair_base", ctypes.c_int64)]


class AlnOut(ctypes.Structure):
    _fields_ = [("flag", ctypes.c_void_p), ("pos", ctypes.c_void_p), ("score", ctypes.c_void_p),
                ("n_cigar", ctypes.c_void_p), ("hits", ctypes.c_void_p), ("cigar", ctypes.c_void_p)]


class S6Set(ctypes.Structure):
    """af_s6_set: S6 query rows with their BLAT rows, spill pool and per-query cap counters."""
    _fields_ = [("q", ctypes.c_void_p), ("stride", ctypes.c_int32), ("pad0", ctypes.c_int32),
                ("lens", ctypes.c_void_p), ("src", ctypes.c_void_p), ("n", ctypes.c_void_p), ("over", ctypes.c_void_p),
                ("n_over", ctypes.c_void_p), ("rows", ctypes.c_void_p), ("n_rows", ctypes.c_void_p),
                ("caps", ctypes.c_void_p), ("spill_rows", ctypes.c_void_p), ("spill_query", ctypes.c_void_p),
                ("spill_n", ctypes.c_void_p), ("spill_cap", ctypes.c_int64), ("cap", ctypes.c_int64)]


def build(force=False):
    """Compiles libafgpu.so for gfx950 (hipcc cross-compiles without a GPU)."""
    if force and os.path.exists(LIB_PATH):
        os.remove(LIB_PATH)
    subprocess.run(["make", "-s", "-C", CSRC], check=True)


_L = None

_vp, _i32, _i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64


def lib():
    """Loads libafgpu.so (raises if it has not been built -- no silent fallback)."""
    global _L
    if _L is not None:
        return _L
    if not os.path.exists(LIB_PATH):
        raise AFError(f"{LIB_PATH} is missing: run __graft_entry__.build() (make -C {CSRC})")
    L = ctypes.CDLL(LIB_PATH)
    L.af_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(_vp)]
    L.af_ctx_create.restype = ctypes.c_int
    L.af_ctx_destroy.argtypes = [_vp]
    L.af_ctx_destroy.restype = None
    L.af_last_error.argtypes = [_vp]
    L.af_last_error.restype = ctypes.c_char_p
    L.af_params_default.argtypes = [ctypes.POINTER(Params)]
    L.af_params_default.restype = None
    L.af_index_build.argtypes = [_vp, ctypes.c_char_p, _i64, ctypes.POINTER(_vp)]
    L.af_index_build.restype = ctypes.c_int
    L.af_index_free.argtypes = [_vp]
    L.af_index_free.restype = None
    L.af_index_anchor_len.argtypes = [_vp]
    L.af_index_anchor_len.restype = _i64
    L.af_index_filter_words.argtypes = [_vp]
    L.af_index_filter_words.restype = _i32
    L.af_index_filter_table.argtypes = [_vp, _vp, _i64]
    L.af_index_filter_table.restype = ctypes.c_int
    L.af_pe_default.argtypes = [ctypes.POINTER(Pe)]
    L.af_pe_default.restype = None
    _pe = ctypes.POINTER(Pe)
    L.af_align_pairs.argtypes = [_vp, _vp, _vp, _i64, _i32, _vp, ctypes.POINTER(Params), _pe, ctypes.POINTER(AlnOut)]
    L.af_align_pairs.restype = ctypes.c_int
    L.af_align_pairs_device.argtypes = [_vp, _vp, _vp, _i64, _i32, _vp, ctypes.POINTER(Params), _pe,
                                        ctypes.POINTER(AlnOut), _vp]
    L.af_align_pairs_device.restype = ctypes.c_int
    L.af_align_candidates_device.argtypes = [_vp, _vp, _vp, _i64, _i32, _vp, ctypes.POINTER(Params), _pe,
                                             ctypes.POINTER(AlnOut), _vp]
    L.af_align_candidates_device.restype = ctypes.c_int
    L.af_partition_device.argtypes = [_vp, _vp, _vp, _i64, _i64, _vp, _vp, _vp, _vp, _vp]
    L.af_partition_device.restype = ctypes.c_int
    L.af_seed_filter_device.argtypes = [_vp, _vp, _vp, _i64, _i32, _vp, _vp, _vp]
    L.af_seed_filter_device.restype = ctypes.c_int
    L.af_last_candidates.argtypes = [_vp]
    L.af_last_candidates.restype = _i64
    L.af_split_tails_device.argtypes = [_vp, _vp, _i64, _i32, _vp, ctypes.POINTER(AlnOut), _i32, _i64, _i32, _i64,
                                        _vp, _vp, _vp, _vp, _vp]
    L.af_split_tails_device.restype = ctypes.c_int
    L.af_align_candidates_tails_device.argtypes = [_vp, _vp, _vp, _i64, _i32, _vp, ctypes.POINTER(Params), _pe,
                                                   ctypes.POINTER(AlnOut), _i32, _i64, _i32, _i64, _vp, _vp, _vp,
                                                   _vp, _vp]
    L.af_align_candidates_tails_device.restype = ctypes.c_int
    L.af_gather_reads_device.argtypes = [_vp, _vp, _i32, _vp, _vp, _i64, _i32, ctypes.POINTER(AlnOut), _i64, _i64,
                                         _i64, _vp, _vp, _vp, _vp, _vp]
    L.af_gather_reads_device.restype = ctypes.c_int
    L.af_blat_params_default.argtypes = [_vp]
    L.af_blat_params_default.restype = None
    L.af_tile_index_build.argtypes = [_vp, ctypes.c_char_p, _i64, _i32, ctypes.POINTER(_vp)]
    L.af_tile_index_build.restype = ctypes.c_int
    L.af_tile_index_build_device.argtypes = [_vp, _vp, _i64, _i32, ctypes.POINTER(_vp)]
    L.af_tile_index_build_device.restype = ctypes.c_int
    L.af_blat.argtypes = [_vp, _vp, _vp, _i64, _i32, _vp, _vp, _i32, _vp, _vp]
    L.af_blat.restype = ctypes.c_int
    L.af_blat_device.argtypes = [_vp, _vp, _vp, _vp, _i64, _i32, _vp, _vp, _i32, _vp, _vp, _vp]
    L.af_blat_device.restype = ctypes.c_int
    L.af_blat_device_range.argtypes = [_vp, _vp, _vp, _vp, _vp, _i64, _i32, _vp, _vp, _i32, _vp, _vp, _vp]
    L.af_blat_device_range.restype = ctypes.c_int
    L.af_fastq_open.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(_vp)]
    L.af_fastq_open.restype = ctypes.c_int
    L.af_fastq_next.argtypes = [_vp, _i64, ctypes.POINTER(_i64), ctypes.POINTER(_i32), ctypes.POINTER(_i64)]
    L.af_fastq_next.restype = ctypes.c_int
    L.af_fastq_export.argtypes = [_vp, _i32, _vp, _vp, _vp, _i64, _vp]
    L.af_fastq_export.restype = ctypes.c_int
    L.af_fastq_error.argtypes = [_vp]
    L.af_fastq_error.restype = ctypes.c_char_p
    L.af_fastq_close.argtypes = [_vp]
    L.af_fastq_close.restype = None
    L.af_fastq_part_read.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(_vp),
                                     ctypes.POINTER(_i64), ctypes.POINTER(_i32), ctypes.POINTER(_i64)]
    L.af_fastq_part_read.restype = ctypes.c_int
    L.af_fastq_part_export.argtypes = [_vp, _i32, _vp, _vp, _vp, _i64, _vp]
    L.af_fastq_part_export.restype = ctypes.c_int
    L.af_fastq_part_error.argtypes = [_vp]
    L.af_fastq_part_error.restype = ctypes.c_char_p
    L.af_fastq_part_free.argtypes = [_vp]
    L.af_fastq_part_free.restype = None
    _pp = ctypes.POINTER(Params)
    L.af_genome_build.argtypes = [_vp, _vp, _i64, _vp, _vp, _i32, ctypes.POINTER(_vp)]
    L.af_genome_build.restype = ctypes.c_int
    L.af_genome_build_device.argtypes = [_vp, _vp, _i64, _vp, _vp, _i32, ctypes.POINTER(_vp)]
    L.af_genome_build_device.restype = ctypes.c_int
    L.af_genome_free.argtypes = [_vp]
    L.af_genome_free.restype = None
    L.af_genome_lpac.argtypes = [_vp]
    L.af_genome_lpac.restype = _i64
    L.af_genome_primary.argtypes = [_vp]
    L.af_genome_primary.restype = _i64
    L.af_genome_read.argtypes = [_vp, _vp, _i32, _i64, _i64, _vp]
    L.af_genome_read.restype = ctypes.c_int
    L.af_genome_align_se_device.argtypes = [_vp, _vp, _vp, _i64, _i32, _vp, _pp, _pe, _i64, _vp, _vp, _vp]
    L.af_genome_align_se_device.restype = ctypes.c_int
    L.af_genome_align_se_ids_device.argtypes = [_vp, _vp, _vp, _i64, _i32, _vp, _pp, _pe, _vp, _vp, _vp, _vp]
    L.af_genome_align_se_ids_device.restype = ctypes.c_int
    L.af_genome_align_pe_device.argtypes = [_vp, _vp, _vp, _i64, _i32, _vp, _pp, _pe, _vp, _vp, _vp]
    L.af_genome_align_pe_device.restype = ctypes.c_int
    L.af_genome_align_pe_se_device.argtypes = [_vp, _vp, _vp, _i64, _i64, _i32, _vp, _pp, _pe, _pe, _i64, _vp, _vp,
                                               _vp, _vp, _vp]
    L.af_genome_align_pe_se_device.restype = ctypes.c_int
    L.af_genome_align_se.argtypes = [_vp, _vp, _vp, _i64, _i32, _vp, _pp, _pe, _i64, _vp, _vp]
    L.af_genome_align_se.restype = ctypes.c_int
    L.af_genome_align_pe.argtypes = [_vp, _vp, _vp, _i64, _i32, _vp, _pp, _pe, _vp, _vp]
    L.af_genome_align_pe.restype = ctypes.c_int
    L.af_genome_regions.argtypes = [_vp, _vp, _vp, _i64, _i32, _vp, _pp, _pe, _i32, _vp, _vp]
    L.af_genome_intervals.argtypes = [_vp, _vp, _vp, _i64, _i32, _vp, _pp, _pe, _i32, _vp, _vp]
    L.af_genome_intervals.restype = ctypes.c_int
    L.af_genome_regions.restype = ctypes.c_int
    L.af_genome_stats.argtypes = [_vp, _vp]
    L.af_genome_stats.restype = ctypes.c_int
    L.af_s5_filter_device.argtypes = [_vp, _vp, _vp, _i64, _vp, _i32, _vp, _vp, ctypes.POINTER(AlnOut), _vp, _i64, _vp,
                                      _i32, _vp, _vp, _vp, _vp, _vp]
    L.af_s5_filter_device.restype = ctypes.c_int
    L.af_s5_rules_host.argtypes = [_vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _vp, _vp, _vp, _i32, _vp, _vp]
    L.af_s5_rules_host.restype = ctypes.c_int
    L.af_blat_caps.argtypes = [_vp, _vp, ctypes.c_int]
    L.af_blat_caps.restype = ctypes.c_int
    L.af_blat_spill.argtypes = [_vp, _vp, _vp, _vp, _i64]
    L.af_blat_spill.restype = ctypes.c_int
    L.af_blat_query_caps.argtypes = [_vp, _vp, _i64]
    L.af_blat_query_caps.restype = ctypes.c_int
    _s6 = ctypes.POINTER(S6Set)
    L.af_s6_queries_device.argtypes = [_vp, _i64, _vp, _i32, _vp, _vp, ctypes.POINTER(AlnOut), _vp, _s6, _vp]
    L.af_s6_queries_device.restype = ctypes.c_int
    L.af_s6_check_device.argtypes = [_vp, _vp, _vp, _i64, _vp, ctypes.POINTER(AlnOut), _vp, _s6, _vp, _vp]
    L.af_s6_check_device.restype = ctypes.c_int
    L.af_s6_compact_device.argtypes = [_vp, _s6, _vp, _s6, _i32, _vp]
    L.af_s6_compact_device.restype = ctypes.c_int
    L.af_blat_device_begin.argtypes = [_vp, _vp, _vp, _vp, _i64, _i32, _vp, _vp, _i32, _vp, _vp, _vp]
    L.af_blat_device_begin.restype = ctypes.c_int
    L.af_blat_device_end.argtypes = [_vp, _vp, _vp]
    L.af_blat_device_end.restype = ctypes.c_int
    L.af_blat_long.argtypes = [_vp, _vp, ctypes.c_char_p, _i32, _vp, _i32, _vp, _vp, _vp, _i64, _vp, _vp]
    L.af_blat_long.restype = ctypes.c_int
    L.af_blat_heavy_stats.argtypes = [_vp, _vp]
    L.af_blat_heavy_stats.restype = ctypes.c_int
    _L = L
    return L


def default_params():
    p = Params()
    lib().af_params_default(ctypes.byref(p))
    return p


def default_pe(**kw):
    """af_pe_default (bwa 0.7.17 paired-end options, 10 Mbase chunks) with overrides."""
    e = Pe()
    lib().af_pe_default(ctypes.byref(e))
    for k, v in kw.items():
        setattr(e, k, v)
    return e


def check(ctx, rc, what):
    if rc != AF_OK:
        msg = lib().af_last_error(ctx) if ctx else b""
        raise AFError(f"{what} failed (rc={rc}): {(msg or b'').decode(errors='replace')}")
