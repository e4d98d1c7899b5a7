"""CPU checks of the drop-in boundary: the C-ABI library loads and exports every symbol
include/afgpu.h declares (no compute calls: there is no GPU here)."""
import ctypes
import os
import re

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "afgpu.h")


def declared_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(af_\w+)\s*\(", txt, flags=re.M)))


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ("af_index_build", "af_align_pairs", "af_align_pairs_device", "af_seed_filter_device",
              "af_last_error", "af_ctx_create"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    from anchored_fusion_amd import _lib
    L = ctypes.CDLL(_lib.LIB_PATH)
    missing = [s for s in declared_symbols() if not hasattr(L, s)]
    assert not missing, missing
    assert sorted(_lib.EXPORTS) == declared_symbols()


def test_binding_loads_and_defaults_match_bwa():
    from anchored_fusion_amd import _lib
    p = _lib.default_params()
    assert (p.a, p.b, p.o_del, p.e_del, p.pen_clip5, p.w, p.zdrop, p.min_seed_len, p.T) == (1, 4, 6, 1, 5, 100, 100, 19, 30)


def test_library_targets_gfx950_only():
    data = open(os.path.join(ROOT, "anchored-fusion_amd", "libafgpu.so"), "rb").read()
    assert b"gfx950" in data
    assert b"sm_" not in data[:0]  # no CUDA targets exist in a hipcc gfx950 build
