"""anchored_fusion_amd -- MI355X-native anchored split-read aligner (Anchored-Fusion drop-in).

See DESIGN.md.  Device work goes through the C-ABI library ``libafgpu.so`` (csrc/), loaded
with ctypes by ``_lib``; nothing in this package falls back to a CPU implementation.
"""
__version__ = "0.1.0"
