#!/usr/bin/env python3
"""Entry point of the single-cell GPU pipeline (flags of the reference's Anchored_Fusion_singlecell.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import afpkg  # noqa: E402,F401
from anchored_fusion_amd.cli import main_singlecell  # noqa: E402

if __name__ == "__main__":
    sys.exit(main_singlecell())
