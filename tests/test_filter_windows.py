"""The filter's window builder (filter_model.get_test_reads, functions.py:1642-1721)
against the reference's own function run on the same synthetic candidates
(tests/golden/filter_windows.json, tests/golden/make_filter_windows_fixture.py)."""
import json
import os

import afpkg  # noqa: F401
import fake_tools
from anchored_fusion_amd.annotation import ExonIndex
from anchored_fusion_amd.filter_model import get_test_reads
from anchored_fusion_amd.report import Candidate

FX = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "filter_windows.json")))


def _getfasta(rows):
    return [(f"{name}::{chrom}:{s}-{e}", fake_tools.genome_seq(chrom, s, e)) for chrom, s, e, name in rows]


def _cands(spec):
    out = []
    for c in spec:
        obj = Candidate(c["type"])
        for a in c["adds"]:
            obj.add_reads(a["target"], list(a["other"]), a["left"], a["right"], a["mid"], a["cnt"],
                          list(a["spanning"]), list(a["split"]))
        out.append(obj)
    return out


def test_windows_match_reference():
    index = ExonIndex.from_lines(FX["gtf"])
    n = 0
    for t in FX["trials"]:
        assert t["error"] is None
        got = get_test_reads(_cands(t["spec"]), FX["anchor"], index, _getfasta)
        assert got == t["lines"]
        n += len(got)
    assert n >= 40


def test_window_lengths_show_the_flank_quirk():
    """Every partner flank lands right of 'H' (the tag parse never sees 'left'): MS windows are
    100 + 1 + ~200 long, SM windows before any '-' strand 201."""
    lens = {len(ln.split("\t")[0]) for t in FX["trials"] for ln in t["lines"]}
    assert 201 in lens and any(x > 201 for x in lens)
