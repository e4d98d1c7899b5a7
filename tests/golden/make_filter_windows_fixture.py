"""Golden fixture of the filter's window builder, `get_test_reads` (functions.py:1642-1721), by
running the reference's own function on synthetic candidates.

Run HERE only (needs /root/reference; nothing on the GPU box reads it):

    PYTHONHASHSEED=0 python tests/golden/make_filter_windows_fixture.py

`bedtools getfasta -s -nameOnly` is replaced by a stand-in that writes one header (the BED name)
and one sequence line per row from tests/fake_tools.genome_seq; the BED rows carry the strand in
column 5 (the score column), so `-s` sees no strand and nothing is reverse-complemented.  The
reference's Candidate_reads / Gene_co build the inputs.  Inputs and outputs go to
tests/golden/filter_windows.json (data only; no reference source is copied).
"""
import json
import os
import random
import tempfile

from make_fixtures import HERE, candidates_spec, fake_tools, load_reference, make_gtf, rand_seq


class GetfastaStub:
    def __init__(self, fn):
        self.fn, self.orig = fn, fn.os.system

    def __enter__(self):
        self.fn.os.system = self.system
        return self

    def __exit__(self, *a):
        self.fn.os.system = self.orig

    @staticmethod
    def system(cmd):
        toks = cmd.split()
        assert toks[:2] == ["bedtools", "getfasta"] and "-s" in toks and "-nameOnly" in toks, cmd
        with open(toks[toks.index("-bed") + 1]) as fh:
            rows = [ln.rstrip("\n").split("\t") for ln in fh if ln.strip()]
        with open(toks[toks.index("-fo") + 1], "w") as fh:
            for r in rows:
                fh.write(f">{r[3]}\n{fake_tools.genome_seq(r[0], int(r[1]), int(r[2]))}\n")
        return 0


def main():
    fn = load_reference()
    rng = random.Random(7177)
    gtf, genes = make_gtf(rng)
    work = tempfile.mkdtemp(prefix="afgpu_fw_")
    gtf_path = os.path.join(work, "ann.gtf")
    with open(gtf_path, "w") as fh:
        fh.writelines(gtf)
    gc = fn.Gene_co()
    gc.Build_dic(gtf_path)
    anchor = rand_seq(rng, 6000)
    anchor_path = os.path.join(work, "anchor.fa")
    with open(anchor_path, "w") as fh:
        fh.write(">NM_000000.1 ANC transcript\n")
        for i in range(0, len(anchor), 70):
            fh.write(anchor[i:i + 70] + "\n")
    trials = []
    for trial in range(12):
        spec = candidates_spec(rng, [g for g in genes if g[0] != "chrM"], rng.randint(1, 10))
        cands = []
        for c in spec:
            obj = fn.Candidate_reads(c["type"])
            for a in c["adds"]:
                obj.add_reads(a["target"], list(a["other"]), a["left"], a["right"], a["mid"], a["cnt"],
                              list(a["spanning"]), list(a["split"]))
            cands.append(obj)
        test_file = os.path.join(work, f"test{trial}.txt")
        try:
            with GetfastaStub(fn):
                fn.get_test_reads(os.path.join(work, f"w{trial}"), test_file, cands, anchor_path, "ref.fa", gc)
            with open(test_file) as fh:
                trials.append(dict(spec=spec, lines=fh.readlines(), error=None))
        except Exception as e:  # noqa: BLE001 -- the reference's own failure is the expected output
            trials.append(dict(spec=spec, lines=None, error=type(e).__name__))
    with open(os.path.join(HERE, "filter_windows.json"), "w") as fh:
        json.dump(dict(gtf=gtf, anchor=anchor, trials=trials), fh, separators=(",", ":"))
    print("wrote filter_windows.json:", len(trials), "trials,",
          sum(len(t["lines"] or []) for t in trials), "windows,", sum(t["error"] is not None for t in trials), "errors")


if __name__ == "__main__":
    main()
