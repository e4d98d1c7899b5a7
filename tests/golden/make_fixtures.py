"""Generates the golden fixtures of the split-read consumer stages (SURVEY.md §8 a4-a8, a11,
a12, a14) by running the reference's own `functions.py` on synthetic inputs.

Run HERE only (needs /root/reference; nothing on the GPU box reads it):

    PYTHONHASHSEED=0 python tests/golden/make_fixtures.py

It follows SURVEY.md §8(c):

- `Bio.Align` is stubbed. Biopython is absent, and the PairwiseAligner that functions.py
  configures is never called.
- `sys.dont_write_bytecode` keeps /root/reference free of __pycache__.
- `os.popen` / `os.system` are intercepted to hand the functions canned `samtools view`, `bwa`
  and `blat` outputs. bwa, samtools and BLAT are absent here, so these are synthetic records
  of the right shape.

Inputs and outputs are written to tests/golden/consumers.json. Fixtures are data; no
reference source is copied.
"""
import json
import os
import random
import sys
import tempfile
import types

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.path.insert(0, os.path.dirname(HERE))          # tests/ (fake_tools)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))  # repo root (afpkg)
import fake_tools  # noqa: E402
import afpkg  # noqa: E402,F401
from anchored_fusion_amd.partner import PRESETS  # noqa: E402


def load_reference():
    sys.dont_write_bytecode = True
    bio = types.ModuleType("Bio")
    align = types.ModuleType("Bio.Align")

    class PairwiseAligner:  # configured, never called, by functions.py
        pass

    align.PairwiseAligner = PairwiseAligner
    bio.Align = align
    sys.modules.setdefault("Bio", bio)
    sys.modules.setdefault("Bio.Align", align)
    sys.path.insert(0, REF)
    import functions  # noqa: E402
    return functions


class Canned:
    """Replaces os.popen / os.system inside functions.py with canned tool outputs."""

    def __init__(self, fn):
        self.fn = fn
        self.popen_text = ""
        self.system_payload = ""
        self.orig_popen, self.orig_system = fn.os.popen, fn.os.system

    def __enter__(self):
        outer = self

        class _P:
            def __init__(self, text):
                self.text = text

            def read(self):
                return self.text

        def popen(cmd):
            return _P(outer.popen_text)

        def system(cmd):
            # the output path is the last token (blat) or follows '>' (bwa)
            toks = cmd.split()
            path = toks[toks.index(">") + 1] if ">" in toks else toks[-1]
            with open(path, "w") as fh:
                fh.write(outer.system_payload)
            return 0

        self.fn.os.popen, self.fn.os.system = popen, system
        return self

    def __exit__(self, *a):
        self.fn.os.popen, self.fn.os.system = self.orig_popen, self.orig_system


class ToolSim:
    """Runs the fake tools (tests/fake_tools.py) in place of blat / bedtools / bwa index, reading
    the files functions.py wrote and writing where the tool would have written."""

    def __init__(self, fn, genome_path, genome_targets):
        self.fn, self.genome_path, self.genome = fn, genome_path, genome_targets
        self.orig = fn.os.system
        self.calls = []  # (preset, queries) of every blat call, in order

    def __enter__(self):
        self.fn.os.system = self.system
        return self

    def __exit__(self, *a):
        self.fn.os.system = self.orig

    def _fasta(self, path):
        if path == self.genome_path:
            return self.genome
        with open(path) as fh:
            return fake_tools.read_fasta_text(fh.read())

    def system(self, cmd):
        head, _, redirect = cmd.partition(">")
        toks = head.split()
        if toks[0] == "blat":
            opts = " ".join(t for t in toks[1:] if t.startswith("-"))
            files = [t for t in toks[1:] if not t.startswith("-")]
            preset = next(k for k, v in PRESETS.items() if v == opts)
            queries = self._fasta(files[1])
            self.calls.append([preset, [list(q) for q in queries]])
            out = fake_tools.blat(self._fasta(files[0]), queries, preset)
            with open(files[2], "w") as fh:
                fh.writelines(out)
        elif toks[:2] == ["bedtools", "getfasta"]:
            with open(toks[toks.index("-bed") + 1]) as fh:
                rows = [ln.rstrip("\n").split("\t") for ln in fh if ln.strip()]
            recs = [(f"{r[3]}::{r[0]}:{r[1]}-{r[2]}", fake_tools.genome_seq(r[0], int(r[1]), int(r[2]))) for r in rows]
            with open(redirect.strip(), "w") as fh:
                fh.write(fake_tools.fasta_text(recs))
        elif toks[:2] == ["bedtools", "intersect"]:
            a, b = toks[toks.index("-a") + 1], toks[toks.index("-b") + 1]
            rows = []
            for path in (a, b):
                with open(path) as fh:
                    rows.append([ln.rstrip("\n").split("\t") for ln in fh if ln.strip()])
            with open(redirect.strip(), "w") as fh:
                fh.writelines("\t".join(r) + "\n" for r in fake_tools.intersect_wa(rows[0], rows[1]))
        elif toks[:2] == ["bwa", "index"]:
            pass
        else:
            raise RuntimeError("unexpected tool call: " + cmd)
        return 0


# ---------------------------------------------------------------------------------------------
# synthetic world
# ---------------------------------------------------------------------------------------------
def make_gtf(rng):
    lines = ["##description: synthetic fixture annotation\n", "##provider: afgpu tests\n"]
    genes = []
    gid = 0
    for chrom in ("chr1", "chr2", "chr3", "chr14", "chrM"):
        pos = 10000
        for g in range(8 if chrom != "chrM" else 1):
            gid += 1
            name = f"G{gid}"
            gene_id = f"ENSG{gid:07d}.1"
            tt_gene = rng.choice(["protein_coding"] * 6 + ["lncRNA", "processed_pseudogene"])
            exons = []
            p = pos
            for e in range(rng.randint(2, 7)):
                ln = rng.randint(60, 400)
                exons.append((p, p + ln))
                p += ln + rng.randint(150, 3000)
            genes.append((chrom, gene_id, name, exons))
            lines.append("\t".join([chrom, "SYN", "gene", str(exons[0][0]), str(exons[-1][1]), ".",
                                    rng.choice("+-"), ".", f'gene_id "{gene_id}"; gene_type "{tt_gene}"; '
                                    f'gene_name "{name}"; level 2;']) + "\n")
            for t in range(rng.randint(1, 3)):
                tt = tt_gene if t == 0 else rng.choice(["protein_coding", "artifact", "retained_intron",
                                                         "protein_coding_LoF", "unprocessed_pseudogene"])
                for (s, e) in exons:
                    if rng.random() < 0.2 and t > 0:
                        continue
                    s2 = s + rng.randint(-30, 30) if t > 0 else s
                    e2 = e + rng.randint(-30, 30) if t > 0 else e
                    attrs = [f'gene_id "{gene_id}"', f'transcript_id "ENST{gid:07d}.{t}"', f'gene_name "{name}"',
                             f'transcript_type "{tt}"', "exon_number 1"]
                    if rng.random() < 0.3:
                        attrs = attrs[::-1]
                    lines.append("\t".join([chrom, "SYN", "exon", str(s2), str(e2), ".", "+", ".",
                                            "; ".join(attrs) + ";"]) + "\n")
                lines.append("\t".join([chrom, "SYN", "transcript", str(exons[0][0]), str(exons[-1][1]), ".", "+",
                                        ".", f'gene_id "{gene_id}"; transcript_type "{tt}";']) + "\n")
            pos = p + rng.randint(500, 5000)
    return lines, genes


def rand_seq(rng, n):
    return "".join(rng.choice("ACGT") for _ in range(n))


def mutate(rng, s, rate):
    return "".join(rng.choice("ACGT") if rng.random() < rate else c for c in s)


def make_cigars(rng, n):
    out = []
    for _ in range(n):
        ops = []
        if rng.random() < 0.5:
            ops.append((rng.randint(1, 60), rng.choice("SH")))
        for _ in range(rng.randint(1, 4)):
            ops.append((rng.randint(1, 80), "M"))
            if rng.random() < 0.5:
                ops.append((rng.randint(1, 6), rng.choice("IDN")))
        if rng.random() < 0.5:
            ops.append((rng.randint(1, 60), rng.choice("SH")))
        if rng.random() < 0.1:
            ops.insert(0, (rng.randint(1, 5), rng.choice("DI")))
        cig = "".join(f"{n}{o}" for n, o in ops)
        qlen = sum(n for n, o in ops if o in "MIS")
        out.append((cig, rand_seq(rng, qlen)))
    return out


def split_sam_lines(rng, anchor_chrom, n_bp, reads_per_bp):
    """Pseudo-SAM of anchored split reads around a few anchor breakpoints (a5 output shape)."""
    lines = []
    for b in range(n_bp):
        bp = rng.randint(300, 3000)
        kind = rng.choice(["SM", "MS"])
        left_true = rand_seq(rng, 220)
        right_true = rand_seq(rng, 220)
        for r in range(reads_per_bp):
            jitter = rng.choice([0, 0, 0, 1, -1, 2, 3, -3])
            L = rng.randint(70, 150)
            cut = rng.randint(10, L - 10)
            left = mutate(rng, left_true[220 - cut:], 0.02)
            right = mutate(rng, right_true[:L - cut], 0.02)
            seq = left + right
            if kind == "SM":
                cig = f"{cut}S{L - cut}M"
                pos = bp + jitter
            else:
                cig = f"{cut}M{L - cut}S"
                pos = bp + jitter - cut + 1
            if rng.random() < 0.1:
                cig = f"{cut}M2D{L - cut}M"  # not a split read after normalisation
            lines.append(f"r{b}_{r}\t0\t{anchor_chrom}\t{pos}\t60\t{cig}\t=\t1111\t0\t{seq}\tA\n")
    rng.shuffle(lines)
    return lines


def spanning_records(rng, genes, homo_gene_ids, n_pairs):
    """`samtools view` of genome alignments of one-end-anchored pairs (S4 output shape)."""
    homo = [g for g in genes if g[1] in homo_gene_ids]
    others = [g for g in genes if g[1] not in homo_gene_ids and g[0] != "chrM"]
    lines = []
    for p in range(n_pairs):
        name = f"sp{p}"
        recs = []
        h = rng.choice(homo)
        ex = rng.choice(h[3])
        recs.append((h[0], rng.randint(ex[0], max(ex[0], ex[1] - 60))))
        o = rng.choice(others) if rng.random() < 0.85 else rng.choice(homo)
        ex = rng.choice(o[3])
        recs.append((o[0], rng.randint(ex[0] - 5, max(ex[0], ex[1] - 40))))
        if rng.random() < 0.1:
            o2 = rng.choice(others)
            ex = rng.choice(o2[3])
            recs.append((o2[0], rng.randint(ex[0], ex[1])))
        if rng.random() < 0.05:
            recs = recs[:1]
        for (chrom, pos) in recs:
            cig = rng.choice(["100M", "30S70M", "70M30S", "50M2I48M", "20H80M"])
            lines.append(f"{name}\t{rng.choice([65, 129, 97, 145])}\t{chrom}\t{pos}\t60\t{cig}\t=\t0\t0\t"
                         f"{rand_seq(rng, 100)}\tF\n")
    return lines


def psl_lines(rng, tails, genes, homo_gene_ids):
    """BLAT PSL of the split-read tails (S6 output shape; columns the consumer reads are real)."""
    homo = [g for g in genes if g[1] in homo_gene_ids]
    others = [g for g in genes if g[1] not in homo_gene_ids and g[0] != "chrM"]
    out = ["psLayout version 3\n", "\n", "match\tmis-\trep.\n", "-" * 40 + "\n"]
    for qid, (kind, L, R) in enumerate(tails):
        hits = []
        for _ in range(rng.randint(1, 4)):
            roll = rng.random()
            g = rng.choice(homo if roll < 0.4 else others)
            ex = rng.choice(g[3])
            ts = rng.randint(ex[0], max(ex[0], ex[1] - 20))
            if kind == "MS":
                choices = [(rng.randint(0, 4), L + rng.randint(-4, 4)),            # anchored half
                           (L + rng.randint(-4, 4), L + R - rng.randint(0, 4)),    # tail
                           (rng.randint(0, L // 2), L + R)]                         # whole read (bad)
            else:
                choices = [(rng.randint(0, 4), L + rng.randint(-4, 4)),            # tail
                           (L + rng.randint(-4, 4), L + R - rng.randint(0, 4)),    # anchored half
                           (rng.randint(0, max(0, L - 6)), L + R)]
            w = [0.45, 0.45, 0.1]
            qs, qe = rng.choices(choices, weights=w)[0]
            te = ts + (qe - qs) + (rng.randint(0, 300) if rng.random() < 0.1 else 0)
            f = [str(max(qe - qs, 1)), "0", "0", "0", "0", "0", "0", "0", rng.choice("+-"), str(qid), str(L + R),
                 str(qs), str(qe), g[0], "100000000", str(ts), str(te), "1", f"{qe - qs},", f"{qs},", f"{ts},"]
            hits.append("\t".join(f) + "\n")
        out.extend(hits)
    return out


def genome_sam(rng, fasta):
    """`bwa mem` genome records for the split-read queries (the fn:716 call's output shape)."""
    out = ["@HD\tVN:1.6\tSO:unsorted\n", "@SQ\tSN:chr1\tLN:1000000\n"]
    for name, seq in fasta:
        anchored_cigar = name.split("$")[3]
        L = len(seq)
        n_rec = rng.choice([1, 1, 2, 2, 3])
        for k in range(n_rec):
            flag = rng.choice([0, 16, 256, 272, 2048 + 16]) if k else rng.choice([0, 16])
            roll = rng.random()
            if roll < 0.2:
                cig = f"{L}M"
            elif roll < 0.6:
                c = rng.randint(10, L - 10)
                cig = f"{c}S{L - c}M"
            elif roll < 0.9:
                c = rng.randint(10, L - 10)
                cig = f"{c}M{L - c}S"
            else:
                c = rng.randint(10, L - 10)
                cig = f"{c}H{L - c}M"
            rec_seq = seq if not (flag & 16) else "".join({"A": "T", "C": "G", "G": "C", "T": "A"}[b]
                                                          for b in reversed(seq))
            if "H" in cig:
                rec_seq = rec_seq[int(cig.split("H")[0]):]
            out.append(f"{name}\t{flag}\tchr{rng.randint(1, 3)}\t{rng.randint(1, 900000)}\t60\t{cig}\t*\t0\t0\t"
                       f"{rec_seq}\t*\n")
        del anchored_cigar
    return out


def candidates_spec(rng, genes, n):
    spec = []
    for c in range(n):
        kind = rng.choice(["SM", "MS"])
        adds = []
        bps = [(rng.randint(100, 5000), rng.choice(genes)) for _ in range(rng.randint(1, 3))]
        for _ in range(rng.randint(1, 5)):
            tbp, g = rng.choice(bps)
            ex = rng.choice(g[3])
            other = [g[0], rng.randint(ex[0], ex[1]), rng.choice("+-"), rng.randint(0, 100), rng.randint(0, 30)]
            adds.append(dict(target=tbp, other=other, left=rand_seq(rng, rng.randint(0, 120)),
                             right=rand_seq(rng, rng.randint(0, 120)), mid=rand_seq(rng, rng.randint(0, 20)),
                             cnt=rng.randint(1, 6),
                             spanning=[f"s{rng.randint(0, 30)}" for _ in range(rng.randint(0, 6))],
                             split=[f"t{rng.randint(0, 30)}" for _ in range(rng.randint(0, 6))]))
        spec.append(dict(type=kind, adds=adds, score=round(rng.random(), 3)))
    return spec


def dump_breakpoints(bps):
    return [[b.chrom, b.breakpoint, b.type_, b.seq_left, b.seq_right, b.cnt, list(b.reads),
             [list(o) for o in b.other_breakpoints]] for b in bps]


def dump_candidate(c):
    return dict(type=c.type_, pos=[list(p) for p in c.pos], left=c.return_seq_left(), right=c.return_seq_right(),
                mid=c.return_seq_mid(), l=[c.l_left, c.l_mid, c.l_right], spanning=list(c.spanning_reads),
                split=list(c.split_reads))


def partner_trials(fn, rng, genes, gc, gtf_path, homo_ids, work):
    """a9-a11, a13 and a14 chained on one synthetic sample per trial."""
    chroms = sorted({g[0] for g in genes})
    genome_targets = [(c, 400000) for c in chroms]
    genome_path = os.path.join(work, "genome.fa")
    anchor = ("BCR", rand_seq(rng, 3000))
    anchor_path = os.path.join(work, "anchor.fa")
    with open(anchor_path, "w") as fh:
        fh.write(fake_tools.fasta_text([anchor]))
    trials = []
    homo = []
    small_genome = [(c, 90000) for c in chroms]
    with ToolSim(fn, genome_path, small_genome):
        for k in range(12):
            anc = (f"A{k}", rand_seq(rng, rng.randint(200, 3000)))
            with open(anchor_path, "w") as fh:
                fh.write(fake_tools.fasta_text([anc]))
            bad = os.path.join(work, "homo.bed")
            fn.Find_homo_genes(genome_path, anchor_path, gtf_path, os.path.join(work, "hg"), bad)
            with open(bad) as fh:
                homo.append([list(anc), fh.readlines()])
    with open(anchor_path, "w") as fh:
        fh.write(fake_tools.fasta_text([anchor]))
    for trial in range(14):
        if True:
            spans = spanning_records(rng, genes, homo_ids, rng.randint(60, 200))
            split = split_sam_lines(rng, "BCR", rng.randint(6, 16), rng.randint(2, 10))
            with Canned(fn) as cn:
                cn.popen_text = "".join(spans)
                blocks_chr = fn.Find_blocks("spanning.bam", gc, homo_ids)
            # the reference's widening can leave '' as a block end (find_positions found no
            # downstream interval); Build_candidate_fasta would then raise TypeError.  The chain
            # drops such blocks (the tests do the same: test_consumers.sanitize_blocks).
            for c in list(blocks_chr):
                blocks_chr[c] = [b for b in blocks_chr[c] if isinstance(b.start, int) and isinstance(b.end, int)]
            cand_fa = os.path.join(work, f"cand{trial}.fa")
            with ToolSim(fn, genome_path, genome_targets) as sim:
                fn.Build_candidate_fasta(cand_fa, os.path.join(work, f"bc{trial}"), genome_path, anchor_path,
                                         blocks_chr)
                with open(cand_fa) as fh:
                    cand_recs = fake_tools.read_fasta_text(fh.read())
                split_path = os.path.join(work, f"psplit{trial}.sam")
                with open(split_path, "w") as fh:
                    fh.writelines(split)
                bps = fn.contact_reads(split_path, work, genome_path, "1")
                good = fn.Find_Anchored_split(os.path.join(work, f"fa{trial}"), cand_fa, blocks_chr, bps, gc,
                                              anchor_path)
                after_a9 = dict(good=sorted(good), breakpoints=dump_breakpoints(bps),
                                anchored={c: [sorted(b.anchored_split_breakpoints) for b in bl]
                                          for c, bl in blocks_chr.items()})
                try:
                    cands, cnt_max = fn.Find_candidate_genes(os.path.join(work, f"cg{trial}"), genome_path, good,
                                                             bps, blocks_chr, gc, "1")
                    a11 = dict(candidates=[dump_candidate(c) for c in cands], cnt_max=cnt_max, error=None)
                except Exception as e:  # noqa: BLE001
                    cands, a11 = [], dict(candidates=None, cnt_max=None, error=type(e).__name__)
            prefix = os.path.join(work, f"final{trial}")
            fn.Final_fusion(prefix, cands, "BCR", gc, [], a11["cnt_max"] or 0, True)
            with open(prefix + "_predictions_abridged.txt") as fa, open(prefix + "_predictions.txt") as fo:
                final = dict(abridged=fa.readlines(), full=fo.readlines())
            trials.append(dict(spanning=spans, split=split, blocks_after_a10={
                c: [[b.chrom, b.start, b.end, b.count] for b in bl] for c, bl in blocks_chr.items()},
                candidate_records=cand_recs, a9=after_a9, a11=a11, final=final, blat_calls=sim.calls))
    return dict(genome=genome_targets, small_genome=small_genome, anchor=list(anchor), homologs=homo,
                trials=trials)


def main():
    fn = load_reference()
    rng = random.Random(20251015)
    gtf, genes = make_gtf(rng)
    fx = {"gtf": gtf}
    work = tempfile.mkdtemp(prefix="afgpu_fx_")
    gtf_path = os.path.join(work, "ann.gtf")
    with open(gtf_path, "w") as fh:
        fh.writelines(gtf)
    gc = fn.Gene_co()
    gc.Build_dic(gtf_path)
    fx["gene_co"] = gc.dic
    # a12: Find_exon / find_positions
    q = []
    for _ in range(600):
        chrom = rng.choice(["chr1", "chr2", "chr3", "chr14", "chrM", "chrX", "KI270846.1"])
        s = rng.randint(9000, 120000)
        q.append([chrom, s, s + rng.randint(0, 300)])
    fx["find_exon"] = [[a, b, c] + list(gc.Find_exon(a, b, c)) for a, b, c in q]
    walk = []
    for chrom, gene_id, name, exons in genes:
        if chrom not in gc.dic:
            continue
        for _ in range(4):
            ex = rng.choice(exons)
            p = rng.randint(ex[0], ex[1])
            ln = rng.choice([200, 200, 50, 700])
            try:
                res = fn.find_positions(gc, chrom, p, ln)
                walk.append([chrom, p, ln, [list(x) for x in res], None])
            except Exception as e:  # noqa: BLE001 -- the reference's own failure is the expected output
                walk.append([chrom, p, ln, None, type(e).__name__])
    fx["find_positions"] = walk
    # a6: deal_cigar
    dc = []
    for cig, seq in make_cigars(rng, 400):
        ops, seq2 = fn.deal_cigar(cig, seq)
        dc.append([cig, seq, ops, seq2])
    fx["deal_cigar"] = dc
    fx["reverse"] = [[s, fn.reverse(s)] for s in (rand_seq(rng, rng.randint(0, 40)) + "N" for _ in range(20))]
    # a8: contact_reads (+ combine_split_reads)
    cr = []
    for trial in range(6):
        lines = split_sam_lines(rng, "ANCHOR", rng.randint(1, 6), rng.randint(1, 25))
        path = os.path.join(work, f"split_{trial}.sam")
        with open(path, "w") as fh:
            fh.writelines(lines)
        res = fn.contact_reads(path, work, "ref.fa", "1")
        cr.append([lines, [[r.chrom, r.breakpoint, r.type_, r.seq_left, r.seq_right, r.cnt, list(r.reads)]
                           for r in res]])
    fx["contact_reads"] = cr
    # homologous genes = two genes on chr1 (the "anchor locus")
    homo_ids = [g[1] for g in genes if g[0] == "chr1"][:2]
    fx["homo_genes"] = homo_ids

    def dump_blocks(bc):
        return {c: [[b.chrom, b.start, b.end, list(b.gene), b.count, list(b.reads), b.min_exon_num, b.max_exon_num]
                    for b in bl] for c, bl in bc.items()}

    # a4: Find_blocks
    fb = []
    with Canned(fn) as cn:
        for trial in range(4):
            recs = spanning_records(rng, genes, homo_ids, rng.randint(20, 200))
            cn.popen_text = "".join(recs)
            try:
                out = dump_blocks(fn.Find_blocks("spanning.bam", gc, homo_ids))
                fb.append([recs, out, None])
            except Exception as e:  # noqa: BLE001
                fb.append([recs, None, type(e).__name__])
    fx["find_blocks"] = fb
    # a7: Find_fine_block on top of an existing block set
    ff = []
    with Canned(fn) as cn:
        for trial in range(4):
            lines = split_sam_lines(rng, "ANCHOR", rng.randint(2, 6), rng.randint(2, 12))
            path = os.path.join(work, f"anch_{trial}.sam")
            with open(path, "w") as fh:
                fh.writelines(lines)
            tails = []
            for ln in lines:
                f = ln.split("\t")
                ops, _ = fn.deal_cigar(f[5], f[9])
                if len(ops) == 2:
                    kind = "SM" if (ops[0][2] == "S" and ops[1][2] == "M") else "MS"
                    tails.append((kind, ops[0][1], ops[1][1]))
            psl = psl_lines(rng, tails, genes, homo_ids)
            cn.popen_text = "".join(spanning_records(rng, genes, homo_ids, 80))
            base_recs = cn.popen_text.splitlines(keepends=True)
            try:
                base = fn.Find_blocks("spanning.bam", gc, homo_ids)
            except Exception:  # noqa: BLE001
                base, base_recs = {}, []
            cn.system_payload = "".join(psl)
            try:
                out = dump_blocks(fn.Find_fine_block(path, "ref.fa", os.path.join(work, f"fine{trial}"), gc,
                                                     homo_ids, base))
                ff.append([lines, psl, base_recs, out, None])
            except Exception as e:  # noqa: BLE001
                ff.append([lines, psl, base_recs, None, type(e).__name__])
    fx["find_fine_block"] = ff
    # a5: del_too_many_reads
    dt = []
    with Canned(fn) as cn:
        for trial in range(5):
            anch = split_sam_lines(rng, "ANCHOR", rng.randint(2, 6), rng.randint(2, 10))
            anch = [ln.replace("\t0\tANCHOR", "\t" + rng.choice(["0", "16"]) + "\tANCHOR", 1) for ln in anch]
            fasta = []
            for ln in anch:
                f = ln.split("\t")
                ops, _ = fn.deal_cigar(f[5], f[9])
                if len(ops) == 2:
                    fasta.append(("$".join([f[0], f[2], f[3], f[5]]), f[9]))
            gsam = genome_sam(rng, fasta)
            cn.popen_text = "".join(anch)
            cn.system_payload = "".join(gsam)
            out_sam = os.path.join(work, f"filt{trial}.sam")
            fn.del_too_many_reads("anchored.bam", out_sam, os.path.join(work, f"del{trial}"), "ref.fa", "1")
            with open(out_sam) as fh:
                dt.append([anch, gsam, fh.readlines()])
    fx["del_too_many_reads"] = dt
    # a11/a14: Candidate_reads consensus + Final_fusion
    fin = []
    for trial in range(4):
        spec = candidates_spec(rng, [g for g in genes if g[0] != "chrM"], rng.randint(1, 12))
        cands = []
        for c in spec:
            obj = fn.Candidate_reads(c["type"])
            for a in c["adds"]:
                obj.add_reads(a["target"], list(a["other"]), a["left"], a["right"], a["mid"], a["cnt"],
                              list(a["spanning"]), list(a["split"]))
            obj.score = c["score"]
            cands.append(obj)
        maxpos = [list(o.find_max_pos()[0]) + [o.find_max_pos()[1]] for o in cands]
        prefix = os.path.join(work, f"pred{trial}")
        no_filter = trial % 2 == 0
        scores = [c["score"] for c in spec]
        cnt_max = rng.randint(0, 40)
        fn.Final_fusion(prefix, cands, "BCR", gc, scores, cnt_max, no_filter)
        with open(prefix + "_predictions_abridged.txt") as fa, open(prefix + "_predictions.txt") as fo:
            fin.append(dict(spec=spec, no_filter=no_filter, cnt_max=cnt_max, maxpos=maxpos,
                            abridged=fa.readlines(), full=fo.readlines()))
    fx["final_fusion"] = fin
    fx["partner"] = partner_trials(fn, rng, genes, gc, gtf_path, homo_ids, work)
    with open(os.path.join(HERE, "consumers.json"), "w") as fh:
        json.dump(fx, fh, separators=(",", ":"))
    print("wrote", os.path.join(HERE, "consumers.json"), {k: len(v) for k, v in fx.items() if isinstance(v, list)})


if __name__ == "__main__":
    main()
