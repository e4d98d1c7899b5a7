"""Fusion candidates and the prediction tables (SURVEY.md §8 a11 consensus, a14 output).

* `Candidate` restates `Candidate_reads` (functions.py:230-333). It keeps vote profiles of
  the flank sequences (200 left, 200 right, 100 middle columns, with the reference's Python
  list indexing), the placements with their read counts, and the spanning and split read
  names. `find_max_pos` picks the first placement with the highest count.
* `write_predictions` restates `Final_fusion` (functions.py:1723-1795) and writes
  `<prefix>_predictions_abridged.txt` and `<prefix>_predictions.txt`:
  - rows are deduplicated by (anchor bp, chrom, partner bp, strand);
  - the 10x spanning/split balance rule is applied;
  - with the filter model, a row is kept in the full table only when score > 0.1 and
    either 10 x reads > cnt_max or score > 0.9.

Read-name lists are joined in `list(set(...))` order in the reference. That order depends
on the process's string hashing, so callers comparing outputs compare those columns as sets.
"""
_CODE = {"A": 0, "T": 1, "G": 2, "C": 3}
_BASE = "ATGC"


def _vote_call(col):
    top = max(col)
    return "N" if col.count(top) > 1 else _BASE[col.index(top)]


class Candidate:
    def __init__(self, type_):
        self.pos = []
        self.type_ = type_
        self.spanning_reads = []
        self.split_reads = []
        self.l_left = self.l_right = self.l_mid = 0
        self.seq_left = [[0, 0, 0, 0] for _ in range(200)]
        self.seq_right = [[0, 0, 0, 0] for _ in range(200)]
        self.seq_mid = [[0, 0, 0, 0] for _ in range(100)]
        self.score = 0

    def add_reads(self, target_breakpoint, other_breakpoint, seq_left, seq_right, seq_mid, cnt, spanning_reads,
                  split_reads):
        for off, b in enumerate(reversed(seq_left)):
            if b in _CODE:
                self.seq_left[199 - off][_CODE[b]] += cnt
        for off, b in enumerate(seq_right):
            if b in _CODE:
                self.seq_right[off][_CODE[b]] += cnt
        for off, b in enumerate(seq_mid):
            if b in _CODE:
                self.seq_mid[off][_CODE[b]] += cnt
        self.l_left = max(self.l_left, len(seq_left))
        self.l_right = max(self.l_right, len(seq_right))
        self.l_mid = max(self.l_mid, len(seq_mid))
        key = [target_breakpoint] + list(other_breakpoint[:4])
        for p in self.pos:
            if p[:5] == key:
                p[5] += cnt
                break
        else:
            self.pos.append([target_breakpoint] + list(other_breakpoint) + [cnt])
        self.spanning_reads.extend(spanning_reads)
        self.split_reads.extend(split_reads)

    def left_seq(self):
        return "".join(_vote_call(self.seq_left[c]) for c in range(200 - self.l_left, 200))

    def right_seq(self):
        return "".join(_vote_call(self.seq_right[c]) for c in range(self.l_right))

    def mid_seq(self):
        return "".join(_vote_call(self.seq_mid[c]) for c in range(self.l_mid))

    def find_max_pos(self):
        best, best_cnt = 0, 0
        for k, p in enumerate(self.pos):
            if p[6] > best_cnt:
                best, best_cnt = k, p[6]
        return self.pos[best] + [self.left_seq(), self.right_seq(), self.type_, self.mid_seq()], best


_HEAD = ["Fusion_gene", "Anchored_gene_X", "X_clip_location", "Partner_gene_Y", "Y_clip_location"]


def _partner(index, chrom, bp):
    return index.find_exon(chrom, bp, bp + 1)[0]


def _row_head(pos, gene_name, index):
    anchor_bp, chrom, other_bp = pos[0], pos[1], pos[2]
    other = _partner(index, chrom, other_bp)
    fusion = (other[1] + "--" + gene_name) if pos[9] == "SM" else (gene_name + "--" + other[1])
    return "\t".join([fusion, gene_name, f"{gene_name}:{anchor_bp}", f"{other[1]}:{other[0]}", f"{chrom}:{other_bp}"])


def _alt_name(type_, pos, gene_name, index):
    anchor_bp, chrom, other_bp = pos[0], pos[1], pos[2]
    other = _partner(index, chrom, other_bp)
    if type_ == "SM":
        return f"{other[1]}:{chrom}:{other_bp}--{gene_name}:{anchor_bp}"
    return f"{gene_name}:{anchor_bp}--{other[1]}:{chrom}:{other_bp}"


def prediction_rows(candidates, gene_name, index, scores, cnt_max, no_filter=True):
    """The rows of both tables as lists of strings (no header, no newline)."""
    abridged, full = [], []
    seen = []
    for j, cand in enumerate(candidates):
        pos, best = cand.find_max_pos()
        head = _row_head(pos, gene_name, index)
        key = (pos[0], pos[1], pos[2], pos[3])
        if key in seen:
            continue
        seen.append(key)
        span = list(set(cand.spanning_reads))
        split = list(set(cand.split_reads))
        if len(span) * 10 < len(split) or len(split) * 10 < len(span):
            continue
        if not span and not split:
            continue
        counts = [str(len(span)), str(len(split))]
        alts = [_alt_name(cand.type_, p, gene_name, index) for k, p in enumerate(cand.pos) if k != best]
        tail = [";".join(span), ";".join(split), ";".join(alts)]
        if no_filter:
            abridged.append("\t".join([head] + counts))
            full.append("\t".join([head] + counts + tail))
        else:
            abridged.append("\t".join([head, str(cand.score)] + counts))
            sc = scores[j]
            if sc > 0.1 and (len(set(span + split)) * 10 > cnt_max or sc > 0.9):
                full.append("\t".join([head, str(sc)] + counts + tail))
    return abridged, full


def write_predictions(prefix, candidates, gene_name, index, scores, cnt_max, no_filter=True):
    abridged, full = prediction_rows(candidates, gene_name, index, scores, cnt_max, no_filter)
    counts = ["Spanning_read_count", "Breakpoint_read_count"]
    mid = [] if no_filter else ["Natural_score"]
    tail = ["Spanning_reads", "Breakpoint_reads", "Breakpoint_site_reads_1", "Breakpoint_site_reads_2", "Homo_genes"]
    with open(prefix + "_predictions_abridged.txt", "w") as fa:
        fa.write("\t".join(_HEAD + mid + counts) + "\n")
        fa.writelines(r + "\n" for r in abridged)
    with open(prefix + "_predictions.txt", "w") as fo:
        fo.write("\t".join(_HEAD + mid + counts + tail) + "\n")
        fo.writelines(r + "\n" for r in full)
