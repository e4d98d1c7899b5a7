"""Exon annotation index.

Restates `Gene_co` (functions.py:7-86) and `find_positions` (functions.py:1331-1391):

* exons of every non-pseudogene transcript (GTF `exon` rows; transcript types containing
  "pseudogene", "artifact" and "protein_coding_LoF" are skipped), per chromosome, sorted and
  merged when overlapping within the same gene (or inside the hard-coded IGH@/TRA@ loci,
  which the reference adds for hg38);
* `find_exon` is the ±10 nt tolerant lookup (binary search on starts, then the neighbour
  below, then a forward scan);
* `walk` walks `length` transcript bases upstream and downstream of a position along the
  same gene's exons (used to widen breakpoint blocks by 200 nt).

GTF attribute parsing follows the reference exactly, including that gene_id / gene_name /
transcript_type carry over from the previous exon row when a row lacks them, and that a GTF
without any transcript_type fails (the reference raises NameError).
"""

NO_GENE = ["", "", "", "", ""]

# hard-coded hg38 loci the reference appends (functions.py:40-46)
_EXTRA = (("chr14", [105586337, 106879944, "IGH@", "IGH@"]),
          ("chr14", [21621804, 22552332, "TRA@", "TRA@"]),
          ("KI270846.1", [0, 1351393, "IGH@", "IGH@"]))


class ExonIndex:
    """chrom -> sorted list of [start, end, gene_id, gene_name] (1-based closed, GTF)."""

    def __init__(self, table=None):
        self.dic = table if table is not None else {}

    # -- construction -------------------------------------------------------------------
    @classmethod
    def from_gtf(cls, path):
        with open(path) as fh:
            return cls.from_lines(fh.readlines())

    @classmethod
    def from_lines(cls, lines):
        dic = {}
        state = {}
        for line in lines:
            if line.startswith("##"):
                continue
            col = line.split("\t")
            if col[2] != "exon":
                continue
            for item in col[8].rstrip().split(";"):
                item = item.rstrip()
                if not item:
                    continue
                if item[0] == " ":
                    item = item[1:]
                kv = item.split(" ")
                if len(kv) == 2 and kv[0] in ("gene_id", "gene_name", "transcript_type"):
                    state[kv[0]] = kv[1][1:-1]
            if "transcript_type" not in state:
                raise NameError("GTF exon row without transcript_type (reference: functions.py:34)")
            tt = state["transcript_type"]
            if "pseudogene" in tt or tt in ("artifact", "protein_coding_LoF"):
                continue
            if "gene_id" not in state or "gene_name" not in state:
                raise NameError("GTF exon row without gene_id/gene_name")
            dic.setdefault(col[0], []).append([int(col[3]), int(col[4]), state["gene_id"], state["gene_name"]])
        for chrom, rec in _EXTRA:
            dic.setdefault(chrom, []).append(list(rec))
        for rows in dic.values():
            rows.sort()
            merged = []
            for r in rows:
                if merged and merged[-1][1] >= r[0] and (merged[-1][2] == r[2] or merged[-1][2] in ("IGH@", "TRA@")):
                    if r[1] > merged[-1][1]:
                        merged[-1][1] = r[1]
                    continue
                merged.append(r)
            rows[:] = merged
        return cls(dic)

    # -- lookups ---------------------------------------------------------------------------
    def find_exon(self, chrom, start, end):
        """(gene_id, gene_name, chrom, exon_start, exon_end), exon index -- or NO_GENE, -1."""
        rows = self.dic.get(chrom)
        if rows is None or chrom == "chrM":
            return list(NO_GENE), -1

        def hit(k):
            r = rows[k]
            return [r[2], r[3], chrom, r[0], r[1]], k

        lo, hi = 0, len(rows)
        while hi - lo > 1:                      # last row whose start <= start (or row 0)
            mid = (lo + hi) // 2
            if rows[mid][0] <= start:
                lo = mid
            else:
                hi = mid
        near = lambda k: rows[k][0] - 10 <= start and rows[k][1] + 10 >= end  # noqa: E731
        if near(lo):
            return hit(lo)
        if lo >= 1 and near(lo - 1):
            return hit(lo - 1)
        k = lo + 1
        while k < len(rows) and rows[k][0] - 10 <= start:
            if rows[k][1] + 10 >= end:
                return hit(k)
            k += 1
        return list(NO_GENE), -1

    def walk(self, chrom, pos, length):
        """Exon intervals covering `length` bases on each side of `pos` within its gene.

        Returns [(s, e), ... upstream ..., ['H', ''], ... downstream ...] with 0-based starts,
        as find_positions (functions.py:1331-1391); [] when pos is in no gene."""
        gene, k0 = self.find_exon(chrom, pos, pos)
        if gene[0] == "":
            return []
        rows = self.dic[chrom]
        name = gene[1]

        def inside(k, p):
            return rows[k][3] == name and rows[k][0] <= p < rows[k][1] + 1

        up = []
        left, k, p = length, k0, pos - 1
        while left > 0:
            if not inside(k, p):
                k -= 1
                if not 0 <= k < len(rows):
                    break
                p = rows[k][1]
                continue
            span = p - rows[k][0] + 1
            if span >= left:
                up.append((p - left, p))
                left -= span
            elif span != 0:
                left -= span
                up.append((rows[k][0] - 1, p))
                k -= 1
                if k < 0:
                    break
                p = rows[k][1]
            else:
                k -= 1
                if k < 0:
                    break
                p = rows[k][1]
        out = up[::-1] + [["H", ""]]
        right, k, p = length, k0, pos
        while right > 0:
            if not inside(k, p):
                k += 1
                if not 0 <= k < len(rows):
                    break
                p = rows[k][0]
                continue
            span = rows[k][1] + 1 - p
            if span >= right:
                out.append((p - 1, p + right - 1))
                right = 0
            elif span != 0:
                right -= span
                out.append((p - 1, rows[k][1]))
                k += 1
                if k >= len(rows):
                    break
                p = rows[k][0]
            else:
                k += 1
                if k >= len(rows):
                    break
                p = rows[k][0]
        return out
