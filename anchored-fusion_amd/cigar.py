"""CIGAR normalisation used by every split-read consumer.

Restates `deal_cigar` (functions.py:656-702) behaviour, including its quirks, because the
downstream stages key on its exact output:

* ops become ``[end, length, op]`` where ``end`` is the running sum of op lengths;
* ``N`` and ``H`` ops are dropped and the ends after them move back by their length;
* ``D`` is dropped, its length is added to the NEXT op (whose end is left as it was), and
  the sequence gets ``'N' * len`` inserted at the end of the PREVIOUS op -- for a leading
  ``D`` "previous" is the last op (Python's ``[-1]``), as in the reference;
* ``I`` is dropped, later ends move back, and the read bases between the previous op's end
  and the ``I``'s own end are removed (same ``[-1]`` rule for a leading ``I``);
* adjacent ``M`` runs (after the removals) are merged.

A read is a "split read" when exactly two ops remain (S+M or M+S).
"""
import re

_OP = re.compile(r"(\d+)([A-Za-z=])")


def parse(cigar):
    """'30S70M' -> [[30, 30, 'S'], [100, 70, 'M']] (running end, length, op)."""
    out, end = [], 0
    for n, op in _OP.findall(cigar):
        end += int(n)
        out.append([end, int(n), op])
    return out


def normalize(cigar, seq):
    """Returns (ops, seq') with the semantics of functions.py:656-702 (module docstring)."""
    ops = parse(cigar)
    k = 0
    while k < len(ops):
        end, ln, op = ops[k]
        if op in ("N", "H", "I"):
            for later in ops[k + 1:]:
                later[0] -= ln
            if op == "I":
                cut = ops[k - 1][0]           # k == 0 reads ops[-1], as the reference does
                seq = seq[:cut] + seq[end:]
            del ops[k]
        elif op == "D":
            if k + 1 < len(ops):
                ops[k + 1][1] += ln
            at = ops[k - 1][0]
            seq = seq[:at] + "N" * ln + seq[at:]
            del ops[k]
        else:
            k += 1
    merged = []
    for e in ops:
        if merged and merged[-1][2] == "M" and e[2] == "M":
            merged[-1][0] = e[0]
            merged[-1][1] += e[1]
        else:
            merged.append(e)
    return merged, seq


_RC = {"A": "T", "T": "A", "G": "C", "C": "G", "N": "N", "H": "H"}


def revcomp(seq):
    """functions.py:498-503 (`reverse`): reverse complement over ACGTNH (other bytes raise)."""
    return "".join(_RC[c] for c in reversed(seq))
