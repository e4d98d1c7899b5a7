"""False-positive filter network on PyTorch-ROCm (SURVEY.md §8 f rank 4; Model.py, off the hot path).

The reference scores each fusion candidate with a small network over a one-hot window of the
junction (`Test_model`, Model.py:314-333): 6 input channels (A T G C, 'H' = the junction, 'D'),
an input projection, two conv blocks each feeding a softmax head, a one-layer transformer
encoder and a third head whose class-1 probability is the score `Final_fusion` thresholds
(functions.py:1786-1791).  This module rebuilds that network so that a `model.pt` trained by the
reference loads as-is (same parameter names and shapes; `torch.load(weights_only=True)`), and
restates the scoring entry point:

| reference | here |
|---|---|
| `read_lines` (MD:170-187) | `one_hot` |
| `Model` and its blocks (MD:46-131) | `FusionFilter` |
| `Test_model` (MD:314-333), `test` (MD:263-268) | `score_windows`, `score_test_file` |

As in the reference, scoring runs the network in float64 WITHOUT switching it to eval mode: the
batch norms use the batch's statistics and the heads' dropout (p = 0.2) is live, so scores are
random unless the caller seeds torch.  `score_windows(..., train_mode=False)` gives the
deterministic eval-mode scores.

Pinned by tests/golden/filter_model.json: the reference `Model` (imported here only, by
tests/golden/make_filter_fixture.py) and this network, loaded with the same seeded weights, give
the same outputs in eval mode and, under the same torch seed, in train mode; and the reference's
own `Test_model` (file in, scores out, seeded before the network is built) gives the scores
`score_test_file` gives under the same seed, which also pins the parameter-creation order.

`get_test_reads` (fn:1642-1721), the input-window builder, is `get_test_reads` here: per distinct
candidate breakpoint, 100 exon bases on each side of the partner breakpoint (`find_positions`,
`ExonIndex.walk`) fetched as `bedtools getfasta -s -nameOnly` would (the BED rows carry the
strand in column 5, the score column, so `-s` sees no strand and nothing is reverse-complemented),
and 100 anchor bases on each side of the anchor breakpoint.  Its quirks are kept: the flank tag is
read as `line[1:-3].split('$')[2]`, which cuts "ft\n" (">0$+$left\n" gives 'le') or "+)\n" and
so never equals 'left' -- every partner flank base (about 200) lands in the right-hand sequence;
the id written beside each window is the previous header's; a '-' strand swaps and
reverse-complements the partner flanks of the NEXT candidate (`strand_last`).  MS windows, and
SM windows after a '-' strand, are therefore about 301 positions long instead of the 201 a
trained model expects; scoring such a file fails in the reference's `Test_model` as it does in
`score_test_file` (ragged windows, or a 33-row position table against a model trained on 22).
Only a missing model file is caught (AF:214-225): the run then proceeds as
`--not_filter_false_positive`, which is what the reference does with its default
`--model_file ./data/model.pt` (not shipped).
"""
import os

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

# Test_model's hyper-parameters (MD:318-329)
HPARAMS = dict(input_dim=6, block_dim=256, embed_dim=256, class_dim=256, window=3, maxpool_dim=3,
               class_shrink_dim=4, transformer_dim=128, num_class=2, dropout=0.2)
_CHANNEL = {"A": 0, "T": 1, "G": 2, "C": 3, "H": 4, "D": 5}


def one_hot(windows):
    """read_lines (MD:170-187) on the window strings: float64 [n, L, 6]; characters outside
    A/T/G/C/H/D (N padding) are all-zero rows.  All windows must have the same length."""
    seqs = [w.upper().replace("\n", "") for w in windows]
    n = len(seqs)
    L = len(seqs[0]) if n else 0
    if any(len(s) != L for s in seqs):
        raise ValueError("windows of different lengths")
    codes = np.frombuffer("".join(seqs).encode(), dtype=np.uint8).reshape(n, L) if n else np.zeros((0, 0), np.uint8)
    lut = np.full(256, -1, np.int64)
    for ch, k in _CHANNEL.items():
        lut[ord(ch)] = k
    idx = lut[codes]
    x = np.zeros((n, L, 6), np.float64)
    rows, cols = np.nonzero(idx >= 0)
    x[rows, cols, idx[rows, cols]] = 1.0
    return torch.from_numpy(x)


class _Head(nn.Module):
    """prj -> flatten -> fc1/relu/dropout -> fc2, softmax at temperature t (MD:79-92)."""

    def __init__(self, width, hidden, positions, shrink, num_class):
        super().__init__()
        self.prj = nn.Linear(width, width // shrink)
        self.flatten = nn.Flatten()
        self.classify = _Mlp(positions * width // shrink, hidden, num_class, p_drop=0.2)

    def forward(self, x, temperature=1.0):
        return F.softmax(self.classify(self.flatten(self.prj(x))) / temperature, dim=1)


class _Mlp(nn.Module):
    def __init__(self, n_in, n_mid, n_out, p_drop):
        super().__init__()
        self.fc1 = nn.Linear(n_in, n_mid)
        self.dropout = nn.Dropout(p_drop)
        self.fc2 = nn.Linear(n_mid, n_out)
        self.relu = nn.ReLU()

    def forward(self, x):
        return self.fc2(self.dropout(self.relu(self.fc1(x))))


class _ConvBlock(nn.Module):
    """conv(window) -> batch norm -> relu -> conv(window) -> relu -> average pool, over the
    position axis (MD:61-77)."""

    def __init__(self, c_in, c_mid, c_out, window, pool):
        super().__init__()
        self.normal_layer1 = nn.BatchNorm1d(c_mid)
        self.conv1 = nn.Conv1d(c_in, c_mid, window, padding=window // 2)
        self.conv2 = nn.Conv1d(c_mid, c_out, window, padding=window // 2)
        self.relu = nn.ReLU()
        self.avgpool = nn.AvgPool1d(pool, stride=pool)

    def forward(self, x):  # x: [n, positions, channels]
        y = self.relu(self.normal_layer1(self.conv1(x.transpose(1, 2))))
        return self.avgpool(self.relu(self.conv2(y))).transpose(1, 2)


class _Encoder(nn.Module):
    """Linear embedding + learned positions + one post-norm transformer layer (2 heads, no
    dropout) + relu (MD:94-111)."""

    def __init__(self, width, positions, hidden, layers, heads):
        super().__init__()
        self.len_seq = positions
        self.input_embedding = nn.Linear(width, hidden)
        self.position_encoding = nn.Embedding(positions, hidden)
        nn.init.normal_(self.position_encoding.weight, std=0.02)
        layer = nn.TransformerEncoderLayer(hidden, heads, dropout=0.0, batch_first=True)
        self.transformer_encoder = nn.TransformerEncoder(layer, num_layers=layers)
        self.relu = nn.ReLU()

    def forward(self, x):
        pos = self.position_encoding(torch.arange(self.len_seq, device=x.device).unsqueeze(0))
        return self.relu(self.transformer_encoder(self.input_embedding(x) + pos))


class FusionFilter(nn.Module):
    """Model (MD:113-131): returns ((head1, head2), head3), each [n, num_class] probabilities;
    head3[:, 1] is the candidate score."""

    def __init__(self, len_seq, input_dim=6, block_dim=256, embed_dim=256, class_dim=256, window=3, maxpool_dim=3,
                 class_shrink_dim=4, transformer_dim=128, num_class=2, dropout=0.2):
        super().__init__()
        del dropout  # the reference hard-codes p = 0.2 in its heads
        p1, p2 = len_seq // maxpool_dim, len_seq // maxpool_dim ** 2
        self.embed_dim, self.num_class = embed_dim, num_class
        self.relu = nn.ReLU()
        self.input_embedding = nn.Linear(input_dim, embed_dim)
        self.block1 = _ConvBlock(embed_dim, block_dim, embed_dim, window, maxpool_dim)
        self.classify1 = _Head(embed_dim, class_dim, p1, class_shrink_dim, num_class)
        self.block2 = _ConvBlock(embed_dim, block_dim, embed_dim, window, maxpool_dim)
        self.classify2 = _Head(embed_dim, class_dim, p2, class_shrink_dim, num_class)
        self.transformer = _Encoder(embed_dim, p2, transformer_dim, 1, 2)
        self.classify3 = _Head(transformer_dim, class_dim, p2, class_shrink_dim, num_class)

    def forward(self, x):
        x = self.block1(self.relu(self.input_embedding(x)))
        h1 = self.classify1(x, 0.25)
        x = self.block2(x)
        h2 = self.classify2(x, 0.25)
        return (h1, h2), self.classify3(self.transformer(x))


def load_filter(len_seq, model_file=None, device="cpu"):
    """The network for windows of len_seq positions, float64 on `device`; weights from
    model_file when it exists (state_dict saved by the reference's training), else the
    initialisation (as Test_model does when the file is missing)."""
    net = FusionFilter(len_seq, **HPARAMS)
    if model_file and os.path.exists(model_file):
        net.load_state_dict(torch.load(model_file, map_location="cpu", weights_only=True))
    return net.to(device).double()


@torch.no_grad()
def score_windows(windows, model_file=None, device="cpu", train_mode=True, net=None):
    """Test_model (MD:314-333) on window strings: the class-1 probability of head 3 per window.
    train_mode=True keeps the reference's behaviour (module left in training mode)."""
    x = one_hot(windows)
    if net is None:
        net = load_filter(x.shape[1], model_file, device)
    net.train(train_mode)
    return net(x.to(device))[1][:, 1].cpu().numpy().tolist()


def score_test_file(test_file, model_file, device="cpu"):
    """Test_model on a `<window>\\t<id>` file as get_test_reads writes it."""
    with open(test_file) as fh:
        windows = [ln.split("\t")[0].upper().replace("\n", "") for ln in fh]
    return score_windows(windows, model_file, device)


_RC = {"A": "T", "T": "A", "G": "C", "C": "G", "N": "N", "H": "H"}


def _reverse(seq):
    """functions.py:498 `reverse`: reverse complement over A/C/G/T/N/H (KeyError otherwise)."""
    return "".join(_RC[c] for c in seq[::-1])


def get_test_reads(candidates, anchor_seq, index, getfasta):
    """get_test_reads (fn:1642-1721): the `<window>\t<id>` lines of the test file, in the
    reference's order and with its quirks (module docstring).  candidates: report.Candidate list
    (Find_candidate_genes' order); anchor_seq: the anchored transcript (the FASTA's sequence lines
    joined, fn:1646-1649); index: annotation.ExonIndex; getfasta(rows): `bedtools getfasta` of
    (chrom, start, end, name) rows -> [(header, seq)], intervals outside a contig skipped."""
    bed, seen, id_ = [], [], 0
    for cand in candidates:
        pos, _ = cand.find_max_pos()
        target_bp, chrom, other_bp, strand = pos[0], pos[1], pos[2], pos[3]
        key = (target_bp, chrom, other_bp, strand)
        if key in seen:
            continue
        seen.append(key)
        t = cand.type_
        at = other_bp + 1 if (t == "SM" and strand == "+") or (t == "MS" and strand == "-") else other_bp
        flag = "left"
        for p in index.walk(chrom, at, 100):
            if p[0] == "H":
                flag = "right"
                continue
            bed.append((chrom, int(p[0]), int(p[1]), f"{id_}${strand}${flag}"))
        id_ += 1
    # bedtools getfasta -s -nameOnly: one header line (the name) and one sequence line per row
    lines = []
    for hdr, seq in getfasta(bed):  # rows outside a contig are skipped, as bedtools does
        lines.append(">" + hdr.split("::")[0] + "\n")
        lines.append(seq + "\n")
    if not lines:
        raise IndexError("get_test_reads: no flank sequence (the reference indexes lines[0] here)")
    out, seen = [], []
    last_id = "0"
    strand_last = lines[0][1:-3].split("$")[1]
    fusion_id, strand, dir_ = last_id, strand_last, ""
    i = 0
    for cand in candidates:
        pos, _ = cand.find_max_pos()
        target_bp, chrom, other_bp, strand_c = pos[0], pos[1], pos[2], pos[3]
        key = (target_bp, chrom, other_bp, strand_c)
        if key in seen:
            continue
        seen.append(key)
        seq_left2 = seq_right2 = ""
        while i < len(lines):
            if lines[i].startswith(">"):
                fusion_id, strand, dir_ = lines[i][1:-3].split("$")
                if fusion_id != last_id or i == len(lines) - 1:
                    break
            else:
                if dir_ == "left":
                    seq_left2 += lines[i][:-1].upper()
                else:
                    seq_right2 += lines[i][:-1].upper()
            i += 1
        if strand_last == "-":
            seq_left2, seq_right2 = _reverse(seq_right2), _reverse(seq_left2)
        lo = target_bp - min(101, target_bp)
        seq_left1 = anchor_seq[lo:target_bp - 1]
        seq_right1 = anchor_seq[target_bp - 1:min(target_bp + 99, len(anchor_seq))]
        if cand.type_ == "MS":
            w = "N" * (100 - len(seq_left1)) + seq_left1 + "H" + seq_right2 + "N" * (100 - len(seq_right2))
        else:
            w = "N" * (100 - len(seq_left2)) + seq_left2 + "H" + seq_right1 + "N" * (100 - len(seq_right1))
        out.append(w + "\t" + last_id + "\n")
        last_id = fusion_id
        strand_last = strand
    return out



def score_candidates(candidates, anchor_seq, index, getfasta, model_file, out_prefix, device="cpu", log=print):
    """The filter step of Anchored_Fusion.py:212-225: (scores, no_filter).  A missing model file
    is reported and the run continues without the filter, as the reference's FileNotFoundError
    branch does; otherwise the windows are written to `<out_prefix>_test_reads.txt`
    (get_test_reads), scored by Test_model and set on the candidates by candidate index (a
    duplicate breakpoint leaves fewer windows than candidates and raises IndexError there, as in
    the reference)."""
    try:
        with open(model_file):
            pass
    except FileNotFoundError:
        log("Error: model file not found!, not performing filter false positives.")
        return [], True
    lines = get_test_reads(candidates, anchor_seq, index, getfasta)
    test_file = out_prefix + "_test_reads.txt"
    with open(test_file, "w") as fh:
        fh.writelines(lines)
    scores = [float(x) for x in score_test_file(test_file, model_file, device)]
    for i, cand in enumerate(candidates):
        cand.score = scores[i]
    return scores, False
