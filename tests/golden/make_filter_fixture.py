"""Golden outputs of the reference filter network (Model.py `Model`) for the parity test of
anchored_fusion_amd.filter_model (SURVEY.md §8 f rank 4).

Run HERE only (imports /root/reference/Model.py; nothing on the GPU box reads it):

    python tests/golden/make_filter_fixture.py

The reference network is built with Test_model's hyper-parameters (Model.py:318-329) for
201-position windows, loaded with the seeded weights of tests/filter_cases.py (strict: the
parameter names and shapes must match), converted to float64 as Test_model does, and run on the
windows of tests/filter_cases.py (encoded by the reference's read_lines) in eval mode and in train mode (Test_model's mode) under
torch.manual_seed(99); and Test_model itself (file in, scores out) under torch.manual_seed(77).
Inputs and outputs go to tests/golden/filter_model.json.
"""
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import afpkg  # noqa: E402,F401
from filter_cases import seeded_state, windows  # noqa: E402



def main():
    sys.dont_write_bytecode = True
    sys.path.insert(0, "/root/reference")
    import Model as ref  # noqa: N813
    import tempfile
    wins = windows()
    with tempfile.NamedTemporaryFile("w", suffix=".txt", delete=False) as fh:  # get_test_reads' layout
        fh.writelines(f"{w}\t{k}\n" for k, w in enumerate(wins))
    x = ref.read_lines(fh.name)  # the reference's own encoding (Model.py:170-187)
    net = ref.Model(6, 256, 256, 256, 3, 3, 4, 128, 2, x.shape[1], 0.2)
    net.load_state_dict(seeded_state(net), strict=True)
    net = net.double()
    code = torch.where(x.sum(-1) > 0, x.argmax(-1), torch.full(x.shape[:2], -1))
    out = {"windows": wins, "len_seq": int(x.shape[1]), "channel": code.tolist()}
    with torch.no_grad():
        net.eval()
        (a, b), c = net(x)
        out["eval"] = [a.tolist(), b.tolist(), c.tolist()]
        net.train()
        torch.manual_seed(99)
        (a, b), c = net(x)
        out["train_seed99"] = [a.tolist(), b.tolist(), c.tolist()]
    # Test_model end to end (its training-mode forward) under torch.manual_seed(77): the seed is
    # set before the network is built, so the scores also pin the parameter-creation order
    model_file = fh.name + ".pt"
    torch.save(seeded_state(net), model_file)
    torch.manual_seed(77)
    out["test_model_seed77"] = [float(v) for v in ref.Test_model(fh.name, model_file, "-1")]
    os.remove(model_file)
    os.remove(fh.name)
    with open(os.path.join(HERE, "filter_model.json"), "w") as out_fh:
        json.dump(out, out_fh, indent=1)


if __name__ == "__main__":
    main()
