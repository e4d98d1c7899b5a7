"""Filter network (anchored_fusion_amd.filter_model; SURVEY.md §8 f rank 4) against the
reference Model.py: outputs of the reference network with the same seeded weights on the same
windows (tests/golden/filter_model.json, made by tests/golden/make_filter_fixture.py).
Float64 throughout; the bar is 1e-10 absolute on probabilities."""
import json
import os

import numpy as np
import pytest
import torch

import afpkg  # noqa: F401
from anchored_fusion_amd import filter_model as fm
from filter_cases import seeded_state

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "filter_model.json")))


def _net(device="cpu"):
    net = fm.FusionFilter(GOLD["len_seq"], **fm.HPARAMS)
    net.load_state_dict(seeded_state(net), strict=True)
    return net.to(device).double()


def test_one_hot_matches_read_lines():
    x = fm.one_hot(GOLD["windows"])
    code = torch.where(x.sum(-1) > 0, x.argmax(-1), torch.full(x.shape[:2], -1))
    assert code.tolist() == GOLD["channel"]
    assert float(x.sum(-1).max()) == 1.0


@pytest.mark.parametrize("mode", ["eval", "train_seed99"])
def test_outputs_match_reference(mode):
    net = _net()
    x = fm.one_hot(GOLD["windows"])
    with torch.no_grad():
        net.train(mode != "eval")
        if mode != "eval":
            torch.manual_seed(99)
        (a, b), c = net(x)
    for got, want in zip((a, b, c), GOLD[mode]):
        assert np.allclose(got.numpy(), np.array(want), atol=1e-10, rtol=0)


def test_score_windows_is_head3_class1(tmp_path):
    net = _net()
    want = np.array(GOLD["eval"][2])[:, 1]
    got = fm.score_windows(GOLD["windows"], net=net, train_mode=False)
    assert np.allclose(got, want, atol=1e-10, rtol=0)
    # a reference-trained state_dict file loads as-is (weights_only)
    path = str(tmp_path / "model.pt")
    torch.save(seeded_state(net), path)
    test_file = tmp_path / "test_reads.txt"
    test_file.write_text("".join(f"{w}\t{k}\n" for k, w in enumerate(GOLD["windows"])))
    torch.manual_seed(77)  # as the fixture: seeded before the network is built
    s = fm.score_test_file(str(test_file), path)  # Test_model's (train-mode) behaviour
    assert np.allclose(s, np.array(GOLD["test_model_seed77"]), atol=1e-10, rtol=0)


@pytest.mark.gpu
def test_outputs_on_gpu():
    net = _net("cuda:0")
    got = fm.score_windows(GOLD["windows"], device="cuda:0", net=net, train_mode=False)
    assert np.allclose(got, np.array(GOLD["eval"][2])[:, 1], atol=1e-8, rtol=0)
