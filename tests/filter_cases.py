"""Seeded weights and junction windows for the filter-network parity tests (TEST INFRASTRUCTURE)."""
import numpy as np
import torch


def seeded_state(net):
    """A deterministic state_dict for a network with FusionFilter's parameter names: every float
    tensor N(0, 0.05^2) from its own seed (sorted names), batch-norm variances in [0.5, 1.5),
    counters 0."""
    state = {}
    for i, (k, v) in enumerate(sorted(net.state_dict().items())):
        g = torch.Generator().manual_seed(1000 + i)
        if not v.is_floating_point():
            state[k] = torch.zeros_like(v)
        elif k.endswith("running_var"):
            state[k] = 0.5 + torch.rand(v.shape, generator=g, dtype=torch.float64)
        else:
            state[k] = 0.05 * torch.randn(v.shape, generator=g, dtype=torch.float64)
    return state


def windows(n=6, half=100, seed=5):
    """Junction windows as get_test_reads lays them out: N-padded left flank, 'H', right flank."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        a, b = int(rng.integers(40, half + 1)), int(rng.integers(40, half + 1))
        left = "".join(rng.choice(list("ACGT"), a))
        right = "".join(rng.choice(list("acgtD"), b))
        out.append("N" * (half - a) + left + "H" + right + "N" * (half - b))
    return out
