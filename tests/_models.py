"""Small modules shared by the golden-vector generator and the tests."""
import torch
import torch.nn as nn


class TinyNet(nn.Module):
    """Covers every entry kind the reference models have: conv (cosine column kind, B=9),
    BatchNorm (running stats + int64 num_batches_tracked), 1x1 conv (row kind), linear with
    odd sizes (n % 4 tails)."""

    def __init__(self):
        super().__init__()
        self.conv = nn.Conv2d(3, 4, 3)
        self.bn = nn.BatchNorm2d(4)
        self.pw = nn.Conv2d(4, 6, 1, bias=False)
        self.fc = nn.Linear(13, 5)
        self.bn2 = nn.BatchNorm1d(5)


class Vec(nn.Module):
    def __init__(self, m):
        super().__init__()
        self.v = nn.Parameter(torch.zeros(m))


def cos_pair_state(layout, sa, sb, entries, mix):
    """Two seeded synthetic state_dicts (topology_aware_learning_amd.synth); with `mix`, the
    second is a + mix * b (fp32, a multiply then an add: a neighbor close to the first, as
    trained neighbors are).  tests/golden/cosine_threads.json's inputs."""
    from topology_aware_learning_amd import synth

    a = synth.synth_state_dict(layout, sa, entries=entries)
    b = synth.synth_state_dict(layout, sb, entries=entries)
    if mix:
        b = type(b)((k, a[k] + b[k] * mix) for k in b)
    return a, b
