"""Host-side dispatch of aido1_amd/train_ops.py (no GPU): which layers the
update's kernels take.  The GPU parity of those kernels is
tests/test_gpu_upd_conv.py."""
import torch

from conftest import golden
from test_trainer import no_dropout

from aido1_amd import train_ops
from aido1_amd.actor import ConfigActor, ConfigCritic


def test_cpu_tensors_stay_on_torch():
    cfg = golden('reference_config.json')
    crit = ConfigCritic(no_dropout(cfg['model']['critic'])).train()
    mods = crit.net.input_nets[0].internal_modules
    x = torch.zeros(2, 3, 120, 160)
    assert train_ops.trunk_len(x, mods, 0, len(mods)) == 0       # CPU: torch modules run
    lin = torch.nn.Linear(4032, 256)
    assert not train_ops.linear_applicable(torch.zeros(2, 4032), lin)


def test_config_layers_are_the_kernels_geometries():
    """config.json's four conv layers at 120 x 160 are exactly
    UPD_CONV_LAYERS (so the whole trunk is one chain on the GPU)."""
    cfg = golden('reference_config.json')
    actor = ConfigActor(cfg['model']['actor'])
    convs, _, lin1, _ = actor.layers()
    shape = (3, 120, 160)
    got = set()
    for c in convs:
        ks, st = c.weight.shape[2], c.stride[0]
        got.add((shape[0], ks, st, shape[1], shape[2]))
        shape = (32, (shape[1] - ks) // st + 1, (shape[2] - ks) // st + 1)
    assert got == train_ops.UPD_CONV_LAYERS
    assert 32 * shape[1] * shape[2] == lin1.in_features == 4032
    assert lin1.in_features >= train_ops.LINEAR_MIN_K and lin1.out_features % 32 == 0
