"""Actor: the reference's two actor layouts reproduced with
identical parameter names, against golden outputs of the reference's own
modules (tests/golden/actor.npz, formula weights from tests/golden/formulas.py),
and the BN-folded inference copy against the eval-mode actor."""
import os
import sys

import numpy as np
import pytest
import torch

from conftest import GOLDEN, golden

sys.path.insert(0, GOLDEN)
from formulas import formula_input, formula_state_dict  # noqa: E402


def test_actor_cnn_golden():
    from aido1_amd.actor import ActorCNN
    g = golden('actor.npz')
    a = ActorCNN(2, 1.0)
    assert list(a.state_dict().keys()) == [str(k) for k in g['actor_cnn_keys']]
    a.load_state_dict(formula_state_dict(a.state_dict()))
    a.eval()
    with torch.no_grad():
        y = a(formula_input(4)).numpy()
    assert np.max(np.abs(y - g['actor_cnn'])) < 1e-5


def test_config_actor_golden():
    from aido1_amd.actor import ConfigActor
    g = golden('actor.npz')
    cfg = golden('reference_config.json')
    a = ConfigActor(cfg['model']['actor'])
    assert list(a.state_dict().keys()) == [str(k) for k in g['config_actor_keys']]
    a.load_state_dict(formula_state_dict(a.state_dict()))
    a.eval()
    with torch.no_grad():
        y = a(formula_input(4)).numpy()
    assert np.max(np.abs(y - g['config_actor'])) < 1e-5


@pytest.mark.parametrize('kind', ['cnn', 'config'])
def test_fused_actor_matches_eval_fp32(kind):
    from aido1_amd.actor import ActorCNN, ConfigActor, FusedActor
    a = ActorCNN(2, 1.0) if kind == 'cnn' else ConfigActor(golden('reference_config.json')['model']['actor'])
    a.load_state_dict(formula_state_dict(a.state_dict()))
    a.eval()
    f = FusedActor(a, dtype=torch.float32)
    x = formula_input(4)
    with torch.no_grad():
        ref = a(x)
    assert torch.max(torch.abs(f(x) - ref)) < 1e-4
    # ring order: feeding the slots in ring order with `order` == feeding the stack
    order = [2, 0, 1]
    ring = torch.empty_like(x)
    for c, sl in enumerate(order):
        ring[:, sl] = x[:, c]
    assert torch.max(torch.abs(f(ring, order) - ref)) < 1e-4


def test_flops_figure():
    from aido1_amd.actor import flops_per_sample
    # 50.8 M MAC = 101.6 MFLOP per env per decision
    assert abs(flops_per_sample() / 1e6 - 101.6) < 0.2


def _per_sample_train_mode(actor, x):
    """The reference's acting: train-mode modules, one observation per call."""
    import copy as _copy
    a = _copy.deepcopy(actor)
    a.train()
    with torch.no_grad():
        return torch.cat([a(x[i:i + 1]) for i in range(x.shape[0])])


def test_fused_reference_mode_equals_per_sample_train_mode():
    from aido1_amd.actor import ConfigActor, FusedActor
    from test_trainer import no_dropout
    a = ConfigActor(no_dropout(golden('reference_config.json')['model']['actor']))
    a.load_state_dict(formula_state_dict(a.state_dict()))
    x = formula_input(4)
    ref = _per_sample_train_mode(a, x)
    f = FusedActor(a, dtype=torch.float32, mode='reference')
    y = f(x)
    np.testing.assert_allclose(y.numpy(), ref.numpy(), rtol=1e-4, atol=1e-5)
    # ring order: the same stack stored in rotated slots
    order = [2, 0, 1]
    ring = torch.empty_like(x)
    ring[:, order] = x
    np.testing.assert_allclose(f(ring, order).numpy(), ref.numpy(), rtol=1e-4, atol=1e-5)


def test_fused_reference_mode_dropout_live_and_refresh():
    from aido1_amd.actor import ConfigActor, FusedActor
    a = ConfigActor(golden('reference_config.json')['model']['actor'])
    f = FusedActor(a, dtype=torch.float32, mode='reference')
    assert f.p_drop == 0.5
    x = formula_input(4)
    assert not torch.equal(f(x), f(x))              # dropout is live in train mode
    b = ConfigActor(golden('reference_config.json')['model']['actor'])
    f.refresh(b)
    assert torch.equal(f.w[2], b.layers()[0][2].weight.contiguous(memory_format=torch.channels_last))


@pytest.mark.parametrize('mode', ['reference', 'eval'])
def test_refresh_fragments_match_fragment_builders(mode):
    """refresh() gathers the MFMA fragments through index maps; they equal
    conv1_fragments / conv32_fragments of the weights it derives, and the f32
    biases are the layers' (folded) biases."""
    from aido1_amd.actor import (ConfigActor, FusedActor, conv1_fragments,
                                 conv32_fragments)
    torch.manual_seed(3)
    a = ConfigActor(golden('reference_config.json')['model']['actor'])
    for m in a.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.running_mean.uniform_(-0.5, 0.5)
            m.running_var.uniform_(0.5, 2.0)
    f = FusedActor(a, dtype=torch.float16, mode=mode)
    assert torch.equal(f.w0frag, conv1_fragments(f.w[0].float()))
    for i in range(1, 4):
        assert torch.equal(f.wfrag[i - 1], conv32_fragments(f.w[i].float()))
    convs = a.layers()[0]
    if mode == 'reference':
        for i in range(4):
            assert torch.equal(f.bf[i], convs[i].bias.detach())
    else:
        assert torch.allclose(f.bf, torch.stack([b.float() for b in f.b]), rtol=1e-3, atol=1e-3)


def test_bench_actor_f64_is_batch_of_one_train_mode():
    """bench.actor_f64 (configs 4 / 5's precision yardstick) = the reference's
    act: the train-mode ConfigActor on ONE observation at a time, in float64,
    dropout off (models/ddpg/model.py:74-88)."""
    import bench
    from aido1_amd.actor import ConfigActor
    from test_trainer import no_dropout
    cfg = golden('reference_config.json')
    torch.manual_seed(3)
    a = ConfigActor(no_dropout(cfg['model']['actor']))
    x = torch.rand(3, 3, 120, 160)
    got = bench.actor_f64(a, x)
    a64 = ConfigActor(no_dropout(cfg['model']['actor']))
    a64.load_state_dict(a.state_dict())
    a64.double().train()
    with torch.no_grad():
        want = torch.cat([a64(x[i:i + 1].double()) for i in range(3)])
    torch.testing.assert_close(got, want, rtol=1e-12, atol=1e-12)


def test_bench_actor_f64_eval_mode_uses_running_statistics():
    """bench.actor_f64(mode='eval') = the eval-mode ConfigActor in float64
    (the running statistics: the folded-BN policy's reference)."""
    import bench
    from aido1_amd.actor import ConfigActor
    from test_trainer import no_dropout
    cfg = golden('reference_config.json')
    torch.manual_seed(4)
    a = ConfigActor(no_dropout(cfg['model']['actor']))
    for bn in [m for m in a.modules() if isinstance(m, torch.nn.BatchNorm2d)]:
        bn.running_mean.uniform_(-0.2, 0.2)
        bn.running_var.uniform_(0.5, 2.0)
    x = torch.rand(3, 3, 120, 160)
    got = bench.actor_f64(a, x, 'eval')
    a64 = ConfigActor(no_dropout(cfg['model']['actor']))
    a64.load_state_dict(a.state_dict())
    a64.double().eval()
    with torch.no_grad():
        want = a64(x.double())
    torch.testing.assert_close(got, want, rtol=1e-12, atol=1e-12)
